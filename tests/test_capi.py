"""The C-ABI library: loads without a GPU, exports every symbol include/iqpt.h declares, and the
host-only entry points (scene builder, camera, PPM, errors) behave; no kernel is launched here."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import iqpt
from iqpt import _lib

HEADER = Path(__file__).resolve().parent.parent / "include" / "iqpt.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(iqpt_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound():
    lib = iqpt.load()
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_abi_version_and_error_strings():
    lib = iqpt.load()
    # 2: packet material table; 3: split mode, prepare, frame copy; 4: RCCL gather; 5: gather_read_select;
    # 6: CHAIN / FAN launch modes refused (archived)
    assert lib.iqpt_abi_version() == 6
    assert lib.iqpt_error_string(0) == b"IQPT_OK"
    assert lib.iqpt_error_string(4) == b"IQPT_ERR_NO_DEVICE"
    assert lib.iqpt_error_string(99) == b"IQPT_ERR_UNKNOWN"


def test_create_validates_arguments_before_touching_the_device():
    lib = iqpt.load()
    h = C.c_void_p()
    assert lib.iqpt_create(0, 0, 10, None, 1984, 5, C.byref(h)) == 1
    assert b"frame" in lib.iqpt_last_error()
    assert lib.iqpt_create(0, 10, 10, None, 1984, 0, C.byref(h)) == 1
    assert lib.iqpt_create(0, 10, 10, None, 1984, 99, C.byref(h)) == 6
    bad = _lib.PixelSet(0, 11, 0, 1, 10)
    assert lib.iqpt_create(0, 10, 10, C.byref(bad), 1984, 5, C.byref(h)) == 1
    with pytest.raises(iqpt.IqptError) as e:
        iqpt.PathTracer(10, 10, max_depth=0)
    assert e.value.status == 1
    assert lib.iqpt_render(None, 1) == 1
    assert lib.iqpt_read(None, None, None) == 1


def test_scene_preset_stats_match_the_survey():
    expect = {"c1_plumbing": (224, 1), "cornell": (10, 2), "mesh10k": (10_000, 0), "mixed": (50_000, 1000),
              "app_default": (12, 2)}
    for preset, (t, s) in expect.items():
        sc = iqpt.Scene()
        sc.add_preset(preset)
        st = iqpt.packet_stats(sc.build_packet())
        assert (st["triangles"], st["spheres"]) == (t, s), preset
    with pytest.raises(iqpt.IqptError):
        iqpt.Scene().add_preset("nope")


@pytest.mark.parametrize("segments,rings", [(16, 8), (32, 16), (100, 51), (3, 3), (7, 5)])
def test_uv_sphere_counts_and_indices(segments, rings):
    """mesh.cu:190-279: (rings-1)*segments + 2 vertices, 2*segments*(rings-1) triangles."""
    sc = iqpt.Scene()
    sc.add_mesh_uv_sphere("m", False, segments, rings, iqpt.MESH_TRIANGLES)
    sc.add_model("x", "m")
    pk = sc.build_packet()
    m = pk.tri_meshes[0]
    assert m.num_vertices == (rings - 1) * segments + 2
    assert m.num_indices == 3 * 2 * segments * (rings - 1)
    idx = np.ctypeslib.as_array(m.indices, shape=(m.num_indices,))
    assert idx.max() < m.num_vertices
    v = np.ctypeslib.as_array(C.cast(m.vertices, C.POINTER(C.c_float)), shape=(m.num_vertices * 6,)).reshape(-1, 6)
    r = np.linalg.norm(v[:, :3], axis=1)
    assert np.allclose(r, 1.0, atol=1e-5)                     # unit sphere, normals = positions
    assert np.array_equal(v[:, :3], v[:, 3:])


def test_quad_cube_polygon_tri():
    sc = iqpt.Scene()
    sc.add_mesh_quad("a_quad")
    sc.add_mesh_cube("b_cube")
    sc.add_mesh_reg_polygon("c_poly", 6)
    sc.add_mesh_tri("d_tri")
    for n, m in (("q", "a_quad"), ("c", "b_cube"), ("p", "c_poly"), ("t", "d_tri")):
        sc.add_model(n, m)
    pk = sc.build_packet()
    got = [(pk.tri_meshes[i].num_vertices, pk.tri_meshes[i].num_indices) for i in range(pk.num_tri_meshes)]
    assert got == [(4, 6), (24, 36), (7, 18), (3, 3)]
    assert [pk.tri_mesh_dcs[i].mesh_id for i in range(4)] == [0, 1, 2, 3]


def test_build_packet_sorted_names_and_mesh_id_quirk():
    """scene.cu:161-181: drawcalls in mesh-name order, mesh_id = position among ALL mesh names —
    so a sphere mesh sorting before a triangle mesh makes mesh_id skip past the compacted array."""
    sc = iqpt.Scene()
    sc.add_mesh_uv_sphere("a_sphere")                          # SPHERES, sorts first
    sc.add_mesh_quad("b_quad")
    sc.add_model("q", "b_quad", translation=(1, 2, 3))
    sc.add_model("s", "a_sphere", scale=0.5, translation=(4, 5, 6))
    pk = sc.build_packet()
    assert pk.num_tri_meshes == 1
    assert pk.num_drawcalls[0] == 1 and pk.num_drawcalls[1] == 1
    assert pk.tri_mesh_dcs[0].mesh_id == 1                     # out of range of tri_meshes[1]
    assert pk.sphere_dcs[0].radius == np.float32(0.5)
    assert list(pk.sphere_dcs[0].center)[:3] == [4.0, 5.0, 6.0]
    t = np.array(pk.tri_mesh_dcs[0].transform).reshape(4, 4)
    assert list(t[3, :3]) == [1.0, 2.0, 3.0]                   # translation in row 3 (row vectors)


def test_model_transform_order_scale_rotation_translation():
    """model.cu:11-18: s * rx * ry * rz * t with row vectors."""
    sc = iqpt.Scene()
    sc.add_mesh_quad("q")
    sc.add_model("m", "q", scale=(2, 3, 4, 1), rotation=(0, np.pi / 2, 0, 0), translation=(1, 0, 0, 0))
    t = np.array(sc.build_packet().tri_mesh_dcs[0].transform, dtype=np.float64).reshape(4, 4)
    c, s = np.cos(np.float32(np.pi / 2)), np.sin(np.float32(np.pi / 2))
    ry = np.eye(4); ry[0, 0] = c; ry[0, 2] = -s; ry[2, 0] = s; ry[2, 2] = c
    expect = np.diag([2, 3, 4, 1]) @ ry
    expect[3, :3] += [1, 0, 0]
    assert np.allclose(t, expect, atol=1e-6)


def test_camera_matrices():
    """camera.cu:5-18: inverse matrices invert view/projection; the defaults of camera.h."""
    cam = iqpt.make_camera(1920, 1080)
    assert (cam.width, cam.height) == (1920, 1080) and cam.fovh == 45.0
    for a, b in (("view", "inv_view"), ("projection", "inv_proj")):
        m = np.array(getattr(cam, a), dtype=np.float64).reshape(4, 4)
        mi = np.array(getattr(cam, b), dtype=np.float64).reshape(4, 4)
        assert np.allclose(m @ mi, np.eye(4), atol=1e-5)
    p = np.array(cam.projection).reshape(4, 4)
    assert np.isclose(p[1, 1], 1 / np.tan(np.radians(22.5)), rtol=1e-6)
    assert np.isclose(p[0, 0], p[1, 1] / (1920 / 1080), rtol=1e-6)
    assert p[2, 3] == 1.0
    assert list(cam.position) == [0.0, 0.5, -3.0, 0.0] and list(cam.forward) == [0.0, -0.5, 3.0, 0.0]


def test_write_ppm(tmp_path):
    bgra = np.zeros((2, 3, 4), dtype=np.uint8)
    bgra[..., 0] = 10; bgra[..., 1] = 20; bgra[..., 2] = 30; bgra[..., 3] = 255
    p = tmp_path / "x.ppm"
    iqpt.write_ppm(str(p), 3, 2, bgra.reshape(-1, 4))
    data = p.read_bytes()
    assert data.startswith(b"P6\n3 2\n255\n")
    assert data[len(b"P6\n3 2\n255\n"):][:3] == bytes([30, 20, 10])
