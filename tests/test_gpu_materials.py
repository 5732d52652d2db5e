"""Material-table kernel variant (kOptMaterials) vs the oracle, bit for bit: Oren–Nayar
triangles (interpolated vertex normals, front-face flip, shape.cu:93-101), emissive spheres, coloured
albedo (RGB scatter records), roughness range, the LDS-streamed path, and a table that spells out the
reference's own materials (which must reproduce the default kernel's frame exactly)."""
import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import MAT_EMISSIVE, MAT_OREN_NAYAR, PathTracer, Scene, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def run_both(scene, w, h, launches, depth, pixels=None, seed=1984):
    pk = scene.build_packet()
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=pixels, seed=seed, max_depth=depth)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=pixels, seed=seed, max_depth=depth)
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    return pt, fr


@pytest.mark.parametrize("depth", [1, 3, 8])
def test_lit_cornell_box(require_gpu, depth):
    sc = Scene()
    sc.add_preset("cornell_lit")
    run_both(sc, 96, 64, [3, 2], depth)


def test_lit_cornell_box_full_width_band(require_gpu):
    sc = Scene()
    sc.add_preset("cornell_lit")
    run_both(sc, 320, 180, [4], 8, pixels=pixel_set(320, 180, 0, 320, 60, 1, 24))


def test_reference_materials_as_a_table_equal_the_default_kernel(require_gpu):
    a = Scene()
    a.add_preset("cornell")
    b = Scene()
    b.add_preset("cornell")
    em = b.add_material(MAT_EMISSIVE, (1.0, 1.0, 1.0, 1.0), 10.0)
    on = b.add_material(MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 1.0)
    for m in ("back", "floor", "ceiling", "left", "right"):
        b.set_model_material(m, em)
    for m in ("sphere_big", "sphere_small"):
        b.set_model_material(m, on)
    pa, _ = run_both(a, 80, 48, [3], 8)
    pb, _ = run_both(b, 80, 48, [3], 8)
    assert np.array_equal(pa.read()[0].view(np.uint32), pb.read()[0].view(np.uint32))


def test_emissive_spheres_and_rough_triangles(require_gpu):
    sc2 = Scene()
    sc2.add_mesh_cube("cube")
    sc2.add_mesh_uv_sphere("sphere")
    sc2.add_model("cube", "cube", 0.6, (0.3, 0.5, 0.0), (0.0, 0.3, 0.5))
    sc2.add_model("lamp", "sphere", 0.2, 0.0, (0.7, 0.9, 0.2))
    sc2.add_model("ground", "sphere", 10.0, 0.0, (0.0, -10.0, 0.0))
    sc2.set_model_material("cube", sc2.add_material(MAT_OREN_NAYAR, (0.8, 0.3, 0.1, 0.0), 0.0))
    sc2.set_model_material("lamp", sc2.add_material(MAT_EMISSIVE, (1.0, 0.8, 0.6, 1.0), 6.0))
    sc2.set_model_material("ground", sc2.add_material(MAT_OREN_NAYAR, (0.4, 0.4, 0.45, 0.0), 0.7))
    run_both(sc2, 80, 60, [4], 6)


def test_streamed_scene_with_materials(require_gpu):
    """> 32 KiB of triangles: the LDS-batch path with Oren–Nayar mesh triangles."""
    sc = Scene()
    sc.add_mesh_uv_sphere("ball", False, 30, 16, 0)          # 900 triangles
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("ball", "ball", 0.5, (0.2, 0.1, 0.0), (0.0, 0.4, 0.3))
    sc.add_model("light", "sphere", 0.3, 0.0, (0.8, 1.2, -0.4))
    sc.add_model("ground", "sphere", 10.0, 0.0, (0.0, -10.0, 0.0))
    sc.set_model_material("ball", sc.add_material(MAT_OREN_NAYAR, (0.9, 0.9, 0.9, 0.0), 0.4))
    sc.set_model_material("light", sc.add_material(MAT_EMISSIVE, (1.0, 1.0, 1.0, 1.0), 8.0))
    run_both(sc, 96, 64, [2], 5, pixels=pixel_set(96, 64, 16, 80, 8, 1, 40))


@pytest.mark.parametrize("frame0", [0, 2 ** 33, 2 ** 40])
def test_tiny_colours_and_large_frame_counters(require_gpu, frame0):
    """The running mean's short division (Markstein with RN(1/n) from the table) is exact only while
    c / n is normal: colours near 2^-90 after 2^33 or 2^40 frames give subnormal quotients and must
    take the IEEE division (kparams::mean_tiny), colours near 2^-100 and exact zeros too."""
    import ctypes as C
    from iqpt import _lib
    sc = Scene()
    sc.add_mesh_quad("quad")
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("wall", "quad", 3.0, 0.0, (0.0, 0.5, 1.0))
    sc.add_model("floor", "quad", 3.0, (1.5707963267948966, 0, 0), (0.0, -0.5, 0.0))
    sc.add_model("ball", "sphere", 0.35, 0.0, (0.0, 0.1, 0.3))
    sc.set_model_material("wall", sc.add_material(MAT_EMISSIVE, (2.0 ** -88, 2.0 ** -92, 0.25, 1.0), 1.0))
    sc.set_model_material("floor", sc.add_material(MAT_EMISSIVE, (2.0 ** -100, 0.0, 2.0 ** -80, 1.0), 1.0))
    sc.set_model_material("ball", sc.add_material(MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 0.5))
    pk = sc.build_packet()
    w, h = 64, 48
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=4)
    lib = _lib.load()
    lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
    _lib.check(lib.iqpt_debug_set_frame(pt._h, frame0), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=4)
    fr.frame = frame0
    for s in (3, 2):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    if frame0:
        assert np.any((lin[:, :3] > 0) & (lin[:, :3] < 2.0 ** -126))   # subnormal means were produced
