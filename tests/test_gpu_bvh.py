"""Exact BVH for secondary rays (csrc/iq_bvh.hpp) vs the oracle's brute-force loop
(path_tracer.cu:257-295), bit for bit. Scenes are chosen to stress what could break exactness:
grazing bounces off a finely tessellated floor, duplicated geometry (equal t: the last triangle in
packet order must win), large triangles on the always-tested list next to BVH triangles, and the
C5-style mesh + pebbles with Oren–Nayar mesh triangles."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import MAT_EMISSIVE, MAT_OREN_NAYAR, PathTracer, Scene, _lib, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def bvh_info(pt):
    lib = _lib.load()
    f = lib.iqpt_debug_bvh_info
    f.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    n, a = C.c_uint32(), C.c_uint32()
    _lib.check(f(pt._h, C.byref(n), C.byref(a)), "iqpt_debug_bvh_info")
    return n.value, a.value


def run_both(scene, w, h, spp, depth, pixels=None, seed=1984, cam=None, launches=None):
    pk = scene.build_packet()
    cam = cam or make_camera(w, h)
    pt = PathTracer(w, h, pixels=pixels, seed=seed, max_depth=depth)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=pixels, seed=seed, max_depth=depth)
    for s in (launches or [spp]):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    return pt, fr


def grid(n, size):
    """n x n quads in the xz plane, [-size/2, size/2]^2, normals +y."""
    xs = np.linspace(-size / 2, size / 2, n + 1, dtype=np.float64)
    X, Z = np.meshgrid(xs, xs, indexing="ij")
    v = np.zeros(((n + 1) ** 2, 6), np.float32)
    v[:, 0], v[:, 2], v[:, 4] = X.ravel(), Z.ravel(), 1.0
    idx = []
    for i in range(n):
        for j in range(n):
            a, b, c, d = i * (n + 1) + j, (i + 1) * (n + 1) + j, (i + 1) * (n + 1) + j + 1, i * (n + 1) + j + 1
            idx += [a, b, c, a, c, d]
    return v, np.array(idx, np.uint32)


def test_grazing_bounces_on_a_tessellated_floor(require_gpu):
    sc = Scene()
    v, i = grid(40, 4.0)                                  # 3200 triangles of 0.1
    sc.add_mesh("floor", v, i)
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("floor", "floor", 1.0, 0.0, (0.0, 0.0, 0.0))
    sc.add_model("ball", "sphere", 0.3, 0.0, (0.0, 0.3, 0.4))
    sc.add_model("lamp", "sphere", 0.25, 0.0, (0.9, 1.4, 0.2))
    sc.set_model_material("floor", sc.add_material(MAT_OREN_NAYAR, (0.8, 0.8, 0.8, 0.0), 0.3))
    sc.set_model_material("ball", sc.add_material(MAT_OREN_NAYAR, (0.9, 0.5, 0.3, 0.0), 0.8))
    sc.set_model_material("lamp", sc.add_material(MAT_EMISSIVE, (1.0, 1.0, 1.0, 1.0), 9.0))
    # a low camera: primary rays graze the floor, bounces off the ball's base skim it
    cam = make_camera(96, 64, position=(0.0, 0.06, -2.0, 0.0), forward=(0.0, -0.01, 1.0, 0.0))
    pt, _ = run_both(sc, 96, 64, 3, 6, cam=cam)
    nodes, always = bvh_info(pt)
    assert nodes > 0 and always == 0


def test_duplicated_mesh_resolves_ties_like_the_loop(require_gpu):
    """Two copies of the same mesh at the same place: every hit is an exact tie, which the reference
    resolves to the later triangle (t == closest is accepted, path_tracer.cu:266)."""
    sc = Scene()
    sc.add_mesh_uv_sphere("ball", False, 24, 12, 0)      # 576 triangles
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("a", "ball", 0.5, (0.1, 0.2, 0.0), (0.0, 0.5, 0.0))
    sc.add_model("b", "ball", 0.5, (0.1, 0.2, 0.0), (0.0, 0.5, 0.0))
    sc.add_model("ground", "sphere", 10.0, 0.0, (0.0, -10.0, 0.0))
    sc.add_model("lamp", "sphere", 0.3, 0.0, (0.8, 1.3, -0.5))
    sc.set_model_material("a", sc.add_material(MAT_OREN_NAYAR, (0.9, 0.1, 0.1, 0.0), 0.5))
    sc.set_model_material("b", sc.add_material(MAT_OREN_NAYAR, (0.1, 0.9, 0.1, 0.0), 0.5))
    sc.set_model_material("lamp", sc.add_material(MAT_EMISSIVE, (1.0, 1.0, 1.0, 1.0), 8.0))
    pt, fr = run_both(sc, 80, 60, 3, 6)
    assert bvh_info(pt)[0] > 0
    # the second copy's colour wins wherever the ball is seen
    rgb = fr.lin[:, :3]
    assert (rgb[:, 1] > rgb[:, 0]).sum() > (rgb[:, 0] > rgb[:, 1]).sum()


def test_large_walls_stay_out_of_the_bvh(require_gpu):
    """Cornell walls (R > 1/4: tested by every ray) around a dense Oren–Nayar mesh in the BVH."""
    sc = Scene()
    sc.add_preset("cornell_lit")
    sc.add_mesh_uv_sphere("ball", False, 40, 20, 0)      # 1600 triangles
    sc.add_model("mesh", "ball", 0.3, 0.0, (0.2, 0.0, 0.3))
    sc.set_model_material("mesh", sc.add_material(MAT_OREN_NAYAR, (0.6, 0.6, 0.9, 0.0), 0.6))
    pt, _ = run_both(sc, 96, 64, 3, 8)
    nodes, always = bvh_info(pt)
    assert nodes > 0 and always >= 12                     # the six quads' 12 triangles


@pytest.mark.parametrize("preset,w,h,crop", [
    ("mesh10k", 1920, 1080, (900, 1000, 300, 7, 16)),
    ("mixed", 3840, 2160, (1700, 2100, 900, 11, 12)),
])
def test_presets_with_materials(require_gpu, preset, w, h, crop):
    """C4 / C5 geometry with an Oren–Nayar mesh and an emissive lamp: long secondary paths through
    the BVH (with the reference's materials a mesh hit ends the path)."""
    sc = Scene()
    sc.add_preset(preset)
    sc.add_mesh_uv_sphere("lampmesh")
    sc.add_model("lamp", "lampmesh", 0.4, 0.0, (1.0, 1.6, -0.6))
    sc.set_model_material("ball", sc.add_material(MAT_OREN_NAYAR, (0.7, 0.7, 0.7, 0.0), 0.4))
    sc.set_model_material("lamp", sc.add_material(MAT_EMISSIVE, (1.0, 0.9, 0.8, 1.0), 10.0))
    pt, _ = run_both(sc, w, h, 2, 8, pixels=pixel_set(w, h, *crop))
    assert bvh_info(pt)[0] > 0


def test_camera_ray_path_switch_between_launches(require_gpu):
    """The first two launches of a streamed scene with a BVH time the tile-mask and the BVH camera-ray
    kernels, later launches use the faster: every launch continues the same frame sequence."""
    sc = Scene()
    sc.add_preset("mixed")
    w, h = 3840, 2160
    pt, _ = run_both(sc, w, h, 0, 8, pixels=pixel_set(w, h, 1800, 2000, 1000, 13, 8), launches=[1, 2, 1, 1])
    assert pt.frames() == 5


@pytest.mark.parametrize("anyhit", [1, 0])
def test_anyhit_variants_on_c4(require_gpu, anyhit):
    """C4 geometry (triangles only, the reference's materials: every triangle emissive) over launches that
    time and then use both camera-ray paths (tile lists and the BVH): with any-hit on, the launches run the
    kOptAnyHit variants (first accepted triangle ends a ray, lists ordered by hit count), off the closest-hit
    ones; both equal the oracle bit for bit (round 5)."""
    import ctypes as C
    from iqpt import _lib
    sc = Scene()
    sc.add_preset("mesh10k")
    w, h = 1920, 1080
    pk = sc.build_packet()
    cam = make_camera(w, h)
    ps = pixel_set(w, h, 880, 1040, 420, 9, 14)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    lb = _lib.load()
    lb.iqpt_debug_set_anyhit.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_anyhit(pt._h, anyhit), "iqpt_debug_set_anyhit")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    for s in (2, 1, 1, 1, 3):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    opt = C.c_int(0)
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(opt)), "iqpt_debug_last_options")
    assert bool(opt.value & (1 << 20)) == bool(anyhit), hex(opt.value)      # kOptAnyHit


@pytest.mark.parametrize("preset,w,h,ps_args,launches", [
    ("mixed", 3840, 2160, (1700, 2100, 1000, 11, 6), [16, 3, 16]),      # C5 geometry, the bench's 16 spp
    ("mesh10k", 1920, 1080, (860, 1060, 420, 9, 10), [8, 1, 5]),        # C4 geometry (any-hit variants)
])
@pytest.mark.parametrize("refill", [1, 16, 64])
def test_stream_refill_group_sizes(require_gpu, preset, w, h, ps_args, launches, refill):
    """Streamed-scene launches whose waves take new pixels only once `refill` lanes are idle (64, whole waves, by
    default since round 5: a tile's pixels together; 1 = a refill at every iteration with an idle lane): the
    pixels' results do not depend on when a lane takes them — bit-exact against the oracle."""
    sc = Scene()
    sc.add_preset(preset)
    pk = sc.build_packet()
    cam = make_camera(w, h)
    ps = pixel_set(w, h, *ps_args)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    lb = _lib.load()
    lb.iqpt_debug_set_stream_refill.argtypes = [C.c_void_p, C.c_uint32]
    _lib.check(lb.iqpt_debug_set_stream_refill(pt._h, refill), "iqpt_debug_set_stream_refill")
    assert lb.iqpt_debug_set_stream_refill(pt._h, 0) != 0 and lb.iqpt_debug_set_stream_refill(pt._h, 65) != 0
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("preset,w,h,ps_args,launches", [
    ("mesh10k", 1920, 1080, (0, 1920, 300, 7, 9), [2, 1]),            # C4 geometry, 17,280 pixels
    ("mixed", 3840, 2160, (0, 3840, 900, 9, 5), [1]),                 # C5 geometry, 19,200 pixels
])
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_stream_xcd_tile_lists(require_gpu, preset, w, h, ps_args, launches, mode):
    """Streamed-scene launches whose tiles are dealt to the 8 XCDs (iqpt_debug_set_stream_xcd: 1 the cost order
    round-robin, 2 bands of tile rows round-robin, 3 the default: 1 for launches of up to 4 samples), each XCD
    taking its own list from its own queue word; the kernel's last block checks that every list was taken. Pixel
    sets of more than 64 blocks, so the lists are used — and the launches must report that they were (bit 30 of
    iqpt_debug_last_options; the runtime falls back to one queue silently on other devices or grids).
    Bit-exact against the oracle."""
    sc = Scene()
    sc.add_preset(preset)
    pk = sc.build_packet()
    cam = make_camera(w, h)
    ps = pixel_set(w, h, *ps_args)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    lb = _lib.load()
    lb.iqpt_debug_set_stream_xcd.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_stream_xcd(pt._h, mode), "iqpt_debug_set_stream_xcd")
    # (the plain kernel's lists: C4's any-hit scene would otherwise take iqpt_anyhit_kernel, which has no queue)
    lb.iqpt_debug_set_pixel_masks.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_pixel_masks(pt._h, 1), "iqpt_debug_set_pixel_masks")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
        o = C.c_int(0)
        _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
        assert o.value & (1 << 30), hex(o.value)     # every launch here has <= 4 spp: per-XCD lists in mode 3 too
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
