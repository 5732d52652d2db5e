"""Certain-miss pixels (kparams::miss, iqpt_sky_kernel): a pixel whose own camera-ray bundle
culls every candidate primitive of its tile (iq_interval.h tri_culled / sphere_culled) ends every sample on the
sky gradient of its camera ray after the camera's two draws (path_tracer.cu:307-316, camera.cu:24-25). Plain
launches hand such pixels to the sky kernel and the plain kernel skips them. Bit for bit against the oracle
(accumulator, BGRA8, RNG states, ray counts) and against the same launches with the path off. RMSE < 1e-5."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5


def _lib():
    from iqpt import _lib as L
    lib = L.load()
    lib.iqpt_debug_set_sky.argtypes = [C.c_void_p, C.c_int]
    lib.iqpt_debug_sky_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    return L, lib


def _render(preset, w, h, launches, sky=True, ps=None, overlap=True, frame0=None, depth=8):
    from iqpt import PathTracer, make_camera
    L, lib = _lib()
    sc, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=depth)
    pt.set_split(L.SPLIT_OFF)
    if not overlap:
        pt.set_overlap(L.OVERLAP_OFF)
    L.check(lib.iqpt_debug_set_sky(pt.handle, 1 if sky else 0), "iqpt_debug_set_sky")
    if frame0 is not None:
        lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
        L.check(lib.iqpt_debug_set_frame(pt.handle, frame0), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
    lin, bgra = pt.read()
    px, tl = C.c_uint32(0), C.c_uint32(0)
    L.check(lib.iqpt_debug_sky_info(pt.handle, C.byref(px), C.byref(tl)), "iqpt_debug_sky_info")
    pt._scene = sc                      # the scene owns the packet's arrays: keep it alive with the context
    return pt, lin, bgra, px.value, pk, cam


def _oracle(pk, cam, w, h, launches, ps=None, frame0=None, depth=8):
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=depth)
    if frame0 is not None:
        fr.frame = frame0
    for s in launches:
        fr.render(pk, cam, s)
    return fr


@pytest.mark.parametrize("overlap", [True, False])
def test_sky_pixels_cornell_match_oracle(require_gpu, overlap):
    """A 480x270 Cornell frame (a third of it sky beside and below the box) over three launches: the sky
    kernel's pixels and the plain kernel's together are the oracle's frame bit for bit."""
    w, h, launches = 480, 270, [7, 64, 3]
    pt, lin, bgra, nsky, pk, cam = _render("cornell", w, h, launches, overlap=overlap)
    assert nsky > w * h // 5, nsky
    fr = _oracle(pk, cam, w, h, launches)
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()


def test_sky_on_equals_sky_off(require_gpu):
    """The same launches with certain misses traced by the plain kernel: identical state and ray counts."""
    w, h, launches = 320, 180, [16, 5]
    a, lin_a, bgra_a, n_a, _, _ = _render("cornell", w, h, launches, sky=True)
    b, lin_b, bgra_b, n_b, _, _ = _render("cornell", w, h, launches, sky=False)
    assert n_a > 0
    assert np.array_equal(lin_a.view(np.uint32), lin_b.view(np.uint32))
    assert np.array_equal(bgra_a, bgra_b)
    assert np.array_equal(a.read_rng(), b.read_rng())
    assert a.rays() == b.rays()
    a.close()
    b.close()


@pytest.mark.parametrize("preset,depth", [("app_default", 5), ("c1_plumbing", 2)])
def test_sky_pixels_other_scenes(require_gpu, preset, depth):
    """Scenes with a triangle light and spheres over open sky: ragged edge tiles (W, H not multiples of 8)."""
    w, h, launches = 203, 117, [9, 2]
    pt, lin, bgra, nsky, pk, cam = _render(preset, w, h, launches, depth=depth)
    fr = _oracle(pk, cam, w, h, launches, depth=depth)
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()


def test_sky_row_share_and_large_frame_counter(require_gpu):
    """Rank 1's rows of a 3-way split, frame counter beyond 2^32 (the table's n and the mean's tiny threshold)."""
    w, h, launches = 256, 144, [4, 4]
    ps = pixel_set(w, h, 0, w, 1, 3)
    f0 = (1 << 33) + 17
    pt, lin, bgra, nsky, pk, cam = _render("cornell", w, h, launches, ps=ps, frame0=f0)
    fr = _oracle(pk, cam, w, h, launches, ps=ps, frame0=f0)
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(pt.read_rng(), fr.states)
    pt.close()


@pytest.mark.parametrize("after", [0, 1])
def test_sky_kernel_ahead_of_and_behind_the_plain_kernel(require_gpu, after):
    """Overlapped launches with the sky kernel queued ahead of or behind (the default) the plain kernel
    (iqpt_debug_set_sky_order): the oracle's bits, four launches on alternating streams."""
    from iqpt import PathTracer, make_camera
    L, lib = _lib()
    lib.iqpt_debug_set_sky_order.argtypes = [C.c_void_p, C.c_int]
    w, h, launches = 480, 270, [16, 8, 64, 3]
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt._scene = sc
    pt.set_split(L.SPLIT_OFF)
    L.check(lib.iqpt_debug_set_sky_order(pt.handle, after), "iqpt_debug_set_sky_order")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
    lin, bgra = pt.read()
    fr = _oracle(pk, cam, w, h, launches)
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()


@pytest.mark.parametrize("split", ["spec"])
def test_sky_with_more_than_64_spheres(require_gpu, split):
    """a resident scene of more than 64 spheres skips the per-pixel sphere test of the split
    tiles, so every pixel of a split tile went to the spec / chain kernel's list — the certain misses too, which
    the sky kernel also renders on the other stream. The Cornell box plus 70 small spheres (a grid above the
    floor, resident in LDS), a row share, spec and chain launches with the sky kernel on: bit for bit against
    the oracle, and the sky kernel still has pixels. (Round 6 archived the chain kernel and queue mode.)"""
    from iqpt import PathTracer, make_camera
    L, lib = _lib()
    from iqpt.scene import Scene
    sc = Scene()
    sc.add_preset("cornell")
    for i in range(70):
        x, z = -0.9 + 0.26 * (i % 7), -0.4 + 0.12 * (i // 7)
        sc.add_model(f"ball{i}", "sphere", scale=0.04, translation=(x, -0.45, z, 0.0))
    pk = sc.build_packet()
    assert int(pk.num_drawcalls[L.MESH_SPHERES]) == 72
    w, h, world, rank = 480, 270, 4, 1
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(L.SPLIT_SPEC)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    for s in (8, 24):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    px, tiles = C.c_uint32(0), C.c_uint32(0)
    L.check(lib.iqpt_debug_sky_info(pt.handle, C.byref(px), C.byref(tiles)), "iqpt_debug_sky_info")
    assert px.value > 0
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()
