"""Sample-parallel chains (kOptSplit) vs the CPU oracle, bit for bit.

Split mode evaluates a sample at every even XORWOW offset of a window in parallel and stitches the
chain afterwards (iqpt_split_prep_kernel, the render kernel's rounds 1 and 2, iqpt_split_stitch_kernel).
It must reproduce the reference's sequential chain exactly: the accumulator, BGRA8, the final RNG
states and the ray count (path_tracer.cu:330-366, random.cu:66-107). Tolerance stated anyway: RMSE < 1e-5.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, gpu_render, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5
K_OPT_SPLIT = 1 << 16
SPLIT_ON, SPLIT_OFF = 1, 0


def last_options(pt):
    from iqpt import _lib
    lb = _lib.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    o = C.c_int()
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
    return o.value


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches", [[16], [8, 8, 8], [3, 1, 40]])
def test_cornell_crop_split(require_gpu, launches):
    """C2 crop through both spheres; later launches size their windows from the previous chains."""
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    pt, lin, bgra = gpu_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches, split=SPLIT_ON)
    assert last_options(pt) & K_OPT_SPLIT
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (1, 3)])
def test_row_share_split(require_gpu, rank, world):
    """A rank's cyclic row share of a 480x270 Cornell frame (the multi-GPU partition)."""
    w, h = 480, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12], split=SPLIT_ON)
    assert last_options(pt) & K_OPT_SPLIT
    fr = oracle_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("depth", [1, 2, 8])
def test_material_table_split(require_gpu, depth):
    """Lit Cornell box (Oren-Nayar walls: every tile is split, RGB records) at several depths."""
    ps = pixel_set(320, 180, 96, 224, 40, 2, 48)
    pt, lin, bgra = gpu_render("cornell_lit", 320, 180, 0, depth, pixels=ps, launches=[6, 10], split=SPLIT_ON)
    assert last_options(pt) & K_OPT_SPLIT
    fr = oracle_render("cornell_lit", 320, 180, 0, depth, pixels=ps, launches=[6, 10])
    _check(pt, lin, bgra, fr)


def test_deep_paths_split(require_gpu):
    """max_depth 16 (the MAXD-16 variant): long chains of sphere bounces, windows capped at 3 spp."""
    pt, lin, bgra = gpu_render("app_default", 160, 90, 0, 16, launches=[20, 20], split=SPLIT_ON)
    assert last_options(pt) & K_OPT_SPLIT
    fr = oracle_render("app_default", 160, 90, 0, 16, launches=[20, 20])
    _check(pt, lin, bgra, fr)


def test_long_launch_split(require_gpu):
    """One launch of 300 samples (windows of 450 slots, run length 57) over a small crop."""
    ps = pixel_set(640, 360, 300, 332, 150, 1, 16)
    pt, lin, bgra = gpu_render("cornell", 640, 360, 300, 8, pixels=ps, split=SPLIT_ON)
    fr = oracle_render("cornell", 640, 360, 300, 8, pixels=ps)
    _check(pt, lin, bgra, fr)


def test_split_on_off_identical(require_gpu):
    """The same context state rendered with and without split: identical bits everywhere."""
    w, h = 320, 180
    outs = []
    for mode in (SPLIT_OFF, SPLIT_ON):
        pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, launches=[5, 7], split=mode)
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), last_options(pt)))
        pt.close()
    assert not outs[0][4] & K_OPT_SPLIT and outs[1][4] & K_OPT_SPLIT
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


def test_large_frame_counter_split(require_gpu):
    """Running mean at frame counters beyond 2^32 (the 64-bit conversions and the tiny-colour path)."""
    from iqpt import PathTracer, _lib, make_camera
    frame0 = 1 << 33
    w, h = 96, 64
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_ON)
    lib = _lib.load()
    lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
    _lib.check(lib.iqpt_debug_set_frame(pt._h, frame0), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    fr.frame = frame0
    for s in (4, 9):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert last_options(pt) & K_OPT_SPLIT
    _check(pt, lin, bgra, fr)
