"""Chain-parallel pixels (IQPT_SPLIT_CHAIN, iqpt_chain_kernel) vs the CPU oracle, bit for bit.

The split set's pixels are evaluated by groups of lanes at consecutive even XORWOW offsets and folded in
sample order as the results arrive, beside the plain kernel over the other tiles. That must reproduce the
reference's sequential per-pixel chain exactly: accumulator, BGRA8, final RNG states and the ray count
(path_tracer.cu:330-366, random.cu:66-107). Tolerance stated anyway: RMSE < 1e-5.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, gpu_render, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5
SPLIT_OFF, SPLIT_CHAIN = 0, 2


def ran_chain(pt) -> bool:
    from iqpt import _lib
    lb = _lib.load()
    lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    info = (C.c_ulonglong * 8)()
    _lib.check(lb.iqpt_debug_split_info(pt._h, info), "iqpt_debug_split_info")
    return info[7] in (2, 4)     # chain (anchored tiles plain) or chain + fan


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches", [[16], [8, 8, 8], [3, 1, 40]])
def test_cornell_crop_chain(require_gpu, launches):
    """C2 crop through both spheres: long scatter chains, several launches (frame counter continues)."""
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    pt, lin, bgra = gpu_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches, split=SPLIT_CHAIN)
    assert ran_chain(pt)
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (1, 3), (0, 2)])
def test_row_share_chain(require_gpu, rank, world):
    """A rank's cyclic row share of a 480x270 Cornell frame (the multi-GPU partition)."""
    w, h = 480, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12], split=SPLIT_CHAIN)
    assert ran_chain(pt)
    fr = oracle_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("depth", [1, 2, 3, 16])
def test_depths_chain(require_gpu, depth):
    """max_depth 1 (every sphere hit ends on a scatter: two slots per sample), 2, 3 and 16 (MAXD 16)."""
    pt, lin, bgra = gpu_render("app_default", 160, 90, 0, depth, launches=[20, 7], split=SPLIT_CHAIN)
    assert ran_chain(pt)
    fr = oracle_render("app_default", 160, 90, 0, depth, launches=[20, 7])
    _check(pt, lin, bgra, fr)


def test_long_launch_chain(require_gpu):
    """One launch of 300 samples over a small crop (many ring wraps per pixel)."""
    ps = pixel_set(640, 360, 300, 332, 150, 1, 16)
    pt, lin, bgra = gpu_render("cornell", 640, 360, 300, 8, pixels=ps, split=SPLIT_CHAIN)
    assert ran_chain(pt)
    fr = oracle_render("cornell", 640, 360, 300, 8, pixels=ps)
    _check(pt, lin, bgra, fr)


def test_one_sample_chain(require_gpu):
    """spp = 1 per launch: the chain ends at its first slot every launch."""
    pt, lin, bgra = gpu_render("cornell", 200, 120, 0, 8, launches=[1, 1, 1, 2], split=SPLIT_CHAIN)
    assert ran_chain(pt)
    fr = oracle_render("cornell", 200, 120, 0, 8, launches=[1, 1, 1, 2])
    _check(pt, lin, bgra, fr)


def test_materials_fall_back(require_gpu):
    """A packet with a material table is not taken by the chain kernel; results stay exact."""
    ps = pixel_set(320, 180, 96, 224, 40, 2, 48)
    pt, lin, bgra = gpu_render("cornell_lit", 320, 180, 0, 8, pixels=ps, launches=[6, 10], split=SPLIT_CHAIN)
    assert not ran_chain(pt)
    fr = oracle_render("cornell_lit", 320, 180, 0, 8, pixels=ps, launches=[6, 10])
    _check(pt, lin, bgra, fr)


def test_c3_share_chain_vs_plain(require_gpu):
    """Rank 0's N = 8 row share of the full C3 frame (1920x1080, 64 spp, 8 bounces), two launches: the chain
    launch equals the plain kernel bit for bit (the plain kernel equals the oracle: test_gpu_fullframe)."""
    w, h = 1920, 1080
    n = len(range(0, h, 8))
    ps = pixel_set(w, h, 0, w, 0, 8, n)
    outs = []
    for mode in (SPLIT_OFF, SPLIT_CHAIN):
        pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[64, 64], split=mode)
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), ran_chain(pt)))
        pt.close()
    assert not outs[0][4] and outs[1][4]
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


def test_large_frame_counter_chain(require_gpu):
    """Running mean at frame counters beyond 2^32 (64-bit conversions and the tiny-colour path)."""
    from iqpt import PathTracer, _lib, make_camera
    frame0 = 1 << 33
    w, h = 96, 64
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_CHAIN)
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
    assert ran_chain(pt)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("lanes,waves", [(4, 16), (8, 4), (4, 1)])
def test_lanes_and_waves_chain(require_gpu, lanes, waves):
    """4 lanes per pixel (16 pixels per wave) and other chain-kernel grid sizes: the same bits."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 480, 270
    n = len(range(2, h, 4))
    ps = pixel_set(w, h, 0, w, 2, 4, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(SPLIT_CHAIN)
    lib = _lib.load()
    lib.iqpt_debug_set_chain_waves.argtypes = [C.c_void_p, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_chain_waves(pt._h, waves | (lanes << 8)), "iqpt_debug_set_chain_waves")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for s in (10, 3):
        pt.render(s)
    lin, bgra = pt.read()
    assert ran_chain(pt)
    fr = oracle_render("cornell", w, h, 0, 8, pixels=ps, launches=[10, 3])
    _check(pt, lin, bgra, fr)
