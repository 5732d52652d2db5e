"""Slot-parallel sphere pixels (IQPT_SPLIT_SPEC) vs the CPU oracle, bit for bit.

Only the pixels whose own camera-ray bundle may reach a sphere can take more than two draws per sample.
The slots of a window (slot j: the sample that starts 2j draws into the pixel's XORWOW stream) are evaluated
in parallel, the chain 0 -> j + n_j -> ... is walked afterwards and folded in sample order, and a chain
that leaves its window continues in a new window (another round of the same block); every other pixel
runs in the fan kernel beside it (or after it on one stream). The result must be the reference's sequential chain (path_tracer.cu:330-366, random.cu:66-107):
accumulator, BGRA8, final RNG states, ray count. RMSE < 1e-5 stated.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, gpu_render, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5
SPLIT_OFF, SPLIT_SPEC = 0, 4
def mode_of(pt, queue_fits=True) -> int:
    """The last launch's mode (6: spec). (queue_fits: kept for the callers; round 6 archived queue mode.)"""
    from iqpt import _lib
    lb = _lib.load()
    lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    info = (C.c_ulonglong * 8)()
    _lib.check(lb.iqpt_debug_split_info(pt._h, info), "iqpt_debug_split_info")
    return int(info[7])


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches", [[16], [8, 8, 8], [3, 1, 40], [64, 64], [300]])
def test_cornell_crop_spec(require_gpu, launches):
    """C2 crop through both spheres: long scatter chains, several launches (history-sized windows)."""
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    pt, lin, bgra = gpu_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches, split=SPLIT_SPEC)
    assert mode_of(pt) == 6
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches)
    _check(pt, lin, bgra, fr)


def test_spec_at_the_launch_limit(require_gpu):
    """One launch of kAccTableMax = 1,024 samples, the largest a render is cut into: the spec block's slot
    marks take 32 pixels x 3,072 bytes of LDS, so the runtime checks the block against the device's limit and
    one resident block and otherwise falls back to the plain kernel — the bits either way."""
    ps = pixel_set(1920, 1080, 920, 952, 480, 1, 8)
    pt, lin, bgra = gpu_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=[1024], split=SPLIT_SPEC)
    assert mode_of(pt, queue_fits=False) in (0, 6)   # (queue mode: 4 waves x 6 pixels x 3,072 slot counts)
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=[1024])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (1, 3), (0, 2), (3, 4)])
def test_row_share_spec(require_gpu, rank, world):
    """A rank's cyclic row share of a 484x270 Cornell frame (ragged tiles at the right edge)."""
    w, h = 484, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12], split=SPLIT_SPEC)
    assert mode_of(pt) == 6
    fr = oracle_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("depth", [1, 2, 3, 16])
def test_depths_spec(require_gpu, depth):
    """max_depth 1 (every sphere hit ends on a scatter at max depth: two slots, one ray), 2, 3, 16."""
    pt, lin, bgra = gpu_render("app_default", 160, 90, 0, depth, launches=[20, 7], split=SPLIT_SPEC)
    assert mode_of(pt) == 6
    fr = oracle_render("app_default", 160, 90, 0, depth, launches=[20, 7])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("spp", [1, 2, 5, 130])
def test_launch_sizes_spec(require_gpu, spp):
    pt, lin, bgra = gpu_render("cornell", 203, 117, 0, 8, launches=[spp, 7], split=SPLIT_SPEC)
    assert mode_of(pt) == 6
    fr = oracle_render("cornell", 203, 117, 0, 8, launches=[spp, 7])
    _check(pt, lin, bgra, fr)


def test_chains_leaving_their_window_spec(require_gpu):
    """Windows sized for one slot per sample: the sphere pixels' chains leave them in the first launch and
    further rounds finish them; the second launch sizes the windows from that history."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 320, 180
    sc, pk = scene_for("cornell")          # the scene owns the packet's arrays: keep it alive
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    lib = _lib.load()
    lib.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_spec(pt._h, 256, 0), "iqpt_debug_set_spec")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s in (24, 24):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


def test_large_frame_counter_spec(require_gpu):
    from iqpt import PathTracer, _lib, make_camera
    frame0 = (1 << 33) + 3
    w, h = 96, 64
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_SPEC)
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
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


def test_c3_share8_spec_vs_plain(require_gpu):
    """Rank 0's N = 8 row share of the full C3 frame (1920x1080, 64 spp, 8 bounces), three launches: the
    spec launches equal the plain kernel bit for bit (the plain kernel equals the oracle on the whole
    frame: test_gpu_fullframe)."""
    w, h = 1920, 1080
    n = len(range(0, h, 8))
    ps = pixel_set(w, h, 0, w, 0, 8, n)
    outs = []
    for mode in (SPLIT_OFF, SPLIT_SPEC):
        pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[64, 64, 64], split=mode)
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), mode_of(pt)))
        pt.close()
    assert [o[4] for o in outs] == [0, 6]
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


@pytest.mark.parametrize("margin_div", [1, 16])
def test_window_margins_spec(require_gpu, margin_div):
    """Wide (margin = all the extra slots) and tight windows: the same bits."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 256, 144
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    lib = _lib.load()
    lib.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_spec(pt._h, 0, margin_div), "iqpt_debug_set_spec")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s in (16, 40, 40):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("specfan", [(0, 0), (1, 0)])
@pytest.mark.parametrize("rank,world", [(0, 8), (3, 4)])
def test_specfan_layouts(require_gpu, specfan, rank, world):
    """The fan tiles beside the sphere pixels on a second stream (0) or after them on one stream (1)."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 484, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    lib = _lib.load()
    lib.iqpt_debug_set_specfan.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_specfan(pt._h, specfan[0], specfan[1]), "iqpt_debug_set_specfan")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    for s in (12, 20):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("plan", [0, 2, 3, 4, 5])
@pytest.mark.parametrize("specfan", [0, 1])
def test_spec_plans(require_gpu, plan, specfan):
    """Spec plans (the sphere pixels reordered by their last chain's work, 16 / 32 / 64 lanes per pixel):
    none, rebuilt before every launch from the history, every pixel on 32 or on 64 lanes, mixed lane counts.
    Four launches (the first without history), beside the fan tiles or after them on one stream."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 484, 270
    n = len(range(1, h, 3))
    ps = pixel_set(w, h, 0, w, 1, 3, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    lib = _lib.load()
    lib.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lib.iqpt_debug_spec_plan(pt._h, plan), "iqpt_debug_spec_plan")
    lib.iqpt_debug_set_specfan.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_specfan(pt._h, specfan, 0xffffffff), "iqpt_debug_set_specfan")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    for s in (10, 17, 3, 24):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    info = (C.c_ulonglong * 8)()
    lib.iqpt_debug_spec_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    _lib.check(lib.iqpt_debug_spec_info(pt._h, info), "iqpt_debug_spec_info")
    if plan >= 2:
        assert info[4] > 0                   # the last launch ran a plan
    _check(pt, lin, bgra, fr)


def test_spec_plan_async_c3_share8(require_gpu):
    """The default (asynchronous) plan on rank 0's N = 8 share of C3 over six launches (the history read
    after a launch is used once it has arrived: a sync after each launch makes that the next launch) equals
    the plain kernel bit for bit, and a plan is in use by the last launch."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 1920, 1080
    n = len(range(0, h, 8))
    ps = pixel_set(w, h, 0, w, 0, 8, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    lib = _lib.load()
    outs = []
    for mode in (SPLIT_OFF, SPLIT_SPEC):
        pt = PathTracer(w, h, pixels=ps, max_depth=8)
        pt.set_split(mode)
        pt.set_camera(cam)
        pt.upload_packet(pk)
        for _ in range(6):
            pt.render(64)
            pt.sync()
        if mode == SPLIT_SPEC:
            info = (C.c_ulonglong * 8)()
            lib.iqpt_debug_spec_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
            _lib.check(lib.iqpt_debug_spec_info(pt._h, info), "iqpt_debug_spec_info")
            assert info[4] > 0
        lin, bgra = pt.read()
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), mode_of(pt)))
        pt.close()
    assert [o[4] for o in outs] == [0, 6]
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


@pytest.mark.parametrize("split,expect", [(SPLIT_SPEC, 6)])
def test_pipelined_async_copies(require_gpu, split, expect):
    """Pipelined spec launches (the fan stream runs ahead, no join per launch) with a stream-ordered
    frame copy after every launch, as the multi-GPU gather issues them: copy k holds exactly launch k's frame
    (the launches write two frame buffers in turn), a reset in the middle joins the streams, and the final
    state is the oracle's bit for bit."""
    import torch
    from iqpt import PathTracer, _lib, make_camera
    w, h = 484, 270
    n = len(range(0, h, 4))
    ps = pixel_set(w, h, 0, w, 0, 4, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(split)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    npix = w * n
    bufs, want = [], []
    for i, s in enumerate((6, 9, 4, 12, 7, 5)):
        if i == 3:
            pt.reset()
            fr.reset()
        pt.render(s)
        fr.render(pk, cam, s)
        b = torch.zeros(npix, dtype=torch.int32, device="cuda")
        stream = torch.cuda.ExternalStream(pt.frame_stream_handle())
        pt.copy_frame_device_async(b.data_ptr(), b.numel() * 4)
        done = torch.cuda.Event()
        done.record(stream)
        torch.cuda.current_stream().wait_event(done)
        bufs.append(b)
        want.append(fr.bgra.copy())
    torch.cuda.synchronize()
    assert mode_of(pt) == expect
    for b, wv in zip(bufs, want):
        assert np.array_equal(b.cpu().numpy().view(np.uint8).reshape(-1, 4), wv)
    lin, bgra = pt.read()
    _check(pt, lin, bgra, fr)


def _set_parity(pt, rho256):
    from iqpt import _lib
    lb = _lib.load()
    lb.iqpt_debug_set_spec_parity.argtypes = [C.c_void_p, C.c_uint32]
    _lib.check(lb.iqpt_debug_set_spec_parity(pt._h, rho256), "iqpt_debug_set_spec_parity")


@pytest.mark.parametrize("parity", [0, 1, 480, 2000])
@pytest.mark.parametrize("launches", [[16, 16, 16], [5, 64]])
def test_parity_pixels(require_gpu, parity, launches):
    """Parity pixels (round 5): round 0 traces the even slots, the walk stops at the first odd
    slot the chain lands on, and the block's lanes share the odd slots from there on (fix-up pass). Threshold
    0 (off: every slot), 1 (every sphere pixel, edge pixels whose camera rays often miss the sphere included:
    many fix-ups), 480 (the default, 1.875 slots per sample) and 2000 (none). A C2 crop through both spheres
    over several launches (history-sized windows), bit for bit."""
    from iqpt import PathTracer, make_camera
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    sc, pk = scene_for("cornell")
    cam = make_camera(1920, 1080)
    pt = PathTracer(1920, 1080, pixels=ps, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    _set_parity(pt, parity)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(1920, 1080, pixels=ps, max_depth=8)
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rho0,plan", [(256, 0), (256, 2), (384, 4), (576, 3)])
def test_parity_pixels_leaving_windows_and_plans(require_gpu, rho0, plan):
    """Parity pixels whose chains leave their windows (a short first window: rho0 one slot per sample, the
    parity threshold at 1) — the fix-up pass, then trace-all rounds from the window's end — under plans none /
    rebuilt / 64 / 32 lanes, with a frame counter beyond 2^32; row share 3 of 8."""
    from iqpt import PathTracer, _lib, make_camera
    w, h = 484, 270
    n = len(range(3, h, 8))
    ps = pixel_set(w, h, 0, w, 3, 8, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    _set_parity(pt, 1)
    lib = _lib.load()
    lib.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    _lib.check(lib.iqpt_debug_set_spec(pt._h, rho0, 0), "iqpt_debug_set_spec")
    lib.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lib.iqpt_debug_spec_plan(pt._h, plan), "iqpt_debug_spec_plan")
    lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
    _lib.check(lib.iqpt_debug_set_frame(pt._h, (1 << 32) + 5), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    fr.frame = (1 << 32) + 5
    for s in (24, 40):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == 6
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("world", [8, 4])
def test_parity_on_equals_off_on_the_share(require_gpu, world):
    """Rank 0's whole C3 share, two 64-spp launches with parity pixels (default) and without: the same bits."""
    from iqpt import PathTracer, make_camera
    w, h = 1920, 1080
    n = len(range(0, h, world))
    ps = pixel_set(w, h, 0, w, 0, world, n)
    sc, pk = scene_for("cornell")
    cam = make_camera(w, h)
    out = []
    for parity in (480, 0):
        pt = PathTracer(w, h, pixels=ps, max_depth=8)
        pt.set_split(SPLIT_SPEC)
        _set_parity(pt, parity)
        pt.set_camera(cam)
        pt.upload_packet(pk)
        pt.render(64)
        pt.render(64)
        lin, bgra = pt.read()
        out.append((lin.view(np.uint32).copy(), bgra.copy(), pt.read_rng(), pt.rays()))
        pt.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2], out[1][2]) and out[0][3] == out[1][3]
