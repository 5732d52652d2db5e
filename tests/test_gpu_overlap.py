"""Overlapped launches (kOptOverlap): consecutive iqpt_render calls alternate between two
HIP streams and each screen tile waits, on its XCD, for the previous launch to finish it. The results must
be the bits of one stream (and of the oracle): accumulator, BGRA8, XORWOW states and ray counts, for
chains of launches, chains cut by reads / camera changes / resets, and the full C2 frame."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, scene_for
from iqpt import PathTracer, _lib, make_camera
from iqpt.render import pixel_set

pytestmark = pytest.mark.gpu

K_OPT_OVERLAP = 1 << 19


def last_options(pt):
    lb = _lib.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    o = C.c_int(0)
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
    return o.value


def run(preset, w, h, launches, depth=8, pixels=None, overlap=True, cut=None):
    """launches: spp per render call; cut: {index: action} applied before that render."""
    _, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=pixels, max_depth=depth)
    pt.set_split(_lib.SPLIT_OFF)      # small pixel sets would take the split mode, which never overlaps
    pt.set_overlap(_lib.OVERLAP_AUTO if overlap else _lib.OVERLAP_OFF)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    opts = []
    for i, s in enumerate(launches):
        if cut and i in cut:
            cut[i](pt, cam)
        pt.render(s)
        opts.append(last_options(pt))
    pt.sync()
    lin, bgra = pt.read()
    out = (lin, bgra, pt.read_rng(), pt.rays(), pt.frames())
    pt.close()
    return out, opts


def same(a, b):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[2], b[2])
    assert a[3] == b[3] and a[4] == b[4]


def test_chain_equals_one_stream_and_oracle(require_gpu):
    w, h = 256, 144
    launches = [4, 3, 5, 1, 2, 6, 4, 4]
    on, opts = run("cornell", w, h, launches)
    assert all(o & K_OPT_OVERLAP for o in opts), opts
    off, opts_off = run("cornell", w, h, launches, overlap=False)
    assert not any(o & K_OPT_OVERLAP for o in opts_off)
    same(on, off)
    _, pk = scene_for("cornell")
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s in launches:
        fr.render(pk, make_camera(w, h), s)
    c = compare(on[0], fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(on[2], fr.states)
    assert on[3] == int(fr.rays.sum())


def test_chain_cut_by_reads_camera_and_reset(require_gpu):
    w, h = 200, 120
    launches = [3] * 9

    def read(pt, cam):
        pt.read()

    def recam(pt, cam):
        pt.set_camera(cam)            # same view: masks and XCD tile lists rebuilt, the chain restarts

    def reset(pt, cam):
        pt.reset()

    cuts = {2: read, 4: recam, 6: reset, 7: read}
    on, _ = run("cornell", w, h, launches, cut=dict(cuts))
    off, _ = run("cornell", w, h, launches, overlap=False, cut=dict(cuts))
    same(on, off)


@pytest.mark.parametrize("preset,w,h,depth,crop", [
    ("app_default", 320, 180, 5, None),
    ("cornell", 1920, 1080, 8, (640, 1280, 400, 2, 96)),       # a C3-like row share (every other row)
    ("cornell_lit", 160, 96, 8, None),                         # material table variant
])
def test_other_scenes_and_shares(require_gpu, preset, w, h, depth, crop):
    ps = pixel_set(w, h, *crop) if crop else None
    launches = [2, 2, 2, 2, 2]
    on, opts = run(preset, w, h, launches, depth=depth, pixels=ps)
    off, _ = run(preset, w, h, launches, depth=depth, pixels=ps, overlap=False)
    same(on, off)


def test_full_c2_frame_three_overlapped_launches(require_gpu):
    """The bench's step sequence: 64-spp launches back to back on the full 1920x1080 frame."""
    w, h = 1920, 1080
    on, opts = run("cornell", w, h, [64, 64, 64])
    assert all(o & K_OPT_OVERLAP for o in opts)
    off, _ = run("cornell", w, h, [64, 64, 64], overlap=False)
    same(on, off)


def test_kernel_span_not_longer_than_sum(require_gpu):
    _, pk = scene_for("cornell")
    w, h = 640, 360
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(_lib.SPLIT_OFF)
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(pk)
    pt.render(8)
    pt.sync()
    pt.kernel_time()
    for _ in range(6):
        pt.render(8)
    total, n = pt.kernel_time()
    span = pt.kernel_span()
    assert n == 6 and 0.0 < span <= total * 1.0001
    pt.close()


@pytest.mark.parametrize("preset,w,h,crop", [
    ("cornell", 256, 144, None),
    ("cornell", 1920, 1080, (640, 1280, 400, 2, 96)),          # the C3 N = 2 share shape
])
def test_async_frame_copies_keep_overlap(require_gpu, preset, w, h, crop):
    """bench.py's stream-ordered gather: after every render a copy of the frame on iqpt_frame_stream,
    without joining the streams. Launches keep overlapping (two frame buffers in turn) and every copy
    is the frame of its own launch: the BGRA8 a one-stream context presents after the same launch."""
    import torch
    _, pk = scene_for(preset)
    ps = pixel_set(w, h, *crop) if crop else None
    launches = [3, 4, 2, 5, 3, 3]
    cam = make_camera(w, h)

    def ctx(overlap):
        pt = PathTracer(w, h, pixels=ps, max_depth=8)
        pt.set_split(_lib.SPLIT_OFF)
        pt.set_overlap(_lib.OVERLAP_AUTO if overlap else _lib.OVERLAP_OFF)
        pt.set_camera(cam)
        pt.upload_packet(pk)
        return pt

    ref = ctx(False)
    want = []
    for s in launches:
        ref.render(s)
        want.append(ref.read()[1].view(np.uint32).ravel().copy())
    ref_state = (ref.read()[0], ref.read()[1], ref.read_rng(), ref.rays(), ref.frames())
    ref.close()

    pt = ctx(True)
    npix = want[0].size
    bufs = [torch.empty(npix, dtype=torch.int32, device="cuda") for _ in launches]
    opts, streams = [], set()
    for s, b in zip(launches, bufs):
        pt.render(s)
        opts.append(last_options(pt))
        streams.add(pt.frame_stream_handle())
        pt.copy_frame_device_async(b.data_ptr(), b.numel() * 4)
    assert all(o & K_OPT_OVERLAP for o in opts), opts
    assert len(streams) == 2                   # copies followed their launches on both streams
    pt.sync()
    torch.cuda.synchronize()
    for i, b in enumerate(bufs):
        got = b.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want[i]), f"copy after launch {i}"
    lin, bgra = pt.read()
    same((lin, bgra, pt.read_rng(), pt.rays(), pt.frames()), ref_state)
    pt.close()


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("refill", [16, 64])
def test_resident_refill_group_sizes(require_gpu, overlap, refill):
    """Resident plain launches whose waves take new pixels only once `refill` lanes are idle
    (iqpt_debug_set_resident_refill; 1 by default): overlapped chains of launches and single-stream ones
    keep the oracle's bits (accumulator, BGRA8, RNG states, ray counts)."""
    w, h = 256, 144
    sc, pk = scene_for("cornell")              # (the packet points into the scene's arrays)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(_lib.SPLIT_OFF)
    pt.set_overlap(_lib.OVERLAP_AUTO if overlap else _lib.OVERLAP_OFF)
    lb = _lib.load()
    lb.iqpt_debug_set_resident_refill.argtypes = [C.c_void_p, C.c_uint32]
    _lib.check(lb.iqpt_debug_set_resident_refill(pt._h, refill), "iqpt_debug_set_resident_refill")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    opts = []
    for s in (4, 9, 2, 7):
        pt.render(s)
        opts.append(last_options(pt))
        fr.render(pk, cam, s)
    assert all(bool(o & K_OPT_OVERLAP) == overlap for o in opts), opts
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()
