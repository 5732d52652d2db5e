"""libiqpt's own multi-GPU frame delivery (iqpt_comm_init / iqpt_gather_*),
through the C ABI on one GPU with one-rank RCCL communicators (RCCL refuses two ranks on one device; the
2..8-rank exchange runs on the driver's 8-GPU node). The gathered and assembled frame must equal the
context's own frame and the oracle's bit for bit: a whole frame; rank 0's share of an N-way cyclic row
split (the root places rows 0, N, 2N, ... only); and every rank of an N-way split rehearsed in turn, each
placing its rows into one device frame, which must then be the single-GPU frame."""
import ctypes as C

import numpy as np
import pytest
import torch

import iqpt
from iqpt import dist as iqdist
from iqpt.render import pixel_set
from helpers import oracle_render, scene_for

pytestmark = pytest.mark.gpu


def _ctx(w, h, ps, depth=8, spp=4, launches=1, preset="cornell"):
    _, pk = scene_for(preset)
    pt = iqpt.PathTracer(w, h, pixels=ps, max_depth=depth)
    pt.set_camera(iqpt.make_camera(w, h))
    pt.upload_packet(pk)
    return pt, pk, spp, launches


def test_full_frame_gather_equals_read_and_oracle(require_gpu):
    w, h = 160, 90
    pt, _, spp, _ = _ctx(w, h, None)
    pt.comm_init(0, 1, iqpt.comm_unique_id())
    frame = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    for _ in range(3):                       # stream-ordered gathers behind consecutive renders
        pt.render(spp)
        pt.gather_frame_async(0, frame.data_ptr(), frame.numel() * 4)
    pt.sync()                                # joins the communicator stream
    lin, bgra = pt.read()
    assert np.array_equal(frame.cpu().numpy(), bgra.view(np.int32).reshape(-1))
    glin, gbgra = pt.gather_read(0)
    assert np.array_equal(glin.view(np.uint32), lin.view(np.uint32))
    assert np.array_equal(gbgra, bgra)
    acc = torch.zeros((w * h, 4), dtype=torch.float32, device="cuda")
    pt.gather_accum(0, acc.data_ptr(), acc.numel() * 4)
    assert np.array_equal(acc.cpu().numpy().view(np.uint32), lin.view(np.uint32))
    ms, n = pt.comm_time()
    assert n == 6 and ms > 0.0               # 3 frame gathers, 2 in gather_read (accumulators, frame), 1 accum
    # the select form runs only the collectives asked for (a present needs the BGRA8 frame alone)
    flin, fbgra = pt.gather_read(0, "frame")
    assert flin is None and np.array_equal(fbgra, bgra)
    alin, abgra = pt.gather_read(0, "accum")
    assert abgra is None and np.array_equal(alin.view(np.uint32), lin.view(np.uint32))
    assert pt.comm_time()[1] == 2
    fr = oracle_render("cornell", w, h, spp, 8, launches=[spp] * 3)
    assert np.array_equal(lin.view(np.uint32), fr.lin.view(np.uint32))
    pt.close()


@pytest.mark.parametrize("split,mode", [(8, iqpt._lib.SPLIT_AUTO), (2, iqpt._lib.SPLIT_AUTO), (4, iqpt._lib.SPLIT_OFF)])
def test_share_rehearsal_places_rank0_rows(require_gpu, split, mode):
    """Rank 0's rows of a split-way cyclic split, gathered by a one-rank communicator: the root assembles
    them at rows 0, split, 2 split, ... of the frame and leaves every other row untouched."""
    w, h = 256, 144
    ps = iqdist.pixel_set_for_rank(w, h, 0, split)
    pt, _, spp, _ = _ctx(w, h, ps, spp=8)
    pt.set_split(mode)
    pt.comm_init(0, 1, iqpt.comm_unique_id())
    sentinel = -12345
    frame = torch.full((h * w,), sentinel, dtype=torch.int32, device="cuda")
    for _ in range(3):
        pt.render(spp)
        pt.gather_frame_async(0, frame.data_ptr(), frame.numel() * 4)
    pt.sync()
    _, bgra = pt.read()
    got = frame.cpu().numpy().reshape(h, w)
    own = bgra.view(np.int32).reshape(-1, w)
    assert np.array_equal(got[0::split], own)
    mask = np.ones(h, bool)
    mask[0::split] = False
    assert np.all(got[mask] == sentinel)
    pt.close()


@pytest.mark.parametrize("n", [3, 4, 8])
def test_n_rehearsals_assemble_the_whole_frame(require_gpu, n):
    """Every rank r of an n-way split rehearsed by a one-rank communicator whose root places rank r's rows
    (r, r + n, ...; H not a multiple of n: ragged last rows) into ONE device frame: the assembled frame and
    the accumulators equal the oracle's single-GPU frame bit for bit, and equal iqpt.dist.assemble of the
    ranks' own frames."""
    w, h, spp = 96, 45, 4
    frame = torch.full((h * w,), -1, dtype=torch.int32, device="cuda")
    acc = torch.zeros((h * w, 4), dtype=torch.float32, device="cuda")
    parts = []
    for r in range(n):
        ps = iqdist.pixel_set_for_rank(w, h, r, n)
        pt, _, _, _ = _ctx(w, h, ps, spp=spp)
        pt.comm_init(0, 1, iqpt.comm_unique_id())
        pt.render(spp)
        pt.gather_frame_async(0, frame.data_ptr(), frame.numel() * 4)
        pt.gather_accum(0, acc.data_ptr(), acc.numel() * 4)
        _, bgra = pt.read()
        blk = np.zeros((iqdist.max_rows(h, n) * w, 4), np.uint8)
        blk[: bgra.shape[0]] = bgra
        parts.append(blk)
        pt.close()
    one = oracle_render("cornell", w, h, spp, 8)
    assert np.array_equal(frame.cpu().numpy(), one.bgra.view(np.int32).reshape(-1))
    assert np.array_equal(acc.cpu().numpy().view(np.uint32), one.lin.view(np.uint32))
    assert np.array_equal(iqdist.assemble(parts, w, h, n, 4).view(np.int32).reshape(-1), frame.cpu().numpy())


def _last_options(pt):
    lb = iqpt.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    o = C.c_int(0)
    iqpt._lib.check(lb.iqpt_debug_last_options(pt.handle, C.byref(o)), "iqpt_debug_last_options")
    return o.value


def _split_mode(pt):
    lb = iqpt.load()
    lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    info = (C.c_ulonglong * 8)()
    iqpt._lib.check(lb.iqpt_debug_split_info(pt.handle, info), "iqpt_debug_split_info")
    return int(info[7])


def test_comm_init_pads_every_frame_buffer_of_a_ragged_rank(require_gpu):
    """A ragged rank (fewer rows than the rank block) whose context already made the overlapped launches'
    second frame buffer and the pipelined launches' ring — and whose second-buffer view points into that
    ring — before iqpt_comm_init. The pipelined gather sends the launch's own frame buffer as it is, rank
    block long: every frame buffer must be padded, none left dangling. Gathers after it, from overlapped
    and from pipelined spec launches in turn, each hold their launch's frame (the oracle's), and the final
    state is the oracle's."""
    import oracle
    L = iqpt._lib
    w, h, n, r = 640, 130, 4, 3                   # rank 3 of 4: 32 rows, the rank block 33 (overlap: >= 16384 px)
    ps = iqdist.pixel_set_for_rank(w, h, r, n)
    pt, _, _, _ = _ctx(w, h, ps)
    sc, pk = scene_for("cornell")                 # (the packet points into the scene's arrays: keep both)
    cam = iqpt.make_camera(w, h)
    fr = oracle.OracleFrame(w, h, pixels=oracle.pixel_set(w, h, 0, w, r, n, ps.nrows), max_depth=8)
    npix = w * len(range(r, h, n))
    assert npix < iqdist.max_rows(h, n) * w

    def render(mode, s):
        if mode == "ovl":
            pt.set_split(L.SPLIT_OFF)
            pt.set_overlap(L.OVERLAP_AUTO)
        else:
            pt.set_split(4)                       # IQPT_SPLIT_SPEC: pipelined spec + fan launches
        pt.render(s)
        fr.render(pk, cam, s)
        if mode == "ovl":
            assert _last_options(pt) & (1 << 19), hex(_last_options(pt))
        else:
            assert _split_mode(pt) == 6

    keep = []
    for mode, s in (("ovl", 3), ("ovl", 4), ("spec", 5), ("spec", 6), ("ovl", 3)):
        render(mode, s)
        b = torch.zeros(npix, dtype=torch.int32, device="cuda")
        pt.copy_frame_device_async(b.data_ptr(), b.numel() * 4)
        keep.append(b)                            # (the copies read the buffers comm_init replaces)
    pt.comm_init(0, 1, iqpt.comm_unique_id())
    frames, want = [], []
    for mode, s in (("spec", 4), ("ovl", 5), ("spec", 3), ("ovl", 2), ("spec", 6)):
        render(mode, s)
        f = torch.full((h * w,), -7, dtype=torch.int32, device="cuda")
        pt.gather_frame_async(0, f.data_ptr(), f.numel() * 4)
        frames.append(f)
        want.append(fr.bgra.view(np.int32).reshape(-1).copy())
    pt.sync()
    torch.cuda.synchronize()
    for i, (f, wv) in enumerate(zip(frames, want)):
        got = f.cpu().numpy().reshape(h, w)
        assert np.array_equal(got[r::n].reshape(-1), wv), f"gather after launch {i}"
        mask = np.ones(h, bool)
        mask[r::n] = False
        assert np.all(got[mask] == -7)
    lin, bgra = pt.read()
    assert np.array_equal(lin.view(np.uint32), fr.lin.view(np.uint32))
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    pt.close()


def test_comm_init_rejects_a_pixel_set_it_cannot_assemble(require_gpu):
    w, h = 64, 32
    lib = iqpt.load()
    uid = iqpt.comm_unique_id()
    buf = (C.c_uint8 * 128).from_buffer_copy(uid)
    # partial columns; rows 2, 4, ... of a 2-way split (no rank of a one-rank world owns them); a wrong row count
    for ps in (pixel_set(w, h, 0, 32), pixel_set(w, h, 0, w, 2, 2), pixel_set(w, h, 0, w, 0, 2, 3)):
        pt = iqpt.PathTracer(w, h, pixels=ps, max_depth=2)
        assert lib.iqpt_comm_init(pt.handle, 0, 1, buf, 128) == 1
        assert b"cyclic rows" in lib.iqpt_last_error()
        pt.close()
    pt = iqpt.PathTracer(w, h, max_depth=2)
    assert lib.iqpt_comm_init(pt.handle, 1, 1, buf, 128) == 1            # rank out of range
    assert lib.iqpt_gather_frame_async(pt.handle, 0, None, 0) == 5       # no communicator yet
    pt.close()
