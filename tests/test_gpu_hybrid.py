"""Hybrid launches: overlapped plain launches whose sphere pixels — the pixels whose own
camera-ray bundle may reach a sphere, the longest per-pixel chains — run in the spec kernel on a stream of
their own, pipelined across launches, while the plain kernel skips them (and the certain misses, which the
sky kernel renders). Bit for bit against the oracle (accumulator, BGRA8, RNG states, ray counts) and against
the plain launches on the full C2 frame. RMSE < 1e-5 stated."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, scene_for

pytestmark = pytest.mark.gpu


def _render(w, h, launches, hybrid=True, sky=True, preset="cornell", copies=False, rho=0, sync_each=False):
    from iqpt import PathTracer, _lib, make_camera
    lib = _lib.load()
    lib.iqpt_debug_set_hybrid.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
    lib.iqpt_debug_set_sky.argtypes = [C.c_void_p, C.c_int]
    sc, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt._scene = sc
    pt.set_split(_lib.SPLIT_OFF)             # small frames: AUTO would take spec launches (no overlapped plain kernel)
    _lib.check(lib.iqpt_debug_set_hybrid(pt.handle, 1 if hybrid else 0, rho), "iqpt_debug_set_hybrid")
    _lib.check(lib.iqpt_debug_set_sky(pt.handle, 1 if sky else 0), "iqpt_debug_set_sky")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    frames = []
    for s in launches:
        pt.render(s)
        if sync_each:
            pt.sync()                        # the chain history arrives: the next launch selects
        if copies:
            import torch
            buf = torch.zeros(pt.npix, dtype=torch.int32, device="cuda")
            pt.copy_frame_device_async(buf.data_ptr(), buf.numel() * 4)
            frames.append(buf)
    mode = pt.launch_mode()
    lin, bgra = pt.read()
    lib.iqpt_debug_hybrid_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    a, b = C.c_uint32(0), C.c_uint32(0)
    _lib.check(lib.iqpt_debug_hybrid_info(pt.handle, C.byref(a), C.byref(b)), "iqpt_debug_hybrid_info")
    pt.selected, pt.sphere_pixels = a.value, b.value
    return pt, lin, bgra, mode, pk, cam, frames


@pytest.mark.parametrize("sky", [True, False])
def test_hybrid_cornell_matches_oracle(require_gpu, sky):
    w, h, launches = 480, 270, [16, 64, 5]
    pt, lin, bgra, mode, pk, cam, _ = _render(w, h, launches, sky=sky)
    assert mode == "hybrid"
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s in launches:
        fr.render(pk, cam, s)
    c = compare(lin, fr.lin)
    assert c["rmse"] < 1e-5 and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()


def test_hybrid_frame_copies_after_every_launch(require_gpu):
    """A stream-ordered frame copy after every hybrid launch (the spec kernel writes its pixels of the frame on
    its own stream): copy k is the oracle's frame after launch k."""
    w, h, launches = 320, 180, [8, 8, 8]
    pt, lin, bgra, mode, pk, cam, frames = _render(w, h, launches, copies=True)
    assert mode == "hybrid"
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s, got in zip(launches, frames):
        fr.render(pk, cam, s)
        pt.sync()
        assert np.array_equal(got.cpu().numpy(), fr.bgra.view(np.int32).reshape(-1))
    pt.close()


def test_hybrid_full_c2_frame_equals_plain(require_gpu):
    """The whole C2 bench frame (1920x1080, 64 spp, 8 bounces) over three launches: hybrid equals the plain
    overlapped launches bit for bit (the plain kernel equals the oracle on this frame: test_gpu_fullframe)."""
    outs = []
    for hybrid in (False, True):
        pt, lin, bgra, mode, _, _, _ = _render(1920, 1080, [64, 64, 64], hybrid=hybrid)
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), mode))
        pt.close()
    assert [o[4] for o in outs] == ["plain", "hybrid"]
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


def _first_launch_history(w, h, spp):
    """The sphere pixels' slots per sample x 256 after one hybrid launch of `spp` (the history the selection of
    the second launch reads): the spec plan rebuilt synchronously, then read back with the history."""
    from iqpt import PathTracer, _lib, make_camera
    lib = _lib.load()
    lib.iqpt_debug_set_hybrid.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
    lib.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
    sc, pk = scene_for("cornell")
    pt = PathTracer(w, h, max_depth=8)
    pt._scene = sc
    pt.set_split(_lib.SPLIT_OFF)
    _lib.check(lib.iqpt_debug_set_hybrid(pt.handle, 1, 0), "iqpt_debug_set_hybrid")
    _lib.check(lib.iqpt_debug_spec_plan(pt.handle, 2), "iqpt_debug_spec_plan")
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(pk)
    pt.render(spp)
    assert pt.launch_mode() == "hybrid"
    cap = w * h
    order, blocks, rho = (C.c_uint32 * cap)(), (C.c_uint32 * (2 * cap))(), (C.c_uint32 * cap)()
    n, nb = C.c_uint32(0), C.c_uint32(0)
    lib.iqpt_debug_read_spec_plan.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint32)]
    _lib.check(lib.iqpt_debug_read_spec_plan(pt.handle, order, blocks, rho, cap, C.byref(n), C.byref(nb)),
               "iqpt_debug_read_spec_plan")
    out = np.frombuffer(rho, dtype=np.uint32, count=n.value).copy()
    pt.close()
    return out


@pytest.mark.parametrize("q", [40, 80])
def test_hybrid_selection_matches_oracle(require_gpu, q):
    """After the first launch's chain history, only the sphere pixels whose chains used >= rho / 256 slots per
    sample stay in the spec kernel; the plain kernel takes the others back (plan and skip masks change together
    at a join). The threshold is the q-th percentile of that history (so both kernels keep some sphere pixels).
    Five launches, the selection active from the second: the oracle's bits."""
    w, h, launches = 480, 270, [16, 16, 32, 8, 64]
    hist = _first_launch_history(w, h, launches[0])
    assert hist.size > 0 and hist.min() > 0
    rho = int(np.percentile(hist, q))
    if not (0 < int((hist >= rho).sum()) < hist.size):
        rho += 1
    want = int((hist >= rho).sum())
    assert 0 < want < hist.size, (rho, np.unique(hist))
    pt, lin, bgra, mode, pk, cam, _ = _render(w, h, launches, rho=rho, sync_each=True)
    assert mode == "hybrid"
    assert pt.selected == want and pt.sphere_pixels == hist.size, (pt.selected, want, pt.sphere_pixels)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    for s in launches:
        fr.render(pk, cam, s)
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()
