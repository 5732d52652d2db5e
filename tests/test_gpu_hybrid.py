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


def _render(w, h, launches, hybrid=True, sky=True, preset="cornell", copies=False):
    from iqpt import PathTracer, _lib, make_camera
    lib = _lib.load()
    lib.iqpt_debug_set_hybrid.argtypes = [C.c_void_p, C.c_int]
    lib.iqpt_debug_set_sky.argtypes = [C.c_void_p, C.c_int]
    sc, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt._scene = sc
    pt.set_split(_lib.SPLIT_OFF)             # small frames: AUTO would take spec launches (no overlapped plain kernel)
    _lib.check(lib.iqpt_debug_set_hybrid(pt.handle, 1 if hybrid else 0), "iqpt_debug_set_hybrid")
    _lib.check(lib.iqpt_debug_set_sky(pt.handle, 1 if sky else 0), "iqpt_debug_set_sky")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    frames = []
    for s in launches:
        pt.render(s)
        if copies:
            import torch
            buf = torch.zeros(pt.npix, dtype=torch.int32, device="cuda")
            pt.copy_frame_device_async(buf.data_ptr(), buf.numel() * 4)
            frames.append(buf)
    mode = pt.launch_mode()
    lin, bgra = pt.read()
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
