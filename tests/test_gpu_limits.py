"""The forward-progress guards and what a caller sees when one fires.

Overlapped launches wait per tile for the previous launch (bounded polls, kparams::spin_limit; round 6
archived the chain kernel and its iteration bound). The bound is never reached by a real launch.
iqpt_debug_set_limits lowers it (and can bias the per-tile wait targets so that a wait can never be
satisfied), which forces the path here. Once a kernel reports either error, the pixel state
is undefined: iqpt_sync, iqpt_read, iqpt_read_rng, the device copies and iqpt_checkpoint_save must all
fail (the error is latched in the context) until iqpt_checkpoint_load replaces the whole state.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import scene_for
from iqpt import PathTracer, Scene, _lib, make_camera
from iqpt._lib import IqptError
from iqpt.render import pixel_set

pytestmark = pytest.mark.gpu


def set_limits(pt, spin=0, iters=0, bias=0):
    lb = _lib.load()
    lb.iqpt_debug_set_limits.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]
    _lib.check(lb.iqpt_debug_set_limits(pt._h, spin, iters, bias), "iqpt_debug_set_limits")


def expect_latched(pt, tmp_path, what):
    with pytest.raises(IqptError, match=what):
        pt.sync()
    for call in (pt.read, pt.read_rng, lambda: pt.checkpoint_save(str(tmp_path / "bad.ckpt"))):
        with pytest.raises(IqptError, match=what):
            call()
    assert not (tmp_path / "bad.ckpt").exists()
    import torch
    dst = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    with pytest.raises(IqptError, match=what):
        pt.copy_frame_device(dst.data_ptr(), dst.numel() * 4)


def test_overlap_wait_timeout_is_reported_and_latched(require_gpu, tmp_path):
    w, h = 256, 144                        # 144 blocks: overlapped launches run (>= 64 blocks, 8 XCDs)
    sc, pk = scene_for("cornell")          # the scene owns the packet's arrays: keep it alive
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(_lib.SPLIT_OFF)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    pt.render(2)
    pt.sync()
    good = tmp_path / "good.ckpt"
    pt.checkpoint_save(str(good))          # the state after 2 samples, before any error
    lin_good, bgra_good = pt.read()
    # the next overlapped launch waits for a completion count no launch reaches: every wait gives up
    # after 4 polls and the error word is set
    set_limits(pt, spin=4, bias=1000)
    pt.render(2)
    pt.render(2)
    expect_latched(pt, tmp_path, "per-tile wait timed out")
    # back to defined state: the checkpoint replaces everything and clears the latch
    set_limits(pt)
    pt.checkpoint_load(str(good))
    lin, bgra = pt.read()
    assert np.array_equal(lin.view(np.uint32), lin_good.view(np.uint32)) and np.array_equal(bgra, bgra_good)
    pt.render(3)
    pt.sync()
    lin, _ = pt.read()
    fr = oracle.OracleFrame(w, h, max_depth=8)
    fr.render(pk, cam, 5)
    assert np.array_equal(lin.view(np.uint32), fr.lin.view(np.uint32))
    pt.close()


def walls_packet():
    """The Cornell box without its spheres: triangles only (every camera ray ends on its first hit).
    Returns (scene, packet): the scene owns the packet's arrays."""
    sc = Scene()
    sc.add_mesh_quad("quad")
    wall = (2.0, 2.0, 1.0, 1.0)
    sc.add_model("back", "quad", wall, 0.0, (0.0, 0.5, 1.0))
    sc.add_model("floor", "quad", wall, (1.5707963267948966, 0, 0), (0.0, -0.5, 0.0))
    sc.add_model("ceiling", "quad", wall, (-1.5707963267948966, 0, 0), (0.0, 1.5, 0.0))
    sc.add_model("left", "quad", wall, (0, 1.5707963267948966, 0), (-1.0, 0.5, 0.0))
    sc.add_model("right", "quad", wall, (0, -1.5707963267948966, 0), (1.0, 0.5, 0.0))
    return sc, sc.build_packet()


def test_small_frames_do_not_overlap_and_stay_exact(require_gpu):
    """Frames of fewer than 64 blocks (16,384 pixels) never take overlapped launches: with few blocks an
    XCD may get none and its tiles would not be rendered. A 32x32 frame, a triangle-only scene and the
    lit Cornell box stay bit-exact vs the oracle over several launches."""
    K_OPT_OVERLAP = 1 << 19
    lb = _lib.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    for preset in ("cornell_lit", "walls", "cornell"):
        w, h = 32, 32
        sc, pk = walls_packet() if preset == "walls" else scene_for(preset)
        cam = make_camera(w, h)
        pt = PathTracer(w, h, max_depth=8)
        pt.set_split(_lib.SPLIT_OFF)
        pt.set_camera(cam)
        pt.upload_packet(pk)
        fr = oracle.OracleFrame(w, h, max_depth=8)
        for s in (3, 1, 4):
            pt.render(s)
            o = C.c_int(0)
            _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
            assert not o.value & K_OPT_OVERLAP, (preset, hex(o.value))
            fr.render(pk, cam, s)
        pt.sync()
        lin, bgra = pt.read()
        assert np.array_equal(lin.view(np.uint32), fr.lin.view(np.uint32)), preset
        assert np.array_equal(bgra, fr.bgra), preset
        assert np.array_equal(pt.read_rng(), fr.states), preset
        pt.close()
