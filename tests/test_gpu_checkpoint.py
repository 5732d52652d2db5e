"""Checkpoint / resume of the progressive accumulation (iqpt_checkpoint_save / _load).

render(a); save; load into a fresh context; render(b) must be bit-identical to render(a + b) in one
context — accumulator, BGRA, XORWOW states, frame counter and ray count — including across a
reset and on a row-partitioned context. Damaged or mismatched files are refused.
"""
import numpy as np
import pytest

from iqpt import IqptError, PathTracer, Scene, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def setup(w, h, pixels=None, seed=1984, depth=8, preset="cornell"):
    sc = Scene()
    sc.add_preset(preset)
    pt = PathTracer(w, h, pixels=pixels, seed=seed, max_depth=depth)
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(sc.build_packet())
    return pt


def state(pt):
    lin, bgra = pt.read()
    return lin.view(np.uint32).copy(), bgra.copy(), pt.read_rng(), pt.frames(), pt.rays()


def same(a, b):
    for x, y in zip(a, b):
        if isinstance(x, np.ndarray):
            assert np.array_equal(x, y)
        else:
            assert x == y


@pytest.mark.parametrize("pixels", [None, (0, 96, 1, 3, 18)])
def test_resume_equals_uninterrupted(require_gpu, tmp_path, pixels):
    ps = pixel_set(96, 54, *pixels) if pixels else None
    a = setup(96, 54, ps)
    a.render(3)
    ck = tmp_path / "a.ckpt"
    a.checkpoint_save(ck)
    a.render(2)
    a.render(1)
    ref = state(a)
    b = setup(96, 54, ps)
    b.checkpoint_load(ck)
    assert b.frames() == 3
    b.render(2)
    b.render(1)
    same(state(b), ref)


def test_resume_after_reset(require_gpu, tmp_path):
    a = setup(64, 48)
    a.render(4)
    a.reset()
    ck = tmp_path / "r.ckpt"
    a.checkpoint_save(ck)
    a.render(2)
    ref = state(a)
    b = setup(64, 48)
    b.render(7)                      # whatever b held is replaced by the checkpoint
    b.checkpoint_load(ck)
    b.render(2)
    same(state(b), ref)


def test_damaged_or_mismatched_checkpoints_are_refused(require_gpu, tmp_path):
    a = setup(40, 30)
    a.render(2)
    ck = tmp_path / "c.ckpt"
    a.checkpoint_save(ck)
    before = state(a)
    raw = bytearray(ck.read_bytes())
    raw[-5] ^= 0x40                                   # one flipped bit in the RNG planes
    bad = tmp_path / "bad.ckpt"
    bad.write_bytes(bytes(raw))
    with pytest.raises(IqptError):
        a.checkpoint_load(bad)
    short = tmp_path / "short.ckpt"
    short.write_bytes(ck.read_bytes()[:-4])
    with pytest.raises(IqptError):
        a.checkpoint_load(short)
    with pytest.raises(IqptError):
        a.checkpoint_load(tmp_path / "missing.ckpt")
    same(state(a), before)                             # a refused load leaves the context untouched
    other_seed = setup(40, 30, seed=7)
    with pytest.raises(IqptError):
        other_seed.checkpoint_load(ck)
    other_size = setup(40, 31)
    with pytest.raises(IqptError):
        other_size.checkpoint_load(ck)
