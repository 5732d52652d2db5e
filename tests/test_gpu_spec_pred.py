"""Predicted chains in the spec kernel (kspec::pred, off by default; iqpt_debug_set_spec_pred):
phase A traces the camera ray of every slot of a window (all lanes at depth 0, tile masks), phase B completes
the samples whose camera ray hit a sphere only at the chain's positions as predicted (two slots each), checks
the prediction against their true slot counts and continues from where a sample really ended. Bit for bit
against the oracle (accumulator, BGRA8, RNG states, ray counts) and against every slot traced whole. RMSE < 1e-5
stated."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
SPLIT_SPEC = 4


def _render(ps, launches, pred, depth=8, plan=1, frame0=None, rho0=None, w=1920, h=1080):
    from iqpt import PathTracer, _lib, make_camera
    lb = _lib.load()
    lb.iqpt_debug_set_spec_pred.argtypes = [C.c_void_p, C.c_int]
    lb.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
    sc, pk = scene_for("cornell")
    pt = PathTracer(w, h, pixels=ps, max_depth=depth)
    pt._scene = sc
    pt.set_split(SPLIT_SPEC)
    _lib.check(lb.iqpt_debug_set_spec_pred(pt.handle, 1 if pred else 0), "iqpt_debug_set_spec_pred")
    _lib.check(lb.iqpt_debug_spec_plan(pt.handle, plan), "iqpt_debug_spec_plan")
    if frame0 is not None:
        lb.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
        _lib.check(lb.iqpt_debug_set_frame(pt.handle, frame0), "iqpt_debug_set_frame")
    if rho0 is not None:
        lb.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_spec(pt.handle, rho0, 0), "iqpt_debug_set_spec")
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
    lin, bgra = pt.read()
    return pt, lin, bgra


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < 1e-5 and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches,plan", [([16], 1), ([8, 8, 8], 1), ([3, 1, 40], 2), ([64, 64], 3), ([64, 64], 4),
                                           ([300], 1)])
def test_pred_cornell_crop(require_gpu, launches, plan):
    """A crop through both spheres (sphere interiors, rims, the gap between them: second sphere hits that break
    the prediction), launch sizes 1-300, plans none / rebuilt / 32 / 64 lanes."""
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    pt, lin, bgra = _render(ps, launches, True, plan=plan)
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("depth", [1, 2, 3, 16])
def test_pred_depths(require_gpu, depth):
    """max_depth 1 (a sphere hit ends on its scatter at once: two slots), 2, 3 and 16."""
    ps = pixel_set(1920, 1080, 900, 980, 480, 1, 24)
    pt, lin, bgra = _render(ps, [16, 16], True, depth=depth)
    fr = oracle_render("cornell", 1920, 1080, 0, depth, pixels=ps, launches=[16, 16])
    _check(pt, lin, bgra, fr)


def test_pred_chains_leaving_their_window(require_gpu):
    """Windows far too small (one slot per sample before any history): chains leave them and continue in new
    rounds, each with its own phases A and B; a frame counter beyond 2^32."""
    ps = pixel_set(1920, 1080, 900, 980, 480, 1, 24)
    f0 = (1 << 33) + 3
    pt, lin, bgra = _render(ps, [32, 8], True, frame0=f0, rho0=256)
    sc, pk = scene_for("cornell")
    from iqpt import make_camera
    fr = oracle.OracleFrame(1920, 1080, pixels=ps, max_depth=8)
    fr.frame = f0
    for s in [32, 8]:
        fr.render(pk, make_camera(1920, 1080), s)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (3, 4), (1, 2)])
def test_pred_row_share_equals_whole_slots(require_gpu, rank, world):
    """A C3 row share over three 64-spp launches: predicted chains = every slot traced whole, bit for bit."""
    from iqpt import dist as iqdist
    ps = iqdist.pixel_set_for_rank(1920, 1080, rank, world)
    outs = []
    for pred in (True, False):
        pt, lin, bgra = _render(ps, [64, 64, 64], pred)
        outs.append((lin, bgra, pt.read_rng(), pt.rays()))
        pt.close()
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]
