"""Even slots of 2-slot sphere pixels in the spec kernel (kspec::even2, iqpt_debug_set_spec_even; DESIGN.md
§3.11 "Round 4"): round 0 of a pixel whose last chain took exactly two slots per sample traces only the
even slots of its window; where the chain lands on an odd slot (a sample of one or three slots) the round
ends and the next one traces every slot from there. The launches after the first (which builds the
history) run that path; bit for bit against the oracle (accumulator, BGRA8, RNG states, ray counts) and
against the same launches with every slot traced. RMSE < 1e-5 stated."""
import ctypes as C

import numpy as np
import pytest

from helpers import compare, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
SPLIT_SPEC = 4


def _render(w, h, ps, launches, even, plan=1, frame0=None, depth=8):
    from iqpt import PathTracer, _lib, make_camera
    lb = _lib.load()
    lb.iqpt_debug_set_spec_even.argtypes = [C.c_void_p, C.c_int]
    lb.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
    sc, pk = scene_for("cornell")
    pt = PathTracer(w, h, pixels=ps, max_depth=depth)
    pt._scene = sc
    pt.set_split(SPLIT_SPEC)
    _lib.check(lb.iqpt_debug_set_spec_even(pt.handle, 1 if even else 0), "iqpt_debug_set_spec_even")
    _lib.check(lb.iqpt_debug_spec_plan(pt.handle, plan), "iqpt_debug_spec_plan")
    if frame0 is not None:
        lb.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
        _lib.check(lb.iqpt_debug_set_frame(pt.handle, frame0), "iqpt_debug_set_frame")
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
        pt.sync()                          # the history of each launch is there for the next one's plan
    lin, bgra = pt.read()
    return pt, lin, bgra


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < 1e-5 and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches,plan", [([16, 16, 16], 1), ([64, 64, 64], 1), ([64, 64, 64], 2),
                                           ([8, 64, 3, 40], 2), ([32, 1, 32], 3), ([64, 64], 4)])
def test_even_slots_cornell_crop(require_gpu, launches, plan):
    """A crop through both spheres (sphere interiors at exactly two slots per sample, rims and the gap
    between the spheres at one or three): launches of several sizes, plans none / async / rebuilt / 32 / 64 lanes."""
    ps = pixel_set(1920, 1080, 880, 1000, 470, 1, 48)
    pt, lin, bgra = _render(1920, 1080, ps, launches, True, plan=plan)
    fr = oracle_render("cornell", 1920, 1080, 0, 8, pixels=ps, launches=launches)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (1, 2)])
def test_even_slots_row_share_equals_every_slot(require_gpu, rank, world):
    """A C3 row share over four 64-spp launches: even slots on = off, bit for bit (state and ray counts)."""
    from iqpt import dist as iqdist
    ps = iqdist.pixel_set_for_rank(1920, 1080, rank, world)
    outs = []
    for even in (True, False):
        pt, lin, bgra = _render(1920, 1080, ps, [64, 64, 64, 64], even)
        outs.append((lin, bgra, pt.read_rng(), pt.rays()))
        pt.close()
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


def test_even_slots_depths_and_frame_counter(require_gpu):
    """Depth 2 (a sphere hit at the last bounce ends on the scatter) and a frame counter beyond 2^32."""
    ps = pixel_set(1920, 1080, 900, 980, 480, 1, 24)
    f0 = (1 << 33) + 5
    pt, lin, bgra = _render(1920, 1080, ps, [16, 16, 16], True, frame0=f0, depth=2)
    from iqpt import make_camera
    import oracle
    sc, pk = scene_for("cornell")
    fr = oracle.OracleFrame(1920, 1080, pixels=ps, max_depth=2)
    fr.frame = f0
    for s in [16, 16, 16]:
        fr.render(pk, make_camera(1920, 1080), s)
    _check(pt, lin, bgra, fr)
