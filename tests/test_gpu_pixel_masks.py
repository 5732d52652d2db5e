"""Per-pixel candidate masks over the streamed kernel's tile lists (round 6, kparams::pmask): a lane
walks only the list entries its own pixel's camera rays may meet (iq_interval.h tri_culled on the pixel's jitter
square). The C4 geometry (a 10k-triangle ball, every triangle emissive: any-hit) and the same scene under the
closest-hit search, in full-width bands that cross both silhouettes and the poles, must equal the oracle bit for bit
— accumulator, BGRA8, XORWOW states and ray counts — and equal the launches without masks."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import PathTracer, Scene, _lib, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def run(w, h, ps, launches, masks=True, anyhit=True, depth=8):
    sc = Scene()
    sc.add_preset("mesh10k")
    pk = sc.build_packet()
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=depth)
    lb = _lib.load()
    lb.iqpt_debug_set_pixel_masks.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_pixel_masks(pt._h, 1 if masks else 0), "iqpt_debug_set_pixel_masks")
    lb.iqpt_debug_set_anyhit.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_anyhit(pt._h, 1 if anyhit else 0), "iqpt_debug_set_anyhit")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
    pt.sync()
    lb.iqpt_debug_pixel_mask_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    n = C.c_uint32(0)
    _lib.check(lb.iqpt_debug_pixel_mask_info(pt._h, C.byref(n)), "iqpt_debug_pixel_mask_info")
    lin, bgra = pt.read()
    out = (lin, bgra, pt.read_rng(), pt.rays(), n.value)
    pt.close()
    return out, (sc, pk), cam


def check_oracle(out, scene, cam, w, h, ps, launches, depth=8):
    _, pk = scene                       # the packet's arrays live as long as its Scene
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=depth)
    for s in launches:
        fr.render(pk, cam, s)
    lin, bgra, rng, rays, _ = out
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(rng, fr.states)
    assert rays == int(fr.rays.sum())


@pytest.mark.parametrize("anyhit", [1, 0])
def test_bands_match_oracle(require_gpu, anyhit):
    """Full-width bands through the ball's silhouettes and pole rows, launches of 2 and 1 samples."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 0, w, 150, 97, 9)
    launches = [2, 1]
    out, scene, cam = run(w, h, ps, launches, anyhit=bool(anyhit))
    assert out[4] > 0, "no tile got per-pixel masks"
    check_oracle(out, scene, cam, w, h, ps, launches)


def test_masks_on_equals_off(require_gpu):
    """A crop around the ball's upper silhouette, 16 samples in three launches: masks on and off, same bits."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 700, 1220, 180, 1, 80)
    on, _, _ = run(w, h, ps, [8, 5, 3])
    off, _, _ = run(w, h, ps, [8, 5, 3], masks=False)
    assert on[4] > 0 and off[4] == 0
    assert np.array_equal(on[0].view(np.uint32), off[0].view(np.uint32))
    assert np.array_equal(on[1], off[1])
    assert np.array_equal(on[2], off[2])
    assert on[3] == off[3]
