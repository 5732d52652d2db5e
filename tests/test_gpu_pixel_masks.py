"""Per-pixel candidate masks over the streamed kernel's tile lists (round 6, kparams::pmask): a lane
walks only the list entries its own pixel's camera rays may meet (iq_interval.h tri_culled on the pixel's jitter
square) — in the plain kernel (mode 1) or, for any-hit scenes whose every tile has masks, in iqpt_anyhit_kernel
(mode 2, the default; bit 29 of iqpt_debug_last_options). The C4 geometry (a 10k-triangle ball, every triangle
emissive: any-hit) and the same scene under the closest-hit search, in full-width bands that cross both silhouettes
and the poles, must equal the oracle bit for bit — accumulator, BGRA8, XORWOW states and ray counts — and equal
the launches without masks."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import PathTracer, Scene, _lib, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def run(w, h, ps, launches, mode=2, anyhit=True, depth=8):
    sc = Scene()
    sc.add_preset("mesh10k")
    pk = sc.build_packet()
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=depth)
    lb = _lib.load()
    lb.iqpt_debug_set_pixel_masks.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_pixel_masks(pt._h, mode), "iqpt_debug_set_pixel_masks")
    lb.iqpt_debug_set_anyhit.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_anyhit(pt._h, 1 if anyhit else 0), "iqpt_debug_set_anyhit")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    anyk = []
    for s in launches:
        pt.render(s)
        o = C.c_int(0)
        _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
        anyk.append(bool(o.value & (1 << 29)))
    pt.sync()
    lb.iqpt_debug_pixel_mask_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_int),
                                              C.POINTER(C.c_uint32)]
    n, every = C.c_uint32(0), C.c_int(0)
    _lib.check(lb.iqpt_debug_pixel_mask_info(pt._h, C.byref(n), C.byref(every), None), "iqpt_debug_pixel_mask_info")
    # iqpt_anyhit_kernel runs exactly where it applies: mode 2, an any-hit scene, masks on every tile
    assert all(a == (mode == 2 and anyhit and bool(every.value)) for a in anyk), (mode, anyhit, every.value, anyk)
    lin, bgra = pt.read()
    out = (lin, bgra, pt.read_rng(), pt.rays(), n.value, bool(every.value))
    pt.close()
    return out, (sc, pk), cam


def check_oracle(out, scene, cam, w, h, ps, launches, depth=8):
    _, pk = scene                       # the packet's arrays live as long as its Scene
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=depth)
    for s in launches:
        fr.render(pk, cam, s)
    lin, bgra, rng, rays = out[:4]
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(rng, fr.states)
    assert rays == int(fr.rays.sum())


@pytest.mark.parametrize("mode,anyhit", [(2, 1), (1, 1), (2, 0)])
@pytest.mark.parametrize("y0,ystep,rows,every", [(150, 97, 9, None), (180, 1, 24, True), (520, 1, 16, True),
                                                  (500, 3, 16, None)])
def test_bands_match_oracle(require_gpu, mode, anyhit, y0, ystep, rows, every):
    """Full-width bands through the ball's silhouettes: rows 97 apart (tiles of owned rows span the frame: long
    lists), contiguous bands through the upper cap and the middle (every tile masked: iqpt_anyhit_kernel in
    mode 2) and every third row (a 3-way row split's share); launches of 2 and 1 samples."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 0, w, y0, ystep, rows)
    launches = [2, 1]
    out, scene, cam = run(w, h, ps, launches, mode=mode, anyhit=bool(anyhit))
    assert out[4] > 0, "no tile got per-pixel masks"
    assert every is None or out[5] == every, out[5]
    check_oracle(out, scene, cam, w, h, ps, launches)


@pytest.mark.parametrize("mode", [2, 1])
def test_masks_on_equals_off(require_gpu, mode):
    """A crop around the ball's upper silhouette, 16 samples in three launches: masks (mode 2 / 1) and none, same
    bits."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 700, 1220, 180, 1, 80)
    on, _, _ = run(w, h, ps, [8, 5, 3], mode=mode)
    off, _, _ = run(w, h, ps, [8, 5, 3], mode=0)
    assert on[4] > 0 and off[4] == 0
    assert np.array_equal(on[0].view(np.uint32), off[0].view(np.uint32))
    assert np.array_equal(on[1], off[1])
    assert np.array_equal(on[2], off[2])
    assert on[3] == off[3]


def test_full_frame_and_frame_counter(require_gpu):
    """The whole C4 scene in a 322 x 181 frame (ragged last tile column and row), two launches, a frame counter past
    2^32."""
    w, h = 322, 181
    sc = Scene()
    sc.add_preset("mesh10k")
    pk = sc.build_packet()
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    lb = _lib.load()
    lb.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
    _lib.check(lb.iqpt_debug_set_frame(pt._h, (1 << 32) + 3), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    fr.frame = (1 << 32) + 3
    for s in (3, 2):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    pt.close()
