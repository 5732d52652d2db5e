"""The fan kernel (iqpt_fan_kernel) vs the CPU oracle, bit for bit, as spec launches run it
(IQPT_SPLIT_SPEC: the sphere pixels in iqpt_spec_kernel, every other pixel in the fan kernel on a second stream).

A pixel whose camera rays cannot reach a sphere ends every path on its first ray (every triangle is
emissive under the reference's materials, path_tracer.cu:248-249, 278), so its sample k starts 2k draws
into the pixel's XORWOW stream (camera.cu:24-25). The fan kernel spreads each pixel's samples over four
waves and folds them in sample order; the result must be the reference's sequential chain: accumulator,
BGRA8, final RNG states and the ray count (path_tracer.cu:330-366). RMSE < 1e-5 stated. Covered: row
shares, ragged edge tiles, chunked launches (spp > 64, partial last chunk, spp < 4: empty wave ranges),
depths 1 and 16, frame counters beyond 2^32. Round 6 archived the FAN and CHAIN launch modes (the fan
kernel beside the plain or the chain kernel): the library refuses them.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, gpu_render, oracle_render, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5
SPLIT_OFF, SPLIT_CHAIN, SPLIT_FAN, SPLIT_SPEC = 0, 2, 3, 4
MODE_SPEC = 6          # iqpt_debug_split_info's launch mode of a spec launch (spec + fan kernels)


def mode_of(pt) -> int:
    from iqpt import _lib
    lb = _lib.load()
    lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    info = (C.c_ulonglong * 8)()
    _lib.check(lb.iqpt_debug_split_info(pt._h, info), "iqpt_debug_split_info")
    return int(info[7])


def _check(pt, lin, bgra, fr):
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("launches", [[16], [8, 8, 8], [3, 1, 40], [64, 64]])
def test_cornell_fan(require_gpu, launches):
    """A 320x180 Cornell frame: wall / sky pixels in the fan kernel beside the sphere pixels' spec kernel."""
    pt, lin, bgra = gpu_render("cornell", 320, 180, 0, 8, launches=launches, split=SPLIT_SPEC)
    assert mode_of(pt) == MODE_SPEC
    fr = oracle_render("cornell", 320, 180, 0, 8, launches=launches)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("rank,world", [(0, 8), (5, 8), (1, 3), (0, 2), (3, 4)])
def test_row_share_fan(require_gpu, rank, world):
    """A rank's cyclic row share of a 484x270 Cornell frame (ragged tiles at the right edge)."""
    w, h = 484, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12], split=SPLIT_SPEC)
    assert mode_of(pt) == MODE_SPEC
    fr = oracle_render("cornell", w, h, 0, 8, pixels=ps, launches=[12, 12])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("spp", [1, 2, 3, 5, 65, 130, 200])
def test_chunks_fan(require_gpu, spp):
    """Launch sizes around the chunk of 64 samples and the four wave ranges (some empty for spp < 4)."""
    pt, lin, bgra = gpu_render("cornell", 203, 117, 0, 8, launches=[spp, 7], split=SPLIT_SPEC)
    assert mode_of(pt) == MODE_SPEC
    fr = oracle_render("cornell", 203, 117, 0, 8, launches=[spp, 7])
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("depth", [1, 16])
def test_depths_fan(require_gpu, depth):
    """max_depth 1 and 16 (the MAXD-16 spec variant beside the fan kernel)."""
    pt, lin, bgra = gpu_render("app_default", 160, 90, 0, depth, launches=[20, 7], split=SPLIT_SPEC)
    assert mode_of(pt) == MODE_SPEC
    fr = oracle_render("app_default", 160, 90, 0, depth, launches=[20, 7])
    _check(pt, lin, bgra, fr)


def test_large_frame_counter_fan(require_gpu):
    """The running mean at frame counters beyond 2^32 (64-bit conversions and the tiny-colour path)."""
    from iqpt import PathTracer, _lib, make_camera
    frame0 = (1 << 33) + 5
    w, h = 96, 64
    sc, pk = scene_for("cornell")          # the scene owns the packet's arrays: keep it alive
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=8)
    pt.set_split(SPLIT_SPEC)
    lib = _lib.load()
    lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
    _lib.check(lib.iqpt_debug_set_frame(pt._h, frame0), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    fr.frame = frame0
    for s in (4, 9):
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    assert mode_of(pt) == MODE_SPEC
    _check(pt, lin, bgra, fr)


def test_archived_modes_refused(require_gpu):
    """IQPT_SPLIT_CHAIN and IQPT_SPLIT_FAN (archived in round 6) are refused with IQPT_ERR_UNSUPPORTED."""
    from iqpt import PathTracer, _lib
    pt = PathTracer(64, 48, max_depth=8)
    for mode in (SPLIT_CHAIN, SPLIT_FAN):
        with pytest.raises(_lib.IqptError) as e:
            pt.set_split(mode)
        assert e.value.status == 6
    pt.close()


def test_c3_share8_fan_vs_plain(require_gpu):
    """Rank 0's N = 8 row share of the full C3 frame (1920x1080, 64 spp, 8 bounces), two launches: spec launches
    (the fan kernel beside the spec kernel) equal the plain kernel bit for bit (the plain kernel equals the oracle
    on the whole frame: test_gpu_fullframe)."""
    w, h = 1920, 1080
    n = len(range(0, h, 8))
    ps = pixel_set(w, h, 0, w, 0, 8, n)
    outs = []
    for mode in (SPLIT_OFF, SPLIT_SPEC):
        pt, lin, bgra = gpu_render("cornell", w, h, 0, 8, pixels=ps, launches=[64, 64], split=mode)
        outs.append((lin, bgra, pt.read_rng(), pt.rays(), mode_of(pt)))
        pt.close()
    assert [o[4] for o in outs] == [0, MODE_SPEC]
    for o in outs[1:]:
        assert np.array_equal(outs[0][0].view(np.uint32), o[0].view(np.uint32))
        assert np.array_equal(outs[0][1], o[1])
        assert np.array_equal(outs[0][2], o[2])
        assert outs[0][3] == o[3]
