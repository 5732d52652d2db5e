"""Certain pixels (kparams::certain): a pixel of a tile without a sphere candidate whose every
camera ray is proven to hit one candidate triangle (iq_interval.h tri_certain) folds its samples at once — two draws and
the emissive colour (1, 1, 1) per sample (path_tracer.cu:278, 341-358; camera.cu:24-25) — in the plain
kernel's refill and in the fan kernel. Bit for bit against the oracle, and against the same launches with
the certain path off. RMSE < 1e-5 stated."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, pixel_set, scene_for

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5


def _certain_tiles(pt):
    from iqpt import _lib
    lib = _lib.load()
    lib.iqpt_debug_certain_tiles.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                             C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32]
    n, nt, ntx = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    _lib.check(lib.iqpt_debug_certain_tiles(pt._h, C.byref(n), C.byref(nt), C.byref(ntx), None, 0),
               "iqpt_debug_certain_tiles")
    return n.value, nt.value


def _render(preset, w, h, ps, launches, split, certain, overlap=True, frame0=None):
    from iqpt import PathTracer, _lib, make_camera
    sc, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=ps, max_depth=8)
    pt.set_split(split)
    if not overlap:
        pt.set_overlap(_lib.OVERLAP_OFF)
    lib = _lib.load()
    lib.iqpt_debug_set_certain.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lib.iqpt_debug_set_certain(pt._h, 1 if certain else 0), "iqpt_debug_set_certain")
    if frame0 is not None:
        lib.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
        _lib.check(lib.iqpt_debug_set_frame(pt._h, frame0), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=ps, max_depth=8)
    if frame0 is not None:
        fr.frame = frame0
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    return pt, lin, bgra, fr, sc


@pytest.mark.parametrize("split", [0, 4])
@pytest.mark.parametrize("overlap", [True, False])
def test_certain_tiles_cornell(require_gpu, split, overlap):
    """A 484x270 Cornell frame over three launches in the plain kernel (overlapped or not) and in spec launches
    (the fan kernel's certain path): the oracle's bits, most wall tiles certain."""
    w, h = 484, 270
    pt, lin, bgra, fr, _sc = _render("cornell", w, h, None, [16, 5, 64], split, True, overlap)
    n, nt = _certain_tiles(pt)
    assert nt > 0 and n > 16 * nt, (n, nt)      # certain pixels: over a quarter of the frame
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL and c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())


@pytest.mark.parametrize("rank,world", [(0, 8), (3, 4), (1, 2)])
def test_certain_tiles_row_shares(require_gpu, rank, world):
    """Row shares (ragged tiles at the right and bottom edge): certain on equals certain off bit for bit."""
    w, h = 484, 270
    n = len(range(rank, h, world))
    ps = pixel_set(w, h, 0, w, rank, world, n)
    outs = []
    for certain in (True, False):
        pt, lin, bgra, fr, _sc = _render("cornell", w, h, ps, [12, 12], -1, certain)
        outs.append((lin, bgra, pt.read_rng(), pt.rays()))
        if certain:
            assert _certain_tiles(pt)[0] > 0
            c = compare(lin, fr.lin)
            assert c["bitexact"] == c["npix"], c
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


def test_certain_tiles_large_frame_counter(require_gpu):
    """The fold at frame counters beyond 2^32 (the table's 1/n and (n - 1)/n)."""
    w, h = 256, 144
    pt, lin, bgra, fr, _sc = _render("cornell", w, h, None, [4, 9], 0, True, frame0=(1 << 33) + 7)
    assert _certain_tiles(pt)[0] > 0
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(pt.read_rng(), fr.states)


def test_no_certain_tiles_with_materials(require_gpu):
    """A material table (non-emissive triangles possible): no tile is certain."""
    from iqpt import PathTracer, make_camera
    sc, pk = scene_for("cornell_lit")
    w, h = 160, 96
    pt = PathTracer(w, h, max_depth=8)
    pt.set_camera(make_camera(w, h))
    pt.upload_packet(pk)
    pt.render(2)
    assert _certain_tiles(pt)[0] == 0
