"""GPU parity: the HIP kernel (through the C ABI) vs the CPU oracle on identical packets and seeds.

The bar is bit-exactness of the float accumulator, the BGRA8 frame, the XORWOW states and the ray
counts (tolerance stated anyway: per-pixel RMSE < 1e-5, BASELINE.json north_star).
"""
import numpy as np
import pytest

from helpers import compare, gpu_render, oracle_render, pixel_set

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5


def _check(pt, lin, bgra, fr, expect_rays=True):
    c = compare(lin, fr.lin)
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    if expect_rays:
        assert pt.rays() == int(fr.rays.sum())


def test_c1_full_frame(require_gpu):
    """C1: 256x256, 1 spp, 2 bounces — the whole frame."""
    pt, lin, bgra = gpu_render("c1_plumbing", 256, 256, 1, 2)
    fr = oracle_render("c1_plumbing", 256, 256, 1, 2)
    _check(pt, lin, bgra, fr)


@pytest.mark.parametrize("preset,w,h,spp,depth,crop", [
    ("cornell", 1920, 1080, 8, 8, (896, 960, 500, 1, 40)),     # C2 crop through both spheres
    ("mesh10k", 1920, 1080, 2, 8, (930, 970, 380, 1, 12)),     # C4 crop (streams 10k tris through LDS)
    ("mixed", 3840, 2160, 1, 8, (1900, 1940, 1100, 1, 8)),     # C5 crop (50k tris + 1k spheres)
    ("app_default", 320, 180, 16, 5, None),                    # IoniqRE default scene, full frame
])
def test_config_crops(require_gpu, preset, w, h, spp, depth, crop):
    ps = pixel_set(w, h, crop[0], crop[1], crop[2], crop[3], crop[4]) if crop else None
    pt, lin, bgra = gpu_render(preset, w, h, spp, depth, pixels=ps)
    fr = oracle_render(preset, w, h, spp, depth, pixels=ps)
    _check(pt, lin, bgra, fr)


def test_multi_launch_equals_reference_launch_sequence(require_gpu):
    """render(3)+render(2)+render(1) == six 1-spp reference launches (frame counter continues)."""
    ps = pixel_set(640, 360, 200, 440, 100, 1, 64)
    pt, lin, bgra = gpu_render("cornell", 640, 360, 0, 8, pixels=ps, launches=[3, 2, 1])
    fr = oracle_render("cornell", 640, 360, 0, 8, pixels=ps, launches=[1] * 6)
    assert pt.frames() == 6
    _check(pt, lin, bgra, fr)


def test_reset_keeps_rng_and_restarts_mean(require_gpu):
    import oracle
    from iqpt import PathTracer, make_camera
    from helpers import scene_for
    w, h = 160, 90
    sc, pk = scene_for("app_default")
    cam = make_camera(w, h)
    pt = PathTracer(w, h, max_depth=5)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=5)
    pt.render(3)
    fr.render(pk, cam, 3)
    pt.reset()
    fr.reset()
    lin0, bgra0 = pt.read()
    assert not bgra0.any()
    pt.render(2)
    fr.render(pk, cam, 2)
    lin, bgra = pt.read()
    _check(pt, lin, bgra, fr)


def test_row_partition_matches_full_frame(require_gpu):
    """Cyclic row tiles (the multi-GPU partition) reassemble the 1-GPU frame bit for bit."""
    w, h, n = 256, 144, 3
    _, full, _ = gpu_render("cornell", w, h, 4, 8)
    out = np.zeros_like(full)
    for r in range(n):
        ps = pixel_set(w, h, 0, w, r, n, (h - r + n - 1) // n)
        _, lin, _ = gpu_render("cornell", w, h, 4, 8, pixels=ps)
        rows = np.arange(r, h, n)
        out.reshape(h, w, 4)[rows] = lin.reshape(len(rows), w, 4)
    assert np.array_equal(out.view(np.uint32), full.view(np.uint32))
