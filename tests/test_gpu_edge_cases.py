"""GPU parity on edge cases of the kernel's layouts and limits (vs the oracle, bit for bit):
odd triangle / sphere counts (pair tails), the LDS-streamed path with ragged batches, every
max_depth bound, spp above the running-mean table, 1-pixel and 1-row frames, non-default cameras,
singular normal matrices (the reference's mat3x3(INFINITY) quirk) and empty scenes."""
import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import PathTracer, Scene, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def run_both(scene, w, h, launches, depth, pixels=None, camera=None):
    pk = scene.build_packet()
    cam = camera or make_camera(w, h)
    pt = PathTracer(w, h, pixels=pixels, max_depth=depth)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, pixels=pixels, max_depth=depth)
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    return fr


def odd_scene(n_extra_spheres=3):
    sc = Scene()
    sc.add_mesh_tri("a_tri")                    # 1 triangle
    sc.add_mesh_quad("b_quad")                  # 2 triangles
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("t1", "a_tri", 0.8, 0.0, (0.3, 0.4, 0.6))
    sc.add_model("q1", "b_quad", (3.0, 3.0, 1.0), (1.2, 0.0, 0.0), (0.0, -0.6, 0.5))
    sc.add_model("q2", "b_quad", (1.5, 1.5, 1.0), (0.0, 0.5, 0.0), (-0.9, 0.5, 0.8))
    for i in range(n_extra_spheres):
        sc.add_model(f"s{i}", "sphere", 0.2 + 0.05 * i, 0.0, (-0.5 + 0.45 * i, 0.1 * i, 0.2))
    return sc


@pytest.mark.parametrize("depth", [1, 2, 5, 8, 9, 16])
def test_odd_counts_every_depth(require_gpu, depth):
    run_both(odd_scene(3), 96, 64, [3], depth)      # 5 triangles, 3 spheres: both pair tails


def test_streamed_path_with_ragged_batches(require_gpu):
    """601 triangles x 3 models + 7 spheres > the 32 KiB resident budget: LDS batches of 256 pairs
    with a ragged last batch and an odd triangle count."""
    sc = Scene()
    sc.add_mesh_uv_sphere("ball", False, 21, 15, 1 - 1)      # TRIANGLES: 2*21*14 = 588 tris
    sc.add_mesh_tri("c_tri")
    sc.add_mesh_uv_sphere("sphere")
    for i in range(3):
        sc.add_model(f"b{i}", "ball", 0.3, (0.1 * i, 0.2, 0.0), (-0.7 + 0.7 * i, 0.4, 0.3))
    sc.add_model("t", "c_tri", 2.0, 0.0, (0.0, 0.0, 1.5))
    for i in range(7):
        sc.add_model(f"s{i}", "sphere", 0.12, 0.0, (-0.9 + 0.3 * i, -0.2, -0.4))
    ps = pixel_set(160, 90, 40, 120, 10, 2, 35)
    run_both(sc, 160, 90, [2, 1], 8, pixels=ps)


def test_spp_above_the_mean_table(require_gpu):
    """1100 spp in one launch exceeds kAccTableMax (1024): the kernel falls back to the divisions."""
    ps = pixel_set(64, 36, 30, 34, 16, 1, 2)
    sc = Scene()
    sc.add_preset("cornell")
    run_both(sc, 64, 36, [1100], 8, pixels=ps)


@pytest.mark.parametrize("w,h,ps", [(1, 1, None), (257, 1, None), (1, 300, None), (300, 200, (299, 300, 0, 7, 29))])
def test_tiny_and_ragged_frames(require_gpu, w, h, ps):
    sc = Scene()
    sc.add_preset("app_default")
    pixels = pixel_set(w, h, *ps) if ps else None
    run_both(sc, w, h, [2], 5, pixels=pixels)


def test_non_default_camera(require_gpu):
    cam = make_camera(120, 80, fovh=70.0, znear=0.05, zfar=50.0, position=(0.3, 1.2, -2.0, 0.0),
                      forward=(-0.1, -0.6, 1.0, 0.0))
    sc = Scene()
    sc.add_preset("cornell")
    run_both(sc, 120, 80, [4], 8, camera=cam)


def test_singular_normal_matrix_and_empty_scene(require_gpu):
    sc = Scene()
    sc.add_mesh_quad("q")
    sc.add_model("tiny", "q", 0.01, 0.0, (0.0, 0.5, 0.0))  # det 1e-6 < 1e-5: infinite normal matrix
    sc.add_model("wall", "q", 3.0, 0.0, (0.0, 0.5, 1.0))
    run_both(sc, 64, 48, [2], 5)
    run_both(Scene(), 48, 32, [3], 5)


@pytest.mark.parametrize("case", ["edges_2^59", "edges_2^61", "denormal_radius", "huge_radius"])
def test_fast_division_range(require_gpu, case):
    """kOptFastDiv (iq_fastdiv.h) is exact only for reciprocals in [2^-126, 2^126): packets whose edge
    components stay within 2^60 keep the fast variant (here with determinants near 2^118), larger
    edges or radii outside the range switch the launch to the generic-division variant. Both must
    match the oracle bit for bit."""
    sc = odd_scene(2)
    if case.startswith("edges"):
        s = 2.0 ** (59 if case.endswith("59") else 61)
        sc.add_model("giant", "b_quad", (s, s, 1.0), 0.0, (0.0, 0.0, 2.0 ** 62))
        sc.add_model("near", "b_quad", (s, s, 1.0), (0.3, 0.2, 0.0), (0.0, 0.5, 3.0))
    elif case == "denormal_radius":
        sc.add_model("dust", "sphere", 1e-40, 0.0, (0.0, 0.5, 0.5))
    else:
        sc.add_model("shell", "sphere", 2.0 ** 126, 0.0, (0.0, 0.0, 0.0))
    run_both(sc, 80, 60, [3], 8)
