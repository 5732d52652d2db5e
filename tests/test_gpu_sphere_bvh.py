"""Exact sphere BVH (iq_bvh.hpp, iqpt_kernels.hip sbvh_closest) vs the oracle's brute-force fold, bit for
bit: a C5-like grid of small spheres with the ground sphere on the always-tested list, ray origins
inside spheres (the fold's order-dependent far-root case, both from the camera and after bounces),
nested and overlapping spheres, duplicated spheres (every hit an exact t tie: the later sphere must
win) with different emissive colours, and camera rays through the BVH as well."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import MAT_EMISSIVE, MAT_OREN_NAYAR, PathTracer, Scene, _lib, make_camera, pixel_set

pytestmark = pytest.mark.gpu


def sbvh_info(pt):
    lb = _lib.load()
    lb.iqpt_debug_sbvh_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    n, a = C.c_uint32(0), C.c_uint32(0)
    _lib.check(lb.iqpt_debug_sbvh_info(pt._h, C.byref(n), C.byref(a)), "iqpt_debug_sbvh_info")
    return n.value, a.value


def prim_opt():
    """kOptDefault | kOptBvhPrimary, a production variant (read from the library: no GPU needed)."""
    return _lib.load().iqpt_debug_default_options() | (1 << 12)


def run_both(scene, w, h, launches, depth, camera=None, pixels=None, opt=None):
    pk = scene.build_packet()
    cam = camera or make_camera(w, h)
    pt = PathTracer(w, h, max_depth=depth, pixels=pixels)
    if opt == "prim":
        opt = prim_opt()
    if opt is not None:
        lb = _lib.load()
        lb.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_kernel_options(pt._h, opt), "iqpt_debug_set_kernel_options")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    fr = oracle.OracleFrame(w, h, max_depth=depth, pixels=pixels)
    for s in launches:
        pt.render(s)
        fr.render(pk, cam, s)
    lin, bgra = pt.read()
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    info = sbvh_info(pt)
    pt.close()
    return info


def streamed_base(sc):
    """A 900-triangle mesh: the scene exceeds the LDS-resident budget (the streamed kernel, where the
    BVHs live)."""
    sc.add_mesh_uv_sphere("ball", False, 30, 16, 0)
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("ball", "ball", 0.3, (0.2, 0.1, 0.0), (0.9, 0.35, 0.6))


def grid(sc, n, r=0.04, y=0.04, prefix="s"):
    for i in range(n):
        sc.add_model(f"{prefix}{i:04d}", "sphere", r, 0.0, (-1.2 + 0.1 * (i % 25), y, -0.3 + 0.1 * (i // 25)))


@pytest.mark.parametrize("opt", [None, "prim"], ids=["auto", "prim"])
def test_grid_with_ground_on_always_list(require_gpu, opt):
    sc = Scene()
    streamed_base(sc)
    grid(sc, 300)
    sc.add_model("ground", "sphere", 10.0, 0.0, (0.0, -10.0, 0.0))
    nodes, always = run_both(sc, 96, 64, [2, 1], 8, opt=opt)
    assert nodes > 0 and always == 1


@pytest.mark.parametrize("opt", [None, "prim"], ids=["auto", "prim"])
def test_origins_inside_spheres(require_gpu, opt):
    """Camera inside a sphere of the BVH (every camera ray takes that sphere's far root), plus nested and
    overlapping spheres so that bounces also start inside spheres."""
    sc = Scene()
    streamed_base(sc)
    grid(sc, 120, r=0.08, y=0.0)
    sc.add_model("bubble", "sphere", 0.3, 0.0, (0.0, 0.5, -3.0))           # the camera sits in it
    sc.add_model("nest_a", "sphere", 0.35, 0.0, (0.0, 0.45, 0.4))
    sc.add_model("nest_b", "sphere", 0.2, 0.0, (0.05, 0.45, 0.4))          # inside nest_a
    sc.add_model("nest_c", "sphere", 0.25, 0.0, (0.3, 0.5, 0.4))           # overlaps nest_a
    nodes, always = run_both(sc, 80, 60, [2], 8, opt=opt)
    assert nodes > 0 and always == 0


@pytest.mark.parametrize("opt", [None, "prim"], ids=["auto", "prim"])
def test_duplicate_spheres_tie_to_the_later_one(require_gpu, opt):
    """Every sphere twice at the same place: each hit is an exact t tie and the later (second) sphere's
    material must be the one shaded — the duplicates are emissive with different colours."""
    sc = Scene()
    streamed_base(sc)
    red = sc.add_material(MAT_EMISSIVE, (1.0, 0.1, 0.1, 1.0), 2.0)
    blue = sc.add_material(MAT_EMISSIVE, (0.1, 0.1, 1.0, 1.0), 2.0)
    rough = sc.add_material(MAT_OREN_NAYAR, (0.6, 0.6, 0.6, 0.0), 0.8)
    for i in range(80):
        x, z = -1.0 + 0.25 * (i % 10), 0.0 + 0.2 * (i // 10)
        for tag, m in (("a", red), ("b", blue)):
            name = f"d{i:03d}{tag}"
            sc.add_model(name, "sphere", 0.09, 0.0, (x, 0.1, z))
            sc.set_model_material(name, m)
    sc.add_model("floor", "sphere", 10.0, 0.0, (0.0, -10.0, 0.0))
    sc.set_model_material("floor", rough)
    sc.set_model_material("ball", rough)
    nodes, always = run_both(sc, 96, 64, [3], 6, opt=opt)
    assert nodes > 0


def test_c5_band_through_both_bvhs(require_gpu):
    """The C5 scene (50k triangles, 1000 spheres) on a band of 4K rows, several launches (camera rays
    switch between tile masks and the BVHs after the first two)."""
    sc = Scene()
    sc.add_preset("mixed")
    ps = pixel_set(3840, 2160, 1200, 1520, 1500, 2, 12)
    nodes, always = run_both(sc, 3840, 2160, [1, 1, 1], 8, pixels=ps)
    assert nodes > 0 and always == 1
