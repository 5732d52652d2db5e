"""Soundness of the sphere-BVH bound (csrc/iq_bvh.hpp `sphere_growth`) used to skip spheres.

A node may be skipped only if none of its spheres is "non-inert" for the ray: the reference's own
float32 sphere test (shape.cu:13-46, the kernel's operation sequence, replayed here in numpy binary32,
which has no FMA) must find delta < 0 or a far root below t_min. The bound says: when the float test
finds delta >= 0 and t_far >= t_min, the exact ray line passes within r + growth(S) of the centre
(S >= |c - o|), the grown sphere's far crossing lies beyond t_min - 20 u S, and the computed near root
is no earlier than the grown sphere's entry minus 20 u S (what lets a node be skipped behind the running
closest hit). This test attacks the bound with rays chosen to be badly conditioned — lines tangent to
the sphere within a few ulp, origins from 1e-3 to 1e4 away, tiny and huge radii, directions whose
|d|^2 is off by up to 2^-10 — and checks every non-inert case in float64 (exact to ~1e-16 relative).
"""
import ctypes as C

import numpy as np
import pytest

from iqpt import _lib

f32 = np.float32
U = 2.0 ** -24
T_MIN = f32(0.000001)


def growth(rmin, rmax, S, eps=8 * U):
    """The kernel's growth with the ray's |d|^2 deviation eps folded in (iqpt_kernels.hip sbvh_pass),
    in double; checked against the library's host restatement for eps at its floor."""
    K = (24 * U * rmax * rmax + (86 * U + 2.01 * eps) * S * S) * (1 + 2 ** -8) + 2.01 * eps * rmax * rmax
    return K / (np.sqrt(rmin * rmin + K) + rmin) + 4 * U * S + 8 * U * rmax


def test_growth_matches_library():
    lib = _lib.load()
    lib.iqpt_debug_sphere_growth.argtypes = [C.c_double, C.c_double, C.c_double]
    lib.iqpt_debug_sphere_growth.restype = C.c_double
    for r, S in [(0.04, 5.0), (10.0, 30.0), (1e-3, 100.0), (2.0, 0.01)]:
        lib_g = lib.iqpt_debug_sphere_growth(r, r, S)
        K = 24 * U * r * r + 86 * U * S * S
        assert abs(lib_g - (K / (np.sqrt(r * r + K) + r) + 4 * U * S + 8 * U * r)) <= 1e-12 * max(1.0, lib_g)
        assert growth(r, r, S) >= lib_g


def float_test(c, r, o, d):
    """(delta, t_near, t_far) as float32, shape.cu:13-46 in the kernel's operation order."""
    c, o, d, r = (np.asarray(v, f32) for v in (c, o, d, r))
    oc = c - o
    halfb = (d[..., 0] * oc[..., 0] + d[..., 1] * oc[..., 1]) + d[..., 2] * oc[..., 2]
    cc = ((oc[..., 0] * oc[..., 0] + oc[..., 1] * oc[..., 1]) + oc[..., 2] * oc[..., 2]) - r * r
    delta = halfb * halfb - cc
    with np.errstate(invalid="ignore"):
        sd = np.sqrt(np.maximum(delta, f32(0)))
    return delta, halfb - sd, halfb + sd


def check_cases(c, r, o, d):
    """Every non-inert case must satisfy the bound; returns how many were non-inert."""
    delta, tn, tf = float_test(c, r, o, d)
    live = (delta >= 0) & (tf >= T_MIN)
    c64, o64, d64 = (np.asarray(v, np.float64) for v in (c, o, d))
    r64 = np.asarray(r, np.float64)
    w = c64 - o64
    S = np.linalg.norm(w, axis=-1)
    dd = np.sum(d64 * d64, axis=-1)
    eps = np.abs(np.sum(np.asarray(d, f32).astype(np.float64) ** 2, axis=-1) - 1.0) + 8 * U
    rho = np.linalg.norm(np.cross(w, d64), axis=-1) / np.sqrt(dd)
    R = r64 + growth(r64, r64, S, eps)
    assert np.all(rho[live] <= R[live]), np.max((rho - R)[live])
    # the grown sphere's crossings along the (non-unit) direction: s = (w.d -+ sqrt(...)) / |d|^2
    wd = np.sum(w * d64, axis=-1)
    disc = np.maximum(wd * wd - dd * (S * S - R * R), 0.0)
    s_near = (wd - np.sqrt(disc)) / dd
    s_far = (wd + np.sqrt(disc)) / dd
    slack = (20 * U + 4 * eps) * S
    assert np.all(s_far[live] >= T_MIN - slack[live])
    assert np.all(tn[live] >= s_near[live] - slack[live] - 1e-30)
    return int(live.sum())


def unit(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


@pytest.mark.parametrize("seed", range(4))
def test_tangent_rays(seed):
    """Lines whose exact distance to the centre is r (1 +- 1e-7): the float test's decision flips."""
    rng = np.random.default_rng(seed)
    n = 200000
    r = (10.0 ** rng.uniform(-3, 1, n))
    c = rng.uniform(-20, 20, (n, 3))
    dist = 10.0 ** rng.uniform(-3, 4, n)
    d = unit(rng.normal(size=(n, 3)))
    perp = unit(np.cross(d, rng.normal(size=(n, 3))))
    # closest approach at parameter s0 (ahead, behind, or at the origin), at distance r (1 + tiny)
    s0 = dist * rng.choice([-1.0, 0.0, 1.0], n)
    rho = r * (1.0 + rng.uniform(-3e-7, 3e-7, n))
    o = c - perp * rho[:, None] - d * s0[:, None]
    live = check_cases(c.astype(f32), r.astype(f32), o.astype(f32), d.astype(f32))
    assert live > 1000


@pytest.mark.parametrize("seed", range(3))
def test_origins_near_and_inside(seed):
    """Origins on, just outside and inside the surface (secondary rays leave a sphere 1e-4 off it)."""
    rng = np.random.default_rng(100 + seed)
    n = 200000
    r = 10.0 ** rng.uniform(-2, 1, n)
    c = rng.uniform(-5, 5, (n, 3))
    nrm = unit(rng.normal(size=(n, 3)))
    o = c + nrm * (r * (1.0 + rng.choice([-1e-3, -1e-7, 0.0, 1e-7, 1e-4 / 0.5], n)))[:, None]
    d = unit(rng.normal(size=(n, 3)))
    live = check_cases(c.astype(f32), r.astype(f32), o.astype(f32), d.astype(f32))
    assert live > 1000


def test_non_unit_directions():
    """|d|^2 off by up to 2^-10 (the sphere BVH's limit; the pdf fallback's direction is a hit normal)."""
    rng = np.random.default_rng(7)
    n = 200000
    r = 10.0 ** rng.uniform(-2, 0.5, n)
    c = rng.uniform(-10, 10, (n, 3))
    d = unit(rng.normal(size=(n, 3))) * (1.0 + rng.uniform(-2 ** -11, 2 ** -11, n))[:, None]
    perp = unit(np.cross(d, rng.normal(size=(n, 3))))
    s0 = 10.0 ** rng.uniform(-2, 2, n)
    o = c - perp * (r * (1.0 + rng.uniform(-1e-6, 1e-6, n)))[:, None] - d * s0[:, None]
    live = check_cases(c.astype(f32), r.astype(f32), o.astype(f32), d.astype(f32))
    assert live > 1000


def test_c5_like_grid():
    """The C5 layout: 0.04-radius spheres on a ground plane, rays leaving the ground at all angles."""
    rng = np.random.default_rng(11)
    n = 200000
    k = rng.integers(0, 999, n)
    c = np.stack([-2 + 0.1 * (k % 40), np.full(n, 0.04), -0.5 + 0.1 * (k // 40)], axis=-1)
    r = np.full(n, 0.04)
    o = np.stack([rng.uniform(-2.2, 2.2, n), rng.uniform(-1e-3, 0.2, n), rng.uniform(-0.7, 2.1, n)], axis=-1)
    d = unit(np.stack([rng.normal(size=n), np.abs(rng.normal(size=n)) * rng.uniform(0, 0.3, n),
                       rng.normal(size=n)], axis=-1))
    live = check_cases(c.astype(f32), r.astype(f32), o.astype(f32), d.astype(f32))
    assert live > 100
