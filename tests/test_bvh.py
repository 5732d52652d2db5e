"""Soundness of the BVH error bound (csrc/iq_bvh.hpp) used to skip triangles for secondary rays.

A BVH node may be skipped only if the reference's own Möller–Trumbore test (shape.cu:62-103, float32
round-to-nearest, as the oracle and the kernel evaluate it) cannot accept any of its triangles. The
bound says: when the float test accepts with t^, the exact line point o + t d (solved exactly, here in
float64 — its own error is ~1e-16 relative) lies in the triangle's box grown by `delta`, at a t within
dt_a + dt_b t^ of the accepted t^; delta and dt_a grow linearly with S = max_i |o_i - v0_i|, and the
test evaluates them at each ray's own S (the kernel uses an upper bound of it per node). This test attacks it with rays chosen to be badly conditioned —
grazing directions with determinants just above the 1e-6 reject threshold, hits on edges and
vertices, far origins — and checks every accepted hit against the bound. The GPU parity tests then
render streamed scenes whose secondary rays use the BVH and compare with the oracle bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from iqpt import _lib

FP = C.POINTER(C.c_float)
DP = C.POINTER(C.c_double)
T_MIN = np.float32(0.000001)
FLT_MAX = np.float32(3.4028235e38)


def bound(e1, e2, S, Md=1.001, D=0.0):
    """(eligible, [growth, dt_a, dt_b]) of iq_bvh.hpp at distance S and determinant lower bound D."""
    ok, out = bound4(e1, e2, S, Md, D)
    return ok, out[:3]


def bound4(e1, e2, S, Md=1.001, D=0.0):
    lib = _lib.load()
    f = lib.iqpt_debug_bvh_bound
    f.argtypes = [FP, FP, C.c_double, C.c_double, C.c_double, DP]
    f.restype = C.c_int
    e1 = np.ascontiguousarray(e1, np.float32)
    e2 = np.ascontiguousarray(e2, np.float32)
    out = np.zeros(4)
    ok = f(e1.ctypes.data_as(FP), e2.ctypes.data_as(FP), S, Md, D, out.ctypes.data_as(DP))
    return ok == 1, out


def mt(v0, v1, v2, o, d):
    lib = oracle.load()
    z = np.zeros(4, np.float32)
    t = C.c_float()
    p4 = np.zeros(4, np.float32)
    n4 = np.zeros(4, np.float32)
    front = C.c_int()
    a = [np.append(v, np.float32(1)).astype(np.float32) for v in (v0, v1, v2)]
    o4 = np.append(o, np.float32(1)).astype(np.float32)
    d4 = np.append(d, np.float32(0)).astype(np.float32)
    hit = lib.iqo_triangle_intersect(a[0].ctypes.data_as(FP), a[1].ctypes.data_as(FP), a[2].ctypes.data_as(FP),
                                     z.ctypes.data_as(FP), z.ctypes.data_as(FP), z.ctypes.data_as(FP),
                                     o4.ctypes.data_as(FP), d4.ctypes.data_as(FP), T_MIN, FLT_MAX, C.byref(t),
                                     p4.ctypes.data_as(FP), n4.ctypes.data_as(FP), C.byref(front))
    return hit, t.value


def exact_solution(v0, e1, e2, o, d):
    """o + t d = v0 + u e1 + v e2 in float64: (t, u, v)."""
    A = np.stack([d.astype(np.float64), -e1.astype(np.float64), -e2.astype(np.float64)], axis=1)
    return np.linalg.solve(A, v0.astype(np.float64) - o.astype(np.float64))


def unit(v):
    v = v / np.linalg.norm(v)
    return v


@pytest.mark.parametrize("seed", range(4))
def test_accepted_hits_lie_inside_the_grown_box(seed):
    rng = np.random.default_rng(seed)
    checked = grazing = 0
    for _ in range(600):
        size = 10 ** rng.uniform(-2.5, -1)
        v0 = rng.uniform(-8, 8, 3).astype(np.float32)
        e1 = (rng.normal(0, size, 3)).astype(np.float32)
        e2 = (rng.normal(0, size, 3)).astype(np.float32)
        ok, _ = bound(e1, e2, 1.0)
        if not ok:
            continue
        n = np.cross(e1.astype(np.float64), e2.astype(np.float64))
        nn = np.linalg.norm(n)
        if nn < 1e-12:
            continue
        # a target near the triangle's edges / vertices (barycentrics slightly outside too)
        u, v = rng.uniform(-0.02, 1.02, 2)
        if rng.random() < 0.5:
            v = 1.0 - u + rng.uniform(-1e-3, 1e-3)
        X = v0 + u * e1.astype(np.float64) + v * e2.astype(np.float64)
        # grazing direction: sin(angle to the plane) such that |det| ~ [1, 30] x 1e-6
        want_det = 10 ** rng.uniform(-6, -4.5) * rng.choice([-1, 1])
        s = np.clip(want_det / nn, -1, 1)
        tang = unit(np.cross(n, rng.normal(size=3)))
        d = unit(tang * np.sqrt(max(0.0, 1 - s * s)) + (n / nn) * s).astype(np.float32)
        d = (d / np.float32(np.sqrt(np.float32(np.dot(d, d))))).astype(np.float32)
        t = 10 ** rng.uniform(-2, 1.5)
        o = (X - t * d.astype(np.float64)).astype(np.float32)
        S = float(np.max(np.abs(o.astype(np.float64) - v0)))
        hit, that = mt(v0, (v0 + e1).astype(np.float32), (v0 + e2).astype(np.float32), o, d)
        if not hit:
            continue
        # the oracle recomputes e1 = v1 - v0: use the edges it saw
        e1o = ((v0 + e1).astype(np.float32) - v0).astype(np.float32)
        e2o = ((v0 + e2).astype(np.float32) - v0).astype(np.float32)
        ok2, (delta, dta, dtb) = bound(e1o, e2o, S)
        assert ok2
        # the normal-cone form: the same bound priced at this ray's own determinant lower bound
        n = np.cross(e1o.astype(np.float64), e2o.astype(np.float64))
        _, (_, _, _, edet) = bound4(e1o, e2o, S)
        D = abs(float(np.dot(d.astype(np.float64), n))) - edet
        _, (delta_c, dta_c, dtb_c) = bound(e1o, e2o, S, D=D)
        te, ue, ve = exact_solution(v0, e1o, e2o, o, d)
        P = o.astype(np.float64) + te * d.astype(np.float64)
        corners = np.stack([v0, v0 + e1o.astype(np.float64), v0 + e2o.astype(np.float64)])
        lo, hi = corners.min(axis=0) - delta, corners.max(axis=0) + delta
        assert np.all(P >= lo) and np.all(P <= hi), (P, lo, hi, delta, ue, ve)
        assert abs(that - te) <= dta + dtb * abs(that), (that, te, dta, dtb)
        lo, hi = corners.min(axis=0) - delta_c, corners.max(axis=0) + delta_c
        assert np.all(P >= lo) and np.all(P <= hi), (P, lo, hi, delta_c, D)
        assert abs(that - te) <= dta_c + dtb_c * abs(that), (that, te, dta_c, dtb_c, D)
        checked += 1
        det = abs(np.dot(e1o.astype(np.float64), np.cross(d.astype(np.float64), e2o.astype(np.float64))))
        grazing += det < 1e-5
    assert checked > 100 and grazing > 20, (checked, grazing)


def test_large_triangles_are_kept_out_of_the_bvh():
    ok, _ = bound(np.array([2.0, 0, 0], np.float32), np.array([0, 2.0, 0], np.float32), 1.0)
    assert not ok                       # Cornell walls: tested by every ray instead
    e1, e2 = np.array([0.015, 0, 0], np.float32), np.array([0, 0.015, 0.001], np.float32)
    ok, (d1, a1, b1) = bound(e1, e2, 1.0)
    assert ok and d1 < 0.02             # C5's small mesh triangles, seen from 1 unit away
    _, (d2, a2, b2) = bound(e1, e2, 2.0)
    assert d2 > d1 and a2 == pytest.approx(2 * a1) and b2 == b1     # linear in S
    # a ray meeting the triangle at 60 deg from its plane: |det| ~ 1.3e-4, the bound shrinks ~100x
    _, (d3, a3, _) = bound(e1, e2, 1.0, D=1.3e-4)
    assert d3 < d1 / 50 and a3 < a1 / 50
