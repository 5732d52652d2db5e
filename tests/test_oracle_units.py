"""Known-answer tests of the oracle's parts against closed-form geometry (the reference ships no
tests: SURVEY.md §4). Each case names the reference routine it pins."""
import ctypes as C

import numpy as np
import pytest

import oracle

FP = C.POINTER(C.c_float)
UP = C.POINTER(C.c_uint32)


def f4(*v):
    a = np.zeros(4, dtype=np.float32)
    a[:len(v)] = v
    return a


def p(a):
    return a.ctypes.data_as(FP)


def tri_hit(v0, v1, v2, o, d, t_min=1e-6, t_max=999.99, n=(0, 0, -1)):
    lib = oracle.load()
    t = C.c_float()
    pt, nn = np.zeros(4, np.float32), np.zeros(4, np.float32)
    front = C.c_int()
    nv = f4(*n)
    hit = lib.iqo_triangle_intersect(p(f4(*v0)), p(f4(*v1)), p(f4(*v2)), p(nv), p(nv.copy()), p(nv.copy()),
                                     p(f4(*o)), p(f4(*d)), t_min, t_max, C.byref(t), p(pt), p(nn), C.byref(front))
    return hit, t.value, pt, nn, front.value


def sph_hit(c, r, o, d, t_min=1e-6, t_max=999.99):
    lib = oracle.load()
    t = C.c_float()
    pt, nn = np.zeros(4, np.float32), np.zeros(4, np.float32)
    front = C.c_int()
    hit = lib.iqo_sphere_intersect(p(f4(*c)), r, p(f4(*o)), p(f4(*d)), t_min, t_max, C.byref(t), p(pt), p(nn),
                                   C.byref(front))
    return hit, t.value, pt, nn, front.value


TRI = ((-1, -1, 0), (0, 1, 0), (1, -1, 0))


def test_triangle_hit_center():
    """shape.cu:62-103 Möller–Trumbore: ray along +z hits z=0 at t=1."""
    hit, t, pt, n, front = tri_hit(*TRI, (0, 0, -1), (0, 0, 1))
    assert hit and t == 1.0 and np.allclose(pt[:3], 0.0)
    # v0v1 x v0v2 = (0, 0, -4): dir·n_g < 0 -> front face, interpolated normal kept (shape.cu:96-101)
    assert front == 1 and np.allclose(n[:3], [0, 0, -1])


def test_triangle_backface_not_culled():
    hit, t, pt, n, front = tri_hit(*TRI, (0, 0, 1), (0, 0, -1))
    assert hit and t == 1.0 and front == 0 and np.allclose(n[:3], [0, 0, 1])   # flipped to face the ray


def test_triangle_t_equal_t_max_is_accepted():
    """`t_max < t` rejects; t == t_max is a hit, so a later primitive at equal t wins."""
    assert tri_hit(*TRI, (0, 0, -1), (0, 0, 1), t_max=1.0)[0] == 1
    assert tri_hit(*TRI, (0, 0, -1), (0, 0, 1), t_max=np.nextafter(np.float32(1), np.float32(0)))[0] == 0


def test_triangle_parallel_and_outside():
    assert tri_hit(*TRI, (0, 0, -1), (1, 0, 0))[0] == 0          # det == 0 (is_zero, iqmath.h:28-31)
    assert tri_hit(*TRI, (5, 0, -1), (0, 0, 1))[0] == 0          # u out of range
    assert tri_hit(*TRI, (0, 2, -1), (0, 0, 1))[0] == 0          # u + v > 1
    assert tri_hit(*TRI, (0, 0, 1), (0, 0, 1))[0] == 0           # t < t_min (behind)


def test_sphere_near_root():
    hit, t, pt, n, front = sph_hit((0, 0, 0), 1.0, (0, 0, -3), (0, 0, 1))
    assert hit and t == 2.0 and front == 1 and np.allclose(n[:3], [0, 0, -1])


def test_sphere_inside_uses_far_root_and_flips_normal():
    hit, t, pt, n, front = sph_hit((0, 0, 0), 1.0, (0, 0, 0), (0, 0, 1))
    assert hit and t == 1.0 and front == 0 and np.allclose(n[:3], [0, 0, -1])


def test_sphere_far_root_not_checked_against_t_max():
    """shape.cu:25-34: the far root is only checked against t_min (reference quirk kept)."""
    hit, t, *_ = sph_hit((0, 0, 0), 1.0, (0, 0, 0), (0, 0, 1), t_max=0.5)
    assert hit and t == 1.0
    assert sph_hit((0, 0, 0), 1.0, (0, 0, -3), (0, 0, 1), t_max=1.5)[0] == 0   # near root > t_max


def test_sphere_miss():
    assert sph_hit((0, 0, 0), 1.0, (0, 2, -3), (0, 0, 1))[0] == 0


def test_onb_orthonormal():
    lib = oracle.load()
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = rng.normal(size=3).astype(np.float32)
        u, v, w = np.zeros(4, np.float32), np.zeros(4, np.float32), np.zeros(4, np.float32)
        lib.iqo_onb(p(f4(*n)), p(u), p(v), p(w))
        m = np.stack([u[:3], v[:3], w[:3]]).astype(np.float64)
        assert np.allclose(m @ m.T, np.eye(3), atol=1e-5)
        assert np.allclose(w[:3], n / np.linalg.norm(n), atol=1e-6)


def test_cosine_weighted_hemisphere():
    lib = oracle.load()
    st = np.zeros(6, np.uint32)
    lib.iqo_xorwow_seed(1984, st.ctypes.data_as(UP))
    zs = []
    for _ in range(2000):
        out = np.zeros(4, np.float32)
        lib.iqo_cosine_weighted(st.ctypes.data_as(UP), p(out))
        assert abs(np.linalg.norm(out[:3].astype(np.float64)) - 1) < 1e-5
        assert out[2] >= 0
        zs.append(out[2])
    assert abs(np.mean(zs) - 2 / 3) < 0.03                         # E[cos θ] = 2/3 for cosine sampling


def test_oren_nayar_record():
    """material.cu:5-43: pdf = cos/π, cos weight = max(0, n·wi), att = albedo·(A + B…)/π ≤ albedo/π·(A+B)."""
    lib = oracle.load()
    st = np.zeros(6, np.uint32)
    lib.iqo_xorwow_seed(7, st.ctypes.data_as(UP))
    sigma2 = np.float32(1.0)
    A = np.float32(1.0) - np.float32(0.5) * sigma2 / (sigma2 + np.float32(0.33))
    B = np.float32(0.45) * sigma2 / (sigma2 + np.float32(0.09))
    for _ in range(300):
        att, pdf, cosw = np.zeros(4, np.float32), C.c_float(), C.c_float()
        ro, rd = np.zeros(4, np.float32), np.zeros(4, np.float32)
        lib.iqo_oren_nayar(p(f4(0, 1, 0)), p(f4(0, 1, 0)), p(f4(0.3, -0.9, 0.1)), st.ctypes.data_as(UP),
                           p(att), C.byref(pdf), C.byref(cosw), p(ro), p(rd))
        assert np.isclose(pdf.value, max(rd[1], 0) / np.pi, rtol=1e-5) or pdf.value == np.float32(1 / np.pi)
        assert cosw.value >= 0 and np.isclose(cosw.value, rd[1], atol=1e-6)
        assert att[0] == att[1] == att[2] and att[3] == 0            # grey albedo (.5,.5,.5,0)
        assert 0 <= att[0] <= 0.5 * (A + B) / np.pi + 1e-6
        assert np.allclose(ro[:3], [0, 1.0001, 0])                   # p + 1e-4 n


def test_normal_matrix_inverse_transpose_and_singular_quirk():
    lib = oracle.load()
    m = np.diag([2.0, 4.0, 8.0, 1.0]).astype(np.float32)
    out = np.zeros(16, np.float32)
    lib.iqo_normal_matrix(p(m.reshape(-1)), p(out))
    assert np.allclose(out.reshape(4, 4), np.diag([0.5, 0.25, 0.125, 1.0]))
    tiny = np.diag([0.01, 0.01, 0.01, 1.0]).astype(np.float32)       # det 1e-6 < 1e-5 -> mat3x3(INFINITY)
    lib.iqo_normal_matrix(p(tiny.reshape(-1)), p(out))
    assert np.isinf(out.reshape(4, 4)[0, 0]) and out.reshape(4, 4)[3, 3] == 1.0


def test_get_ray_center_pixel_points_forward():
    import iqpt
    lib = oracle.load()
    cam = iqpt.make_camera(64, 64)
    st = np.zeros(6, np.uint32)
    lib.iqo_xorwow_seed(1984, st.ctypes.data_as(UP))
    o, d = np.zeros(4, np.float32), np.zeros(4, np.float32)
    lib.iqo_get_ray(C.byref(cam), 32, 32, st.ctypes.data_as(UP), p(o), p(d))
    fwd = np.array([0, -0.5, 3.0]) / np.linalg.norm([0, -0.5, 3.0])
    assert np.dot(d[:3], fwd) > 0.999 and abs(np.linalg.norm(d[:3]) - 1) < 1e-6
    assert np.linalg.norm(o[:3] - np.array([0, 0.5, -3.0])) < 0.02   # near plane at 0.01
