"""kOptCamAxis (the short camera transform for pitch-only cameras, iqpt_kernels.hip camera_ray_axis):
which cameras qualify (host check, iqpt_runtime.cpp cam_axis_constants), and the exactness argument
replayed in numpy binary32 — the general chain of camera_ndc (camera.cu:20-43 as the kernel and the
oracle evaluate it) against the short chain, bit for bit including the signs of zeros, on random
and adversarial NDC inputs (x_ndc = +-0, tiny, large) and on cameras whose kept terms vanish."""
import ctypes as C

import numpy as np
import pytest

from iqpt import _lib, make_camera

f32 = np.float32


def lib():
    lb = _lib.load()
    lb.iqpt_debug_cam_axis.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
    lb.iqpt_debug_cam_axis.restype = C.c_int
    return lb


def cam_axis(cam):
    k = (C.c_float * 16)()
    r = lib().iqpt_debug_cam_axis(C.byref(cam), k)
    assert r in (0, 1)
    return bool(r), np.array(list(k), dtype=f32)


def mats(cam):
    return (np.array(list(cam.inv_proj), dtype=f32).reshape(4, 4),
            np.array(list(cam.inv_view), dtype=f32).reshape(4, 4))


def general(P, V, nrw, frw, x, y):
    """camera_ndc: dot4 with column c, left to right, w = 1 (kOptCamConst's constant 1/w)."""
    with np.errstate(all="ignore"):
        def col(v, M, c):
            return ((v[0] * M[0, c] + v[1] * M[1, c]) + v[2] * M[2, c]) + v[3] * M[3, c]
        one, zero = f32(1), f32(0)
        n = [col((x, y, zero, one), P, c) * nrw for c in range(3)]
        fp = [col((x, y, one, one), P, c) * frw for c in range(3)]
        wn = [col((n[0], n[1], n[2], one), V, c) for c in range(3)]
        wf = [col((fp[0], fp[1], fp[2], one), V, c) for c in range(3)]
        d = [wf[c] - wn[c] for c in range(3)]
        ln = np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
        inv = f32(1) / ln
        return np.stack([wn[0], wn[1], wn[2], d[0] * inv, d[1] * inv, d[2] * inv], axis=-1)


def short(k, x, y):
    """camera_ray_axis with the launch constants of cam_axis_constants."""
    with np.errstate(all="ignore"):
        xw = [(x * k[0] + k[2]) * k[4], (x * k[0] + k[2]) * k[5]]
        yw = [(y * k[1] + k[3]) * k[4], (y * k[1] + k[3]) * k[5]]
        wx = [xw[i] * k[6] + k[7] for i in range(2)]
        wy = [(yw[0] * k[8] + k[12]) + k[10], (yw[1] * k[8] + k[13]) + k[10]]
        wz = [(yw[0] * k[9] + k[14]) + k[11], (yw[1] * k[9] + k[15]) + k[11]]
        d = [wx[1] - wx[0], wy[1] - wy[0], wz[1] - wz[0]]
        ln = np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
        inv = f32(1) / ln
        return np.stack([wx[0], wy[0], wz[0], d[0] * inv, d[1] * inv, d[2] * inv], axis=-1)


def ndc_samples(n=20000, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, n).astype(f32)
    y = rng.uniform(-1, 1, n).astype(f32)
    special = np.array([0.0, -0.0, 1e-30, -1e-30, 1e-45, -1e-45, 1.0, -1.0, 0.5, 3e5, -3e5], dtype=f32)
    xs = np.concatenate([x, np.repeat(special, special.size)])
    ys = np.concatenate([y, np.tile(special, special.size)])
    return xs, ys


def assert_same_bits(cam):
    ok, k = cam_axis(cam)
    assert ok
    P, V = mats(cam)
    nrw, frw = k[4], k[5]
    x, y = ndc_samples()
    g, s = general(P, V, nrw, frw, x, y), short(k, x, y)
    assert np.array_equal(g.view(np.uint32), s.view(np.uint32))
    return g


def pitch_camera(w, h, pitch_y, pos=(0.0, 0.5, -3.0), **kw):
    return make_camera(w, h, position=(*pos, 0.0), forward=(0.0, pitch_y, 3.0, 0.0), **kw)


def test_reference_camera_qualifies():
    cam = make_camera(1920, 1080)
    ok, k = cam_axis(cam)
    assert ok
    P, V = mats(cam)
    assert k[0] == P[0, 0] and k[1] == P[1, 1] and k[6] == V[0, 0] and k[8] == V[1, 1]
    assert_same_bits(cam)


@pytest.mark.parametrize("pitch", [-0.9, -0.5, -0.1, 0.0, 0.3, 1.7])
@pytest.mark.parametrize("pos", [(0.0, 0.5, -3.0), (0.0, 0.0, 0.0), (0.0, -2.0, 4.0)])
def test_pitch_cameras_bit_identical(pitch, pos):
    g = assert_same_bits(pitch_camera(320, 200, pitch, pos, fovh=60.0))
    if pos[0] == 0.0 and pitch == 0.0:
        # x_ndc = +-0 rays have zero x components: the zero signs must agree too (checked above)
        assert np.any(g[:, 0] == 0.0)


def test_degenerate_columns_bit_identical():
    """Kept terms that vanish for every ray (V[0] = 0, P[5] = 0): every output is decided by the zero
    rules; the short chain must still give the general chain's bits."""
    cam = make_camera(64, 48)
    for idx in (0,):
        cam.inv_view[idx] = 0.0
    assert_same_bits(cam)
    cam2 = make_camera(64, 48)
    cam2.inv_proj[5] = 0.0
    assert_same_bits(cam2)


def test_yaw_roll_and_negative_zero_do_not_qualify():
    yaw = make_camera(64, 48, position=(0.0, 0.5, -3.0, 0.0), forward=(0.4, -0.5, 3.0, 0.0))
    assert not cam_axis(yaw)[0]
    for idx in (12, 13, 14):
        cam = make_camera(64, 48)
        cam.inv_view[idx] = -0.0
        assert not cam_axis(cam)[0], idx
    cam = make_camera(64, 48)
    cam.inv_proj[12] = -0.0
    assert not cam_axis(cam)[0]
    cam = make_camera(64, 48)
    cam.inv_proj[1] = 1e-3            # not a standard perspective inverse
    assert not cam_axis(cam)[0]
    cam = make_camera(64, 48)
    cam.inv_view[5] = float("inf")
    assert not cam_axis(cam)[0]
