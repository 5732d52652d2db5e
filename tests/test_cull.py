"""Soundness of the exact camera-ray culling (csrc/iq_interval.h, kernel option kOptCull).

The binning kernel clears a primitive's bit for a screen tile only when interval evaluation of the
kernel's own float operation chain proves that the reference's tests reject it for every camera
ray of the tile. Here the host build of the same header is checked against the oracle: for random
cameras, tiles and primitives (many of them straddling the tile's rays), every primitive reported
culled must be rejected by the oracle's Möller–Trumbore / sphere test for random pixels and jitters
of the tile — with t_max = FLT_MAX, so only the order-independent tests count. The GPU parity tests
then check whole frames rendered with culling against the oracle bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from iqpt import _lib, make_camera

FP = C.POINTER(C.c_float)
U8 = C.POINTER(C.c_uint8)
UP = C.POINTER(C.c_uint32)
T_MIN = np.float32(0.000001)
FLT_MAX = np.float32(3.4028235e38)


def cull_tile(cam, xa, xb, ya, yb, tris9, sph4):
    lib = _lib.load()
    f = lib.iqpt_debug_cull_tile
    f.argtypes = [C.POINTER(type(cam)), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, FP, C.c_uint32, FP,
                  C.c_uint32, U8, U8]
    f.restype = C.c_int
    tris9 = np.ascontiguousarray(tris9, dtype=np.float32).reshape(-1, 9)
    sph4 = np.ascontiguousarray(sph4, dtype=np.float32).reshape(-1, 4)
    tc = np.zeros(len(tris9), np.uint8)
    sc = np.zeros(len(sph4), np.uint8)
    ok = f(C.byref(cam), xa, xb, ya, yb, tris9.ctypes.data_as(FP), len(tris9), sph4.ctypes.data_as(FP), len(sph4),
           tc.ctypes.data_as(U8), sc.ctypes.data_as(U8))
    assert ok >= 0, lib.iqpt_last_error()
    return ok == 1, tc.astype(bool), sc.astype(bool)


def tile_rays(cam, xa, xb, ya, yb, n, rng):
    lib = oracle.load()
    out = []
    for _ in range(n):
        x = int(rng.integers(xa, xb + 1))
        y = int(rng.integers(ya, yb + 1))
        st = rng.integers(1, 1 << 32, 6, dtype=np.uint64).astype(np.uint32)
        o = np.zeros(4, np.float32)
        d = np.zeros(4, np.float32)
        lib.iqo_get_ray(C.byref(cam), x, y, st.ctypes.data_as(UP), o.ctypes.data_as(FP), d.ctypes.data_as(FP))
        out.append((o, d))
    # the tile's extreme pixels with the extreme jitter draws (u = 0 and u = 1 come from these states)
    return out


def tri_hit(v0, v1, v2, o, d):
    lib = oracle.load()
    z = np.zeros(4, np.float32)
    t = C.c_float()
    p4 = np.zeros(4, np.float32)
    n4 = np.zeros(4, np.float32)
    front = C.c_int()
    a = [np.append(v, np.float32(1)).astype(np.float32) for v in (v0, v1, v2)]
    return lib.iqo_triangle_intersect(a[0].ctypes.data_as(FP), a[1].ctypes.data_as(FP), a[2].ctypes.data_as(FP),
                                      z.ctypes.data_as(FP), z.ctypes.data_as(FP), z.ctypes.data_as(FP),
                                      o.ctypes.data_as(FP), d.ctypes.data_as(FP), T_MIN, FLT_MAX, C.byref(t),
                                      p4.ctypes.data_as(FP), n4.ctypes.data_as(FP), C.byref(front))


def sph_hit(c, r, o, d):
    lib = oracle.load()
    c4 = np.append(c, np.float32(1)).astype(np.float32)
    t = C.c_float()
    p4 = np.zeros(4, np.float32)
    n4 = np.zeros(4, np.float32)
    front = C.c_int()
    return lib.iqo_sphere_intersect(c4.ctypes.data_as(FP), C.c_float(r), o.ctypes.data_as(FP), d.ctypes.data_as(FP),
                                    T_MIN, FLT_MAX, C.byref(t), p4.ctypes.data_as(FP), n4.ctypes.data_as(FP),
                                    C.byref(front))


def random_prims(rays, rng, ntri=48, nsph=24):
    """Triangles and spheres placed on and around the tile's rays, so many straddle its edges."""
    tris, sphs = [], []
    for k in range(ntri):
        o, d = rays[rng.integers(len(rays))]
        dist = np.float32(rng.uniform(0.05, 6.0) * (1 if k % 5 else -1))
        c = o[:3] + dist * d[:3]
        size = rng.uniform(0.001, 1.5)
        vs = (c + rng.normal(0, size, (3, 3))).astype(np.float32)
        e1 = (vs[1] - vs[0]).astype(np.float32)
        e2 = (vs[2] - vs[0]).astype(np.float32)
        tris.append((vs, np.concatenate([vs[0], e1, e2]).astype(np.float32)))
    for k in range(nsph):
        o, d = rays[rng.integers(len(rays))]
        dist = np.float32(rng.uniform(-2.0, 6.0))
        c = (o[:3] + dist * d[:3] + rng.normal(0, 0.3, 3)).astype(np.float32)
        sphs.append(np.append(c, np.float32(rng.uniform(0.01, 0.8))).astype(np.float32))
    return tris, sphs


CAMERAS = [
    dict(),
    dict(fovh=70.0, znear=0.05, zfar=50.0, position=(0.3, 1.2, -2.0, 0.0), forward=(-0.1, -0.6, 1.0, 0.0)),
    dict(fovh=20.0, znear=0.5, zfar=1000.0, position=(-3.0, 0.2, 4.0, 0.0), forward=(0.6, 0.0, -0.8, 0.0)),
]


@pytest.mark.parametrize("ci", range(len(CAMERAS)))
def test_culled_primitives_are_rejected_by_every_tile_ray(ci):
    rng = np.random.default_rng(100 + ci)
    w, h = 320, 180
    cam = make_camera(w, h, **CAMERAS[ci])
    n_culled = n_kept = 0
    for _ in range(6):
        xa = int(rng.integers(0, w - 8))
        ya = int(rng.integers(0, h - 8))
        xb, yb = xa + 7, ya + 7
        rays = tile_rays(cam, xa, xb, ya, yb, 96, rng)
        tris, sphs = random_prims(rays, rng)
        ok, tc, sc = cull_tile(cam, xa, xb, ya, yb, np.stack([t[1] for t in tris]), np.stack(sphs))
        assert ok
        for (vs, _), culled in zip(tris, tc):
            if culled:
                for o, d in rays:
                    assert not tri_hit(vs[0], vs[1], vs[2], o, d), "culled triangle hit by a tile ray"
        for s, culled in zip(sphs, sc):
            if culled:
                for o, d in rays:
                    assert not sph_hit(s[:3], s[3], o, d), "culled sphere hit by a tile ray"
        n_culled += int(tc.sum() + sc.sum())
        n_kept += int((~tc).sum() + (~sc).sum())
    # the test is only meaningful if both outcomes occur
    assert n_culled > 20 and n_kept > 20, (n_culled, n_kept)


def test_hit_primitives_are_never_culled():
    """Every primitive that some sampled ray of the tile hits must keep its bit."""
    rng = np.random.default_rng(7)
    w, h = 200, 120
    cam = make_camera(w, h)
    hits = 0
    for _ in range(8):
        xa, ya = int(rng.integers(0, w - 8)), int(rng.integers(0, h - 8))
        rays = tile_rays(cam, xa, xa + 7, ya, ya + 7, 64, rng)
        tris, sphs = random_prims(rays, rng)
        ok, tc, sc = cull_tile(cam, xa, xa + 7, ya, ya + 7, np.stack([t[1] for t in tris]), np.stack(sphs))
        for (vs, _), culled in zip(tris, tc):
            if any(tri_hit(vs[0], vs[1], vs[2], o, d) for o, d in rays):
                hits += 1
                assert not culled
        for s, culled in zip(sphs, sc):
            if any(sph_hit(s[:3], s[3], o, d) for o, d in rays):
                hits += 1
                assert not culled
    assert hits > 20


def test_cornell_walls_are_culled_per_tile():
    """On the bench scene most tiles keep only the walls their camera rays can reach."""
    from iqpt import Scene
    from iqpt.scene import packet_stats  # noqa: F401  (import check)
    sc = Scene()
    sc.add_preset("cornell")
    pk = sc.build_packet()
    cam = make_camera(1920, 1080)
    # world-space triangles of the packet, as the runtime builds them (v0, e1, e2)
    lib = _lib.load()
    tris = []
    for i in range(pk.num_drawcalls[_lib.MESH_TRIANGLES]):
        dc = pk.tri_mesh_dcs[i]
        m = pk.tri_meshes[dc.mesh_id]
        M = np.array(dc.transform, dtype=np.float32).reshape(4, 4)
        for j in range(0, m.num_indices, 3):
            vs = []
            for q in range(3):
                v = m.vertices[m.indices[j + q]]
                p = np.array([v.pos[0], v.pos[1], v.pos[2], 1.0], np.float32)
                # row-vector transform with the reference's association (vector.h:371-383)
                w = [np.float32(((p[0] * M[0, c] + p[1] * M[1, c]) + p[2] * M[2, c]) + p[3] * M[3, c])
                     for c in range(3)]
                vs.append(np.array(w, np.float32))
            tris.append(np.concatenate([vs[0], vs[1] - vs[0], vs[2] - vs[0]]).astype(np.float32))
    del lib
    tris = np.stack(tris)
    culled = []
    for ty in range(0, 1080, 120):
        for tx in range(0, 1920, 160):
            ok, tc, _ = cull_tile(cam, tx, tx + 7, ty, ty + 7, tris, np.zeros((0, 4), np.float32))
            assert ok
            culled.append(tc.mean())
    assert np.mean(culled) > 0.5, np.mean(culled)
