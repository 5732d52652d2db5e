// iq_interval.h — exact conservative culling of primitives for bundles of camera rays, and the
// converse: triangles every ray of a bundle is certain to hit.
//
// The kernel's closest-hit loop must return exactly what the reference's brute-force loop over
// every primitive returns (path_tracer.cu:257-295). A primitive may therefore be skipped for a ray
// only if the reference's own test — with its own float rounding — is certain to reject it. This
// header proves that for a whole screen tile of camera rays at once:
//
//   Every quantity the kernel computes for a camera ray of the tile (camera_ray, then the
//   Möller–Trumbore / sphere tests) is a chain of IEEE binary32 operations with round-to-nearest.
//   RN is monotone (x <= y implies RN(x) <= RN(y)), so if x lies in [a, b] and y in [c, d], then
//   RN(x + y) lies in [RN(a + c), RN(b + d)], RN(x * y) between the RN of the smallest and largest
//   of the four endpoint products, RN(1 / x) in [RN(1 / b), RN(1 / a)] for 0 < a, and so on.
//   Evaluating the kernel's operation chain on intervals whose endpoints are computed with the
//   same RN float operations therefore yields intervals that contain the value every lane of the
//   tile computes, bit for bit, without any widening. A primitive whose interval proves one of the
//   reference's reject tests for the whole tile (|det| < 1e-6, u outside [0, 1], v < 0, u + v > 1,
//   t < t_min, delta < 0, both sphere roots < t_min) is rejected by every ray of the tile, so
//   skipping it cannot change any result. Tests that depend on the running closest hit are never
//   used for culling (they depend on the primitive order), and any interval that becomes NaN or
//   infinite, or a branch of the kernel whose direction is not the same for the whole tile, simply
//   means "cannot cull".
//
// Compiled for the host (unit tests) and the GPU (the binning kernel) from this one source, with
// FP contraction off like the rest of the hot path.
#pragma once

#include <stdint.h>

#include "iq_fp.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace iqiv {

struct ivl {
    float lo, hi;
};

IQ_HD inline ivl pt(float v) { return {v, v}; }
IQ_HD inline float fmin2(float a, float b) { return b < a ? b : a; }
IQ_HD inline float fmax2(float a, float b) { return b > a ? b : a; }
IQ_HD inline bool finite(const ivl& a) {
    // NaN fails both comparisons; infinities fail the bound
    return a.lo >= -3.4e38f && a.hi <= 3.4e38f && a.lo <= a.hi;
}
IQ_HD inline ivl add(ivl a, ivl b) { return {a.lo + b.lo, a.hi + b.hi}; }
IQ_HD inline ivl sub(ivl a, ivl b) { return {a.lo - b.hi, a.hi - b.lo}; }
IQ_HD inline ivl mul(ivl a, ivl b) {
    const float p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    return {fmin2(fmin2(p0, p1), fmin2(p2, p3)), fmax2(fmax2(p0, p1), fmax2(p2, p3))};
}
// x * x of one lane value (the same variable on both sides)
IQ_HD inline ivl sq(ivl a) {
    const float l = a.lo * a.lo, h = a.hi * a.hi;
    if (a.lo >= 0.0f) return {l, h};
    if (a.hi <= 0.0f) return {h, l};
    return {0.0f, fmax2(l, h)};
}
// RN(1 / x) for x of one sign (caller checks)
IQ_HD inline ivl rcp(ivl a) { return {1.0f / a.hi, 1.0f / a.lo}; }
IQ_HD inline ivl sqrt_(ivl a) { return {iq_sqrtf(a.lo), iq_sqrtf(a.hi)}; }
IQ_HD inline ivl neg(ivl a) { return {-a.hi, -a.lo}; }
IQ_HD inline ivl absv(ivl a) {
    if (a.lo >= 0.0f) return a;
    if (a.hi <= 0.0f) return neg(a);
    return {0.0f, fmax2(-a.lo, a.hi)};
}

// dot4(v, column c of M) of iqvec::transformed, the same association as the kernel's dot_col
IQ_HD inline ivl dot_col(ivl x, ivl y, ivl z, ivl w, const float* M, int c) {
    return add(add(add(mul(x, pt(M[c])), mul(y, pt(M[4 + c]))), mul(z, pt(M[8 + c]))), mul(w, pt(M[12 + c])));
}

// Camera description the bundle needs (the kernel's kparams fields).
struct camera_in {
    uint32_t width, height;
    float rcp_width, rcp_height;   // unused: x / W is evaluated as the IEEE quotient it equals
    const float* inv_proj;
    const float* inv_view;
    int cam_const;
    float near_rw, far_rw;
};

struct bundle {
    ivl o[3], d[3];
    ivl len;          // |far - near| before normalization (normalize3's len)
    bool ok;
};

// camera_ray (iqpt_kernels.hip, camera.cu:20-43) for every pixel with x in [xa, xb], y in [ya, yb]
// and every jitter draw.
IQ_HD inline bundle camera_bundle(const camera_in& c, uint32_t xa, uint32_t xb, uint32_t ya, uint32_t yb) {
    bundle b;
    b.ok = false;
    const ivl j = {0.0f * (0.5f - -0.5f) + -0.5f, 1.0f * (0.5f - -0.5f) + -0.5f};   // u in [0, 1]
    const ivl xs = add(ivl{(float)xa, (float)xb}, j);
    const ivl ys = add(ivl{(float)ya, (float)yb}, j);
    const float W = (float)c.width, H = (float)c.height;
    const ivl xq = {xs.lo / W, xs.hi / W};
    const ivl yq = {ys.lo / H, ys.hi / H};
    const ivl x_ndc = sub(mul(xq, pt(2.0f)), pt(1.0f));
    const ivl y_ndc = sub(pt(1.0f), mul(yq, pt(2.0f)));
    const float* P = c.inv_proj;
    const float* V = c.inv_view;
    const ivl z0 = pt(0.0f), one = pt(1.0f);
    ivl n[3], f[3];
    for (int k = 0; k < 3; ++k) {
        n[k] = dot_col(x_ndc, y_ndc, z0, one, P, k);
        f[k] = dot_col(x_ndc, y_ndc, one, one, P, k);
    }
    ivl ninv, finv;
    if (c.cam_const) {
        ninv = pt(c.near_rw);
        finv = pt(c.far_rw);
    } else {
        const ivl wn = dot_col(x_ndc, y_ndc, z0, one, P, 3);
        const ivl wf = dot_col(x_ndc, y_ndc, one, one, P, 3);
        if (!finite(wn) || !finite(wf)) return b;
        if (!((wn.lo > 0.0f || wn.hi < 0.0f) && (wf.lo > 0.0f || wf.hi < 0.0f))) return b;
        ninv = rcp(wn);
        finv = rcp(wf);
    }
    for (int k = 0; k < 3; ++k) {
        n[k] = mul(n[k], ninv);
        f[k] = mul(f[k], finv);
    }
    ivl wn3[3], wf3[3], d[3];
    for (int k = 0; k < 3; ++k) {
        wn3[k] = dot_col(n[0], n[1], n[2], one, V, k);
        wf3[k] = dot_col(f[0], f[1], f[2], one, V, k);
        d[k] = sub(wf3[k], wn3[k]);
        if (!finite(d[k]) || !finite(wn3[k])) return b;
    }
    // normalize3: the zero branch is taken only if all three |d| < 1e-5; it must be excluded
    // for the whole tile
    bool some_big = false;
    for (int k = 0; k < 3; ++k) some_big = some_big || !(absv(d[k]).lo < 0.00001f);
    if (!some_big) return b;
    const ivl len2 = add(add(sq(d[0]), sq(d[1])), sq(d[2]));
    const ivl len = sqrt_(len2);
    if (!(len.lo > 0.0f) || !finite(len)) return b;
    b.len = len;
    const ivl inv = rcp(len);
    for (int k = 0; k < 3; ++k) {
        b.d[k] = mul(d[k], inv);
        b.o[k] = wn3[k];
        if (!finite(b.d[k])) return b;
    }
    b.ok = true;
    return b;
}

constexpr float kTMinIv = 0.000001f;   // path_tracer.cu:241 (the kernel's kTMin)

// true if the Möller–Trumbore test (shape.cu:62-103 as the kernel evaluates it) rejects triangle
// (v0, e1, e2) for every ray of the bundle
IQ_HD inline bool tri_culled(const bundle& b, const float v0[3], const float e1[3], const float e2[3]) {
    const ivl* d = b.d;
    const ivl px = sub(mul(d[1], pt(e2[2])), mul(d[2], pt(e2[1])));
    const ivl py = sub(mul(d[2], pt(e2[0])), mul(d[0], pt(e2[2])));
    const ivl pz = sub(mul(d[0], pt(e2[1])), mul(d[1], pt(e2[0])));
    ivl det = add(add(mul(pt(e1[0]), px), mul(pt(e1[1]), py)), mul(pt(e1[2]), pz));
    if (!finite(det)) return false;
    const float eps = 0.000001f;
    if (det.lo > -eps && det.hi < eps) return true;          // |det| < 1e-6 on every lane
    // lanes with |det| < 1e-6 are rejected; the others must all have one sign
    if (det.lo > -eps) det.lo = fmax2(det.lo, eps);
    else if (det.hi < eps) det.hi = fmin2(det.hi, -eps);
    else return false;
    const ivl inv = rcp(det);
    const ivl tx = sub(b.o[0], pt(v0[0])), ty = sub(b.o[1], pt(v0[1])), tz = sub(b.o[2], pt(v0[2]));
    const ivl u = mul(add(add(mul(tx, px), mul(ty, py)), mul(tz, pz)), inv);
    if (!finite(u)) return false;
    if (u.hi < 0.0f || u.lo > 1.0f) return true;
    const ivl qx = sub(mul(ty, pt(e1[2])), mul(tz, pt(e1[1])));
    const ivl qy = sub(mul(tz, pt(e1[0])), mul(tx, pt(e1[2])));
    const ivl qz = sub(mul(tx, pt(e1[1])), mul(ty, pt(e1[0])));
    const ivl v = mul(add(add(mul(d[0], qx), mul(d[1], qy)), mul(d[2], qz)), inv);
    if (!finite(v)) return false;
    if (v.hi < 0.0f) return true;
    const ivl uv = add(u, v);
    if (uv.lo > 1.0f) return true;
    const ivl t = mul(add(add(mul(pt(e2[0]), qx), mul(pt(e2[1]), qy)), mul(pt(e2[2]), qz)), inv);
    if (!finite(t)) return false;
    return t.hi < kTMinIv;
}

constexpr float kTMaxIv = 999.99f;     // the kernel's kTMax: the closest hit a ray starts with

// true if the Möller–Trumbore test (shape.cu:62-103 as the kernel evaluates it) accepts triangle
// (v0, e1, e2) for every ray of the bundle as a first hit: |det| >= 1e-6 with one sign, u in [0, 1],
// v >= 0, u + v <= 1 and t in [t_min, kTMax] on every lane — each of the reference's reject tests
// fails for the whole bundle. Used for tiles without a sphere candidate under the reference's
// materials, where every camera ray then ends on an emissive triangle (path_tracer.cu:278).
IQ_HD inline bool tri_certain(const bundle& b, const float v0[3], const float e1[3], const float e2[3]) {
    if (!b.ok) return false;
    const ivl* d = b.d;
    const ivl px = sub(mul(d[1], pt(e2[2])), mul(d[2], pt(e2[1])));
    const ivl py = sub(mul(d[2], pt(e2[0])), mul(d[0], pt(e2[2])));
    const ivl pz = sub(mul(d[0], pt(e2[1])), mul(d[1], pt(e2[0])));
    const ivl det = add(add(mul(pt(e1[0]), px), mul(pt(e1[1]), py)), mul(pt(e1[2]), pz));
    if (!finite(det)) return false;
    const float eps = 0.000001f;
    if (!(det.lo >= eps || det.hi <= -eps)) return false;   // every lane |det| >= 1e-6, one sign
    const ivl inv = rcp(det);
    const ivl tx = sub(b.o[0], pt(v0[0])), ty = sub(b.o[1], pt(v0[1])), tz = sub(b.o[2], pt(v0[2]));
    const ivl u = mul(add(add(mul(tx, px), mul(ty, py)), mul(tz, pz)), inv);
    if (!finite(u) || !(u.lo >= 0.0f && u.hi <= 1.0f)) return false;
    const ivl qx = sub(mul(ty, pt(e1[2])), mul(tz, pt(e1[1])));
    const ivl qy = sub(mul(tz, pt(e1[0])), mul(tx, pt(e1[2])));
    const ivl qz = sub(mul(tx, pt(e1[1])), mul(ty, pt(e1[0])));
    const ivl v = mul(add(add(mul(d[0], qx), mul(d[1], qy)), mul(d[2], qz)), inv);
    if (!finite(v) || !(v.lo >= 0.0f)) return false;
    const ivl uv = add(u, v);
    if (!finite(uv) || !(uv.hi <= 1.0f)) return false;
    const ivl t = mul(add(add(mul(pt(e2[0]), qx), mul(pt(e2[1]), qy)), mul(pt(e2[2]), qz)), inv);
    if (!finite(t)) return false;
    return t.lo >= kTMinIv && t.hi <= kTMaxIv;
}

// true if sphere::intersect (shape.cu:13-46 as the kernel evaluates it) rejects sphere (c, r)
// for every ray of the bundle
IQ_HD inline bool sphere_culled(const bundle& b, const float c[3], float r) {
    const ivl ocx = sub(pt(c[0]), b.o[0]), ocy = sub(pt(c[1]), b.o[1]), ocz = sub(pt(c[2]), b.o[2]);
    const ivl halfb = add(add(mul(b.d[0], ocx), mul(b.d[1], ocy)), mul(b.d[2], ocz));
    const ivl cc = sub(add(add(sq(ocx), sq(ocy)), sq(ocz)), pt(r * r));
    const ivl delta = sub(sq(halfb), cc);
    if (!finite(halfb) || !finite(delta)) return false;
    if (delta.hi < 0.0f) return true;
    // lanes with delta < 0 are rejected; for the others both roots are below t_min if the far
    // root t2 = halfb + sqrt(delta) is
    const ivl sd = sqrt_(ivl{fmax2(delta.lo, 0.0f), delta.hi});
    const ivl t2 = add(halfb, sd);
    if (!finite(t2)) return false;
    return t2.hi < kTMinIv;
}

}  // namespace iqiv
