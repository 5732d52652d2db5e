// iq_fp2.h — two-lane (packed FP32) forms of the shared transcendentals of iq_fp.h, device only.
//
// The Oren–Nayar scatter (material.cu:5-43) evaluates its transcendentals in pairs that do not depend
// on each other: atan2 of the outgoing and the incoming direction, acos of their two cosines, sin(alpha)
// next to cos(phi_i - phi_o), and sin / cos of one angle. gfx950 executes v_pk_mul_f32 / v_pk_add_f32 /
// v_pk_fma_f32 on two binary32 values per lane at the issue cost of one scalar VALU instruction, so a
// pair costs about what one scalar evaluation did. The forms below are also branch-free: every range of
// the scalar function is evaluated and the element's own range selects its result (the scalar forms
// branch per lane, and a wave whose lanes fall in different ranges executed all of them anyway, with
// the exec-mask bookkeeping on top). Arguments outside the ranges the scatter produces (|x| > 8192 for
// the trigonometric functions, division operands outside iq_div's short range, reciprocals outside
// iq_rcp's) take a rarely executed branch to the scalar functions.
//
// Exactness: for each element the operation sequence is the scalar function's (iq_fp.h as the kernel
// compiles it, with the iq_fastdiv.h forms): the same IEEE operations on the same operands in the same
// order, contraction off; selecting between fully evaluated ranges instead of branching changes no bit.
// tests/test_gpu_libm.py checks every function here against the oracle's host build, bit for bit.
#pragma once

#include "iq_fp.h"
#include "iq_fastdiv.h"

typedef float iq_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ iq_f2 f2_sel(bool cx, bool cy, iq_f2 a, iq_f2 b) {
    return (iq_f2){cx ? a.x : b.x, cy ? a.y : b.y};
}
__device__ __forceinline__ iq_f2 f2_abs(iq_f2 v) { return (iq_f2){__builtin_fabsf(v.x), __builtin_fabsf(v.y)}; }
__device__ __forceinline__ iq_f2 f2_fma(iq_f2 a, iq_f2 b, iq_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ iq_f2 f2_neg_if(bool nx, bool ny, iq_f2 v) { return f2_sel(nx, ny, -v, v); }
__device__ __forceinline__ bool f_sign(float v) { return (__float_as_uint(v) >> 31) != 0u; }
__device__ __forceinline__ bool f_nan(float v) { return (__float_as_uint(v) & 0x7fffffffu) > 0x7f800000u; }
__device__ __forceinline__ bool f_inf(float v) { return (__float_as_uint(v) & 0x7fffffffu) == 0x7f800000u; }

// iq_rcp per element: v_rcp_f32 and v_div_fixup_f32 have no packed form, the Newton step does.
__device__ __forceinline__ iq_f2 iq_rcp2(iq_f2 x) {
    const iq_f2 y0 = {__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
    const iq_f2 e = f2_fma(-x, y0, (iq_f2){1.0f, 1.0f});
    const iq_f2 y1 = f2_fma(e, y0, y0);
    return (iq_f2){__builtin_amdgcn_div_fixupf(y1.x, x.x, 1.0f), __builtin_amdgcn_div_fixupf(y1.y, x.y, 1.0f)};
}

// iq_div_pre per element (same range conditions).
__device__ __forceinline__ iq_f2 iq_div_pre2(iq_f2 a, iq_f2 b, iq_f2 y) {
    const iq_f2 q = a * y;
    const iq_f2 r = f2_fma(-b, q, a);
    const iq_f2 q1 = f2_fma(r, y, q);
    return (iq_f2){__builtin_amdgcn_div_fixupf(q1.x, b.x, a.x), __builtin_amdgcn_div_fixupf(q1.y, b.y, a.y)};
}

// iq_sqrt_n per element (x = +-0 or >= 2^-96, inf, NaN).
__device__ __forceinline__ iq_f2 iq_sqrt_n2(iq_f2 x) {
    const iq_f2 s = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
    const iq_f2 s_dn = {__uint_as_float(__float_as_uint(s.x) - 1u), __uint_as_float(__float_as_uint(s.y) - 1u)};
    const iq_f2 s_up = {__uint_as_float(__float_as_uint(s.x) + 1u), __uint_as_float(__float_as_uint(s.y) + 1u)};
    const iq_f2 r_dn = f2_fma(-s_dn, s, x);
    const iq_f2 r_up = f2_fma(-s_up, s, x);
    iq_f2 t = f2_sel(r_dn.x <= 0.0f, r_dn.y <= 0.0f, s_dn, s);
    return f2_sel(r_up.x > 0.0f, r_up.y > 0.0f, s_up, t);
}

// iq_atanf for two arguments.
__device__ __forceinline__ iq_f2 iq_atanf2(iq_f2 x) {
    const iq_f2 ax = f2_abs(x);
    const bool b1x = ax.x > 2.414213562373095f, b1y = ax.y > 2.414213562373095f;
    const bool b2x = ax.x > 0.4142135623730950f, b2y = ax.y > 0.4142135623730950f;
    // range 1: -IQ_RCP(ax) (iq_rcp_guarded: the IEEE reciprocal from 2^126 up)
    iq_f2 rc = iq_rcp2(ax);
    const bool gx = b1x && !(ax.x < 0x1p126f), gy = b1y && !(ax.y < 0x1p126f);
    if (__builtin_expect(gx || gy, 0)) {
        asm volatile("" ::: "memory");
        if (gx) rc.x = 1.0f / ax.x;
        if (gy) rc.y = 1.0f / ax.y;
    }
    // range 2: IQ_DIV_N(ax - 1, ax + 1)
    const iq_f2 am1 = ax - 1.0f, ap1 = ax + 1.0f;
    const iq_f2 r2 = iq_div_pre2(am1, ap1, iq_rcp2(ap1));
    const iq_f2 y0 = {b1x ? IQ_PI_DIV_2 : (b2x ? IQ_PI_DIV_4 : 0.0f), b1y ? IQ_PI_DIV_2 : (b2y ? IQ_PI_DIV_4 : 0.0f)};
    const iq_f2 r = {b1x ? -rc.x : (b2x ? r2.x : ax.x), b1y ? -rc.y : (b2y ? r2.y : ax.y)};
    const iq_f2 z = r * r;
    const iq_f2 y = y0 + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
                           - 3.33329491539e-1f) * z * r + r);
    const iq_f2 s = f2_neg_if(f_sign(x.x), f_sign(x.y), y);
    return f2_sel(f_nan(x.x), f_nan(x.y), x, s);
}

// iq_atan2f(y.k, x.k) for k = x, y.
__device__ __forceinline__ iq_f2 iq_atan2f2(iq_f2 y, iq_f2 x) {
    const iq_f2 ay = f2_abs(y), ax = f2_abs(x);
    const bool nanx = f_nan(x.x) || f_nan(y.x), nany = f_nan(x.y) || f_nan(y.y);
    const bool genx = !nanx && y.x != 0.0f && !f_inf(y.x) && x.x != 0.0f && !f_inf(x.x);
    const bool geny = !nany && y.y != 0.0f && !f_inf(y.y) && x.y != 0.0f && !f_inf(x.y);
    // IQ_DIV(ay, ax) = iq_div: the short form inside [2^-62, 2^62], the IEEE division outside
    iq_f2 q = iq_div_pre2(ay, ax, iq_rcp2(ax));
    const bool okx = ay.x >= 0x1p-62f && ay.x <= 0x1p62f && ax.x >= 0x1p-62f && ax.x <= 0x1p62f;
    const bool oky = ay.y >= 0x1p-62f && ay.y <= 0x1p62f && ax.y >= 0x1p-62f && ax.y <= 0x1p62f;
    if (__builtin_expect((genx && !okx) || (geny && !oky), 0)) {
        asm volatile("" ::: "memory");
        if (!okx) q.x = ay.x / ax.x;
        if (!oky) q.y = ay.y / ax.y;
    }
    const iq_f2 z = iq_atanf2(q);
    const bool xsx = f_sign(x.x), xsy = f_sign(x.y);
    iq_f2 res = f2_sel(xsx, xsy, IQ_PI - z, z);
    // the special cases of iq_atan2f, in its order
    const float kx = xsx ? IQ_PI : 0.0f, ky = xsy ? IQ_PI : 0.0f;
    const float ix = f_inf(x.x) ? (xsx ? 3.0f * IQ_PI_DIV_4 : IQ_PI_DIV_4) : IQ_PI_DIV_2;
    const float iy = f_inf(x.y) ? (xsy ? 3.0f * IQ_PI_DIV_4 : IQ_PI_DIV_4) : IQ_PI_DIV_2;
    res.x = y.x == 0.0f ? kx : (f_inf(y.x) ? ix : (x.x == 0.0f ? IQ_PI_DIV_2 : (f_inf(x.x) ? kx : res.x)));
    res.y = y.y == 0.0f ? ky : (f_inf(y.y) ? iy : (x.y == 0.0f ? IQ_PI_DIV_2 : (f_inf(x.y) ? ky : res.y)));
    res = f2_neg_if(f_sign(y.x), f_sign(y.y), res);
    return f2_sel(nanx, nany, (iq_f2){iq_nanf(), iq_nanf()}, res);
}

// iq_acosf for two arguments. Inside acos, asin only sees |a| <= 0.5 (x itself on [-0.5, 0.5], the
// root sqrt(0.5 (1 -+ x)) < 0.5 outside), so asin's |a| > 0.5 range is never taken here.
__device__ __forceinline__ iq_f2 iq_acosf2(iq_f2 x) {
    const bool lox = x.x < -0.5f, loy = x.y < -0.5f, hix = x.x > 0.5f, hiy = x.y > 0.5f;
    const iq_f2 w = f2_sel(lox, loy, 1.0f + x, 1.0f - x);
    const iq_f2 s = iq_sqrt_n2(0.5f * w);
    const iq_f2 a_in = f2_sel(lox || hix, loy || hiy, s, x);
    const iq_f2 a = f2_abs(a_in);
    const iq_f2 zz = a * a;
    const iq_f2 p = ((((4.2163199048e-2f * zz + 2.4181311049e-2f) * zz + 4.5470025998e-2f) * zz
                      + 7.4953002686e-2f) * zz + 1.6666752422e-1f) * zz * a + a;
    const iq_f2 z = f2_sel(a.x < 1.0e-4f, a.y < 1.0e-4f, a, p);
    const iq_f2 as = f2_neg_if(f_sign(a_in.x), f_sign(a_in.y), z);
    const iq_f2 two = 2.0f * as;
    iq_f2 res = f2_sel(lox, loy, IQ_PI - two, f2_sel(hix, hiy, two, IQ_PI_DIV_2 - as));
    res = f2_sel(x.x < -1.0f || x.x > 1.0f, x.y < -1.0f || x.y > 1.0f, (iq_f2){iq_nanf(), iq_nanf()}, res);
    return f2_sel(f_nan(x.x), f_nan(x.y), x, res);
}

// (iq_sinf(v.x), iq_cosf(v.y)) with one packed octant reduction and both polynomials per element.
__device__ __forceinline__ iq_f2 iq_sin_cos2(iq_f2 v) {
    const iq_f2 ax = f2_abs(v);
    // NaN, infinities and |v| > 8192 (the double reduction) in a rarely executed branch
    if (__builtin_expect(!(ax.x <= IQ_TRIG_MAX) || !(ax.y <= IQ_TRIG_MAX), 0)) {
        asm volatile("" ::: "memory");
        return (iq_f2){iq_sinf(v.x), iq_cosf(v.y)};
    }
    const iq_f2 jf = IQ_FOPI * ax;
    int jx = (int)jf.x, jy = (int)jf.y;
    const iq_f2 y0 = {(float)jx, (float)jy};
    const iq_f2 y = f2_sel(jx & 1, jy & 1, y0 + 1.0f, y0);
    jx += jx & 1;
    jy += jy & 1;
    const iq_f2 r = ((ax - y * IQ_DP1) - y * IQ_DP2) - y * IQ_DP3;
    const iq_f2 z = r * r;
    const iq_f2 sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    iq_f2 cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
    cp = cp - 0.5f * z;
    cp = cp + 1.0f;
    const int ox = jx & 7, oy = jy & 7;
    const int qx = ox & 3, qy = oy & 3;
    const bool swx = qx == 1 || qx == 2, swy = qy == 1 || qy == 2;
    const float sx = swx ? cp.x : sp.x;                  // sin: the cosine polynomial in octants 1, 2
    const float cy = swy ? sp.y : cp.y;                  // cos: the sine polynomial there
    const bool nsx = f_sign(v.x) != (ox > 3);
    const bool ncy = (oy > 3) != (qy > 1);
    return (iq_f2){nsx ? -sx : sx, ncy ? -cy : cy};
}

// iq_tanf without branches on the common path (|x| <= 8192, finite).
__device__ __forceinline__ float iq_tanf_bf(float x) {
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(!(ax <= IQ_TRIG_MAX), 0)) {
        asm volatile("" ::: "memory");
        return iq_tanf(x);
    }
    int j = (int)(IQ_FOPI * ax);
    float yj = (float)j;
    if (j & 1) {
        j += 1;
        yj += 1.0f;
    }
    const float r = ((ax - yj * IQ_DP1) - yj * IQ_DP2) - yj * IQ_DP3;
    const float zz = r * r;
    const float p = (((((9.38540185543e-3f * zz + 3.11992232697e-3f) * zz + 2.44301354525e-2f) * zz
                       + 5.34112807005e-2f) * zz + 1.33387994085e-1f) * zz + 3.33331568548e-1f) * zz * r + r;
    float y = ax > 1.0e-4f ? p : r;
    // IQ_RCP = iq_rcp_guarded
    const float ay = __builtin_fabsf(y);
    float rc = iq_rcp(y);
    if (__builtin_expect((j & 2) && !(ay >= 0x1p-126f && ay < 0x1p126f), 0)) {
        asm volatile("" ::: "memory");
        rc = 1.0f / y;
    }
    y = (j & 2) ? -rc : y;
    return f_sign(x) ? -y : y;
}
