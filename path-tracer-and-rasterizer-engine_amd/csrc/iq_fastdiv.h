// iq_fastdiv.h — correctly rounded binary32 reciprocal / division / sqrt on gfx950 with fewer
// instructions than the compiler's generic IEEE expansions (device only).
//
// The kernel must reproduce IEEE `1.0f / x`, `a / b` and `sqrtf(x)` bit for bit. The
// generic expansions hipcc emits under -fhip-fp32-correctly-rounded-divide-sqrt cost 10 VALU
// instructions per division (v_div_scale x2, v_rcp, 5 FMA, v_div_fmas, v_div_fixup) and 15 per
// sqrt. The forms below rely on:
//
//  * v_rcp_f32 is accurate to 1 ulp, so with e = 1 - x*y0 formed exactly by one FMA a single
//    Newton correction y1 = RN(y0 + y0*e) is the correctly rounded reciprocal (Markstein) for
//    normal x with a normal reciprocal, |x| in [2^-126, 2^126). v_rcp_f32 flushes denormal results
//    and inputs, so outside that range the result differs from IEEE 1/x. The claim is not taken on
//    faith: tools/fastdiv_check.hip compares iq_rcp with IEEE 1/x on ALL 2^32 inputs on the GPU
//    (profiles/r01_fastdiv_check.txt) and the division forms on 2^36 pairs per operand class;
//  * Markstein's division theorem: if y = RN(1/b) and q = RN(a*y) (within 1 ulp of a/b), then
//    r = a - b*q is exact in one FMA and RN(q + r*y) = RN(a/b), barring over/underflow of the
//    intermediates (the quotient must be normal too: a denormal quotient is off by an ulp).
//    iq_div_pre is only called where the operand ranges rule that out (each call site states the
//    range), iq_div guards it at run time;
//  * v_div_fixup_f32 maps the special operands (zeros, infinities, NaN) to the IEEE result and
//    otherwise returns its first operand with the quotient's sign.
#pragma once

#include <hip/hip_runtime.h>

// RN(1 / x) for |x| in [2^-126, 2^126), for +-0 (+-inf), +-inf (+-0) and NaN (verified exhaustively,
// see above); denormal x and |x| >= 2^126 are NOT exact — call sites keep them out or use
// iq_rcp_guarded.
__device__ __forceinline__ float iq_rcp(float x) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y0, 1.0f);
    const float y1 = __builtin_fmaf(e, y0, y0);
    return __builtin_amdgcn_div_fixupf(y1, x, 1.0f);
}

// RN(a / b) given y = RN(1 / b), for |a| in {0} U [2^-100, 2^100], |b| in [2^-100, 2^100] and a
// normal quotient |a / b| >= 2^-125 (no intermediate under/overflow); zeros, infinities and NaN of
// a are handled by the fixup.
__device__ __forceinline__ float iq_div_pre(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    const float q1 = __builtin_fmaf(r, y, q);
    return __builtin_amdgcn_div_fixupf(q1, b, a);
}

// RN(a / b) for every a, b: the short form when |a|, |b| are in [2^-62, 2^62] (so the quotient
// is in [2^-124, 2^124]), the generic IEEE expansion otherwise (a divergent, rarely taken branch).
__device__ __forceinline__ float iq_div(float a, float b) {
    const float aa = __builtin_fabsf(a), ab = __builtin_fabsf(b);
    if (__builtin_expect(aa >= 0x1p-62f && aa <= 0x1p62f && ab >= 0x1p-62f && ab <= 0x1p62f, 1))
        return iq_div_pre(a, b, iq_rcp(b));
    return a / b;
}

// RN(1 / x) for every x: iq_rcp inside its exact range, the generic expansion outside.
__device__ __forceinline__ float iq_rcp_guarded(float x) {
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(ax >= 0x1p-126f && ax < 0x1p126f, 1)) return iq_rcp(x);
    return 1.0f / x;
}

// RN(sqrt(x)) for x = +-0, x in [2^-96, +inf], negative normals / -inf (NaN) and NaN (verified on
// all such inputs by
// tools/fastdiv_check.hip): v_sqrt_f32 is within 1 ulp, so the correctly rounded root is one of
// s - 1ulp, s, s + 1ulp, picked by the signs of the residuals x - s'*s (one FMA each). Below 2^-96
// the residuals underflow and the pick can be wrong; the generic expansion pre-scales such x by
// 2^32 and adds a class test for 0 / inf on top. Negative denormals give -0 (v_sqrt_f32 flushes
// them), not NaN.
__device__ __forceinline__ float iq_sqrt_n(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, x);
    const float r_up = __builtin_fmaf(-s_up, s, x);
    float t = r_dn <= 0.0f ? s_dn : s;
    t = r_up > 0.0f ? s_up : t;
    return t;
}

// RN(sqrt(x)) for every x (a rarely taken branch for 0 < |x| < 2^-96).
__device__ __forceinline__ float iq_sqrt_guarded(float x) {
    if (__builtin_expect(__builtin_fabsf(x) < 0x1p-96f && x != 0.0f, 0)) return __builtin_sqrtf(x);
    return iq_sqrt_n(x);
}
