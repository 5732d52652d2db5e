/*
 * iq_fp.h — floating-point policy of the iqpt path tracer.
 *
 * The reference kernel (IoniqRE/path_tracer.cu) is FP32 throughout and is compiled by nvcc without
 * --use_fast_math (IoniqRE.vcxproj:58-86): IEEE division and sqrt, but FMA contraction ON and
 * NVIDIA libdevice transcendentals. Neither of the last two can be reproduced outside nvcc, so the
 * parity target of this project is "the reference algorithm, FMA contraction OFF, IEEE div/sqrt,
 * and the transcendentals below" (flavour B). Every translation unit that evaluates
 * the hot path — the HIP kernel, the host-side packet relayout and the CPU oracle — is compiled with
 * -ffp-contract=off and uses the functions in this header, so the GPU and the CPU execute the same
 * sequence of correctly rounded IEEE-754 binary32 operations and agree bit for bit.
 *
 * The functions are written in the common subset of C99 and HIP C++ (no references, no classes)
 * so the plain-C oracle can include this file too. They use only +, -, *, /, sqrt, comparisons and
 * exact float<->int conversions. Accuracy vs the true function: <= 2 ulp on the argument ranges
 * the kernel produces (tests/test_libm.py measures it), the same error class as CUDA's own
 * sinf/cosf/acosf/atan2f (2-3 ulp) that the reference calls.
 *
 * Polynomial coefficients are the classic single-precision minimax sets of the Cephes library
 * (S. L. Moshier, public distribution); the evaluation order is fixed by the code below.
 */
#ifndef IQ_FP_H
#define IQ_FP_H

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define IQ_HD __host__ __device__
#else
#define IQ_HD
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#define IQ_INLINE static inline IQ_HD

/* Divisions inside the functions below. In the GPU pass of a TU that opts in (IQ_FP_FASTDIV) they
 * use the short correctly rounded forms of iq_fastdiv.h (bit-identical to IEEE division, verified
 * exhaustively / on 2^36 pairs per class by tools/fastdiv_check.hip); everywhere else plain IEEE
 * division. IQ_RCP and IQ_DIV are exact for every operand; IQ_DIV_N needs |a| in {0} U
 * [2^-100, 2^100], |b| in [2^-100, 2^100] and a normal quotient, IQ_SQRT_N an argument that is
 * 0 or >= 2^-96 (stated where they are used). */
#if defined(__HIP_DEVICE_COMPILE__) && defined(IQ_FP_FASTDIV)
#include "iq_fastdiv.h"
#define IQ_RCP(x) iq_rcp_guarded(x)
#define IQ_DIV(a, b) iq_div((a), (b))
#define IQ_DIV_N(a, b) iq_div_pre((a), (b), iq_rcp(b))
#define IQ_SQRT_N(x) iq_sqrt_n(x)
#else
#define IQ_RCP(x) (1.0f / (x))
#define IQ_DIV(a, b) ((a) / (b))
#define IQ_DIV_N(a, b) ((a) / (b))
#define IQ_SQRT_N(x) iq_sqrtf(x)
#endif

/* constants of IoniqRE/iqmath.h:6-11 */
#define IQ_PI        3.1415926535897932384626433832795f
#define IQ_TAU       6.283185307179586476925286766559f
#define IQ_PI_DIV_2  1.5707963267948966192313216916398f
#define IQ_PI_DIV_4  0.78539816339744830961566084581988f

/* ---------------------------------------------------------------- bit helpers */
IQ_INLINE uint32_t iq_f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
IQ_INLINE float iq_u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }
IQ_INLINE int iq_isnan(float x) { return (iq_f2u(x) & 0x7fffffffu) > 0x7f800000u; }
IQ_INLINE int iq_isinf(float x) { return (iq_f2u(x) & 0x7fffffffu) == 0x7f800000u; }
IQ_INLINE float iq_fabsf(float x) { return iq_u2f(iq_f2u(x) & 0x7fffffffu); }
IQ_INLINE float iq_copysignf(float m, float s) {
    return iq_u2f((iq_f2u(m) & 0x7fffffffu) | (iq_f2u(s) & 0x80000000u));
}
IQ_INLINE float iq_nanf(void) { return iq_u2f(0x7fc00000u); }

/* IEEE sqrt (correctly rounded on both sides: SSE sqrtss / hipcc's default
 * -fhip-fp32-correctly-rounded-divide-sqrt expansion). */
#if defined(__HIPCC__)
IQ_INLINE float iq_sqrtf(float x) { return __builtin_sqrtf(x); }
#else
IQ_INLINE float iq_sqrtf(float x) { return __builtin_sqrtf(x); }
#endif

/* fmaxf / fminf with C99 NaN semantics (a NaN operand loses). The tie (+0 vs -0) returns the
 * second operand on both sides; the sign of such a zero never reaches an output of the path
 * tracer (it is washed out by the running mean, path_tracer.cu:356-358). */
IQ_INLINE float iq_fmaxf(float a, float b) {
    if (iq_isnan(a)) return b;
    if (iq_isnan(b)) return a;
    return a > b ? a : b;
}
IQ_INLINE float iq_fminf(float a, float b) {
    if (iq_isnan(a)) return b;
    if (iq_isnan(b)) return a;
    return a < b ? a : b;
}

/* ---------------------------------------------------------------- sin / cos / tan
 * Octant reduction by pi/4 with a three-part Cody-Waite constant (each part has enough trailing
 * zero bits that y*DPk is exact for the octant counts reached below 8192). */
#define IQ_FOPI 1.27323954473516f              /* 4/pi */
#define IQ_DP1  0.78515625f
#define IQ_DP2  2.4187564849853515625e-4f
#define IQ_DP3  3.77489497744594108e-8f
#define IQ_TRIG_MAX 8192.0f

IQ_INLINE float iq__sin_poly(float r, float z) {
    return ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
}
/* 0.5 z, exact scaling with one rounding either way. On the device as v_ldexp_f32: as a multiply the
 * SLP vectorizer pairs it with the polynomial's last multiply into a v_pk_mul_f32 whose constant half
 * (0.5) then lives in a VGPR pair that the register-bound render kernels spill to scratch. */
#if defined(__HIP_DEVICE_COMPILE__)
IQ_INLINE float iq__half(float z) { return __builtin_ldexpf(z, -1); }
#else
IQ_INLINE float iq__half(float z) { return 0.5f * z; }
#endif
IQ_INLINE float iq__cos_poly(float z) {
    float y = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
    y = y - iq__half(z);
    return y + 1.0f;
}

/* Octant reduction of ax >= 0, ax <= IQ_TRIG_MAX: returns the reduced argument, octant in *oct. */
IQ_INLINE float iq__reduce_octant(float ax, int* oct) {
    int j = (int)(IQ_FOPI * ax);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    *oct = j & 7;
    return ((ax - y * IQ_DP1) - y * IQ_DP2) - y * IQ_DP3;
}

/* Arguments outside [-8192, 8192] never occur on the hot path (every angle there is the output
 * of atan2/acos or 2*pi*u with u in [0,1]); they get a deterministic double-precision reduction so
 * host-side callers (model rotations) stay reproducible. */
IQ_INLINE float iq__reduce_big(float ax, int* oct) {
    double xd = (double)ax;
    double k = (double)(int64_t)(xd * 1.2732395447351628);  /* 4/pi */
    if (((int64_t)k) & 1) k += 1.0;
    *oct = (int)(((int64_t)k) & 7);
    double r = ((xd - k * 0.78539816290140151978) - k * 4.9604678871439933374e-10)
               - k * 1.1258708853173288931e-18;
    return (float)r;
}

IQ_INLINE float iq_sinf(float x) {
    if (iq_isnan(x) || iq_isinf(x)) return iq_nanf();
    float ax = iq_fabsf(x);
    float sign = (iq_f2u(x) >> 31) ? -1.0f : 1.0f;      /* sin(-0) = -0 */
    if (ax > 1.0e18f) return 0.0f;
    int j;
    float r = ax <= IQ_TRIG_MAX ? iq__reduce_octant(ax, &j) : iq__reduce_big(ax, &j);
    if (j > 3) { sign = -sign; j -= 4; }
    float z = r * r;
    float y = (j == 1 || j == 2) ? iq__cos_poly(z) : iq__sin_poly(r, z);
    return sign < 0.0f ? -y : y;
}

IQ_INLINE float iq_cosf(float x) {
    if (iq_isnan(x) || iq_isinf(x)) return iq_nanf();
    float ax = iq_fabsf(x);
    if (ax > 1.0e18f) return 1.0f;
    int j;
    float sign = 1.0f;
    float r = ax <= IQ_TRIG_MAX ? iq__reduce_octant(ax, &j) : iq__reduce_big(ax, &j);
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    float z = r * r;
    float y = (j == 1 || j == 2) ? iq__sin_poly(r, z) : iq__cos_poly(z);
    return sign < 0.0f ? -y : y;
}

/* sin and cos of one argument with one shared reduction; bit-identical to iq_sinf / iq_cosf. */
IQ_INLINE void iq_sincosf(float x, float* s_out, float* c_out) {
    if (iq_isnan(x) || iq_isinf(x)) { *s_out = iq_nanf(); *c_out = iq_nanf(); return; }
    float ax = iq_fabsf(x);
    if (ax > 1.0e18f) { *s_out = 0.0f; *c_out = 1.0f; return; }
    int j;
    float r = ax <= IQ_TRIG_MAX ? iq__reduce_octant(ax, &j) : iq__reduce_big(ax, &j);
    float ssign = (iq_f2u(x) >> 31) ? -1.0f : 1.0f;
    float csign = 1.0f;
    if (j > 3) { ssign = -ssign; csign = -csign; j -= 4; }
    if (j > 1) csign = -csign;
    float z = r * r;
    float ps = iq__sin_poly(r, z), pc = iq__cos_poly(z);
    int swap = (j == 1 || j == 2);
    float sy = swap ? pc : ps, cy = swap ? ps : pc;
    *s_out = ssign < 0.0f ? -sy : sy;
    *c_out = csign < 0.0f ? -cy : cy;
}

IQ_INLINE float iq_tanf(float x) {
    if (iq_isnan(x) || iq_isinf(x)) return iq_nanf();
    float ax = iq_fabsf(x);
    if (ax > 1.0e18f) return 0.0f;
    int j;
    float r;
    if (ax <= IQ_TRIG_MAX) {
        j = (int)(IQ_FOPI * ax);
        float yj = (float)j;
        if (j & 1) { j += 1; yj += 1.0f; }
        r = ((ax - yj * IQ_DP1) - yj * IQ_DP2) - yj * IQ_DP3;
    } else {
        r = iq__reduce_big(ax, &j);
    }
    float zz = r * r;
    float y;
    if (ax > 1.0e-4f) {
        y = (((((9.38540185543e-3f * zz + 3.11992232697e-3f) * zz + 2.44301354525e-2f) * zz
              + 5.34112807005e-2f) * zz + 1.33387994085e-1f) * zz + 3.33331568548e-1f) * zz * r + r;
    } else {
        y = r;
    }
    if (j & 2) y = -IQ_RCP(y);
    return (iq_f2u(x) >> 31) ? -y : y;
}

/* ---------------------------------------------------------------- asin / acos */
IQ_INLINE float iq_asinf(float x) {
    if (iq_isnan(x)) return x;
    float a = iq_fabsf(x);
    if (a > 1.0f) return iq_nanf();
    float z;
    if (a < 1.0e-4f) {
        z = a;
    } else {
        float r, zz;
        int flag;
        /* 1 - a is 0 or >= 2^-24 (a <= 1): zz is 0 or normal */
        if (a > 0.5f) { zz = 0.5f * (1.0f - a); r = IQ_SQRT_N(zz); flag = 1; }
        else { r = a; zz = r * r; flag = 0; }
        z = ((((4.2163199048e-2f * zz + 2.4181311049e-2f) * zz + 4.5470025998e-2f) * zz
              + 7.4953002686e-2f) * zz + 1.6666752422e-1f) * zz * r + r;
        if (flag) { z = z + z; z = IQ_PI_DIV_2 - z; }
    }
    return (iq_f2u(x) >> 31) ? -z : z;
}

IQ_INLINE float iq_acosf(float x) {
    if (iq_isnan(x)) return x;
    if (x < -1.0f || x > 1.0f) return iq_nanf();
    /* 1 +- x is 0 or >= 2^-24 here: the root's argument is 0 or normal */
    if (x < -0.5f) return IQ_PI - 2.0f * iq_asinf(IQ_SQRT_N(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * iq_asinf(IQ_SQRT_N(0.5f * (1.0f - x)));
    return IQ_PI_DIV_2 - iq_asinf(x);
}

/* ---------------------------------------------------------------- atan / atan2 */
IQ_INLINE float iq_atanf(float x) {
    if (iq_isnan(x)) return x;
    float ax = iq_fabsf(x);
    float y, r;
    /* (ax - 1) is 0 or in [2^-24, 1.5) and (ax + 1) in (1.4, 3.5): inside IQ_DIV_N's range */
    if (ax > 2.414213562373095f) { y = IQ_PI_DIV_2; r = -IQ_RCP(ax); }
    else if (ax > 0.4142135623730950f) { y = IQ_PI_DIV_4; r = IQ_DIV_N(ax - 1.0f, ax + 1.0f); }
    else { y = 0.0f; r = ax; }
    float z = r * r;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
              - 3.33329491539e-1f) * z * r + r);
    return (iq_f2u(x) >> 31) ? -y : y;
}

/* atan2 with the C99 Annex F special cases (signed zeros, infinities, NaN). */
IQ_INLINE float iq_atan2f(float y, float x) {
    if (iq_isnan(x) || iq_isnan(y)) return iq_nanf();
    int ysign = (iq_f2u(y) >> 31) != 0;
    int xsign = (iq_f2u(x) >> 31) != 0;
    float res;
    if (y == 0.0f) {
        res = xsign ? IQ_PI : 0.0f;                       /* atan2(+-0, -x|-0) = +-pi */
    } else if (iq_isinf(y)) {
        if (iq_isinf(x)) res = xsign ? 3.0f * IQ_PI_DIV_4 : IQ_PI_DIV_4;
        else res = IQ_PI_DIV_2;
    } else if (x == 0.0f) {
        res = IQ_PI_DIV_2;
    } else if (iq_isinf(x)) {
        res = xsign ? IQ_PI : 0.0f;
    } else {
        float ay = iq_fabsf(y);
        float z = iq_atanf(IQ_DIV(ay, iq_fabsf(x)));
        res = xsign ? IQ_PI - z : z;
    }
    return ysign ? -res : res;
}

#endif /* IQ_FP_H */
