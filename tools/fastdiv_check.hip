// fastdiv_check.hip — GPU proof of csrc/iq_fastdiv.h against the IEEE expansions hipcc emits.
//
//  * iq_rcp(x) vs 1.0f / x on all 2^32 bit patterns (plus raw v_rcp_f32 and v_sqrt_f32 counts,
//    for information);
//  * iq_div_pre(a, b, iq_rcp(b)) vs a / b on random pairs with exponents in the documented safe
//    range, and on near-midpoint pairs a = RN(b * (q + ulp(q)/2)) that stress the final rounding;
//  * iq_div(a, b) (guarded) on random pairs over the whole finite range, zeros and infinities.
// Bits must match exactly; NaN results are compared as "both NaN" and payload differences are
// counted separately. Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
// -fhip-fp32-correctly-rounded-divide-sqrt -I<csrc> tools/fastdiv_check.hip -o fastdiv_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "iq_fastdiv.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

struct counters {
    unsigned long long n[8];
    unsigned long long sqrt_bad;   // iq_sqrt_n mismatches on its domain
    unsigned long long sqrt_guarded_bad;   // iq_sqrt_guarded mismatches over all inputs
    uint32_t sqrt_worst_below;     // largest failing positive input below the domain
    uint32_t ex_a[16], ex_b[16], ex_got[16], ex_ref[16];
    uint32_t nex;
};

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ bool isnan_u(uint32_t u) { return (u & 0x7fffffffu) > 0x7f800000u; }

// 0 = equal bits, 1 = NaN with another payload, 2 = mismatch
__device__ __forceinline__ int cmp(float got, float ref) {
    const uint32_t g = f2u(got), r = f2u(ref);
    if (g == r) return 0;
    if (isnan_u(g) && isnan_u(r)) return 1;
    return 2;
}

__device__ void record(counters* c, uint32_t a, uint32_t b, float got, float ref) {
    const uint32_t k = atomicAdd(&c->nex, 1u);
    if (k < 16) {
        c->ex_a[k] = a;
        c->ex_b[k] = b;
        c->ex_got[k] = f2u(got);
        c->ex_ref[k] = f2u(ref);
    }
}

// n[0] rcp mismatches, n[1] rcp NaN-payload diffs, n[2] raw v_rcp mismatches, n[3] raw v_sqrt
// mismatches (x >= 0), n[4] inputs tested, n[5] mismatches with |x| in [2^-126, 2^126) (the
// documented exact range), n[6] mismatches on zeros / infinities / NaN
__global__ void rcp_all(counters* c, uint64_t base, uint64_t count) {
    unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0, m5 = 0, m6 = 0, m7 = 0, m8 = 0, m9 = 0, t = 0;
    for (uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < base + count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)i;
        const float x = u2f(u);
        const float ref = 1.0f / x;
        const float got = iq_rcp(x);
        const int k = cmp(got, ref);
        if (k == 2) {
            ++m0;
            const uint32_t ex = (u >> 23) & 0xffu;
            if (ex >= 1u && ex < 253u) {
                ++m5;
                record(c, u, 0, got, ref);
            }
            if (ex == 0u && (u & 0x7fffffu) == 0u) ++m6;
            if (ex == 255u) ++m6;
        } else if (k == 1) {
            ++m1;
        }
        if (cmp(iq_rcp_guarded(x), ref) == 2) ++m7;
        if (cmp(__builtin_amdgcn_rcpf(x), ref) == 2) ++m2;
        if (!(u >> 31) && cmp(__builtin_amdgcn_sqrtf(x), __builtin_sqrtf(x)) == 2) ++m3;
        // iq_sqrt_n on its documented domain: +-0, [2^-96, +inf], negative normals / -inf and NaN;
        // below it (positive) only the largest failing input is recorded, to show where the short
        // form stops being exact. Negative denormals are outside (v_sqrt_f32 flushes them to -0).
        {
            const uint32_t mag = u & 0x7fffffffu;
            const bool in_domain = mag == 0u || mag >= 0x0f800000u || ((u >> 31) && mag >= 0x00800000u);
            const int k2 = cmp(iq_sqrt_n(x), __builtin_sqrtf(x));
            if (in_domain && k2 == 2) {
                ++m8;
                record(c, u, 1, iq_sqrt_n(x), __builtin_sqrtf(x));
            } else if (!in_domain && !(u >> 31) && k2 == 2) {
                atomicMax(&c->sqrt_worst_below, u);
            }
            if (cmp(iq_sqrt_guarded(x), __builtin_sqrtf(x)) == 2) ++m9;
        }
        ++t;
    }
    atomicAdd(&c->n[0], m0);
    atomicAdd(&c->n[1], m1);
    atomicAdd(&c->n[2], m2);
    atomicAdd(&c->n[3], m3);
    atomicAdd(&c->n[4], t);
    atomicAdd(&c->n[5], m5);
    atomicAdd(&c->n[6], m6);
    atomicAdd(&c->n[7], m7);
    atomicAdd(&c->sqrt_bad, m8);
    atomicAdd(&c->sqrt_guarded_bad, m9);
}

__device__ __forceinline__ uint32_t xs32(uint32_t& s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

// random float with |exponent| <= emax around 0, random sign and mantissa
__device__ __forceinline__ float rnd_float(uint32_t& s, int emin, int emax) {
    const uint32_t m = xs32(s) & 0x7fffffu;
    const uint32_t sg = xs32(s) & 0x80000000u;
    const int e = emin + (int)(xs32(s) % (uint32_t)(emax - emin + 1));
    return u2f(sg | ((uint32_t)(e + 127) << 23) | m);
}

// mode 0: random pairs |a|, |b| in [2^-62, 2^62] through iq_div_pre; mode 1: near-midpoint pairs;
// mode 2: iq_div over random bit patterns (whole range incl. specials); mode 3: b with all-ones
// or all-zeros mantissa; mode 4: camera-like (x + jx) / W, W integer in [1, 2^24], a in
// [2^-32, 2^25); mode 5: running-mean-like c / n, n integer in [1, 2^32), c in [2^-90, 1);
// mode 6: iq_div on random pairs with exponents in [-140, 140] (guard boundaries, denormal
// quotients). n[0] mismatches, n[1] NaN payload diffs, n[4] pairs tested.
__global__ void div_rand(counters* c, uint32_t seed, int iters, int mode) {
    uint32_t s = seed ^ (0x9e3779b9u * (blockIdx.x * blockDim.x + threadIdx.x + 1));
    for (int k = 0; k < 4; ++k) xs32(s);
    unsigned long long m0 = 0, m1 = 0, t = 0;
    for (int it = 0; it < iters; ++it) {
        float a, b;
        if (mode == 0) {
            a = rnd_float(s, -62, 62);
            b = rnd_float(s, -62, 62);
        } else if (mode == 4) {
            b = (float)(1u + xs32(s) % (1u << 24));
            a = fabsf(rnd_float(s, -32, 24));
        } else if (mode == 5) {
            const uint32_t n = 1u + (xs32(s) >> (xs32(s) & 31u));
            b = (float)n;
            a = fabsf(rnd_float(s, -90, -1));
        } else if (mode == 6) {
            a = rnd_float(s, -140, 140);
            b = rnd_float(s, -140, 140);
        } else if (mode == 1) {
            b = rnd_float(s, -60, 60);
            const float q = rnd_float(s, -30, 30);
            const double qd = (double)q;
            const double ulp = (double)(u2f(f2u(fabsf(q)) + 1u) - fabsf(q));
            const double mid = qd + (qd < 0 ? -0.5 : 0.5) * ulp;
            const double off = ((double)(int)(xs32(s) % 7u) - 3.0) * ulp * 0x1p-30;
            a = (float)((double)b * (mid + off));
        } else if (mode == 2) {
            a = u2f(xs32(s));
            b = u2f(xs32(s));
        } else {
            const uint32_t sg = xs32(s) & 0x80000000u;
            const int e = -60 + (int)(xs32(s) % 121u);
            b = u2f(sg | ((uint32_t)(e + 127) << 23) | ((xs32(s) & 1u) ? 0x7fffffu : 0u));
            a = rnd_float(s, -60, 60);
        }
        const float ref = a / b;
        const float got = (mode == 2 || mode == 6) ? iq_div(a, b) : iq_div_pre(a, b, iq_rcp(b));
        const int r = cmp(got, ref);
        if (r == 2) {
            ++m0;
            record(c, f2u(a), f2u(b), got, ref);
        } else if (r == 1) {
            ++m1;
        }
        ++t;
    }
    atomicAdd(&c->n[0], m0);
    atomicAdd(&c->n[1], m1);
    atomicAdd(&c->n[4], t);
}

static void report(const char* what, const counters& h) {
    printf("%-34s tested %llu  mismatches %llu  nan-payload %llu", what, h.n[4], h.n[0], h.n[1]);
    if (h.n[2] || h.n[3])
        printf("\n    in [2^-126, 2^126): %llu, zeros/inf/NaN: %llu, iq_rcp_guarded (all): %llu"
               "  (raw v_rcp wrong %llu, raw v_sqrt wrong %llu)",
               h.n[5], h.n[6], h.n[7], h.n[2], h.n[3]);
    printf("\n");
    for (uint32_t k = 0; k < h.nex && k < 8; ++k)
        printf("    a=%08x b=%08x got=%08x ref=%08x\n", h.ex_a[k], h.ex_b[k], h.ex_got[k], h.ex_ref[k]);
}

int main(int argc, char** argv) {
    const int scale = argc > 1 ? atoi(argv[1]) : 1;   // x 2^32 pairs per division mode
    counters* d;
    CHECK(hipMalloc(&d, sizeof(counters)));
    counters h;
    int fails = 0;

    CHECK(hipMemset(d, 0, sizeof(counters)));
    hipLaunchKernelGGL(rcp_all, dim3(65536), dim3(256), 0, 0, d, 0ull, 1ull << 32);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost));
    report("iq_rcp vs 1/x (all 2^32 inputs)", h);
    printf("iq_sqrt_n vs sqrtf on its domain: mismatches %llu (largest failing positive input below 2^-96: "
           "%08x); iq_sqrt_guarded on all 2^32 inputs: mismatches %llu\n",
           h.sqrt_bad, h.sqrt_worst_below, h.sqrt_guarded_bad);
    fails += h.n[5] != 0 || h.n[6] != 0 || h.n[7] != 0 || h.n[4] != (1ull << 32) || h.sqrt_bad != 0 || h.sqrt_guarded_bad != 0;

    const char* names[7] = {"iq_div_pre |a|,|b| in [2^-62,2^62]", "iq_div_pre near-midpoint",
                            "iq_div random bit patterns", "iq_div_pre b mantissa 0/all-ones",
                            "iq_div_pre camera (x+jx)/W", "iq_div_pre running mean c/n",
                            "iq_div exponents [-140,140]"};
    for (int mode = 0; mode < 7; ++mode) {
        CHECK(hipMemset(d, 0, sizeof(counters)));
        for (int r = 0; r < scale; ++r) {
            hipLaunchKernelGGL(div_rand, dim3(16384), dim3(256), 0, 0, d, 0x1234567u + 977u * r + 31u * mode, 1024, mode);
            CHECK(hipGetLastError());
        }
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost));
        report(names[mode], h);
        fails += h.n[0] != 0;
    }
    printf("%s\n", fails ? "FASTDIV_CHECK FAILED" : "FASTDIV_CHECK PASSED");
    CHECK(hipFree(d));
    return fails ? 1 : 0;
}
