// iqpt_kernels.hip — the MI355X (gfx950, CDNA4, wave64) path-tracing megakernel and RNG init.
//
// Replaces render_kernel + path_tracer::ray_color + renderer_init_kernel of IoniqRE
// (path_tracer.cu:36-46, 231-366) and the device code they inline (camera.cu:20-43,
// shape.cu:13-103, material.cu:5-57, onb.h, random.cu:66-107, cuRAND XORWOW).
//
// Design:
//  * Persistent grid, one lane = one pixel at a time. A lane runs ALL of its pixel's samples of
//    the launch back to back (a pixel's samples are sequential in its XORWOW stream: each sample
//    consumes a data-dependent number of draws), regenerating a camera ray as soon as a path ends,
//    so every iteration traces one ray per live lane. Lanes that finish their pixel refill from a
//    global pixel queue: one atomic per 64-pixel chunk per wave, handed to the empty lanes with a
//    wave64 __ballot + mbcnt prefix sum.
//  * The scene is pre-transformed to world space at upload (the per-ray transforms and the
//    per-drawcall normal-matrix inverse of path_tracer.cu:257-270 are ray-independent) and laid out
//    as SoA primitive PAIRS: one packed v_pk_{mul,add}_f32 instruction advances two Möller–Trumbore
//    (or two sphere) tests, with operand pairs arriving in aligned VGPR pairs from ds_read_b128.
//    Packed FP32 ops round each element exactly like the scalar op, and the closest-hit updates of
//    the two primitives stay sequential, so results are unchanged bit for bit.
//  * Small scenes stay resident in LDS for the whole launch; large scenes are streamed through LDS
//    in batches behind workgroup barriers (workgroup-uniform loop).
//  * The scatter_record stack (path_tracer.cu:243, 321-324) lives in LDS, one float per thread per
//    level (bank-conflict free): under the reference materials every non-terminal record is an
//    Oren–Nayar scatter whose (attenuation * cos/pdf) is the same in x, y and z, so a record is one
//    float, and the backward product reads them newest to oldest in the reference's order.
//  * Every floating-point operation follows the reference's order with contraction off
//    (-ffp-contract=off) and the shared transcendentals of iq_fp.h; every shortcut below is exact
//    (argued where it is taken). Results are bit-identical to the CPU oracle.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

// the transcendentals of iq_fp.h use the short exact division forms in this TU's GPU pass
#define IQ_FP_FASTDIV 1
#include "iq_fastdiv.h"
#include "iq_fp.h"
#include "iq_fp2.h"
#include "iq_interval.h"
#include "iq_xorwow.h"
#include "iqpt_internal.hpp"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace iqpt {
namespace {

constexpr float kTMin = 0.000001f;       // path_tracer.cu:241
constexpr float kTMax = 999.99f;
constexpr int kHitNone = 0, kHitTri = 1, kHitSphere = 2;
constexpr float kRcpPi = 0x1.45f306p-2f;   // RN(1 / IQ_PI) of the float IQ_PI
constexpr uint32_t kStitchBlock = 64;       // iqpt_split_stitch_kernel: one wave per block
static_assert(1.0f / IQ_PI == kRcpPi, "kRcpPi must be the correctly rounded reciprocal of the float pi");

typedef float f2 __attribute__((ext_vector_type(2)));

struct rng6 {
    uint32_t v0, v1, v2, v3, v4, d;
};

__device__ __forceinline__ uint32_t xorwow_next(rng6& s) {     // cuRAND curand() (iq_xorwow.h)
    const uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += IQ_XORWOW_WEYL;
    return s.v4 + s.d;
}

// random::real(state, lo, hi) (random.cu:66-70): u * (hi - lo) + lo with u = curand / 2^32.
__device__ __forceinline__ float rand_real(rng6& s, float lo, float hi) {
    const float u = iq_u32_to_unit(xorwow_next(s));
    return u * (hi - lo) + lo;
}

// kOptStats: per-thread counts of the primitive tests executed (Möller–Trumbore triangle tests, sphere
// tests; a packed pair counts two) for the executed-work roofline (tools/work_counters.py), in LDS.
template <int OPT>
__device__ __forceinline__ uint32_t* stat_tests() {
    __shared__ uint32_t cnt[2 * 256];
    return cnt;
}
template <int OPT>
__device__ __forceinline__ void stat_add(int which, uint32_t n) {
    if (OPT & kOptStats) stat_tests<OPT>()[which * 256 + threadIdx.x] += n;
}

// IEEE 1/x under kOptFastDiv (iq_fastdiv.h), the generic expansion otherwise.
// rcp_scene: x is a Möller–Trumbore determinant with |det| >= 1e-6 or a sphere radius; the runtime
// launches kOptFastDiv variants only when every edge component and radius of the packet is within
// 2^60 (radii 0 or >= 2^-60), so |det| <= |e1| |e2| |dir| < 2^126 and 1/r is in iq_rcp's exact range.
template <int OPT>
__device__ __forceinline__ float rcp_scene(float x) {
    if (OPT & kOptFastDiv) return iq_rcp(x);
    return 1.0f / x;
}
// rcp_any: no range known (a rarely taken branch keeps the generic expansion outside iq_rcp's range).
template <int OPT>
__device__ __forceinline__ float rcp_any(float x) {
    if (OPT & kOptFastDiv) return iq_rcp_guarded(x);
    return 1.0f / x;
}

// IEEE sqrt: iq_sqrt_n (iq_fastdiv.h) where the argument is known to be 0, >= 2^-96, inf or NaN
// (sqrt_n), the guarded form elsewhere (sqrt_any).
template <int OPT>
__device__ __forceinline__ float sqrt_n(float x) {
    if (OPT & kOptFastDiv) return iq_sqrt_n(x);
    return iq_sqrtf(x);
}
template <int OPT>
__device__ __forceinline__ float sqrt_any(float x) {
    if (OPT & kOptFastDiv) return iq_sqrt_guarded(x);
    return iq_sqrtf(x);
}

// normalized3 (vector.h:239-244) in place.
template <int OPT>
__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
    if (iq_fabsf(x) < 0.00001f && iq_fabsf(y) < 0.00001f && iq_fabsf(z) < 0.00001f) {
        x = 0.0f;
        y = 0.0f;
        z = 0.0f;
        return;
    }
    // one component is >= 1e-5 in magnitude, so len^2 >= 1e-10 (or inf / NaN): sqrt_n's domain
    const float len = sqrt_n<OPT>((x * x + y * y) + z * z);
    const float inv = rcp_any<OPT>(len);
    x = x * inv;
    y = y * inv;
    z = z * inv;
}

struct ray3 {
    float ox, oy, oz, dx, dy, dz;
};

// camera::get_ray (camera.cu:20-43): x jitter drawn first, then y.
// kOptCamConst: when the inverse projection has m[0][3] = m[1][3] = 0 and finite non-zero m[2][3],
// m[3][3] (checked exactly on the host), w_near = ((x*0 + y*0) + 0*m23) + m33 = m33 and
// w_far = ((x*0 + y*0) + m23) + m33 = fl(m23 + m33) for every finite x, y, so 1/w are launch
// constants computed by the same IEEE division on the host (p.cam_near_rw / p.cam_far_rw).
template <int OPT>
__device__ __forceinline__ void camera_ndc(const kparams& p, float x_ndc, float y_ndc, ray3& r) {
    // rows of the inverse projection P and inverse view V (row-major m[r][c], camera.h:30-31)
    const float* P = p.inv_proj;
    const float* Vw = p.inv_view;
    const float4 P0 = make_float4(P[0], P[1], P[2], P[3]), P1 = make_float4(P[4], P[5], P[6], P[7]);
    const float4 P2 = make_float4(P[8], P[9], P[10], P[11]), P3 = make_float4(P[12], P[13], P[14], P[15]);
    const float4 V0 = make_float4(Vw[0], Vw[1], Vw[2], Vw[3]), V1 = make_float4(Vw[4], Vw[5], Vw[6], Vw[7]);
    const float4 V2 = make_float4(Vw[8], Vw[9], Vw[10], Vw[11]), V3 = make_float4(Vw[12], Vw[13], Vw[14], Vw[15]);
    // dot4(v, column c) of iqvec::transformed (vector.h:371-383), columns spelled out
    float nx = ((x_ndc * P0.x + y_ndc * P1.x) + 0.0f * P2.x) + 1.0f * P3.x;
    float ny = ((x_ndc * P0.y + y_ndc * P1.y) + 0.0f * P2.y) + 1.0f * P3.y;
    float nz = ((x_ndc * P0.z + y_ndc * P1.z) + 0.0f * P2.z) + 1.0f * P3.z;
    float fx = ((x_ndc * P0.x + y_ndc * P1.x) + 1.0f * P2.x) + 1.0f * P3.x;
    float fy = ((x_ndc * P0.y + y_ndc * P1.y) + 1.0f * P2.y) + 1.0f * P3.y;
    float fz = ((x_ndc * P0.z + y_ndc * P1.z) + 1.0f * P2.z) + 1.0f * P3.z;
    float ninv, finv;
    if ((OPT & kOptCamConst) && p.cam_const) {
        ninv = p.cam_near_rw;
        finv = p.cam_far_rw;
    } else {
        ninv = rcp_any<OPT>(((x_ndc * P0.w + y_ndc * P1.w) + 0.0f * P2.w) + 1.0f * P3.w);
        finv = rcp_any<OPT>(((x_ndc * P0.w + y_ndc * P1.w) + 1.0f * P2.w) + 1.0f * P3.w);
    }
    nx = nx * ninv;
    ny = ny * ninv;
    nz = nz * ninv;
    fx = fx * finv;
    fy = fy * finv;
    fz = fz * finv;
    // to world space: usage POINT forces w = 1 (vector.h:374)
    const float wnx = ((nx * V0.x + ny * V1.x) + nz * V2.x) + 1.0f * V3.x;
    const float wny = ((nx * V0.y + ny * V1.y) + nz * V2.y) + 1.0f * V3.y;
    const float wnz = ((nx * V0.z + ny * V1.z) + nz * V2.z) + 1.0f * V3.z;
    const float wfx = ((fx * V0.x + fy * V1.x) + fz * V2.x) + 1.0f * V3.x;
    const float wfy = ((fx * V0.y + fy * V1.y) + fz * V2.y) + 1.0f * V3.y;
    const float wfz = ((fx * V0.z + fy * V1.z) + fz * V2.z) + 1.0f * V3.z;
    float dx = wfx - wnx, dy = wfy - wny, dz = wfz - wnz;
    normalize3<OPT>(dx, dy, dz);
    r.ox = wnx;
    r.oy = wny;
    r.oz = wnz;
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
}

// kOptCamAxis: the same transform for a pitch-only camera. The runtime enables it when P[1] = P[2] =
// P[4] = P[6] = P[8] = P[9] = 0 (standard perspective inverse, kOptCamConst's w row) and V[1] = V[2] =
// V[4] = V[8] = 0 (no yaw, no roll), every entry finite, and none of P[12], P[13], P[14], V[12], V[13],
// V[14] is -0. Every term of camera_ndc left out here is (finite) * (+-0), so each dot product of
// camera_ndc equals the kept terms' sum s, or both are zeros of possibly opposite sign; the last
// addend of every chain is kept (P[12], P[13], V[12], V[13], V[14]; the z chains are launch
// constants ending in P[14]), and c + z = c for c != 0, +0 + z = +0 for a zero z, so both chains
// end on the same bits. The z terms are computed on the host with the same float operations
// (cam_axis_constants). The runtime also proves with the interval bundle of iq_interval.h over the
// whole frame that normalize3's zero branch is never taken and |far - near| < 2^100, so 1/len is
// iq_rcp's exact case.
template <int OPT>
__device__ __forceinline__ void camera_ray_axis(const kparams& p, float x_ndc, float y_ndc, ray3& r) {
    const float* k = p.cam_ax;
    // (near, far) world-space points, both in one packed register pair
    const f2 nf_rw = {k[4], k[5]};                  // 1 / w_near, 1 / w_far
    const f2 xw = (x_ndc * k[0] + k[2]) * nf_rw;    // (((x P[0] + y P[4]) + z P[8]) + P[12]) / w
    const f2 yw = (y_ndc * k[1] + k[3]) * nf_rw;    // (((x P[1] + y P[5]) + z P[9]) + P[13]) / w
    const f2 kzy = {k[12], k[13]}, kzz = {k[14], k[15]};
    const f2 wx = xw * k[6] + k[7];                 // ((x V[0] + y V[4]) + z V[8]) + V[12]
    const f2 wy = (yw * k[8] + kzy) + k[10];        // ((x V[1] + y V[5]) + z V[9]) + V[13]
    const f2 wz = (yw * k[9] + kzz) + k[11];        // ((x V[2] + y V[6]) + z V[10]) + V[14]
    float dx = wx.y - wx.x, dy = wy.y - wy.x, dz = wz.y - wz.x;
    // normalize3 without the zero branch; len in [1e-5, 2^100): iq_rcp is exact (kOptFastDiv)
    const float len = sqrt_n<OPT>((dx * dx + dy * dy) + dz * dz);
    const float inv = (OPT & kOptFastDiv) ? iq_rcp(len) : 1.0f / len;
    r.ox = wx.x;
    r.oy = wy.x;
    r.oz = wz.x;
    r.dx = dx * inv;
    r.dy = dy * inv;
    r.dz = dz * inv;
}

template <int OPT>
__device__ __forceinline__ void camera_ray(const kparams& p, uint32_t x, uint32_t y, rng6& s, ray3& r) {
    const float jx = rand_real(s, -0.5f, 0.5f);
    // (x + jx) / W: under kOptFastDiv Markstein's correction of (x + jx) * RN(1/W) (RN(1/W) from the
    // host); exact here since x + jx is 0 or in [2^-32, 2^24] and W in [1, 2^24] (iq_fastdiv.h)
    const float xs = (float)x + jx;
    const float x_ndc = ((OPT & kOptFastDiv) ? iq_div_pre(xs, (float)p.width, p.rcp_width)
                                             : xs / (float)p.width) * 2.0f - 1.0f;
    const float jy = rand_real(s, -0.5f, 0.5f);
    const float ys = (float)y + jy;
    const float y_ndc = 1.0f - ((OPT & kOptFastDiv) ? iq_div_pre(ys, (float)p.height, p.rcp_height)
                                                    : ys / (float)p.height) * 2.0f;
    if (OPT & kOptCamAxis) camera_ray_axis<OPT>(p, x_ndc, y_ndc, r);
    else camera_ndc<OPT>(p, x_ndc, y_ndc, r);
}

// n XORWOW steps of the xorshift part (random.cu:66-107; the Weyl word d is the caller's, d += n WEYL).
// Five steps at a time: each new word takes the slot of the word it retires (x_{k+5} = f(x_k, x_{k+4})),
// so after five steps v0..v4 name the state again and no register moves are needed; the rest one by one.
__device__ __forceinline__ uint32_t xorwow_next_word(uint32_t x, uint32_t y) {
    const uint32_t t = x ^ (x >> 2);
    return (y ^ (y << 4)) ^ (t ^ (t << 1));
}

__device__ __forceinline__ void xorwow_skip_v(uint32_t& v0, uint32_t& v1, uint32_t& v2, uint32_t& v3, uint32_t& v4,
                                              uint32_t n) {
    for (uint32_t k = n / 5u; k; --k) {
        v0 = xorwow_next_word(v0, v4);
        v1 = xorwow_next_word(v1, v0);
        v2 = xorwow_next_word(v2, v1);
        v3 = xorwow_next_word(v3, v2);
        v4 = xorwow_next_word(v4, v3);
    }
    for (uint32_t i = n % 5u; i; --i) {
        const uint32_t t = v0 ^ (v0 >> 2);
        v0 = v1;
        v1 = v2;
        v2 = v3;
        v3 = v4;
        v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
    }
}

// CUDA float -> uint8_t: NaN -> 0, saturating, truncating (path_tracer.cu:361-363).
__device__ __forceinline__ uint32_t to_u8(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 255.0f) return 255u;
    return (uint32_t)f;
}

// Möller–Trumbore of shape.cu:62-103 with the hit bookkeeping reduced to (t, index); every reject
// test is the reference's condition, negated, so NaN behaves identically.
template <int OPT>
__device__ __forceinline__ void test_triangle(const float4 a, const float4 b, const float4 c, const ray3 r,
                                              float& closest, int& kind, uint32_t& idx, uint32_t k) {
    stat_add<OPT>(0, 1u);
    const float e1x = a.w, e1y = b.x, e1z = b.y;
    const float e2x = b.z, e2y = b.w, e2z = c.x;
    const float px = r.dy * e2z - r.dz * e2y;                   // dir x v0v2
    const float py = r.dz * e2x - r.dx * e2z;
    const float pz = r.dx * e2y - r.dy * e2x;
    const float det = (e1x * px + e1y * py) + e1z * pz;
    if (iq_fabsf(det) < 0.000001f) return;                      // is_zero(fabs(det))
    const float inv = rcp_scene<OPT>(det);
    const float tx = r.ox - a.x, ty = r.oy - a.y, tz = r.oz - a.z;
    const float u = ((tx * px + ty * py) + tz * pz) * inv;
    if (u < 0.0f || u > 1.0f) return;
    const float qx = ty * e1z - tz * e1y;                       // tvec x v0v1
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    const float v = ((r.dx * qx + r.dy * qy) + r.dz * qz) * inv;
    if (v < 0.0f || u + v > 1.0f) return;
    const float t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    if (t < kTMin || closest < t) return;
    closest = t;
    kind = kHitTri;
    idx = k;
}

// The same Möller–Trumbore for the pair (k, k+1), both in flight in packed registers. Each
// element sees exactly the scalar operation sequence above; `alive` masks the odd tail. The t
// test against the running closest hit is sequential (k first), as in the reference's loop.
// Branchless form (kOptBranchless): all stages always evaluated, the reference's reject tests
// folded into the two `alive` masks; same per-element operations, so the same bits.
template <int OPT>
__device__ __forceinline__ void test_triangle_pair_nb(const float4 q0, const float4 q1, const float4 q2,
                                                      const float4 q3, const float4 q4, const ray3 r,
                                                      float& closest, int& kind, uint32_t& idx, uint32_t k,
                                                      bool second) {
    stat_add<OPT>(0, 2u);
    const f2 v0x = {q0.x, q0.y}, v0y = {q0.z, q0.w}, v0z = {q1.x, q1.y};
    const f2 e1x = {q1.z, q1.w}, e1y = {q2.x, q2.y}, e1z = {q2.z, q2.w};
    const f2 e2x = {q3.x, q3.y}, e2y = {q3.z, q3.w}, e2z = {q4.x, q4.y};
    const f2 px = r.dy * e2z - r.dz * e2y;
    const f2 py = r.dz * e2x - r.dx * e2z;
    const f2 pz = r.dx * e2y - r.dy * e2x;
    const f2 det = (e1x * px + e1y * py) + e1z * pz;
    const f2 inv = {rcp_scene<OPT>(det.x), rcp_scene<OPT>(det.y)};
    const f2 tx = r.ox - v0x, ty = r.oy - v0y, tz = r.oz - v0z;
    const f2 u = ((tx * px + ty * py) + tz * pz) * inv;
    const f2 qx = ty * e1z - tz * e1y;
    const f2 qy = tz * e1x - tx * e1z;
    const f2 qz = tx * e1y - ty * e1x;
    const f2 v = ((r.dx * qx + r.dy * qy) + r.dz * qz) * inv;
    const f2 uv = u + v;
    const f2 t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    const bool a0 = !(iq_fabsf(det.x) < 0.000001f) && !(u.x < 0.0f || u.x > 1.0f) &&
                    !(v.x < 0.0f || uv.x > 1.0f) && !(t.x < kTMin);
    const bool a1 = second && !(iq_fabsf(det.y) < 0.000001f) && !(u.y < 0.0f || u.y > 1.0f) &&
                    !(v.y < 0.0f || uv.y > 1.0f) && !(t.y < kTMin);
    if (a0 && !(closest < t.x)) {
        closest = t.x;
        kind = kHitTri;
        idx = k;
    }
    if (a1 && !(closest < t.y)) {
        closest = t.y;
        kind = kHitTri;
        idx = k + 1;
    }
}

template <int OPT>
__device__ __forceinline__ void test_triangle_pair(const float4 q0, const float4 q1, const float4 q2,
                                                   const float4 q3, const float4 q4, const ray3 r, float& closest,
                                                   int& kind, uint32_t& idx, uint32_t k, bool second) {
    stat_add<OPT>(0, 2u);
    const f2 v0x = {q0.x, q0.y}, v0y = {q0.z, q0.w}, v0z = {q1.x, q1.y};
    const f2 e1x = {q1.z, q1.w}, e1y = {q2.x, q2.y}, e1z = {q2.z, q2.w};
    const f2 e2x = {q3.x, q3.y}, e2y = {q3.z, q3.w}, e2z = {q4.x, q4.y};
    const f2 px = r.dy * e2z - r.dz * e2y;
    const f2 py = r.dz * e2x - r.dx * e2z;
    const f2 pz = r.dx * e2y - r.dy * e2x;
    const f2 det = (e1x * px + e1y * py) + e1z * pz;
    bool a0 = !(iq_fabsf(det.x) < 0.000001f);
    bool a1 = second && !(iq_fabsf(det.y) < 0.000001f);
    if (!(a0 || a1)) return;
    const f2 inv = {rcp_scene<OPT>(det.x), rcp_scene<OPT>(det.y)};
    const f2 tx = r.ox - v0x, ty = r.oy - v0y, tz = r.oz - v0z;
    const f2 u = ((tx * px + ty * py) + tz * pz) * inv;
    a0 = a0 && !(u.x < 0.0f || u.x > 1.0f);
    a1 = a1 && !(u.y < 0.0f || u.y > 1.0f);
    if (!(a0 || a1)) return;
    const f2 qx = ty * e1z - tz * e1y;
    const f2 qy = tz * e1x - tx * e1z;
    const f2 qz = tx * e1y - ty * e1x;
    const f2 v = ((r.dx * qx + r.dy * qy) + r.dz * qz) * inv;
    const f2 uv = u + v;
    a0 = a0 && !(v.x < 0.0f || uv.x > 1.0f);
    a1 = a1 && !(v.y < 0.0f || uv.y > 1.0f);
    if (!(a0 || a1)) return;
    const f2 t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    if (a0 && !(t.x < kTMin || closest < t.x)) {
        closest = t.x;
        kind = kHitTri;
        idx = k;
    }
    if (a1 && !(t.y < kTMin || closest < t.y)) {
        closest = t.y;
        kind = kHitTri;
        idx = k + 1;
    }
}

// sphere::intersect (shape.cu:13-46), far root not checked against t_max (reference quirk).
template <int OPT>
__device__ __forceinline__ void sphere_roots(float halfb, float delta, float& closest, int& kind, uint32_t& idx,
                                             uint32_t k) {
    const float sd = sqrt_any<OPT>(delta);      // delta >= 0 may be tiny (grazing rays)
    float t = halfb - sd;
    if (closest < t) return;
    if (t < kTMin) {
        t = halfb + sd;
        if (t < kTMin) return;
    }
    closest = t;
    kind = kHitSphere;
    idx = k;
}

template <int OPT>
__device__ __forceinline__ void test_sphere(const float4 s, const ray3 r, float& closest, int& kind,
                                            uint32_t& idx, uint32_t k) {
    stat_add<OPT>(1, 1u);
    const float ocx = s.x - r.ox, ocy = s.y - r.oy, ocz = s.z - r.oz;
    const float halfb = (r.dx * ocx + r.dy * ocy) + r.dz * ocz;
    const float cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.w * s.w;
    const float delta = halfb * halfb - cc;
    if (delta < 0.0f) return;
    sphere_roots<OPT>(halfb, delta, closest, kind, idx, k);
}

// Two spheres (k, k+1) with the quadratic set up in packed registers, roots tested in order.
template <int OPT>
__device__ __forceinline__ void test_sphere_pair(const float4 s0, const float4 s1, const ray3 r, float& closest,
                                                 int& kind, uint32_t& idx, uint32_t k, bool second) {
    stat_add<OPT>(1, 2u);
    const f2 cx = {s0.x, s0.y}, cy = {s0.z, s0.w}, cz = {s1.x, s1.y}, rad = {s1.z, s1.w};
    const f2 ocx = cx - r.ox, ocy = cy - r.oy, ocz = cz - r.oz;
    const f2 halfb = (r.dx * ocx + r.dy * ocy) + r.dz * ocz;
    const f2 cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rad * rad;
    const f2 delta = halfb * halfb - cc;
    const bool a0 = !(delta.x < 0.0f);
    const bool a1 = second && !(delta.y < 0.0f);
    if (a0) sphere_roots<OPT>(halfb.x, delta.x, closest, kind, idx, k);
    if (a1) sphere_roots<OPT>(halfb.y, delta.y, closest, kind, idx, k + 1);
}

// Sphere hit record (shape.cu:36-44): hit point h = o + t d and the normal (h - c) / r (reciprocal
// multiply), flipped to face the ray.
template <int OPT>
__device__ __forceinline__ void sphere_hit(const float4 sph, float t, const ray3& r, float& hx, float& hy, float& hz,
                                           float& nx, float& ny, float& nz) {
    hx = r.ox + t * r.dx;
    hy = r.oy + t * r.dy;
    hz = r.oz + t * r.dz;
    const float rinv = rcp_scene<OPT>(sph.w);
    nx = (hx - sph.x) * rinv;
    ny = (hy - sph.y) * rinv;
    nz = (hz - sph.z) * rinv;
    if (!((r.dx * nx + r.dy * ny) + r.dz * nz < 0.0f)) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
}

// oren_nayar::scatter (material.cu:5-43) at hit point h with hit normal n: writes the continuation
// ray into r and returns coeff (A + B cos(phi_i - phi_o) sin(alpha) tan(beta)) and q = cos / pdf; the
// record is att_c * q with att_c = (albedo_c * coeff) * (1 / pi).
template <int OPT>
__device__ __forceinline__ void or_scatter_core(float hx, float hy, float hz, float nx, float ny, float nz, ray3& r,
                                                rng6& s, float A, float B, float& coeff, float& q) {
    // onb (onb.h:7-12)
    float wx = nx, wy = ny, wz = nz;
    normalize3<OPT>(wx, wy, wz);
    float ax, ay, az;
    if (iq_fabsf(wx) > 0.9f) { ax = 0.0f; ay = 1.0f; az = 0.0f; }
    else { ax = 1.0f; ay = 0.0f; az = 0.0f; }
    float vx = wy * az - wz * ay, vy = wz * ax - wx * az, vz = wx * ay - wy * ax;
    normalize3<OPT>(vx, vy, vz);
    const float ux = vy * wz - vz * wy, uy = vz * wx - vx * wz, uz = vx * wy - vy * wx;
    // cosine_weighted (random.cu:96-107)
    const float u1 = rand_real(s, 0.0f, 1.0f);
    const float u2 = rand_real(s, 0.0f, 1.0f);
    const float phi = (2.0f * IQ_PI) * u1;
    float su2, lz;
    if ((OPT & kOptScatter2) && (OPT & kOptFastDiv)) {
        // u2 = k 2^-32: 0 or >= 2^-32; 1 - u2: 0 or >= 2^-24 (iq_sqrt_n's domain)
        const iq_f2 rt = iq_sqrt_n2((iq_f2){u2, 1.0f - u2});
        su2 = rt.x;
        lz = rt.y;
    } else {
        su2 = sqrt_n<OPT>(u2);                                   // u2 = k 2^-32: 0 or >= 2^-32
        lz = sqrt_n<OPT>(1.0f - u2);                             // 1 - u2: 0 or >= 2^-24
    }
    float sphi, cphi;
    if (OPT & kOptScatter2) {
        const iq_f2 sc = iq_sin_cos2((iq_f2){phi, phi});
        sphi = sc.x;
        cphi = sc.y;
    } else if (OPT & kOptSinCos) {
        iq_sincosf(phi, &sphi, &cphi);
    } else {
        cphi = iq_cosf(phi);
        sphi = iq_sinf(phi);
    }
    const float lx = cphi * su2;
    const float ly = sphi * su2;
    float dx = (ux * lx + vx * ly) + wx * lz;                    // onb::transform_to_world
    float dy = (uy * lx + vy * ly) + wy * lz;
    float dz = (uz * lx + vz * ly) + wz * lz;
    const float wox = -r.dx, woy = -r.dy, woz = -r.dz;
    // oren_nayar::pdf (material.cu:45-48). Under kOptFastDiv the dot is divided by Markstein's
    // correction with RN(1/pi): exact for |dot| in {0} U [2^-100, 2^100]; below 2^-100 both the IEEE
    // and the short quotient are < 1e-5 and the pdf is replaced by 1/pi on both paths.
    const float pdot = (nx * dx + ny * dy) + nz * dz;
    float pdf = (OPT & kOptFastDiv) ? iq_div_pre(pdot, IQ_PI, kRcpPi) : pdot / IQ_PI;
    if (pdf < 0.00001f) {
        dx = nx;
        dy = ny;
        dz = nz;
        pdf = 1.0f / IQ_PI;
    }
    const float cosw = iq_fmaxf(0.0f, (nx * dx + ny * dy) + nz * dz);
    const float cto = iq_fmaxf(0.0f, (wox * nx + woy * ny) + woz * nz);
    const float cti = iq_fmaxf(0.0f, (dx * nx + dy * ny) + dz * nz);
    if (OPT & kOptScatter2) {
        // the independent transcendentals in packed pairs, branch-free (iq_fp2.h; same bits)
        const iq_f2 ph = iq_atan2f2((iq_f2){woy, dy}, (iq_f2){wox, dx});   // (phi_o, phi_i)
        const iq_f2 th = iq_acosf2((iq_f2){cto, cti});
        const float theta_o = cto > 1.0f ? 0.0f : th.x;
        const float theta_i = cti > 1.0f ? 0.0f : th.y;
        const float alpha = iq_fmaxf(theta_i, theta_o);
        const float beta = iq_fminf(theta_i, theta_o);
        const iq_f2 sc = iq_sin_cos2((iq_f2){alpha, ph.y - ph.x});       // (sin(alpha), cos(phi_i - phi_o))
        coeff = A + B * sc.y * sc.x * iq_tanf_bf(beta);
    } else {
        const float phi_o = iq_atan2f(woy, wox);
        const float phi_i = iq_atan2f(dy, dx);
        const float theta_o = cto > 1.0f ? 0.0f : iq_acosf(cto);
        const float theta_i = cti > 1.0f ? 0.0f : iq_acosf(cti);
        const float alpha = iq_fmaxf(theta_i, theta_o);
        const float beta = iq_fminf(theta_i, theta_o);
        coeff = A + B * iq_cosf(phi_i - phi_o) * iq_sinf(alpha) * iq_tanf(beta);
    }
    r.ox = hx + nx * 0.0001f;                                    // hr.p + 0.0001f * hr.n
    r.oy = hy + ny * 0.0001f;
    r.oz = hz + nz * 0.0001f;
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
    // pdf is NaN, 1/pi or in [1e-5, 1/pi] and cosw = max(0, dot) >= pi * 1e-5 when the pdf was not
    // replaced (|n|^2 otherwise): inside the exact range of iq_div_pre
    q = (OPT & kOptFastDiv) ? iq_div_pre(cosw, pdf, iq_rcp(pdf)) : cosw / pdf;
}

// The reference's sphere material oren_nayar(albedo .5, sigma 1) at the closest sphere hit
// (path_tracer.cu:248, 292): continuation ray into r, returns the record's scalar att * cos / pdf.
template <int OPT>
__device__ __forceinline__ float oren_nayar_scatter(const float4 sph, float t, ray3& r, rng6& s) {
    float hx, hy, hz, nx, ny, nz;
    sphere_hit<OPT>(sph, t, r, hx, hy, hz, nx, ny, nz);
    const float sigma2 = 1.0f * 1.0f;
    const float A = 1.0f - 0.5f * sigma2 / (sigma2 + 0.33f);
    const float B = 0.45f * sigma2 / (sigma2 + 0.09f);
    float coeff, q;
    or_scatter_core<OPT>(hx, hy, hz, nx, ny, nz, r, s, A, B, coeff, q);
    const float att = (0.5f * coeff) * (1.0f / IQ_PI);           // m_albedo * coeff / pi
    return att * q;
}

// Triangle hit record (shape.cu:62-103) for triangle k hit at t: Möller–Trumbore again for u, v (the
// same operation sequence as test_triangle, so the same bits), the hit point, the interpolated
// vertex normal normalized3((1-u-v) n0 + u n1 + v n2), flipped unless dir . (e1 x e2) < 0.
template <int OPT>
__device__ __forceinline__ void triangle_hit(const float4* __restrict__ tris, const float4* __restrict__ shade,
                                             uint32_t k, float t, const ray3& r, float& hx, float& hy, float& hz,
                                             float& nx, float& ny, float& nz) {
    const float4 a = tris[(size_t)k * kTriFloat4], b = tris[(size_t)k * kTriFloat4 + 1],
                 c = tris[(size_t)k * kTriFloat4 + 2];
    const float e1x = a.w, e1y = b.x, e1z = b.y;
    const float e2x = b.z, e2y = b.w, e2z = c.x;
    const float px = r.dy * e2z - r.dz * e2y;
    const float py = r.dz * e2x - r.dx * e2z;
    const float pz = r.dx * e2y - r.dy * e2x;
    const float det = (e1x * px + e1y * py) + e1z * pz;
    const float inv = rcp_scene<OPT>(det);
    const float tx = r.ox - a.x, ty = r.oy - a.y, tz = r.oz - a.z;
    const float u = ((tx * px + ty * py) + tz * pz) * inv;
    const float qx = ty * e1z - tz * e1y;
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    const float v = ((r.dx * qx + r.dy * qy) + r.dz * qz) * inv;
    hx = r.ox + t * r.dx;
    hy = r.oy + t * r.dy;
    hz = r.oz + t * r.dz;
    const float4 s0 = shade[(size_t)k * kTriShadeFloat4], s1 = shade[(size_t)k * kTriShadeFloat4 + 1],
                 s2 = shade[(size_t)k * kTriShadeFloat4 + 2];
    const float w0 = (1.0f - u) - v;
    nx = (s0.x * w0 + s1.x * u) + s2.x * v;
    ny = (s0.y * w0 + s1.y * u) + s2.y * v;
    nz = (s0.z * w0 + s1.z * u) + s2.z * v;
    normalize3<OPT>(nx, ny, nz);
    if (!((r.dx * s0.w + r.dy * s1.w) + r.dz * s2.w < 0.0f)) {   // front_face: dir . (e1 x e2) < 0
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
}

// Adds a block's (or wave's) closest-hit queries to one of the kRaySlots spread counters.
__device__ __forceinline__ void add_rays(unsigned long long* rays, unsigned long long v) {
    atomicAdd(rays + (size_t)((blockIdx.x + threadIdx.x / 64u) % kRaySlots) * kRaySlotStride, v);
}

__device__ __forceinline__ uint32_t prefix_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// c / n of the running mean (path_tracer.cu:356-358) without the table (variants without
// kOptAccTable): the IEEE division.
// With kOptAccTable (every production variant; the runtime keeps launches within the table) the
// three channels are done together in mean_terms below.
template <int OPT>
__device__ __forceinline__ float mean_term(float c, float nf) {
    return c / nf;
}

// (cx, cy, cz) / n for the clamped colour (each channel in [0, 1] or NaN, never -0: path_color =
// 0 + color) with rc = RN(1/n) from the per-launch table. kOptFastDiv: Markstein's correction
// q + (c - n q) rc, q = c rc, is the IEEE quotient while the quotient is normal and the operands are
// within [2^-100, 2^100] (n < 2^64 is); c = 0 gives +0 (as 0 / n) and NaN stays NaN, so no fixup
// is needed in this domain. Channels 0 < c < p.mean_tiny (a quotient that could be subnormal, or c
// below 2^-99) take the IEEE division: one test for all three ((bits - 1) as unsigned maps +0 and
// NaN above the threshold's bits). Without kOptFastDiv: c = 1 gives rc, c = 0 gives +0, else the
// IEEE division.
template <int OPT>
__device__ __forceinline__ void mean_terms(float cx, float cy, float cz, float nf, float rc, float tiny,
                                           float& qx, float& qy, float& qz) {
    if (OPT & kOptFastDiv) {
        const f2 c2 = {cx, cy};
        const f2 q0 = c2 * rc;
        const f2 r = __builtin_elementwise_fma(-(f2){nf, nf}, q0, c2);
        const f2 q1 = __builtin_elementwise_fma(r, (f2){rc, rc}, q0);
        const float z0 = cz * rc;
        const float zr = __builtin_fmaf(-nf, z0, cz);
        qx = q1.x;
        qy = q1.y;
        qz = __builtin_fmaf(zr, rc, z0);
        const uint32_t lim = __float_as_uint(tiny) - 1u;
        const uint32_t m = min(min(__float_as_uint(cx) - 1u, __float_as_uint(cy) - 1u), __float_as_uint(cz) - 1u);
        if (__builtin_expect(m < lim, 0)) {
            asm volatile("" ::: "memory");   // keep the rare IEEE expansion behind a branch (no if-conversion)
            qx = cx / nf;
            qy = cy / nf;
            qz = cz / nf;
        }
        return;
    }
    qx = cx == 1.0f ? rc : (cx == 0.0f ? 0.0f : cx / nf);
    qy = cy == 1.0f ? rc : (cy == 0.0f ? 0.0f : cy / nf);
    qz = cz == 1.0f ? rc : (cz == 0.0f ? 0.0f : cz / nf);
}

// Closest hit over the primitives in [tri0, tri1) / [sph0, sph1) of the given base arrays (LDS),
// in the reference's order: triangles of every drawcall first, then spheres (path_tracer.cu:257-295).
template <int OPT>
__device__ __forceinline__ void intersect_range(const float4* tri, uint32_t tri_first, uint32_t ntri_local,
                                                const float4* sph, uint32_t sph_first, uint32_t nsph_local,
                                                const ray3 ray, float& closest, int& kind, uint32_t& hidx) {
    if (OPT & kOptPair) {
        // tri points at pair records; tri_first / sph_first are even primitive indices
        const uint32_t tp = (ntri_local + 1) / 2;
        for (uint32_t j = 0; j < tp; ++j) {
            const float4* q = tri + (size_t)j * kTriPairFloat4;
            if (OPT & kOptBranchless)
                test_triangle_pair_nb<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, tri_first + 2 * j,
                                      2 * j + 1 < ntri_local);
            else
                test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, tri_first + 2 * j,
                                   2 * j + 1 < ntri_local);
        }
        const uint32_t sp = (nsph_local + 1) / 2;
        for (uint32_t j = 0; j < sp; ++j) {
            const float4* q = sph + (size_t)j * kSphPairFloat4;
            test_sphere_pair<OPT>(q[0], q[1], ray, closest, kind, hidx, sph_first + 2 * j, 2 * j + 1 < nsph_local);
        }
    } else {
        for (uint32_t k = 0; k < ntri_local; ++k) {
            const float4* q = tri + (size_t)k * kTriFloat4;
            test_triangle<OPT>(q[0], q[1], q[2], ray, closest, kind, hidx, tri_first + k);
        }
        for (uint32_t k = 0; k < nsph_local; ++k) test_sphere<OPT>(sph[k], ray, closest, kind, hidx, sph_first + k);
    }
}

// OR of a 32-bit value over the 64 lanes of the wave (all lanes must be executing): DPP within
// each 16-lane row, then the four row results read as scalars.
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) | (uint32_t)__builtin_amdgcn_readlane((int)v, 31) |
           (uint32_t)__builtin_amdgcn_readlane((int)v, 47) | (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// kOptCull, LDS-resident scene: the closest hit over the pairs whose bit is set in the wave's OR of
// the lanes' tile masks (camera rays, iq_interval.h) — or over every pair when some lane traces a
// secondary ray. Skipped pairs are rejected by the reference's own tests for every camera ray of
// the tile, and the remaining pairs are visited in index order, so results are unchanged. Called by
// all lanes of the wave (wave_or); only active lanes test.
// Word 0 of each mask comes from the lane's registers (cm_t, cm_s: loaded with the pixel). When
// every active lane is in the same tile (uni_mask = that tile's words; the caller has made the first
// lane an active one) the OR is that tile's mask itself: word 0 read from the first lane, the others
// with uniform loads, no DPP.
template <int OPT>
__device__ __forceinline__ void intersect_culled(const float4* tri, uint32_t ntri, const float4* sph, uint32_t nsph,
                                                 const uint32_t* lane_mask, uint32_t cm_t, uint32_t cm_s, bool all,
                                                 bool active, const ray3 ray, float& closest, int& kind,
                                                 uint32_t& hidx, uint32_t wt, const uint32_t* uni_mask,
                                                 unsigned long long* st = nullptr) {
    const uint32_t tp = (ntri + 1) / 2, sp = (nsph + 1) / 2;
    for (uint32_t w = 0; w * 32u < tp; ++w) {
        uint32_t m = all ? ~0u
                         : (uni_mask ? (w == 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cm_t) : uni_mask[w])
                                     : wave_or(lane_mask ? (w == 0 ? cm_t : lane_mask[w]) : 0u));
        if ((OPT & kOptStats) && st) st[0] += (unsigned long long)__builtin_popcount(w * 32u + 32u <= tp ? m : (m & ((1u << (tp - w * 32u)) - 1u)));
        while (m) {
            const uint32_t j = w * 32u + (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            if (j >= tp) break;
            if (active) {
                const float4* q = tri + (size_t)j * kTriPairFloat4;
                test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, 2 * j, 2 * j + 1 < ntri);
            }
        }
    }
    for (uint32_t w = 0; w * 32u < sp; ++w) {
        uint32_t m = all ? ~0u
                         : (uni_mask ? (w == 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cm_s) : uni_mask[wt + w])
                                     : wave_or(lane_mask ? (w == 0 ? cm_s : lane_mask[wt + w]) : 0u));
        if ((OPT & kOptStats) && st) st[1] += (unsigned long long)__builtin_popcount(w * 32u + 32u <= sp ? m : (m & ((1u << (sp - w * 32u)) - 1u)));
        while (m) {
            const uint32_t j = w * 32u + (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            if (j >= sp) break;
            if (active) {
                const float4* q = sph + (size_t)j * kSphPairFloat4;
                test_sphere_pair<OPT>(q[0], q[1], ray, closest, kind, hidx, 2 * j, 2 * j + 1 < nsph);
            }
        }
    }
}

// ---- two rays per lane (kOptPipe): ray a is the lane's current path, ray b the camera
// ray of its pixel's next sample. Each ray sees exactly the operation sequence of test_triangle_pair /
// test_sphere_pair and the pairs in index order, so each keeps its own bits; the two tests share the
// pair's LDS reads and their stages are interleaved, so the two dependent chains overlap.
template <int OPT>
__device__ __forceinline__ void test_triangle_pair2(const float4 q0, const float4 q1, const float4 q2, const float4 q3,
                                                    const float4 q4, const ray3 ra, const ray3 rb, bool ta, bool tb,
                                                    float& ca, int& ka, uint32_t& ia, float& cb, int& kb, uint32_t& ib,
                                                    uint32_t k, bool second) {
    if (ta) stat_add<OPT>(0, 2u);
    if (tb) stat_add<OPT>(0, 2u);
    const f2 v0x = {q0.x, q0.y}, v0y = {q0.z, q0.w}, v0z = {q1.x, q1.y};
    const f2 e1x = {q1.z, q1.w}, e1y = {q2.x, q2.y}, e1z = {q2.z, q2.w};
    const f2 e2x = {q3.x, q3.y}, e2y = {q3.z, q3.w}, e2z = {q4.x, q4.y};
    const f2 pxa = ra.dy * e2z - ra.dz * e2y, pxb = rb.dy * e2z - rb.dz * e2y;
    const f2 pya = ra.dz * e2x - ra.dx * e2z, pyb = rb.dz * e2x - rb.dx * e2z;
    const f2 pza = ra.dx * e2y - ra.dy * e2x, pzb = rb.dx * e2y - rb.dy * e2x;
    const f2 deta = (e1x * pxa + e1y * pya) + e1z * pza, detb = (e1x * pxb + e1y * pyb) + e1z * pzb;
    // T = O - v0 ahead of the determinant test, held there (the empty asm): the pair's v0 and edge records are
    // read from LDS together, one wait instead of a second one after the test (the test rarely rejects a wall)
    f2 txa = ra.ox - v0x, tya = ra.oy - v0y, tza = ra.oz - v0z;
    f2 txb = rb.ox - v0x, tyb = rb.oy - v0y, tzb = rb.oz - v0z;
#ifndef IQPT_PAIR2_PIN
#define IQPT_PAIR2_PIN 1
#endif
    if (IQPT_PAIR2_PIN) asm volatile("" : "+v"(txa), "+v"(tya), "+v"(tza), "+v"(txb), "+v"(tyb), "+v"(tzb));
    bool a0 = ta && !(iq_fabsf(deta.x) < 0.000001f), a1 = ta && second && !(iq_fabsf(deta.y) < 0.000001f);
    bool b0 = tb && !(iq_fabsf(detb.x) < 0.000001f), b1 = tb && second && !(iq_fabsf(detb.y) < 0.000001f);
    if (!(a0 || a1 || b0 || b1)) return;
    const f2 inva = {rcp_scene<OPT>(deta.x), rcp_scene<OPT>(deta.y)};
    const f2 invb = {rcp_scene<OPT>(detb.x), rcp_scene<OPT>(detb.y)};
    const f2 ua = ((txa * pxa + tya * pya) + tza * pza) * inva, ub = ((txb * pxb + tyb * pyb) + tzb * pzb) * invb;
    a0 = a0 && !(ua.x < 0.0f || ua.x > 1.0f);
    a1 = a1 && !(ua.y < 0.0f || ua.y > 1.0f);
    b0 = b0 && !(ub.x < 0.0f || ub.x > 1.0f);
    b1 = b1 && !(ub.y < 0.0f || ub.y > 1.0f);
    if (!(a0 || a1 || b0 || b1)) return;
    const f2 qxa = tya * e1z - tza * e1y, qxb = tyb * e1z - tzb * e1y;
    const f2 qya = tza * e1x - txa * e1z, qyb = tzb * e1x - txb * e1z;
    const f2 qza = txa * e1y - tya * e1x, qzb = txb * e1y - tyb * e1x;
    const f2 va = ((ra.dx * qxa + ra.dy * qya) + ra.dz * qza) * inva;
    const f2 vb = ((rb.dx * qxb + rb.dy * qyb) + rb.dz * qzb) * invb;
    const f2 uva = ua + va, uvb = ub + vb;
    a0 = a0 && !(va.x < 0.0f || uva.x > 1.0f);
    a1 = a1 && !(va.y < 0.0f || uva.y > 1.0f);
    b0 = b0 && !(vb.x < 0.0f || uvb.x > 1.0f);
    b1 = b1 && !(vb.y < 0.0f || uvb.y > 1.0f);
    if (!(a0 || a1 || b0 || b1)) return;
    const f2 t_a = ((e2x * qxa + e2y * qya) + e2z * qza) * inva;
    const f2 t_b = ((e2x * qxb + e2y * qyb) + e2z * qzb) * invb;
    if (a0 && !(t_a.x < kTMin || ca < t_a.x)) { ca = t_a.x; ka = kHitTri; ia = k; }
    if (a1 && !(t_a.y < kTMin || ca < t_a.y)) { ca = t_a.y; ka = kHitTri; ia = k + 1; }
    if (b0 && !(t_b.x < kTMin || cb < t_b.x)) { cb = t_b.x; kb = kHitTri; ib = k; }
    if (b1 && !(t_b.y < kTMin || cb < t_b.y)) { cb = t_b.y; kb = kHitTri; ib = k + 1; }
}

template <int OPT>
__device__ __forceinline__ void test_sphere_pair2(const float4 s0, const float4 s1, const ray3 ra, const ray3 rb, bool ta,
                                                  bool tb, float& ca, int& ka, uint32_t& ia, float& cb, int& kb,
                                                  uint32_t& ib, uint32_t k, bool second) {
    if (ta) stat_add<OPT>(1, 2u);
    if (tb) stat_add<OPT>(1, 2u);
    const f2 cx = {s0.x, s0.y}, cy = {s0.z, s0.w}, cz = {s1.x, s1.y}, rad = {s1.z, s1.w};
    const f2 ocxa = cx - ra.ox, ocya = cy - ra.oy, ocza = cz - ra.oz;
    const f2 ocxb = cx - rb.ox, ocyb = cy - rb.oy, oczb = cz - rb.oz;
    const f2 hba = (ra.dx * ocxa + ra.dy * ocya) + ra.dz * ocza, hbb = (rb.dx * ocxb + rb.dy * ocyb) + rb.dz * oczb;
    const f2 r2 = rad * rad;
    const f2 cca = ((ocxa * ocxa + ocya * ocya) + ocza * ocza) - r2, ccb = ((ocxb * ocxb + ocyb * ocyb) + oczb * oczb) - r2;
    const f2 da = hba * hba - cca, db = hbb * hbb - ccb;
    if (ta && !(da.x < 0.0f)) sphere_roots<OPT>(hba.x, da.x, ca, ka, ia, k);
    if (ta && second && !(da.y < 0.0f)) sphere_roots<OPT>(hba.y, da.y, ca, ka, ia, k + 1);
    if (tb && !(db.x < 0.0f)) sphere_roots<OPT>(hbb.x, db.x, cb, kb, ib, k);
    if (tb && second && !(db.y < 0.0f)) sphere_roots<OPT>(hbb.y, db.y, cb, kb, ib, k + 1);
}

// The closest hits of rays a and b over the LDS-resident pairs (kOptCull): ray b is always a camera ray and
// tests the pairs of the wave's OR of its lanes' tile masks (or the uniform tile's own mask, as
// intersect_culled); ray a tests the same pairs when every active lane's ray a is a camera ray, else every
// pair (all_a). The loop runs over the union in index order, so each ray meets its pairs in the
// reference's order. Called by all lanes of the wave.
template <int OPT>
__device__ __forceinline__ void intersect_culled2(const float4* tri, uint32_t ntri, const float4* sph, uint32_t nsph,
                                                  const uint32_t* lane_mask, uint32_t cm_t, uint32_t cm_s, bool all_a,
                                                  bool act_a, bool act_b, const ray3 ra, const ray3 rb, float& ca,
                                                  int& ka, uint32_t& ia, float& cb, int& kb, uint32_t& ib, uint32_t wt,
                                                  const uint32_t* uni_mask, unsigned long long* st = nullptr) {
    const uint32_t tp = (ntri + 1) / 2, sp = (nsph + 1) / 2;
    for (uint32_t w = 0; w * 32u < tp; ++w) {
        const uint32_t mb = uni_mask ? (w == 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cm_t) : uni_mask[w])
                                     : wave_or(lane_mask ? (w == 0 ? cm_t : lane_mask[w]) : 0u);
        uint32_t m = all_a ? ~0u : mb;
        if ((OPT & kOptStats) && st) st[0] += (unsigned long long)__builtin_popcount(w * 32u + 32u <= tp ? m : (m & ((1u << (tp - w * 32u)) - 1u)));
        while (m) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            const uint32_t j = w * 32u + bit;
            m &= m - 1u;
            if (j >= tp) break;
            const bool in_b = (mb >> bit) & 1u;
            const float4* q = tri + (size_t)j * kTriPairFloat4;
            test_triangle_pair2<OPT>(q[0], q[1], q[2], q[3], q[4], ra, rb, act_a, act_b && in_b, ca, ka, ia, cb, kb, ib,
                                     2 * j, 2 * j + 1 < ntri);
        }
    }
    for (uint32_t w = 0; w * 32u < sp; ++w) {
        const uint32_t mb = uni_mask ? (w == 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cm_s) : uni_mask[wt + w])
                                     : wave_or(lane_mask ? (w == 0 ? cm_s : lane_mask[wt + w]) : 0u);
        uint32_t m = all_a ? ~0u : mb;
        if ((OPT & kOptStats) && st) st[1] += (unsigned long long)__builtin_popcount(w * 32u + 32u <= sp ? m : (m & ((1u << (sp - w * 32u)) - 1u)));
        while (m) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            const uint32_t j = w * 32u + bit;
            m &= m - 1u;
            if (j >= sp) break;
            const bool in_b = (mb >> bit) & 1u;
            const float4* q = sph + (size_t)j * kSphPairFloat4;
            test_sphere_pair2<OPT>(q[0], q[1], ra, rb, act_a, act_b && in_b, ca, ka, ia, cb, kb, ib, 2 * j,
                                   2 * j + 1 < nsph);
        }
    }
}

// Order-free closest-triangle update: the brute-force loop keeps the hit with the smallest t and,
// among equal t, the one with the largest packet index (t == closest is accepted, path_tracer.cu:
// 257-275); a BVH visits triangles in another order, so the tie is decided by index explicitly.
__device__ __forceinline__ void take_triangle(float t, uint32_t k, float& closest, int& kind, uint32_t& idx) {
    if (t < closest || (t == closest && (kind == kHitNone || k > idx))) {
        closest = t;
        kind = kHitTri;
        idx = k;
    }
}

// Möller–Trumbore for a leaf pair with explicit packet indices ka, kb (kb = ~0u: padding); the same
// per-element operation sequence as test_triangle_pair, so accepted hits carry the same bits.
template <int OPT>
__device__ __forceinline__ void test_triangle_pair_ix(const float4 q0, const float4 q1, const float4 q2,
                                                      const float4 q3, const float4 q4, const ray3 r, float& closest,
                                                      int& kind, uint32_t& idx, uint32_t ka, uint32_t kb) {
    stat_add<OPT>(0, 2u);
    const f2 v0x = {q0.x, q0.y}, v0y = {q0.z, q0.w}, v0z = {q1.x, q1.y};
    const f2 e1x = {q1.z, q1.w}, e1y = {q2.x, q2.y}, e1z = {q2.z, q2.w};
    const f2 e2x = {q3.x, q3.y}, e2y = {q3.z, q3.w}, e2z = {q4.x, q4.y};
    const f2 px = r.dy * e2z - r.dz * e2y;
    const f2 py = r.dz * e2x - r.dx * e2z;
    const f2 pz = r.dx * e2y - r.dy * e2x;
    const f2 det = (e1x * px + e1y * py) + e1z * pz;
    bool a0 = !(iq_fabsf(det.x) < 0.000001f);
    bool a1 = kb != ~0u && !(iq_fabsf(det.y) < 0.000001f);
    if (!(a0 || a1)) return;
    const f2 inv = {rcp_scene<OPT>(det.x), rcp_scene<OPT>(det.y)};
    const f2 tx = r.ox - v0x, ty = r.oy - v0y, tz = r.oz - v0z;
    const f2 u = ((tx * px + ty * py) + tz * pz) * inv;
    a0 = a0 && !(u.x < 0.0f || u.x > 1.0f);
    a1 = a1 && !(u.y < 0.0f || u.y > 1.0f);
    if (!(a0 || a1)) return;
    const f2 qx = ty * e1z - tz * e1y;
    const f2 qy = tz * e1x - tx * e1z;
    const f2 qz = tx * e1y - ty * e1x;
    const f2 v = ((r.dx * qx + r.dy * qy) + r.dz * qz) * inv;
    const f2 uv = u + v;
    a0 = a0 && !(v.x < 0.0f || uv.x > 1.0f);
    a1 = a1 && !(v.y < 0.0f || uv.y > 1.0f);
    if (!(a0 || a1)) return;
    const f2 t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    if (a0 && !(t.x < kTMin)) take_triangle(t.x, ka, closest, kind, idx);
    if (a1 && !(t.y < kTMin)) take_triangle(t.y, kb, closest, kind, idx);
}

// True if ray r may use the BVH: the error bound of iq_bvh.hpp assumed its origin inside the grown
// scene box and |d_i| <= md (NaN fails every comparison and falls back to the full loop).
__device__ __forceinline__ bool bvh_ray_ok(const kparams& p, const ray3& r) {
    // finite origin (NaN fails every comparison), normalized direction
    return iq_fabsf(r.ox) <= 1e18f && iq_fabsf(r.oy) <= 1e18f && iq_fabsf(r.oz) <= 1e18f &&
           iq_fabsf(r.dx) <= p.bvh_md && iq_fabsf(r.dy) <= p.bvh_md && iq_fabsf(r.dz) <= p.bvh_md;
}

// Per-ray constants of the BVH node test.
struct bvh_ray {
    float ix, iy, iz;    // 1 / d (IEEE)
    float dd, dl;        // |d|^2 and |d|, rounded up (normal cones)
    bool inf_dir;        // some 1 / d_i is infinite: a slab parameter can be 0 * inf (NaN)
};

__device__ __forceinline__ bvh_ray bvh_ray_setup(const ray3 r) {
    const float up16 = 1.0f + 0x1p-16f;
    bvh_ray b;
    b.ix = 1.0f / r.dx;
    b.iy = 1.0f / r.dy;
    b.iz = 1.0f / r.dz;
    b.dd = ((r.dx * r.dx + r.dy * r.dy) + r.dz * r.dz) * up16;
    b.dl = __builtin_sqrtf(b.dd) * up16;
    b.inf_dir = !(iq_fabsf(b.ix) < INFINITY && iq_fabsf(b.iy) < INFINITY && iq_fabsf(b.iz) < INFINITY);
    return b;
}

// Bounds of sqrt(x), x >= 0, for the node tests only (conservative box growths, not the reference's
// rounding): v_sqrt_f32 is within 1 ulp for x >= 2^-96 (iq_fastdiv.h); below that the upper bound's
// absolute 2^-47 covers sqrt(x) < 2^-48 and the lower bound is 0. One instruction instead of the
// correctly rounded expansion (about 17).
__device__ __forceinline__ float sqrt_up(float x) {
    return __builtin_amdgcn_sqrtf(x) * (1.0f + 0x1p-20f) + 0x1p-47f;
}
__device__ __forceinline__ float sqrt_dn(float x) {
    return x >= 0x1p-96f ? __builtin_amdgcn_sqrtf(x) * (1.0f - 0x1p-20f) : 0.0f;
}

// Box test of node i (iq_bvh.hpp): the segment t in [t_min - dt, closest + dt] against the node's box
// grown by lambda (gR + gB S) + gC, where S bounds the origin's distance to the node's vertices,
// lambda = 1e-6 / D comes from the node's normal cone and dt = lambda tA S + tB closest (each rounded
// up by 1 + 2^-20, the box side by gulp more); the slab test is widened by 8 ulp, more than its own
// rounding. Returns the widened entry parameter and the closest-independent part of dt.
__device__ __forceinline__ bool bvh_node_test(const kparams& p, const float4* __restrict__ nodes, uint32_t i,
                                              const ray3 r, const bvh_ray br, float closest, float& enter_out,
                                              float& dtc_out) {
    const float slack = 8.0f * 0x1p-24f, up = 1.0f + 0x1p-20f, up16 = 1.0f + 0x1p-16f;
    const float4* nd = nodes + (size_t)kBvhNodeFloat4 * i;
    const float4 lo = nd[0], hi = nd[1], ax = nd[2], co = nd[3];
    // x and y in packed pairs (v_pk_add / v_pk_mul: the same IEEE operations, two per instruction)
    const f2 oxy = {r.ox, r.oy}, loxy = {lo.x, lo.y}, hixy = {hi.x, hi.y};
    const f2 dlo = oxy - loxy, dhi = oxy - hixy;
    const float sx = fmaxf(iq_fabsf(dlo.x), iq_fabsf(dhi.x));
    const float sy = fmaxf(iq_fabsf(dlo.y), iq_fabsf(dhi.y));
    const float sz = fmaxf(iq_fabsf(r.oz - lo.z), iq_fabsf(r.oz - hi.z));
    const float S = fmaxf(fmaxf(sx, sy), sz) * up;
    // lambda = 1e-6 / D, D a lower bound of |det^| over the node's triangles for this ray
    // (iq_bvh.hpp normal cones): Nmin |d| cos(theta + beta) = |d| cos(theta) A - |d| sin(theta) B with
    // A = Nmin cos(beta), B = Nmin sin(beta), every step rounded toward a smaller D; an unusable cone
    // (A = 0) or a grazing ray leaves lambda = 1
    float lambda = 1.0f;
    if (co.z > 0.0f) {
        const float c = iq_fabsf((r.dx * ax.x + r.dy * ax.y) + r.dz * ax.z);
        const float c_lo = fmaxf(0.0f, c * (1.0f - 0x1p-16f) - 0x1p-20f * br.dl);
        // |d| sin(theta) <= sqrt(dd - c_lo^2); the subtraction's rounding (<= 2u dd) is covered by
        // adding 2^-20 dd before the root
        const float s_hi = sqrt_up(fmaxf(0.0f, br.dd - c_lo * c_lo) + 0x1p-20f * br.dd) * up16;
        const float nc = ((c_lo * co.z) * (1.0f - 0x1p-16f) - (s_hi * co.w) * up16) * (1.0f - 0x1p-16f);
        const float D = nc - ax.w * up16;
        if (D > 1e-6f) lambda = fminf(1.0f, (1e-6f * __builtin_amdgcn_rcpf(D)) * up16);
    }
    const float g = (lambda * (co.x + co.y * S)) * up + p.bvh_gulp;   // gulp includes gC
    // per axis [t0, t1] of the slab; a NaN (0 * inf: origin on a slab plane of an axis-parallel
    // ray) widens that axis to everything
    const f2 gg = {g, g}, ixy = {br.ix, br.iy};
    const f2 t0xy = ((loxy - gg) - oxy) * ixy, t1xy = ((hixy + gg) - oxy) * ixy;
    float t0x = t0xy.x, t1x = t1xy.x;
    float t0y = t0xy.y, t1y = t1xy.y;
    float t0z = ((lo.z - g) - r.oz) * br.iz, t1z = ((hi.z + g) - r.oz) * br.iz;
    float ax0 = fminf(t0x, t1x), ax1 = fmaxf(t0x, t1x);
    float ay0 = fminf(t0y, t1y), ay1 = fmaxf(t0y, t1y);
    float az0 = fminf(t0z, t1z), az1 = fmaxf(t0z, t1z);
    if (__builtin_expect(br.inf_dir || g != g, 0)) {
        // only an infinite 1 / d_i (or a NaN g) makes a NaN (the other factors are finite); rare, so kept off the
        // common path (the empty asm stops the compiler from if-converting it)
        asm volatile("");
        if (t0x != t0x || t1x != t1x) { ax0 = -INFINITY; ax1 = INFINITY; }
        if (t0y != t0y || t1y != t1y) { ay0 = -INFINITY; ay1 = INFINITY; }
        if (t0z != t0z || t1z != t1z) { az0 = -INFINITY; az1 = INFINITY; }
    }
    // computed slab bounds are within 3 ulp (relative) of the exact ones: widen by 8 ulp
    const uint32_t tab = __float_as_uint(hi.w);                        // tA | tB, bf16 rounded up
    const float tA = __uint_as_float(tab & 0xffff0000u), tB = __uint_as_float(tab << 16);
    const float dtc = ((lambda * tA) * S) * up;
    const float dt = (dtc + tB * closest) * up;
    float enter = fmaxf(fmaxf(ax0, ay0), az0), exit = fminf(fminf(ax1, ay1), az1);
    enter = enter - iq_fabsf(enter) * slack;
    exit = exit + iq_fabsf(exit) * slack;
    enter_out = enter;
    dtc_out = dtc;
    return enter <= exit && enter <= closest + dt && exit >= kTMin - dt;
}

template <int OPT>
__device__ __forceinline__ void bvh_leaf(const kparams& p, uint32_t fc, const ray3 r, float& closest, int& kind,
                                         uint32_t& idx) {
    const float4* __restrict__ pairs = reinterpret_cast<const float4*>(p.bvh_pairs);
    const uint32_t first = fc >> 8, cnt = fc & 0xffu;
    for (uint32_t k = 0; k < cnt; ++k) {
        const float4* q = pairs + (size_t)(first + k) * kTriPairFloat4;
        const float4 q4 = q[4];                                   // (e2z_a, e2z_b, index a, index b)
        test_triangle_pair_ix<OPT>(q[0], q[1], q[2], q[3], q4, r, closest, kind, idx, __float_as_uint(q4.z),
                                   __float_as_uint(q4.w));
    }
}

// Closest triangle for one ray through the exact BVH (iq_bvh.hpp): a stackless DFS in the tree's
// fixed order (skip pointers), leaves tested with the reference's own Möller–Trumbore and the
// triangles left out of the BVH afterwards; the result is the brute-force loop's (min t, max index)
// whatever the visiting order. (A near-child-first traversal with a per-lane LDS stack was measured
// slower on C4/C5 — profiles/ab/r01_ab38_c*_order.json — and is not kept.)
template <int OPT>
__device__ __forceinline__ void bvh_closest(const kparams& p, const ray3 r, float& closest, int& kind, uint32_t& idx,
                                            uint32_t* cnt = nullptr) {
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(p.bvh_nodes);
    const bvh_ray br = bvh_ray_setup(r);
    uint32_t i = 0;
    while (i < p.bvh_nnodes) {
        float enter, dtc;
        const bool hit = bvh_node_test(p, nodes, i, r, br, closest, enter, dtc);
        // link: skip pointer (inner node) or 1 << 31 | first pair << 8 | count (leaf, followed by i + 1)
        const uint32_t link = __float_as_uint(nodes[(size_t)kBvhNodeFloat4 * i].w);
        const bool leaf = (link >> 31) != 0u;
        if ((OPT & kOptStats) && cnt) {
            cnt[0] += 1u;
            if (hit && leaf) cnt[1] += link & 0xffu;
        }
        if (hit && leaf) {
            bvh_leaf<OPT>(p, link & 0x7fffffffu, r, closest, kind, idx);
            // any-hit scenes (kparams::anyhit): an accepted triangle decides the ray, whichever it is
            if ((OPT & kOptAnyHit) && p.anyhit && kind == kHitTri) return;
        }
        i = (hit || leaf) ? i + 1 : link;
    }
    const float4* __restrict__ tris = reinterpret_cast<const float4*>(p.tris);
    for (uint32_t a = 0; a < p.bvh_nalways && !((OPT & kOptAnyHit) && p.anyhit && kind == kHitTri); ++a) {
        const uint32_t k = p.bvh_always[a];
        float c2 = closest;
        int kd = kHitNone;
        uint32_t id = 0;
        test_triangle<OPT>(tris[3 * (size_t)k], tris[3 * (size_t)k + 1], tris[3 * (size_t)k + 2], r, c2, kd, id, k);
        if (kd == kHitTri) take_triangle(c2, k, closest, kind, idx);
    }
}

// ---- exact sphere BVH (iq_bvh.hpp: the fold's inert / normal / inside spheres and the bound) ----
// Order-free state of the sphere fold over the spheres seen so far: the best normal sphere (smallest
// t_near, largest index on ties) among indices >= min_idx, and the last (largest-index) inside sphere.
struct sph_fold {
    float bt;         // best normal t_near (kTMax sentinel with bi = ~0u: none)
    uint32_t bi;
    float tin;        // t_far of the inside sphere iin
    uint32_t iin;     // ~0u: none
};

// One sphere k with the reference's test (shape.cu:13-46, the operation sequence of test_sphere).
template <int OPT>
__device__ __forceinline__ void sph_visit(const float4 s, uint32_t k, const ray3 r, uint32_t min_idx, sph_fold& f,
                                          float& bound) {
    stat_add<OPT>(1, 1u);
    const float ocx = s.x - r.ox, ocy = s.y - r.oy, ocz = s.z - r.oz;
    const float halfb = (r.dx * ocx + r.dy * ocy) + r.dz * ocz;
    const float cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.w * s.w;
    const float delta = halfb * halfb - cc;
    if (delta < 0.0f) return;                                   // inert
    const float sd = sqrt_any<OPT>(delta);
    const float tn = halfb - sd;
    if (tn < kTMin) {
        const float tf = halfb + sd;
        if (tf < kTMin) return;                                 // inert
        if (f.iin == ~0u || k > f.iin) {                        // inside: the last one decides
            f.iin = k;
            f.tin = tf;
        }
        return;
    }
    if (k < min_idx) return;
    if (tn < f.bt || (tn == f.bt && (f.bi == ~0u || k > f.bi))) {
        f.bt = tn;
        f.bi = k;
        bound = fminf(bound, tn);
    }
}

// Stackless traversal of the sphere BVH (skip pointers) plus the always-tested spheres, folding
// into f; nodes whose grown box the ray cannot meet before `bound` (+ slack) are skipped.
template <int OPT>
__device__ __forceinline__ void sbvh_pass(const kparams& p, const ray3 r, const bvh_ray br, float eps,
                                          uint32_t min_idx, float bound, sph_fold& f, uint32_t* cnt = nullptr) {
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(p.sbvh_nodes);
    const float4* __restrict__ leaf = reinterpret_cast<const float4*>(p.sbvh_sph);
    const float u = 0x1p-24f, up = 1.0f + 0x1p-16f, slack = 8.0f * 0x1p-24f;
    // the always-tested spheres first (the large ones: their hits tighten the bound for the traversal;
    // the fold is order-free)
    const float4* __restrict__ sph = reinterpret_cast<const float4*>(p.spheres);
    for (uint32_t a = 0; a < p.sbvh_nalways; ++a) {
        const uint32_t k = p.sbvh_always[a];
        sph_visit<OPT>(sph[k], k, r, min_idx, f, bound);
    }
    uint32_t i = 0;
    while (i < p.sbvh_nnodes) {
        const float4* nd = nodes + (size_t)kSphNodeFloat4 * i;
        const float4 lo = nd[0], hi = nd[1], rr = nd[2];
        const uint32_t skip = __float_as_uint(lo.w), fc = __float_as_uint(hi.w);
        // S >= |c - o| for every centre of the node (box corners), rounded up
        const f2 oxy = {r.ox, r.oy}, loxy = {lo.x, lo.y}, hixy = {hi.x, hi.y};   // packed x, y (bvh_node_test)
        const f2 dlo = oxy - loxy, dhi = oxy - hixy;
        const float sx = fmaxf(iq_fabsf(dlo.x), iq_fabsf(dhi.x));
        const float sy = fmaxf(iq_fabsf(dlo.y), iq_fabsf(dhi.y));
        const float sz = fmaxf(iq_fabsf(r.oz - lo.z), iq_fabsf(r.oz - hi.z));
        const float S2 = ((sx * sx + sy * sy) + sz * sz) * up;
        const float S = sqrt_up(S2) * up;
        // growth(S) of iq_bvh.hpp with the ray's |d|^2 deviation eps folded in (rounded up; the root in
        // the denominator rounded down)
        const float K = ((24.0f * u) * (rr.y * rr.y) + (86.0f * u + 2.01f * eps) * S2) * (1.0f + 0x1p-8f) +
                        (2.01f * eps) * (rr.y * rr.y);
        const float g = (K * __builtin_amdgcn_rcpf(sqrt_dn(rr.x * rr.x + K) + rr.x) * (1.0f + 0x1p-12f) +
                         (4.0f * u) * S + (8.0f * u) * rr.y) * up + p.sbvh_gulp;
        const float dts = ((20.0f * u + 4.0f * eps) * S) * up + 1e-30f;
        const f2 gg = {g, g}, ixy = {br.ix, br.iy};
        const f2 t0xy = ((loxy - gg) - oxy) * ixy, t1xy = ((hixy + gg) - oxy) * ixy;
        float t0x = t0xy.x, t1x = t1xy.x;
        float t0y = t0xy.y, t1y = t1xy.y;
        float t0z = ((lo.z - g) - r.oz) * br.iz, t1z = ((hi.z + g) - r.oz) * br.iz;
        float ax0 = fminf(t0x, t1x), ax1 = fmaxf(t0x, t1x);
        float ay0 = fminf(t0y, t1y), ay1 = fmaxf(t0y, t1y);
        float az0 = fminf(t0z, t1z), az1 = fmaxf(t0z, t1z);
        if (__builtin_expect(br.inf_dir || g != g, 0)) {
            // a NaN needs an infinite 1 / d_i or g = 0 * inf (K = 0 over a zero denominator): rare
            asm volatile("");
            if (t0x != t0x || t1x != t1x) { ax0 = -INFINITY; ax1 = INFINITY; }
            if (t0y != t0y || t1y != t1y) { ay0 = -INFINITY; ay1 = INFINITY; }
            if (t0z != t0z || t1z != t1z) { az0 = -INFINITY; az1 = INFINITY; }
        }
        float enter = fmaxf(fmaxf(ax0, ay0), az0), exit = fminf(fminf(ax1, ay1), az1);
        enter = enter - iq_fabsf(enter) * slack;
        exit = exit + iq_fabsf(exit) * slack;
        const bool hit = enter <= exit && exit >= kTMin - dts && enter <= bound + dts;
        if ((OPT & kOptStats) && cnt) cnt[0] += 1u;
        if (hit && fc != 0u) {
            const uint32_t first = fc >> 8, nl = fc & 0xffu;
            if ((OPT & kOptStats) && cnt) cnt[1] += nl;
            for (uint32_t k = 0; k < nl; ++k)
                sph_visit<OPT>(leaf[first + k], p.sbvh_idx[first + k], r, min_idx, f, bound);
        }
        i = (hit && fc == 0u) ? i + 1 : skip;
    }
}

// The spheres' part of the closest hit (after the triangles) through the sphere BVH: the reference's
// in-order fold (path_tracer.cu:283-295) from its order-free form (iq_bvh.hpp). A ray whose |d|^2 is
// not within 2^-10 of 1 folds over every sphere in packet order instead.
template <int OPT>
__device__ __forceinline__ void sbvh_closest(const kparams& p, const ray3 r, float& closest, int& kind,
                                             uint32_t& idx, uint32_t* cnt = nullptr) {
    const bvh_ray br = bvh_ray_setup(r);
    const float dd = (r.dx * r.dx + r.dy * r.dy) + r.dz * r.dz;
    const float eps = iq_fabsf(dd - 1.0f) + 8.0f * 0x1p-24f;
    if (!(eps <= 0x1p-10f)) {
        const float4* __restrict__ sph = reinterpret_cast<const float4*>(p.spheres);
        for (uint32_t k = 0; k < p.nsph; ++k) test_sphere<OPT>(sph[k], r, closest, kind, idx, k);
        return;
    }
    sph_fold f = {kTMax, ~0u, 0.0f, ~0u};
    sbvh_pass<OPT>(p, r, br, eps, 0u, closest, f, cnt);
    if (f.iin == ~0u) {
        // no inside sphere: min(closest, best normal), the sphere on ties
        if (f.bi != ~0u && !(closest < f.bt)) {
            closest = f.bt;
            kind = kHitSphere;
            idx = f.bi;
        }
        return;
    }
    // the last inside sphere sets closest = its far root; normal spheres after it lower it
    closest = f.tin;
    kind = kHitSphere;
    idx = f.iin;
    sph_fold g = {kTMax, ~0u, 0.0f, ~0u};
    sbvh_pass<OPT>(p, r, br, eps, f.iin + 1u, closest, g);
    if (g.bi != ~0u && !(closest < g.bt)) {
        closest = g.bt;
        idx = g.bi;
    }
}

// Closest hit with the spheres first (the BVH-primary variants): the sphere fold's
// order-free state over every sphere (iq_bvh.hpp), then — unless the origin is inside a sphere, whose
// far root overrides any triangle (shape.cu:27-33 skips the t_max test) — the triangles with the best
// sphere's t as their starting bound, so the triangle BVH prunes everything behind it. Same result as
// triangles-then-spheres (path_tracer.cu:253-295): a triangle wins only with t below the sphere's (the
// sphere takes equal t). Requires a sphere BVH, a finite origin and a ray within the sphere bound's
// |d|^2 limit (sbvh_first_ok).
__device__ __forceinline__ bool sbvh_first_ok(const kparams& p, const ray3 r) {
    const float dd = (r.dx * r.dx + r.dy * r.dy) + r.dz * r.dz;
    return p.sbvh_nodes != nullptr && iq_fabsf(r.ox) <= 1e18f && iq_fabsf(r.oy) <= 1e18f &&
           iq_fabsf(r.oz) <= 1e18f && iq_fabsf(dd - 1.0f) + 8.0f * 0x1p-24f <= 0x1p-10f;
}

template <int OPT>
__device__ __forceinline__ void closest_spheres_first(const kparams& p, const ray3 r, bool tri_bvh, float& closest,
                                                      int& kind, uint32_t& idx, uint32_t* ctri = nullptr,
                                                      uint32_t* csph = nullptr) {
    const bvh_ray br = bvh_ray_setup(r);
    const float dd = (r.dx * r.dx + r.dy * r.dy) + r.dz * r.dz;
    const float eps = iq_fabsf(dd - 1.0f) + 8.0f * 0x1p-24f;
    sph_fold f = {kTMax, ~0u, 0.0f, ~0u};
    sbvh_pass<OPT>(p, r, br, eps, 0u, kTMax, f, csph);
    if (f.iin != ~0u) {
        // the last inside sphere sets closest = its far root; normal spheres after it lower it
        closest = f.tin;
        kind = kHitSphere;
        idx = f.iin;
        sph_fold g = {kTMax, ~0u, 0.0f, ~0u};
        sbvh_pass<OPT>(p, r, br, eps, f.iin + 1u, closest, g);
        if (g.bi != ~0u && !(closest < g.bt)) {
            closest = g.bt;
            idx = g.bi;
        }
        return;
    }
    const bool sph = f.bi != ~0u;
    float c = sph ? f.bt : kTMax;
    int kd = kHitNone;
    uint32_t id = 0;
    if (tri_bvh) {
        bvh_closest<OPT>(p, r, c, kd, id, ctri);
    } else {
        const float4* __restrict__ gp = reinterpret_cast<const float4*>(p.tri_pairs);
        for (uint32_t j = 0; j < p.ntri_pairs; ++j) {
            const float4* q = gp + (size_t)j * kTriPairFloat4;
            test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], r, c, kd, id, 2 * j, 2 * j + 1 < p.ntri);
        }
    }
    if (kd == kHitTri && !(sph && c == f.bt)) {
        closest = c;
        kind = kHitTri;
        idx = id;
    } else if (sph) {
        closest = f.bt;
        kind = kHitSphere;
        idx = f.bi;
    }
}

// The running-mean table occupies spp float2 of dynamic LDS when the launch builds it.
__device__ __forceinline__ bool use_tab_lds(const kparams& p) { return p.acc_tab != 0u; }

// ------------------------------------------------------------------------------------------------
// The megakernel. MAXD bounds max_depth (variant selection; the scatter stack lives in LDS); STREAM selects LDS batch streaming
// (scene larger than the resident budget) with workgroup-uniform iteration; OPT is the kOpt* mask.
template <int OPT, bool STREAM>
constexpr int min_waves_per_simd() {
    // streamed variants (BVH traversal) are held to 4 waves/SIMD (<= 128 VGPRs)
    // kOptSplit variants are built for 4 waves/SIMD (<= 128 VGPRs): with 5 their refill and path-end
    // bookkeeping spilled 9 VGPRs to scratch, and at the low occupancy of a multi-GPU row share a scratch
    // reload's latency is not hidden
    return ((OPT & kOptSplit) || (OPT & kOptPipe)) ? 4
                             : ((OPT & kOptLB6) ? 6 : ((OPT & kOptLB5) ? 5 : (STREAM ? 4 : 1)));
}

template <int MAXD, bool STREAM, int OPT>
__global__ __launch_bounds__(kRenderBlock, (min_waves_per_simd<OPT, STREAM>())) void iqpt_render_kernel(const kparams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    constexpr bool kPair = (OPT & kOptPair) != 0;
    constexpr int kTriRec = kPair ? kTriPairFloat4 : kTriFloat4;   // float4 per LDS record
    constexpr int kSphRec = kPair ? kSphPairFloat4 : 1;
    constexpr uint32_t kTriPer = kPair ? 2u : 1u;                   // primitives per record
    constexpr uint32_t kSphPer = kPair ? 2u : 1u;
    const float4* __restrict__ g_tri = reinterpret_cast<const float4*>(kPair ? p.tri_pairs : p.tris);
    const float4* __restrict__ g_sph = reinterpret_cast<const float4*>(kPair ? p.sph_pairs : p.spheres);
    const float4* __restrict__ g_sph_plain = reinterpret_cast<const float4*>(p.spheres);
    const uint32_t tri_recs = kPair ? p.ntri_pairs : p.ntri;
    const uint32_t sph_recs = kPair ? p.nsph_pairs : p.nsph;
    float4* lds_tri = lds;
    float4* lds_sph = lds + (size_t)p.tri_batch * kTriRec;
    float2* lds_tab = reinterpret_cast<float2*>(lds_sph + (size_t)p.sph_batch * kSphRec);
    // kOptCull: one (mask word 0 of triangles, of spheres, tile, -) slot per thread, 16-B aligned
    // kOptAccTable: (1/n, (n-1)/n) per sample of the launch, then (float)n (padded to 16 B)
    float* lds_tab_n = reinterpret_cast<float*>(lds_tab + (use_tab_lds(p) ? ((p.spp + 1u) & ~1u) : 0u));
    uint4* lds_cm = reinterpret_cast<uint4*>(lds_tab_n + (use_tab_lds(p) ? ((p.spp + 3u) & ~3u) : 0u));
    constexpr bool use_tab = (OPT & kOptAccTable) != 0;   // the runtime keeps every launch within the table
    constexpr bool kCull = (OPT & kOptCull) && (OPT & kOptPair);
    constexpr bool kBvh = STREAM && (OPT & kOptBvh) && (OPT & kOptPair);
    constexpr bool kBvhPrimary = kBvh && (OPT & kOptBvhPrimary);
    // kOptSplit (resident scenes): round 1 serves anchored tiles and speculative runs, round 2 the
    // chains that left their window
    constexpr bool kSplit = (OPT & kOptSplit) && !STREAM;
    // kOptOverlap (resident, culled, not split): this XCD's tile list and queue word, per-tile waits
    constexpr bool kOverlap = (OPT & kOptOverlap) && !STREAM && !kSplit && kCull;
    // streamed scenes with p.xcd_order: the same per-XCD lists and queue words (tiles dealt to the XCDs by the
    // runtime, iqpt_debug_set_stream_xcd), without the waits
    // kOptPipe (resident, culled, reference materials): two rays per lane and iteration
    constexpr bool kPipe = (OPT & kOptPipe) && !STREAM && !kSplit && kCull && !(OPT & kOptMaterials) && (OPT & kOptAccTable);
    const bool kXcdQ = kOverlap || (STREAM && p.xcd_order != nullptr);
    const uint32_t xcd = kXcdQ ? (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u) : 0u;   // HW_REG_XCC_ID
    uint32_t* const queue_word = kXcdQ ? p.queue + 16u * xcd : p.queue;

    if (!STREAM) {
        for (uint32_t i = threadIdx.x; i < tri_recs * kTriRec; i += kRenderBlock) lds_tri[i] = g_tri[i];
        for (uint32_t i = threadIdx.x; i < sph_recs * kSphRec; i += kRenderBlock) lds_sph[i] = g_sph[i];
    }
    if (use_tab) {
        // (1/n, (n-1)/n) of sample s of this launch: the reference's own divisions, once per block
        for (uint32_t s = threadIdx.x; s < p.spp; s += kRenderBlock) {
            const uint64_t n = p.frame0 + s + 1;
            lds_tab[s] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
            lds_tab_n[s] = (float)n;
        }
    }
    __syncthreads();

    const uint32_t lane = __lane_id();
    if (OPT & kOptStats) {
        stat_tests<OPT>()[threadIdx.x] = 0u;
        stat_tests<OPT>()[256 + threadIdx.x] = 0u;
    }
    // ---- per-lane state
    // (the compact pixel index, the tile and the mask words live in LDS / are recomputed at the
    // pixel's end, and the accumulator's untouched w is never loaded: registers are the limit at
    // 5 waves/SIMD)
    bool active = false;
    uint32_t px = 0, py = 0;
    uint32_t done = 0;                 // samples finished for the current pixel
    rng6 st = {0u, 0u, 0u, 0u, 0u, 0u};
    float3 acc = make_float3(0.0f, 0.0f, 0.0f);
    ray3 ray = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    // kOptPipe: the camera ray of the pixel's next sample, made from the state the current path's draws left
    ray3 ray_b = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    bool has_b = false;
    int depth = 0;
    // scatter-record stack (path_tracer.cu:243): record k of the current path at lds_stk[k][thread]
    float* lds_stk = reinterpret_cast<float*>(lds_cm + ((OPT & kOptCull) ? kRenderBlock : 0));
    // kOptSplit: per thread (split slot sp, next slot j | slots so far, run end, 1 speculative / 2 light
    // split pixel / 0 other), then the six words of a speculative lane's base state
    uint4* lds_sp = reinterpret_cast<uint4*>(lds_stk + (size_t)(p.max_depth > 1 ? p.max_depth : 1) * kRenderBlock *
                                                          ((OPT & kOptMaterials) ? 3u : 1u));
    uint32_t* lds_base = reinterpret_cast<uint32_t*>(lds_sp + kRenderBlock);
    uint64_t spec_mask = 0;            // kOptSplit: speculative lanes of the wave (wave-uniform)
    // kOptSplit: the lane starts a sample at the next iteration's top. Refills and path ends only set it,
    // so the camera-ray code runs once per iteration for all lanes that need it (with lanes refilled
    // at different iterations it had run in both the refill and the path-end branch)
    bool need_cam = false;
    uint64_t wave_rays = 0;            // closest-hit queries of this wave (wave-uniform)
    // ---- wave-uniform chunk state
    uint32_t chunk_next = 0, chunk_end = 0;
    bool exhausted = false;
    // ---- stats (kOptStats): wave-level counters
    unsigned long long s_iter = 0, s_ready = 0, s_scatter_exec = 0, s_scatter_lanes = 0, s_term_exec = 0,
                       s_term_lanes = 0;
    unsigned long long s_tests[2] = {0, 0};   // wave-level triangle / sphere pair tests (culled resident path)
    unsigned long long s_full = 0;            // iterations forced to the full loop (a secondary ray in the wave)
    unsigned long long s_refill = 0, s_refill_lanes = 0;   // refills that started pixels, pixels started
    unsigned long long s_spec_lanes = 0;      // kOptSplit: speculative slots started by this wave
    uint32_t s_first_q = 0, s_chunks = 0;     // first queue position taken, chunks taken (timeline)
    // per lane (kOptStats): BVH rays, nodes visited, leaf pairs / spheres tested — triangle and sphere BVH
    uint32_t c_tri[2] = {0u, 0u}, c_sph[2] = {0u, 0u}, c_tri_rays = 0u, c_sph_rays = 0u;

    // ---- wave-uniform chunk state: the current tile [chunk_next, chunk_end) of tile-major storage
    uint32_t chunk_tile = 0;
    // kOptSplit: chunk kind — 0 anchored tile, 1 speculative run chunk_r of the heavy pixels of a split
    // tile, 2 leftovers [chunk_next, chunk_end) of the leftover list, 3 the light pixels of a split tile
    // (anchored) — and the split tile's first slot and storage index
    uint32_t chunk_kind = 0, chunk_sp0 = 0, chunk_first = 0, chunk_r = 0;
    // the chunk's tile's certain pixels (kparams::certain): they take the whole launch at once (refill). Resident
    // scenes only (streamed: DESIGN.md §3.3; round 5 measured the BVH-primary variants with certain pixels and the
    // sky kernel on C4 slower too, 135 -> 161 ms). The instrumented (kOptStats) variants too, so that the
    // executed-work counts are the production launch's (tools/work_counters.py).
    constexpr bool kCertain = !kSplit && !STREAM && (OPT & kOptAccTable) && !(OPT & kOptMaterials);
    uint64_t chunk_certain = 0;
    // ... and its certain-miss pixels (kparams::miss): iqpt_sky_kernel renders them, this kernel skips them
    uint64_t chunk_miss = 0;
    uint32_t queue_total = kXcdQ ? p.xcd_off[xcd + 1] - p.xcd_off[xcd] : (p.nqueue ? p.nqueue : p.ntiles), n_runs = 0;
    if (kSplit) {
        // round 1, longest tasks first: the split tiles' light pixels (anchored chains with scatters, in
        // the masks' cost order), then the heavy pixels' run chunks, then the anchored (wall / sky) tiles
        n_runs = p.split_round == 2 ? 0u : *p.chunk_count;
        queue_total = p.split_round == 2 ? (*p.left_count + kQueueChunk - 1) / kQueueChunk
                                         : n_runs + p.n_anchor + p.n_split_tiles;
    }
    // kOptSplit: the next queue position is taken one chunk ahead (its atomic's latency overlaps the
    // current chunk's work); a taken position is always consumed by this wave's next refill
    uint32_t q_next_v = 0u;            // the prefetched position (lane 0's atomic result, read when needed)
    bool have_next = false;
    // lanes idle before a refill (kOptSplit round 1: speculative runs end at different iterations, and
    // a refill per iteration costs its dependent loads every iteration; streamed scenes: a wave that takes
    // a whole tile at once keeps its rays coherent through the BVHs, C5 -5 %, r05 runs 29-35)
    const uint32_t refill_min = max(p.refill_min, 1u);
    // pixel complete: BGRA8 (:360-365), accumulator and RNG state back to HBM
    auto store_pixel = [&]() {
        const uint32_t r8 = to_u8(255.0f * iq_sqrtf(acc.x));
        const uint32_t g8 = to_u8(255.0f * iq_sqrtf(acc.y));
        const uint32_t b8 = to_u8(255.0f * iq_sqrtf(acc.z));
        const uint32_t pix = tile_store_index(px - p.x0, (py - p.y0) / p.ystep, p.ncols, p.nrows);
        p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
        // one 16-byte store: the reference never writes w (path_tracer.cu:356-358), and w is 0 from
        // iqpt_create's clear on (iqpt_checkpoint_load refuses a non-zero w), so writing 0 keeps its
        // bits while filling whole lines (three 4-byte stores left partial lines: C4 wrote 2.9x)
        reinterpret_cast<float4*>(p.lin)[pix] = make_float4(acc.x, acc.y, acc.z, 0.0f);
        p.rng[pix] = st.v0;
        p.rng[(size_t)p.npix + pix] = st.v1;
        p.rng[2 * (size_t)p.npix + pix] = st.v2;
        p.rng[3 * (size_t)p.npix + pix] = st.v3;
        p.rng[4 * (size_t)p.npix + pix] = st.v4;
        p.rng[5 * (size_t)p.npix + pix] = st.d;
        done = 0;
    };
    auto refill = [&]() {
        uint64_t need = __ballot(!active);
        while (need != 0ull && !exhausted) {
            if (chunk_next >= chunk_end) {
                uint32_t q = 0;
                if (kSplit && have_next) {
                    q = (uint32_t)__builtin_amdgcn_readfirstlane((int)q_next_v);
                } else {
                    if (lane == 0) q = atomicAdd(queue_word, 1u);
                    q = (uint32_t)__builtin_amdgcn_readfirstlane((int)q);   // wave-uniform: scalar registers
                }
                have_next = false;
                if (q >= queue_total) {
                    exhausted = true;
                    break;
                }
                if (OPT & kOptStats) {
                    if (s_chunks == 0) s_first_q = q;
                    ++s_chunks;
                    if (lane == 0 && p.stats && q < kStatsQueueSlots)
                        p.stats[kStatsHeader + 3 * (size_t)kStatsWaveSlots + q] =
                            (__builtin_amdgcn_s_memrealtime() & 0xffffffffffffull) |
                            ((unsigned long long)(blockIdx.x * (kRenderBlock / 64) + threadIdx.x / 64) << 48);
                }
                if (kSplit) {
                    if (lane == 0) q_next_v = atomicAdd(p.queue, 1u);
                    have_next = true;
                }
                if (kSplit && p.split_round == 2) {
                    chunk_kind = 2;
                    chunk_next = q * kQueueChunk;
                    chunk_end = min(chunk_next + kQueueChunk, *p.left_count);
                } else {
                    uint32_t t;
                    if (kSplit) {
                        if (q < p.n_split_tiles) {
                            chunk_kind = 3;
                            t = p.split_tiles[q];
                            chunk_sp0 = q * kQueueChunk;
                        } else if (q < p.n_split_tiles + n_runs) {
                            // (tile, split tile | run << 23) from the prep kernel's chunk list
                            const uint32_t c = q - p.n_split_tiles;
                            chunk_kind = 1;
                            t = p.chunks[2 * (size_t)c];
                            const uint32_t e = p.chunks[2 * (size_t)c + 1];
                            chunk_r = e >> 23;
                            chunk_sp0 = (e & 0x7fffffu) * kQueueChunk;
                        } else {
                            chunk_kind = 0;
                            t = p.anchor_order[q - p.n_split_tiles - n_runs];
                        }
                    } else if (kXcdQ) {
                        t = p.xcd_order[p.xcd_off[xcd] + q];
                        if (kOverlap && p.done_target != 0u && lane == 0) {
                            // wait until the previous launches of the chain have finished tile t: their waves
                            // ran on this XCD, so the counter and the tile's pixel state meet in its L2 (sc1
                            // polls and loads bypass this CU's L1)
                            const uint32_t tx = t % p.ntx, ty = t / p.ntx;
                            const uint32_t need = p.done_target * (min(kCullTile, p.nrows - ty * kCullTile) *
                                                                   min(kCullTile, p.ncols - tx * kCullTile));
                            uint32_t spins = 0;
                            while (__hip_atomic_load(p.tile_done + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
                                __builtin_amdgcn_s_sleep(20);
                                if (++spins > p.spin_limit) {
                                    atomicOr(p.ovl_err, 1u);
                                    break;
                                }
                            }
                        }
                    } else {
                        t = p.tile_order ? p.tile_order[q] : q;
                    }
                    chunk_tile = t;
                    chunk_certain = (kCertain && p.certain != nullptr)
                                        ? ((uint64_t)p.certain[2 * (size_t)t] | ((uint64_t)p.certain[2 * (size_t)t + 1] << 32))
                                        : 0ull;
                    chunk_miss = (kCertain && p.miss != nullptr)
                                     ? ((uint64_t)p.miss[2 * (size_t)t] | ((uint64_t)p.miss[2 * (size_t)t + 1] << 32))
                                     : 0ull;
                    const uint32_t tx = t % p.ntx, ty = t / p.ntx;
                    const uint32_t th = min(kCullTile, p.nrows - ty * kCullTile);
                    const uint32_t tw = min(kCullTile, p.ncols - tx * kCullTile);
                    chunk_next = ty * kCullTile * p.ncols + tx * kCullTile * th;
                    chunk_end = chunk_next + tw * th;
                    chunk_first = chunk_next;

                }
            }
            const uint32_t avail = chunk_end - chunk_next;
            const uint32_t rank = prefix_below(need);
            if (!active && rank < avail) {
                uint32_t pix = chunk_next + rank;                  // tile-major storage index
                uint32_t tile = chunk_tile;
                // a certain-miss pixel is iqpt_sky_kernel's: skipped (no state touched, no ray counted here)
                bool go = !(kCertain && ((chunk_miss >> (pix - chunk_first)) & 1ull)), spec = false;
                uint32_t sp = 0;
                if (kSplit && (chunk_kind == 1 || chunk_kind == 3)) {
                    sp = chunk_sp0 + (pix - chunk_first);
                    const uint32_t m = p.sp_win[sp];                // 0: a light pixel this launch
                    if (chunk_kind == 3) {
                        go = m == 0u;                               // heavy pixels run as speculative runs
                        lds_sp[threadIdx.x] = make_uint4(sp, 0u, 0u, 2u);
                    } else {
                        // speculative run chunk_r of the heavy pixel: slots [r R, min(r R + R, M)) of its
                        // window, from the run's start state (iqpt_split_prep_kernel)
                        const uint32_t j0 = chunk_r * p.split_len, j1 = min(j0 + p.split_len, m);
                        go = j0 < j1;
                        spec = true;
                        if (go) {
                            const size_t pl = (size_t)chunk_r * 6u * p.ns_cap + sp;
                            st.v0 = p.run_st[pl];
                            st.v1 = p.run_st[pl + p.ns_cap];
                            st.v2 = p.run_st[pl + 2 * (size_t)p.ns_cap];
                            st.v3 = p.run_st[pl + 3 * (size_t)p.ns_cap];
                            st.v4 = p.run_st[pl + 4 * (size_t)p.ns_cap];
                            st.d = p.run_st[pl + 5 * (size_t)p.ns_cap];
                            lds_sp[threadIdx.x] = make_uint4(sp, j0, j1, 1u);
                            if (OPT & kOptStats) s_spec_lanes += 1ull;
                        }
                    }
                } else if (kSplit && chunk_kind == 2) {
                    // a chain that left its window: anchored from its chain position (the stitch's state,
                    // accumulator and sample count)
                    const uint32_t sp = p.left[pix];
                    pix = p.sp_pix[sp];
                    st.v0 = p.sp_st[sp];
                    st.v1 = p.sp_st[(size_t)p.ns_cap + sp];
                    st.v2 = p.sp_st[2 * (size_t)p.ns_cap + sp];
                    st.v3 = p.sp_st[3 * (size_t)p.ns_cap + sp];
                    st.v4 = p.sp_st[4 * (size_t)p.ns_cap + sp];
                    st.d = p.sp_st[5 * (size_t)p.ns_cap + sp];
                    lds_sp[threadIdx.x] = make_uint4(sp, 0u, 0u, 0u);
                }
                uint32_t loc = 0;                                   // the pixel's place in its tile (kparams::pmask)
                if (go) {
                    uint32_t col, row;
                    tile_decode(pix, p.ncols, p.nrows, &col, &row);
                    px = p.x0 + col;
                    py = p.y0 + row * p.ystep;
                    if (STREAM)
                        loc = (row % kCullTile) * min(kCullTile, p.ncols - (col / kCullTile) * kCullTile) + col % kCullTile;
                    if (spec) {
                        // state from the run planes (above)
                    } else if (kSplit && chunk_kind == 2) {
                        tile = (row / kCullTile) * p.ntx + col / kCullTile;
                        const float4_storage a = p.sp_acc[p.left[chunk_next + rank]];
                        acc = make_float3(a.x, a.y, a.z);
                        done = __float_as_uint(a.w);
                    } else if (kOverlap) {
                        // written by the previous launch of the chain, possibly from another CU of this XCD
                        auto ld = [](const uint32_t* q) {
                            return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        };
                        st.v0 = ld(p.rng + pix);
                        st.v1 = ld(p.rng + (size_t)p.npix + pix);
                        st.v2 = ld(p.rng + 2 * (size_t)p.npix + pix);
                        st.v3 = ld(p.rng + 3 * (size_t)p.npix + pix);
                        st.v4 = ld(p.rng + 4 * (size_t)p.npix + pix);
                        st.d = ld(p.rng + 5 * (size_t)p.npix + pix);
                        const uint32_t* a = reinterpret_cast<const uint32_t*>(p.lin + pix);
                        acc = make_float3(__uint_as_float(ld(a)), __uint_as_float(ld(a + 1)), __uint_as_float(ld(a + 2)));
                        done = 0;
                    } else {
                        st.v0 = p.rng[pix];
                        st.v1 = p.rng[(size_t)p.npix + pix];
                        st.v2 = p.rng[2 * (size_t)p.npix + pix];
                        st.v3 = p.rng[3 * (size_t)p.npix + pix];
                        st.v4 = p.rng[4 * (size_t)p.npix + pix];
                        st.d = p.rng[5 * (size_t)p.npix + pix];
                        const float* a = reinterpret_cast<const float*>(p.lin + pix);
                        acc = make_float3(a[0], a[1], a[2]);
                        done = 0;
                        if (kSplit && chunk_kind == 0) lds_sp[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
                    }
                    depth = 0;
                    if (kCertain && ((chunk_certain >> (pix - chunk_first)) & 1ull)) {
                        // a certain tile (kparams::certain): every sample takes the camera's two draws and
                        // ends on an emissive triangle, clamped colour (1, 1, 1), whose mean term c / n is the
                        // table's RN(1 / n) (mean_terms): the launch's samples fold at once, in order
                        xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, 2u * p.spp);
                        st.d += 2u * p.spp * IQ_XORWOW_WEYL;
                        for (uint32_t k = 0; k < p.spp; ++k) {
                            const float2 tv = lds_tab[k];
                            acc.x = tv.x + acc.x * tv.y;
                            acc.y = tv.x + acc.y * tv.y;
                            acc.z = tv.x + acc.z * tv.y;
                        }
                        store_pixel();
                        go = false;
                    } else if (kSplit) {
                        need_cam = true;           // one camera_ray call site per iteration (loop top)
                    } else {
                        camera_ray<OPT>(p, px, py, st, ray);
                        if (kPipe) {
                            has_b = 1u < p.spp;
                            if (has_b) {
                                rng6 sb = st;
                                camera_ray<OPT>(p, px, py, sb, ray_b);
                            }
                        }
                    }
                }
                if (go && kCull && p.cull) {
                    // the tile and word 0 of its triangle / sphere masks, kept in this lane's LDS slot for
                    // the pixel's lifetime (the global load latency is paid once per pixel, not per ray)
                    lds_cm[threadIdx.x] = make_uint4(p.cull[(size_t)tile * p.cull_stride],
                                                     p.cull[(size_t)tile * p.cull_stride + p.cull_wt], tile, loc);
                }
                if (go) active = true;
            }
            if (kCertain && (chunk_certain | chunk_miss)) {
                // the certain pixels of this pass are complete: their rays, and (overlapped launches) their
                // tile's completion count once their stores are done; the skipped certain misses count
                // toward the tile's completion only (the sky kernel renders them and counts their rays)
                const uint32_t took = prefix_below(need) < avail && ((need >> lane) & 1ull) ? 1u : 0u;
                const uint32_t nfin = (uint32_t)__popcll(__ballot(took && !active));
                const uint32_t nmiss = (uint32_t)__popcll(
                    __ballot(took && ((chunk_miss >> ((chunk_next + prefix_below(need) - chunk_first) & 63u)) & 1ull)));
                if (nfin) {
                    wave_rays += (uint64_t)(nfin - nmiss) * p.spp;
                    if (kOverlap && p.tile_done) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) atomicAdd(p.tile_done + chunk_tile, nfin);
                    }
                }
            }
            if (OPT & kOptStats) {
                const uint32_t got = min((uint32_t)__popcll(need), avail);
                s_refill += got ? 1ull : 0ull;
                s_refill_lanes += got;
            }
            const uint32_t cnt = (uint32_t)__popcll(need);
            chunk_next += cnt < avail ? cnt : avail;
            need = __ballot(!active);
        }
        if (kSplit) spec_mask = __ballot(active && lds_sp[threadIdx.x].w == 1u);
        if ((OPT & kOptPrio) && kCull && p.cull) {
            // a wave holding pixels of a tile with sphere candidates (chains that scatter: the launch's
            // longest) wins VALU arbitration against wall / sky waves
            if (__ballot(active && lds_cm[threadIdx.x].y != 0u) != 0ull) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(0);
        }
    };

    const uint64_t t_start = (OPT & kOptStats) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (p.spp > 0) refill();

    // kOptBvhPrimary: every ray goes through the BVHs, no LDS batches, so no workgroup barriers: the
    // waves iterate independently, as in the resident kernel
    constexpr bool kBatches = STREAM && !kBvhPrimary;
    // kOptStats: shader-clock cycles per phase of the loop (closest hits, shading, next rays, the rest)
    unsigned long long s_ph[4] = {0ull, 0ull, 0ull, 0ull};
    unsigned long long s_t = (OPT & kOptStats) ? __builtin_amdgcn_s_memtime() : 0ull;
    auto phase = [&](int i) {
        if (OPT & kOptStats) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            s_ph[i] += t - s_t;
            s_t = t;
        }
    };
    while (true) {
        if (kBatches) {
            if (!__syncthreads_or(active ? 1 : 0)) break;
        } else {
            if (!__any(active)) break;
        }
        phase(3);
        if (kSplit && need_cam) {
            camera_ray<OPT>(p, px, py, st, ray);
            need_cam = false;
        }
        if (OPT & kOptStats) {
            ++s_iter;
            s_ready += (unsigned long long)__popcll(__ballot(active));
        }

        bool finished = false;             // kOptOverlap: the lane stored its pixel this iteration
        if constexpr (kPipe) {
            // ---- kOptPipe: the lane's path ray (a = `ray`) and the camera ray of its pixel's next
            // sample (b = `ray_b`, made from the state the path's draws have left) are traced together. Sample k + 1
            // starts where sample k's draws end (path_tracer.cu:338-339), so b is that sample's camera ray exactly
            // when ray a ends the path without drawing again (an emissive triangle or the sky, path_tracer.cu:278,
            // 307-316); then sample k + 1's first query is already done and the lane shades it in the same
            // iteration. A scatter (material.cu:10 draws two numbers) makes b stale: it is dropped, not counted,
            // and made again. Each ray's closest hit is the reference's (its own pairs in index order).
            float cb = kTMax;
            int kb = kHitNone;
            uint32_t ib = 0;
            float closest = kTMax;
            int kind = kHitNone;
            uint32_t hidx = 0;
            {
                uint4 cm = lds_cm[threadIdx.x];
                const uint64_t act = __ballot(active);
                const uint32_t first = act ? (uint32_t)__builtin_ctzll(act) : 0u;
                const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)cm.z, (int)first);
                const bool uni = __ballot(active && cm.z != t0) == 0ull;
                if (uni) {
                    cm.x = (uint32_t)__builtin_amdgcn_readlane((int)cm.x, (int)first);
                    cm.y = (uint32_t)__builtin_amdgcn_readlane((int)cm.y, (int)first);
                }
                const uint32_t* uni_mask = uni ? p.cull + (size_t)t0 * p.cull_stride : nullptr;
                const uint32_t* lane_mask = active ? p.cull + (size_t)cm.z * p.cull_stride : nullptr;
                const bool all_a = __any(active && depth != 0);
                intersect_culled2<OPT>(lds_tri, p.ntri, lds_sph, p.nsph, lane_mask, cm.x, cm.y, all_a, active,
                                       active && has_b, ray, ray_b, closest, kind, hidx, cb, kb, ib, p.cull_wt, uni_mask,
                                       (OPT & kOptStats) ? s_tests : nullptr);
                if (OPT & kOptStats) s_full += all_a ? 1ull : 0ull;
            }
            phase(0);
            wave_rays += (uint64_t)__popcll(__ballot(active));
            // at most two shading rounds: ray a's hit, then (ray a ended the path) ray b's
            bool pend = active, need_a = false;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                bool term = false;
                uint32_t md_end = 0;
                float Lx = 0.0f, Ly = 0.0f, Lz = 0.0f;
                if (pend) {
                    if (kind == kHitSphere) {
                        if (OPT & kOptStats) ++s_scatter_lanes;
                        const float* q = reinterpret_cast<const float*>(lds_sph + (size_t)(hidx >> 1) * kSphPairFloat4) +
                                         (hidx & 1u);
                        const float s = oren_nayar_scatter<OPT>(make_float4(q[0], q[2], q[4], q[6]), closest, ray, st);
                        if (depth + 1 >= p.max_depth) {
                            term = true;             // the last record is this scatter (biased, :252)
                            md_end = 1;
                            Lx = s;
                            Ly = s;
                            Lz = s;
                        } else {
                            lds_stk[(uint32_t)depth * kRenderBlock + threadIdx.x] = s;
                            ++depth;
                        }
                    } else if (kind == kHitTri) {
                        term = true;                 // emissive(1, 10): att 10, cos = pdf = 1
                        Lx = 10.0f;
                        Ly = 10.0f;
                        Lz = 10.0f;
                    } else {
                        term = true;                 // sky gradient, :308-313
                        const float a = (ray.dy + 1.0f) * 0.5f;
                        const float one_a = 1.0f - a;
                        Lx = one_a + a * 0.5f;
                        Ly = one_a + a * 0.7f;
                        Lz = one_a + a * 1.0f;
                    }
                }
                if (OPT & kOptStats) {
                    if (__ballot(pend && kind == kHitSphere)) ++s_scatter_exec;
                    const uint64_t tm = __ballot(term);
                    if (tm) {
                        ++s_term_exec;
                        s_term_lanes += (unsigned long long)__popcll(tm);
                    }
                }
                bool next = false;
                if (term) {
                    // backward product (:321-324), clamp (:345-347), path_color = 0 + color, running mean (:356-358)
                    float cx = Lx, cy = Ly, cz = Lz;
                    for (int i = depth - 1; i >= 0; --i) {
                        const float f = lds_stk[(uint32_t)i * kRenderBlock + threadIdx.x];
                        cx = cx * f;
                        cy = cy * f;
                        cz = cz * f;
                    }
                    cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
                    cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
                    cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
                    const float2 tv = lds_tab[done];
                    float qx, qy, qz;
                    mean_terms<OPT>(0.0f + cx, 0.0f + cy, 0.0f + cz, lds_tab_n[done], tv.x, p.mean_tiny, qx, qy, qz);
                    acc.x = qx + acc.x * tv.y;
                    acc.y = qy + acc.y * tv.y;
                    acc.z = qz + acc.z * tv.y;
                    ++done;
                    depth = 0;
                    if (done == p.spp) {
                        store_pixel();
                        if (kOverlap) finished = true;
                        active = false;
                    } else if (r == 0 && md_end == 0u && has_b) {
                        // the path ended without drawing: ray b is the next sample's camera ray, its query done
                        (void)xorwow_next(st);
                        (void)xorwow_next(st);
                        ray = ray_b;
                        closest = cb;
                        kind = kb;
                        hidx = ib;
                        next = true;
                    } else {
                        need_a = true;
                    }
                }
                if (r == 0) wave_rays += (uint64_t)__popcll(__ballot(next));
                pend = next;
            }
            phase(1);
            // the next iteration's rays: a new path's camera ray where a path ended without taking ray b, and the
            // camera ray of the sample after the current one (ray b is stale after any scatter or path end)
            if (need_a && active) camera_ray<OPT>(p, px, py, st, ray);
            has_b = active && done + 1u < p.spp;
            if (has_b) {
                rng6 sb = st;
                camera_ray<OPT>(p, px, py, sb, ray_b);
            }
            phase(2);
        } else {
            // ------------------------------------------------ closest hit (path_tracer.cu:253-295)
            float closest = kTMax;
            int kind = kHitNone;
            uint32_t hidx = 0;
            // kOptCull: camera rays (depth 0) test only the pairs of their tile's mask; one secondary ray
            // in the wave makes it test everything
            const bool cull = kCull && p.cull != nullptr && !__any(active && depth != 0);
            const uint32_t* lane_mask =
                (cull && active) ? p.cull + (size_t)lds_cm[threadIdx.x].z * p.cull_stride : nullptr;   // null: 0
            // kBvhPrimary: the path state the traversals never read (RNG state, accumulator, pixel, sample
            // count, depth: 13 words) waits in this thread's slots of the unused scene-batch region of LDS
            // (>= 13 x kRenderBlock words, checked by the runtime), so the traversals' live ranges fit the
            // 5-wave register budget instead of spilling to scratch. The empty asm keeps the
            // compiler from forwarding the stores into registers across the traversal.
            uint32_t* const park = reinterpret_cast<uint32_t*>(lds_tri) + threadIdx.x;
            if (kBvhPrimary) {
                park[0 * kRenderBlock] = st.v0;
                park[1 * kRenderBlock] = st.v1;
                park[2 * kRenderBlock] = st.v2;
                park[3 * kRenderBlock] = st.v3;
                park[4 * kRenderBlock] = st.v4;
                park[5 * kRenderBlock] = st.d;
                park[6 * kRenderBlock] = __float_as_uint(acc.x);
                park[7 * kRenderBlock] = __float_as_uint(acc.y);
                park[8 * kRenderBlock] = __float_as_uint(acc.z);
                park[9 * kRenderBlock] = px;
                park[10 * kRenderBlock] = py;
                park[11 * kRenderBlock] = done;
                park[12 * kRenderBlock] = (uint32_t)depth;
                asm volatile("" ::: "memory");
            }
            if (kBvhPrimary) {
                // Triangles through the exact BVH, spheres through the exact sphere BVH (each falls back to
                // the brute-force fold from global memory where its BVH is absent or the ray is outside
                // the bounds' assumptions, bvh_ray_ok). With a sphere BVH the spheres go first and bound the
                // triangle traversal (closest_spheres_first); otherwise triangles first, as in
                // path_tracer.cu:257-295. Both give the reference's result.
                if (active && sbvh_first_ok(p, ray)) {
                    if (OPT & kOptStats) {
                        ++c_sph_rays;
                        if (p.bvh_nodes != nullptr && bvh_ray_ok(p, ray)) ++c_tri_rays;
                    }
                    closest_spheres_first<OPT>(p, ray, p.bvh_nodes != nullptr && bvh_ray_ok(p, ray), closest, kind, hidx,
                                               (OPT & kOptStats) ? c_tri : nullptr, (OPT & kOptStats) ? c_sph : nullptr);
                } else if (active) {
                    const bool ok = bvh_ray_ok(p, ray);
                    if (ok && p.bvh_nodes != nullptr) {
                        if (OPT & kOptStats) ++c_tri_rays;
                        bvh_closest<OPT>(p, ray, closest, kind, hidx, (OPT & kOptStats) ? c_tri : nullptr);
                    } else {
                        const float4* __restrict__ gp = reinterpret_cast<const float4*>(p.tri_pairs);
                        for (uint32_t j = 0; j < p.ntri_pairs; ++j) {
                            const float4* q = gp + (size_t)j * kTriPairFloat4;
                            test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, 2 * j,
                                                    2 * j + 1 < p.ntri);
                        }
                    }
                    if (ok && p.sbvh_nodes != nullptr) {
                        if (OPT & kOptStats) ++c_sph_rays;
                        sbvh_closest<OPT>(p, ray, closest, kind, hidx, (OPT & kOptStats) ? c_sph : nullptr);
                    } else {
                        const float4* __restrict__ gs = reinterpret_cast<const float4*>(p.sph_pairs);
                        for (uint32_t j = 0; j < p.nsph_pairs; ++j) {
                            const float4* q = gs + (size_t)j * kSphPairFloat4;
                            test_sphere_pair<OPT>(q[0], q[1], ray, closest, kind, hidx, 2 * j, 2 * j + 1 < p.nsph);
                        }
                    }
                }
            } else if (STREAM) {
                // Streamed scene. Per lane and mask word: a camera ray contributes its tile's mask (kOptCull),
                // a secondary ray that takes the BVH (kOptBvh) contributes nothing to the triangle batches,
                // any other ray every pair; the wave ORs the words, the block skips a batch nobody needs.
                constexpr bool kWords = kCull || kBvh;
                const bool bvh_ray = kBvh && active && (depth != 0 || kBvhPrimary) &&
                                     (p.bvh_nodes != nullptr || p.sbvh_nodes != nullptr) && bvh_ray_ok(p, ray);
                const bool bvh_lane = bvh_ray && p.bvh_nodes != nullptr;
                const uint32_t* tile_mask =
                    (kCull && p.cull != nullptr && active && depth == 0)
                        ? p.cull + (size_t)lds_cm[threadIdx.x].z * p.cull_stride : nullptr;
                const uint32_t* tri_mask = bvh_lane ? nullptr : tile_mask;
                const bool tri_all = active && tile_mask == nullptr && !bvh_lane;
                // the spheres through the sphere BVH (same rays as the triangle BVH) instead of the batches
                const bool sbvh_lane = bvh_ray && p.sbvh_nodes != nullptr;
                const bool sph_all = active && tile_mask == nullptr && !sbvh_lane;
                const uint32_t* sph_mask = sbvh_lane ? nullptr : tile_mask;
                // One tile for every lane that contributes mask words (and no lane that needs every pair): the
                // wave's OR is that tile's mask, read with uniform loads instead of a DPP OR per word
                // (camera-ray waves, the usual case); no contributing lane at all: every word is 0.
                const uint32_t* uni_tri = nullptr;
                const uint32_t* uni_sph = nullptr;
                bool tri_none = false, sph_none = false;
                uint32_t tt = 0, ts = 0;                      // the uniform tiles
                if (kCull && p.cull != nullptr) {
                    const uint32_t tile = lds_cm[threadIdx.x].z;
                    const uint64_t mt = __ballot(tri_mask != nullptr), ms = __ballot(sph_mask != nullptr);
                    if (__ballot(tri_all) == 0ull) {
                        if (mt == 0ull) {
                            tri_none = true;
                        } else {
                            tt = (uint32_t)__builtin_amdgcn_readlane((int)tile, (int)__builtin_ctzll(mt));
                            if (__ballot(tri_mask != nullptr && tile != tt) == 0ull) uni_tri = p.cull + (size_t)tt * p.cull_stride;
                        }
                    }
                    if (__ballot(sph_all) == 0ull) {
                        if (ms == 0ull) {
                            sph_none = true;
                        } else {
                            ts = (uint32_t)__builtin_amdgcn_readlane((int)tile, (int)__builtin_ctzll(ms));
                            if (__ballot(sph_mask != nullptr && tile != ts) == 0ull) uni_sph = p.cull + (size_t)ts * p.cull_stride;
                        }
                    }
                }
                // A uniform-tile wave takes its tile's candidate pairs from the candidate list (ascending
                // pair indices: the order of the masked batch loop, so the same closest hit), reading each
                // pair straight from global memory with wave-uniform loads, and needs none of the batches.
                const bool list_tri = uni_tri != nullptr && p.list != nullptr;
                const bool list_sph = uni_sph != nullptr && p.list != nullptr;
                const uint32_t la = list_tri ? p.list_off_tri[tt] : 0u, lb = list_tri ? p.list_off_tri[tt + 1] : 0u;
                if (list_tri && p.pmask != nullptr && lb - la <= kPixMaskMax) {
                    // per-pixel candidates (kparams::pmask): each lane walks the entries its own bundle may meet, in
                    // list order; the wave leaves when no lane has one left (or, any-hit, every lane left has its hit)
                    const float4* __restrict__ gp = reinterpret_cast<const float4*>(p.tri_pairs);
                    const uint32_t* pm = p.pmask + p.pmask_off[tt] + lds_cm[threadIdx.x].w;
                    const uint32_t nw = (lb - la + 31u) / 32u;
                    uint32_t wi = 0, cur = tri_mask != nullptr ? pm[0] : 0u;
                    while (true) {
                        while (cur == 0u && tri_mask != nullptr && wi + 1u < nw) cur = pm[(size_t)(++wi) * 64u];
                        const bool want = cur != 0u && !((OPT & kOptAnyHit) && p.anyhit && kind == kHitTri);
                        if (!__any(want)) break;
                        if (want) {
                            const uint32_t e = wi * 32u + (uint32_t)__builtin_ctz(cur);
                            cur &= cur - 1u;
                            const uint32_t j = p.list[la + e];
                            const float4* q = gp + (size_t)j * kTriPairFloat4;
                            test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, 2 * j,
                                                    2 * j + 1 < p.ntri);
                        }
                    }
                    tri_none = true;
                } else if (list_tri) {
                    const float4* __restrict__ gp = reinterpret_cast<const float4*>(p.tri_pairs);
                    const uint32_t a = la, b = lb;
                    // software-pipelined: the next pair's records are loaded while this one is tested (C4 -1.7 %)
                    uint32_t j = a < b ? (uint32_t)__builtin_amdgcn_readfirstlane((int)p.list[a]) : 0u;
                    float4 q0, q1, q2, q3, q4;
                    if (a < b) {
                        const float4* q = gp + (size_t)j * kTriPairFloat4;
                        q0 = q[0]; q1 = q[1]; q2 = q[2]; q3 = q[3]; q4 = q[4];
                    }
                    for (uint32_t e = a; e < b; ++e) {
                        const uint32_t jn = e + 1 < b ? (uint32_t)__builtin_amdgcn_readfirstlane((int)p.list[e + 1]) : j;
                        const float4* qn = gp + (size_t)jn * kTriPairFloat4;
                        const float4 n0 = qn[0], n1 = qn[1], n2 = qn[2], n3 = qn[3], n4 = qn[4];
                        if (tri_mask != nullptr)
                            test_triangle_pair<OPT>(q0, q1, q2, q3, q4, ray, closest, kind, hidx, 2 * j,
                                                    2 * j + 1 < p.ntri);
                        // any-hit scenes: the wave leaves once every list lane has an accepted triangle
                        if ((OPT & kOptAnyHit) && p.anyhit && __ballot(tri_mask != nullptr && kind != kHitTri) == 0ull) break;
                        j = jn;
                        q0 = n0; q1 = n1; q2 = n2; q3 = n3; q4 = n4;
                    }
                    tri_none = true;                          // nothing left for the batches from this wave
                }
                // the whole block skips the triangle batches when every ray takes the BVH or a list
                const bool tri_block =
                    !kWords || __syncthreads_or((tri_all || (tri_mask != nullptr && !list_tri)) ? 1 : 0);
                for (uint32_t base = 0; tri_block && base < tri_recs; base += p.tri_batch) {
                    const uint32_t n = min(p.tri_batch, tri_recs - base);
                    uint32_t wm[kWords ? 8 : 1];
                    bool any = true;
                    if (kWords) {
                        // the batch's mask words (a batch is at most 256 pairs, a multiple of 32: <= 8 aligned words)
                        any = false;
    #pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const uint32_t w = base / 32u + (uint32_t)i;
                            wm[i] = 0u;
                            if ((uint32_t)i * 32u < n)
                                wm[i] = tri_none ? 0u
                                                 : (uni_tri ? uni_tri[w]
                                                            : wave_or(tri_all ? ~0u : (tri_mask ? tri_mask[w] : 0u)));
                            any = any || wm[i] != 0u;
                        }
                        // the barrier also orders this batch's LDS writes after the previous batch's reads
                        if (!__syncthreads_or(any ? 1 : 0)) continue;
                    } else {
                        __syncthreads();
                    }
                    for (uint32_t i = threadIdx.x; i < n * kTriRec; i += kRenderBlock)
                        lds_tri[i] = g_tri[(size_t)base * kTriRec + i];
                    __syncthreads();
                    if (active && !bvh_lane && !list_tri) {
                        const uint32_t first = base * kTriPer;
                        const uint32_t cnt = min(n * kTriPer, p.ntri - first);
                        if (kWords) {
    #pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                uint32_t m = wm[i];
                                while (m) {
                                    const uint32_t j = (uint32_t)i * 32u + (uint32_t)__builtin_ctz(m);   // local pair
                                    m &= m - 1u;
                                    if (j >= n) break;
                                    const float4* q = lds_tri + (size_t)j * kTriPairFloat4;
                                    test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx,
                                                            first + 2 * j, 2 * j + 1 < cnt);
                                }
                            }
                        } else {
                            intersect_range<OPT>(lds_tri, first, cnt, lds_sph, 0, 0, ray, closest, kind, hidx);
                        }
                    }
                }
                // secondary rays: triangles through the exact BVH (iq_bvh.hpp), before the spheres
                if (bvh_lane) {
                    if (OPT & kOptStats) ++c_tri_rays;
                    bvh_closest<OPT>(p, ray, closest, kind, hidx, (OPT & kOptStats) ? c_tri : nullptr);
                }
                if (list_sph) {
                    const float4* __restrict__ gs = reinterpret_cast<const float4*>(p.sph_pairs);
                    const uint32_t a = p.list_off_sph[ts], b = p.list_off_sph[ts + 1];
                    for (uint32_t e = a; e < b; ++e) {
                        const uint32_t j = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.list[e]);
                        if (sph_mask != nullptr) {
                            const float4* q = gs + (size_t)j * kSphPairFloat4;
                            test_sphere_pair<OPT>(q[0], q[1], ray, closest, kind, hidx, 2 * j, 2 * j + 1 < p.nsph);
                        }
                    }
                    sph_none = true;
                }
                for (uint32_t base = 0; base < sph_recs; base += p.sph_batch) {
                    const uint32_t n = min(p.sph_batch, sph_recs - base);
                    uint32_t wm[kWords ? 8 : 1];
                    bool any = true;
                    if (kWords) {
                        any = false;
    #pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const uint32_t w = p.cull_wt + base / 32u + (uint32_t)i;
                            wm[i] = 0u;
                            if ((uint32_t)i * 32u < n)
                                wm[i] = sph_none ? 0u
                                                 : (uni_sph ? uni_sph[w]
                                                            : wave_or(sph_all ? ~0u : (sph_mask ? sph_mask[w] : 0u)));
                            any = any || wm[i] != 0u;
                        }
                        if (!__syncthreads_or(any ? 1 : 0)) continue;
                    } else {
                        __syncthreads();
                    }
                    for (uint32_t i = threadIdx.x; i < n * kSphRec; i += kRenderBlock)
                        lds_sph[i] = g_sph[(size_t)base * kSphRec + i];
                    __syncthreads();
                    if (active && !sbvh_lane && !list_sph) {
                        const uint32_t first = base * kSphPer;
                        const uint32_t cnt = min(n * kSphPer, p.nsph - first);
                        if (kWords) {
    #pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                uint32_t m = wm[i];
                                while (m) {
                                    const uint32_t j = (uint32_t)i * 32u + (uint32_t)__builtin_ctz(m);
                                    m &= m - 1u;
                                    if (j >= n) break;
                                    const float4* q = lds_sph + (size_t)j * kSphPairFloat4;
                                    test_sphere_pair<OPT>(q[0], q[1], ray, closest, kind, hidx, first + 2 * j,
                                                          2 * j + 1 < cnt);
                                }
                            }
                        } else {
                            intersect_range<OPT>(lds_tri, 0, 0, lds_sph, first, cnt, ray, closest, kind, hidx);
                        }
                    }
                }
                if (sbvh_lane) {
                    if (OPT & kOptStats) ++c_sph_rays;
                    sbvh_closest<OPT>(p, ray, closest, kind, hidx, (OPT & kOptStats) ? c_sph : nullptr);
                }
            } else if (kCull && p.cull != nullptr) {
                uint4 cm = lds_cm[threadIdx.x];
                // one tile for every active lane (the usual case: a tile's lanes start together and, on
                // tiles whose camera rays all end on their first hit, finish together): its own mask
                const uint64_t act = __ballot(active);
                const uint32_t first = act ? (uint32_t)__builtin_ctzll(act) : 0u;
                const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)cm.z, (int)first);
                const bool uni = cull && __ballot(active && cm.z != t0) == 0ull;
                if (uni) {
                    // word 0 is read from the first lane: give every lane the first active lane's words
                    cm.x = (uint32_t)__builtin_amdgcn_readlane((int)cm.x, (int)first);
                    cm.y = (uint32_t)__builtin_amdgcn_readlane((int)cm.y, (int)first);
                }
                const uint32_t* uni_mask = uni ? p.cull + (size_t)t0 * p.cull_stride : nullptr;
                intersect_culled<OPT>(lds_tri, p.ntri, lds_sph, p.nsph, lane_mask, cm.x, cm.y, !cull, active, ray,
                                      closest, kind, hidx, p.cull_wt, uni_mask, (OPT & kOptStats) ? s_tests : nullptr);
                if (OPT & kOptStats) s_full += cull ? 0ull : 1ull;
            } else if (active) {
                intersect_range<OPT>(lds_tri, 0, p.ntri, lds_sph, 0, p.nsph, ray, closest, kind, hidx);
            }
            phase(0);
            if (kBvhPrimary) {
                asm volatile("" ::: "memory");
                st.v0 = park[0 * kRenderBlock];
                st.v1 = park[1 * kRenderBlock];
                st.v2 = park[2 * kRenderBlock];
                st.v3 = park[3 * kRenderBlock];
                st.v4 = park[4 * kRenderBlock];
                st.d = park[5 * kRenderBlock];
                acc.x = __uint_as_float(park[6 * kRenderBlock]);
                acc.y = __uint_as_float(park[7 * kRenderBlock]);
                acc.z = __uint_as_float(park[8 * kRenderBlock]);
                px = park[9 * kRenderBlock];
                py = park[10 * kRenderBlock];
                done = park[11 * kRenderBlock];
                depth = (int)park[12 * kRenderBlock];
            }

            // ------------------------------------------------ shade (path_tracer.cu:297-316)
            bool term = false;
            uint32_t md_end = 0;               // the path ended on a scatter at max_depth (kOptSplit slot count)
            float Lx = 0.0f, Ly = 0.0f, Lz = 0.0f;
            // speculative lanes' rays are counted by the stitch, for the slots on the chain only
            wave_rays += (uint64_t)__popcll(__ballot(active) & ~spec_mask);
            // kOptSplit: a speculative lane's first scatter keeps its base state (the RNG state of its next
            // slot: the camera took exactly the slot's two draws) for the restore at the path's end
            auto save_base = [&]() {
                if (kSplit && depth == 0 && ((spec_mask >> lane) & 1ull)) {
                    lds_base[threadIdx.x] = st.v0;
                    lds_base[kRenderBlock + threadIdx.x] = st.v1;
                    lds_base[2 * kRenderBlock + threadIdx.x] = st.v2;
                    lds_base[3 * kRenderBlock + threadIdx.x] = st.v3;
                    lds_base[4 * kRenderBlock + threadIdx.x] = st.v4;
                    lds_base[5 * kRenderBlock + threadIdx.x] = st.d;
                }
            };
            if (active && (OPT & kOptMaterials)) {
                // ---- material table (§8f.3): the hit primitive's material decides the scatter
                if (kind != kHitNone) {
                    const uint32_t mi = kind == kHitTri ? p.tri_mat[hidx] : p.sph_mat[hidx];
                    const float4_storage m0 = p.mats[2 * mi], m1 = p.mats[2 * mi + 1];
                    if (__float_as_uint(m0.w) == IQPT_MAT_EMISSIVE) {
                        term = true;                 // emissive::scatter: strength * albedo, cos = pdf = 1
                        Lx = m1.x * m0.x;
                        Ly = m1.x * m0.y;
                        Lz = m1.x * m0.z;
                    } else {
                        float hx, hy, hz, nx, ny, nz;
                        if (kind == kHitSphere) {
                            float4 sphr;
                            if (!STREAM && kPair) {
                                const float* q = reinterpret_cast<const float*>(lds_sph + (size_t)(hidx >> 1) *
                                                                                              kSphPairFloat4) +
                                                 (hidx & 1u);
                                sphr = make_float4(q[0], q[2], q[4], q[6]);
                            } else {
                                sphr = g_sph_plain[hidx];
                            }
                            sphere_hit<OPT>(sphr, closest, ray, hx, hy, hz, nx, ny, nz);
                        } else {
                            triangle_hit<OPT>(reinterpret_cast<const float4*>(p.tris),
                                              reinterpret_cast<const float4*>(p.tri_shade), hidx, closest, ray, hx, hy,
                                              hz, nx, ny, nz);
                        }
                        float coeff, q;
                        save_base();
                        or_scatter_core<OPT>(hx, hy, hz, nx, ny, nz, ray, st, m1.y, m1.z, coeff, q);
                        // m_albedo * coeff / pi, times cos / pdf (path_tracer.cu:321-324)
                        const float sx = ((m0.x * coeff) * (1.0f / IQ_PI)) * q;
                        const float sy = ((m0.y * coeff) * (1.0f / IQ_PI)) * q;
                        const float sz = ((m0.z * coeff) * (1.0f / IQ_PI)) * q;
                        if (depth + 1 >= p.max_depth) {
                            term = true;             // the last record is this scatter (biased, :252)
                            md_end = 1;
                            Lx = sx;
                            Ly = sy;
                            Lz = sz;
                        } else {
                            const uint32_t b = (uint32_t)depth * 3u * kRenderBlock + threadIdx.x;
                            lds_stk[b] = sx;
                            lds_stk[b + kRenderBlock] = sy;
                            lds_stk[b + 2u * kRenderBlock] = sz;
                            ++depth;
                        }
                    }
                } else {
                    term = true;                     // sky gradient, :308-313
                    const float a = (ray.dy + 1.0f) * 0.5f;
                    const float one_a = 1.0f - a;
                    Lx = one_a + a * 0.5f;
                    Ly = one_a + a * 0.7f;
                    Lz = one_a + a * 1.0f;
                }
            } else if (active) {
                if (kind == kHitSphere) {
                    if (OPT & kOptStats) ++s_scatter_lanes;
                    float4 sphr;
                    if (!STREAM && kPair) {
                        // the pair record in LDS: (cx_a, cx_b, cy_a, cy_b), (cz_a, cz_b, r_a, r_b)
                        const float* q = reinterpret_cast<const float*>(lds_sph + (size_t)(hidx >> 1) * kSphPairFloat4) +
                                         (hidx & 1u);
                        sphr = make_float4(q[0], q[2], q[4], q[6]);
                    } else {
                        sphr = g_sph_plain[hidx];
                    }
                    save_base();
                    const float s = oren_nayar_scatter<OPT>(sphr, closest, ray, st);
                    if (depth + 1 >= p.max_depth) {
                        term = true;                 // the last record is this scatter (biased, :252)
                        md_end = 1;
                        Lx = s;
                        Ly = s;
                        Lz = s;
                    } else {
                        lds_stk[(uint32_t)depth * kRenderBlock + threadIdx.x] = s;
                        ++depth;
                    }
                } else if (kind == kHitTri) {
                    term = true;                     // emissive(1, 10): att 10, cos = pdf = 1
                    Lx = 10.0f;
                    Ly = 10.0f;
                    Lz = 10.0f;
                } else {
                    term = true;                     // sky gradient, :308-313
                    const float a = (ray.dy + 1.0f) * 0.5f;
                    const float one_a = 1.0f - a;
                    Lx = one_a + a * 0.5f;
                    Ly = one_a + a * 0.7f;
                    Lz = one_a + a * 1.0f;
                }
            }
            if (OPT & kOptStats) {
                if (__ballot(active && kind == kHitSphere)) ++s_scatter_exec;
                const uint64_t tm = __ballot(term);
                if (tm) {
                    ++s_term_exec;
                    s_term_lanes += (unsigned long long)__popcll(tm);
                }
            }

            // ------------------------------------------------ path end: product, clamp, running mean
            if (term) {
                // backward product over the stacked records, newest first (:321-324)
                float cx = Lx, cy = Ly, cz = Lz;
                // most paths end on their first ray (depth 0: no records)
                for (int i = depth - 1; i >= 0; --i) {
                    if (OPT & kOptMaterials) {
                        const uint32_t b = (uint32_t)i * 3u * kRenderBlock + threadIdx.x;
                        cx = cx * lds_stk[b];
                        cy = cy * lds_stk[b + kRenderBlock];
                        cz = cz * lds_stk[b + 2u * kRenderBlock];
                    } else {
                        const float r = lds_stk[(uint32_t)i * kRenderBlock + threadIdx.x];
                        cx = cx * r;
                        cy = cy * r;
                        cz = cz * r;
                    }
                }
                // clamp (:345-347), path_color = 0 + color (:341,348), running mean (:356-358)
                cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
                cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
                cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
                cx = 0.0f + cx;
                cy = 0.0f + cy;
                cz = 0.0f + cz;
                if (kSplit && ((spec_mask >> lane) & 1ull)) {
                    // speculative slot j of split slot sp: the clamped colour and the slots it consumed
                    // (1 + its scatters: two draws each), then the next slot of the run from the base state
                    uint4 sl = lds_sp[threadIdx.x];
                    const uint32_t nsl = (uint32_t)depth + 1u + md_end;
                    const size_t at = (size_t)sl.x * p.m_cap + sl.y;
                    reinterpret_cast<float4*>(p.res)[at] = make_float4(cx, cy, cz, __uint_as_float(nsl));
                    p.nres[at] = (uint8_t)nsl;
                    depth = 0;
                    if (++sl.y == sl.z) {
                        active = false;
                    } else {
                        lds_sp[threadIdx.x].y = sl.y;
                        if (nsl > 1u) {              // the path scattered: back to the base state (its next slot)
                            st.v0 = lds_base[threadIdx.x];
                            st.v1 = lds_base[kRenderBlock + threadIdx.x];
                            st.v2 = lds_base[2 * kRenderBlock + threadIdx.x];
                            st.v3 = lds_base[3 * kRenderBlock + threadIdx.x];
                            st.v4 = lds_base[4 * kRenderBlock + threadIdx.x];
                            st.d = lds_base[5 * kRenderBlock + threadIdx.x];
                        }
                        need_cam = true;
                    }
                } else {
                float keep, nf, rc = 0.0f;
                if (use_tab) {
                    const float2 tv = lds_tab[done];
                    rc = tv.x;
                    keep = tv.y;
                    nf = lds_tab_n[done];
                } else {
                    const uint64_t n = p.frame0 + done + 1;
                    // (float)n of the 64-bit frame counter; when every frame of the launch fits 32 bits
                    // the 32-bit conversion is the same correctly rounded value (one v_cvt_f32_u32)
                    nf = p.frames32 ? (float)(uint32_t)n : (float)n;
                    keep = (p.frames32 ? (float)(uint32_t)(n - 1) : (float)(n - 1)) / nf;
                }
                if (use_tab) {
                    float qx, qy, qz;
                    mean_terms<OPT>(cx, cy, cz, nf, rc, p.mean_tiny, qx, qy, qz);
                    acc.x = qx + acc.x * keep;
                    acc.y = qy + acc.y * keep;
                    acc.z = qz + acc.z * keep;
                } else {
                    acc.x = mean_term<OPT>(cx, nf) + acc.x * keep;
                    acc.y = mean_term<OPT>(cy, nf) + acc.y * keep;
                    acc.z = mean_term<OPT>(cz, nf) + acc.z * keep;
                }
                uint32_t light_sp = ~0u, light_slots = 0;
                if (kSplit) {
                    // a split tile's light pixel counts its slots (1 + scatters per sample) for the next
                    // launch's heavy / light decision (iqpt_split_prep_kernel)
                    const uint4 sl = lds_sp[threadIdx.x];
                    if (sl.w == 2u) {
                        light_sp = sl.x;
                        light_slots = sl.y + (uint32_t)depth + 1u + md_end;
                        lds_sp[threadIdx.x].y = light_slots;
                    }
                }
                ++done;
                depth = 0;
                if (done == p.spp) {
                    store_pixel();
                    if (kOverlap) finished = true;
                    if (kSplit && light_sp != ~0u) p.sp_rho[light_sp] = (uint32_t)(((uint64_t)light_slots * 256u) / p.spp);
                    active = false;
                } else {
                    if (kSplit) need_cam = true;   // one camera_ray call site per iteration (loop top)
                    else camera_ray<OPT>(p, px, py, st, ray);
                }
                }
            }
            phase(1);
        }
        if (kOverlap && p.tile_done) {
            // pixels completed this iteration: once their stores are done (vmcnt 0), one counter add per tile
            uint64_t fin = __ballot(finished);
            if (fin) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t my_tile = lds_cm[threadIdx.x].z;
                while (fin) {
                    const int f = __builtin_ctzll(fin);
                    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)my_tile, f);
                    const uint64_t m = __ballot(finished && my_tile == t0);
                    if ((int)lane == f) atomicAdd(p.tile_done + t0, (uint32_t)__popcll(m));
                    fin &= ~m;
                }
                finished = false;
            }
        }
        if (!exhausted && (uint32_t)__popcll(__ballot(!active)) >= refill_min) refill();
    }

    // closest-hit query count: one atomic per wave
    if (lane == 0 && wave_rays) add_rays(p.rays, (unsigned long long)wave_rays);
    if (kXcdQ && p.ovl_err) {
        // HIP promises no workgroup -> XCD placement: the last block to finish checks that every XCD's
        // tile list was taken to its end (a list no wave ran on would leave its tiles unrendered, silently)
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t fin = atomicAdd(p.queue + 16u * 8u, 1u);
            if (fin == gridDim.x - 1u) {
                for (uint32_t x = 0; x < 8u; ++x)
                    if (__hip_atomic_load(p.queue + 16u * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                        p.xcd_off[x + 1] - p.xcd_off[x])
                        atomicOr(p.ovl_err, 4u);
            }
        }
    }
    if (OPT & kOptStats) {
        unsigned long long scat = s_scatter_lanes;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) scat += __shfl_xor(scat, off);
        if (lane == 0 && p.stats) {
            atomicAdd(p.stats + 0, s_iter);
            atomicAdd(p.stats + 1, s_ready);
            atomicAdd(p.stats + 2, s_ready);
            atomicAdd(p.stats + 3, s_scatter_exec);
            atomicAdd(p.stats + 4, scat);
            atomicAdd(p.stats + 5, s_term_exec);
            atomicAdd(p.stats + 6, s_term_lanes);
            atomicAdd(p.stats + 7, 1ull);
            atomicAdd(p.stats + 8, s_tests[0]);
            atomicAdd(p.stats + 9, s_tests[1]);
            atomicAdd(p.stats + 10, s_full);
            atomicAdd(p.stats + 12, s_refill);
            atomicAdd(p.stats + 13, s_refill_lanes);
        }
        {
            // BVH work and the primitive tests executed, summed over the wave's lanes
            unsigned long long v[8] = {c_tri_rays, c_tri[0], c_tri[1], c_sph_rays, c_sph[0], c_sph[1],
                                       stat_tests<OPT>()[threadIdx.x], stat_tests<OPT>()[256 + threadIdx.x]};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
            }
            if (lane == 0 && p.stats) {
#pragma unroll
                for (int k = 0; k < 8; ++k) atomicAdd(p.stats + 14 + k, v[k]);
            }
            // wave timeline (s_memrealtime, 100 MHz): start, end, iterations per wave
            // one record per wave (lane 0; the atomic optimiser would otherwise hand every lane a slot)
            const uint64_t slot = lane == 0 && p.stats ? atomicAdd(p.stats + 11, 1ull) : ~0ull;
            if (slot < kStatsWaveSlots) {
                // start (48 b) | wave id (blockIdx.x * waves per block + wave, 16 b)
                p.stats[kStatsHeader + 3 * slot] =
                    (t_start & 0xffffffffffffull) |
                    ((unsigned long long)(blockIdx.x * (kRenderBlock / 64) + threadIdx.x / 64) << 48);
                p.stats[kStatsHeader + 3 * slot + 1] = __builtin_amdgcn_s_memrealtime();
                unsigned long long* ph = p.stats + kStatsHeader + 3 * (size_t)kStatsWaveSlots + kStatsQueueSlots +
                                         (size_t)kStatsPhaseWords * slot;
                ph[0] = s_ph[0];
                ph[1] = s_ph[1];
                ph[2] = s_ph[2];
                ph[3] = s_ph[3];
                // iterations | (split: speculative lanes; else first queue position (24 b) | chunks (8 b)) << 32
                p.stats[kStatsHeader + 3 * slot + 2] =
                    s_iter | ((kSplit ? s_spec_lanes
                                      : (unsigned long long)(min(s_first_q, 0xffffffu) | (min(s_chunks, 255u) << 24)))
                              << 32);
            }
        }
    }
}

// Device probe of the shared transcendentals and division forms exactly as the render kernel
// compiles them (tests/test_gpu_libm.py compares them with the oracle's host build, bit for bit).
// fn: 0 sin, 1 cos, 2 tan, 3 acos, 4 atan2(a, b), 5 asin, 6 atan (the oracle's iqo_libm_batch
// numbering), 7 / 8 sin / cos of iq_sincosf, 9 iq_sqrt_guarded, 10 iq_rcp_guarded, 11 iq_div.
// Test only (iqpt_debug_poison_lds): fills every byte of its dynamic LDS with `pattern` and leaves. A grid of
// these at the largest allocation a block may have, several per CU, leaves non-zero values wherever the next
// kernels' LDS allocations land, so a kernel that reads an LDS word before writing it sees garbage and its
// results differ from the oracle's (r04 run 16's one-off parity failure).
__global__ __launch_bounds__(256) void iqpt_lds_poison_kernel(uint32_t pattern, uint32_t words) {
    extern __shared__ uint32_t lds_words[];
    for (uint32_t i = threadIdx.x; i < words; i += 256u) lds_words[i] = pattern ^ (i * 0x9e3779b9u);
    __syncthreads();
    // keep the stores (the kernel's only effect is the LDS contents it leaves behind)
    if (lds_words[threadIdx.x % (words ? words : 1u)] == 0x12345678u && pattern == 0x0badf00du) __builtin_trap();
}

__global__ __launch_bounds__(256) void iqpt_libm_kernel(int fn, const float* a, const float* b, float* out,
                                                        uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const float x = a[i], y = b[i];
    float r = 0.0f, s2, c2;
    switch (fn) {
    case 0: r = iq_sinf(x); break;
    case 1: r = iq_cosf(x); break;
    case 2: r = iq_tanf(x); break;
    case 3: r = iq_acosf(x); break;
    case 4: r = iq_atan2f(x, y); break;
    case 5: r = iq_asinf(x); break;
    case 6: r = iq_atanf(x); break;
    case 7: iq_sincosf(x, &s2, &c2); r = s2; break;
    case 8: iq_sincosf(x, &s2, &c2); r = c2; break;
    case 9: r = iq_sqrt_guarded(x); break;
    case 10: r = iq_rcp_guarded(x); break;
    case 11: r = iq_div(x, y); break;
    default: break;
    }
    if (fn >= 12 && fn <= 19) {
        // iq_fp2.h pair forms: element 0 from (a[i], b[i]), element 1 from the mirrored index, so every
        // output is produced once by each lane slot over the two calls (fn even: .x, odd: .y)
        const uint32_t k = n - 1u - i;
        const float xk = a[k], yk = b[k];
        const bool hi = fn & 1;
        const iq_f2 va = hi ? (iq_f2){xk, x} : (iq_f2){x, xk}, vb = hi ? (iq_f2){yk, y} : (iq_f2){y, yk};
        iq_f2 v = {0.0f, 0.0f};
        switch (fn) {
        case 12: case 13: v = iq_atan2f2(va, vb); break;      // atan2(a, b)
        case 14: case 15: v = iq_acosf2(va); break;
        case 16: case 17: v = iq_sin_cos2(va); break;         // 16: sin(a) from .x, 17: cos(a) from .y
        case 18: v = (iq_f2){iq_tanf_bf(x), 0.0f}; break;
        default: v = iq_sqrt_n2(va); break;                   // 19: iq_sqrt_n from .y
        }
        r = hi ? v.y : v.x;
    }
    out[i] = r;
}

// Camera probe (tests/test_gpu_camera.py): the general transform and kOptCamAxis's short one for n
// given (x_ndc, y_ndc), ray components written as 6 floats each (bits compared by the test).
__global__ __launch_bounds__(256) void iqpt_camera_probe_kernel(const kparams p, const float* ndc, float* gen,
                                                                float* axis, uint32_t n, int do_axis) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    constexpr int kOpt = kOptDefault;
    ray3 r;
    camera_ndc<kOpt>(p, ndc[2 * i], ndc[2 * i + 1], r);
    const float g[6] = {r.ox, r.oy, r.oz, r.dx, r.dy, r.dz};
    for (int k = 0; k < 6; ++k) gen[6 * (size_t)i + k] = g[k];
    if (do_axis) {
        camera_ray_axis<kOpt | kOptCamAxis>(p, ndc[2 * i], ndc[2 * i + 1], r);
        const float a[6] = {r.ox, r.oy, r.oz, r.dx, r.dy, r.dz};
        for (int k = 0; k < 6; ++k) axis[6 * (size_t)i + k] = a[k];
    }
}

// kOptCull tile masks: one thread per (tile, mask word), 32 primitive pairs per word. A pair's bit
// is cleared only if iq_interval.h proves that the reference's tests reject both of its primitives
// for every camera ray of the tile (every pixel, every jitter).
__global__ __launch_bounds__(256) void iqpt_bin_kernel(const kbin b) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t ntiles = (uint64_t)b.ntx * b.nty;
    if (gid >= ntiles * b.stride) return;
    const uint32_t w = (uint32_t)(gid % b.stride);
    const uint32_t tile = (uint32_t)(gid / b.stride);
    const uint32_t tx = tile % b.ntx, ty = tile / b.ntx;
    const uint32_t c0 = tx * kCullTile, c1 = min(c0 + kCullTile, b.ncols) - 1u;
    const uint32_t k0 = ty * kCullTile, k1 = min(k0 + kCullTile, b.nrows) - 1u;
    iqiv::camera_in ci;
    ci.width = b.width;
    ci.height = b.height;
    ci.rcp_width = 0.0f;
    ci.rcp_height = 0.0f;
    ci.inv_proj = b.inv_proj;
    ci.inv_view = b.inv_view;
    ci.cam_const = (int)b.cam_const;
    ci.near_rw = b.cam_near_rw;
    ci.far_rw = b.cam_far_rw;
    const iqiv::bundle bd = iqiv::camera_bundle(ci, b.x0 + c0, b.x0 + c1, b.y0 + k0 * b.ystep, b.y0 + k1 * b.ystep);
    uint32_t bits = 0u;
    if (w < b.wt) {
        for (uint32_t i = 0; i < 32u; ++i) {
            const uint32_t j = w * 32u + i;
            if (2u * j >= b.ntri) break;
            bool culled = bd.ok;
            for (uint32_t e = 0; e < 2u && culled; ++e) {
                const uint32_t k = 2u * j + e;
                if (k >= b.ntri) break;
                const float4_storage* t = b.tris + (size_t)k * kTriFloat4;
                const float v0[3] = {t[0].x, t[0].y, t[0].z};
                const float e1[3] = {t[0].w, t[1].x, t[1].y};
                const float e2[3] = {t[1].z, t[1].w, t[2].x};
                culled = iqiv::tri_culled(bd, v0, e1, e2);
            }
            if (!culled) bits |= 1u << i;
        }
    } else {
        for (uint32_t i = 0; i < 32u; ++i) {
            const uint32_t j = (w - b.wt) * 32u + i;
            if (2u * j >= b.nsph) break;
            bool culled = bd.ok;
            for (uint32_t e = 0; e < 2u && culled; ++e) {
                const uint32_t k = 2u * j + e;
                if (k >= b.nsph) break;
                const float4_storage s = b.spheres[k];
                const float c[3] = {s.x, s.y, s.z};
                culled = iqiv::sphere_culled(bd, c, s.w);
            }
            if (!culled) bits |= 1u << i;
        }
    }
    b.cull[gid] = bits;
}

// Per pixel: certain if its tile has no sphere candidate and one of the tile's candidate triangles is
// accepted by every camera ray of the pixel's own bundle (its jitter square; iq_interval.h tri_certain).
// Under the reference's materials (the runtime launches this only without a material table) every
// sample of such a pixel ends on its first ray with the emissive colour, clamped to (1, 1, 1), after the
// two jitter draws (path_tracer.cu:278, 341-358; camera.cu:24-25). One wave per tile, lane = pixel in the
// tile's storage order (row-major inside the tile); certain[2 t], certain[2 t + 1] = the tile's 64-bit
// mask. Run after iqpt_bin_kernel on the same stream.
// Round 4: also the converse per pixel, certain misses — the pixel's own bundle culls every candidate triangle
// and sphere of its tile (iq_interval.h tri_culled / sphere_culled, the tests the tile masks are built with), so
// every camera ray of the pixel misses everything and ends on the sky gradient (path_tracer.cu:307-316) —
// into certain[2 ntiles + 2 t], certain[2 ntiles + 2 t + 1] (iqpt_sky_kernel's pixels).
// Tiles with more candidate pairs than this are left uncertain (both masks 0: traced as usual): a pixel's
// proofs test up to every candidate, and streamed scenes (round 5) can have thousands per tile (C5's mesh).
constexpr uint32_t kCertainMaxPairs = 96;

__global__ __launch_bounds__(64) void iqpt_certain_kernel(const kbin b, uint32_t* certain) {
    const uint32_t t = blockIdx.x, lane = threadIdx.x;
    const uint32_t* m = b.cull + (size_t)t * b.stride;
    bool sph = false;
    uint32_t ncand = 0;
    for (uint32_t w = 0; w < b.stride; ++w) {
        const uint32_t mw = m[w];
        ncand += (uint32_t)__builtin_popcount(mw);
        if (w >= b.wt) sph = sph || mw != 0u;
    }
    const bool small = ncand <= kCertainMaxPairs;
    const uint32_t tx = t % b.ntx, ty = t / b.ntx;
    const uint32_t tw = min(kCullTile, b.ncols - tx * kCullTile), th = min(kCullTile, b.nrows - ty * kCullTile);
    bool ok = false, miss = false;
    if (lane < tw * th && small) {
        const uint32_t col = tx * kCullTile + lane % tw, row = ty * kCullTile + lane / tw;
        iqiv::camera_in ci;
        ci.width = b.width;
        ci.height = b.height;
        ci.rcp_width = 0.0f;
        ci.rcp_height = 0.0f;
        ci.inv_proj = b.inv_proj;
        ci.inv_view = b.inv_view;
        ci.cam_const = (int)b.cam_const;
        ci.near_rw = b.cam_near_rw;
        ci.far_rw = b.cam_far_rw;
        const uint32_t x = b.x0 + col, y = b.y0 + row * b.ystep;
        const iqiv::bundle bd = iqiv::camera_bundle(ci, x, x, y, y);
        // certain hit: no sphere candidate in the tile, some candidate triangle accepts every ray
        for (uint32_t w = 0; !sph && w < b.wt && bd.ok && !ok; ++w) {
            uint32_t bits = m[w];
            while (bits && !ok) {
                const uint32_t j = w * 32u + (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1u;
                for (uint32_t e = 0; e < 2u && !ok; ++e) {
                    const uint32_t k = 2u * j + e;
                    if (k >= b.ntri) break;
                    const float4_storage* tr = b.tris + (size_t)k * kTriFloat4;
                    const float v0[3] = {tr[0].x, tr[0].y, tr[0].z};
                    const float e1[3] = {tr[0].w, tr[1].x, tr[1].y};
                    const float e2[3] = {tr[1].z, tr[1].w, tr[2].x};
                    ok = iqiv::tri_certain(bd, v0, e1, e2);
                }
            }
        }
        // certain miss: every candidate triangle and sphere of the tile culled for the pixel's own bundle
        miss = bd.ok && !ok;
        for (uint32_t w = 0; w < b.stride && miss; ++w) {
            uint32_t bits = m[w];
            while (bits && miss) {
                const uint32_t j = (w < b.wt ? w : w - b.wt) * 32u + (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1u;
                for (uint32_t e = 0; e < 2u && miss; ++e) {
                    const uint32_t k = 2u * j + e;
                    if (w < b.wt) {
                        if (k >= b.ntri) break;
                        const float4_storage* tr = b.tris + (size_t)k * kTriFloat4;
                        const float v0[3] = {tr[0].x, tr[0].y, tr[0].z};
                        const float e1[3] = {tr[0].w, tr[1].x, tr[1].y};
                        const float e2[3] = {tr[1].z, tr[1].w, tr[2].x};
                        miss = iqiv::tri_culled(bd, v0, e1, e2);
                    } else {
                        if (k >= b.nsph) break;
                        const float4_storage sp = b.spheres[k];
                        const float c[3] = {sp.x, sp.y, sp.z};
                        miss = iqiv::sphere_culled(bd, c, sp.w);
                    }
                }
            }
        }
    }
    const uint64_t mask = __ballot(ok), miss_mask = __ballot(miss);
    if (lane == 0) {
        const size_t nt = (size_t)b.ntx * b.nty;
        certain[2 * (size_t)t] = (uint32_t)mask;
        certain[2 * (size_t)t + 1] = (uint32_t)(mask >> 32);
        certain[2 * nt + 2 * (size_t)t] = (uint32_t)miss_mask;
        certain[2 * nt + 2 * (size_t)t + 1] = (uint32_t)(miss_mask >> 32);
    }
}

// Per tile: candidate triangle pairs and sphere pairs of its masks (the queue-order cost and the
// sizes of the candidate lists).
__global__ __launch_bounds__(256) void iqpt_tile_count_kernel(const uint32_t* cull, uint32_t ntiles, uint32_t wt,
                                                              uint32_t stride, uint32_t* cnt_tri, uint32_t* cnt_sph) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= ntiles) return;
    const uint32_t* m = cull + (size_t)t * stride;
    uint32_t a = 0, b = 0;
    for (uint32_t w = 0; w < stride; ++w) {
        if (w < wt) a += (uint32_t)__popc(m[w]);
        else b += (uint32_t)__popc(m[w]);
    }
    cnt_tri[t] = a;
    cnt_sph[t] = b;
}

// Candidate lists: the set bits of each tile's masks as ascending pair indices, triangle pairs at
// off_tri[t], sphere pairs at off_sph[t] (exclusive prefix sums of the counts).
__global__ __launch_bounds__(256) void iqpt_tile_list_kernel(const uint32_t* cull, uint32_t ntiles, uint32_t wt,
                                                             uint32_t stride, const uint32_t* off_tri,
                                                             const uint32_t* off_sph, uint32_t* list) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= ntiles) return;
    const uint32_t* m = cull + (size_t)t * stride;
    uint32_t o = off_tri[t];
    for (uint32_t w = 0; w < wt; ++w)
        for (uint32_t b = m[w]; b; b &= b - 1u) list[o++] = w * 32u + (uint32_t)__builtin_ctz(b);
    o = off_sph[t];
    for (uint32_t w = wt; w < stride; ++w)
        for (uint32_t b = m[w]; b; b &= b - 1u) list[o++] = (w - wt) * 32u + (uint32_t)__builtin_ctz(b);
}

// Any-hit scenes (kparams::anyhit: no sphere, every triangle emissive), round 5: a ray's result is whether some
// triangle accepts it, so the order in which a tile's candidate list is tested changes no bit — only how soon every
// lane of a wave has its hit and the wave leaves the list (the candidate-list loop of iqpt_render_kernel). One
// wave per tile: each lane casts its pixel's central ray (a plain float camera: the score is a heuristic) at every
// candidate pair of the tile, the pair's score is how many of the tile's lanes it hits, and the list is reordered
// by descending score (ties: ascending index). Lists longer than kOrderMax keep their ascending order.
constexpr uint32_t kOrderMax = 1024;

__global__ __launch_bounds__(64) void iqpt_tile_list_order_kernel(const kbin b, const uint32_t* off_tri, uint32_t* list) {
    __shared__ uint32_t sc[kOrderMax];
    __shared__ uint32_t ix[kOrderMax];
    const uint32_t t = blockIdx.x, lane = threadIdx.x;
    const uint32_t a0 = off_tri[t], a1 = off_tri[t + 1];
    const uint32_t n = a1 - a0;
    if (n < 2u || n > kOrderMax) return;
    const uint32_t tx = t % b.ntx, ty = t / b.ntx;
    const uint32_t tw = min(kCullTile, b.ncols - tx * kCullTile), th = min(kCullTile, b.nrows - ty * kCullTile);
    const bool inside = lane < tw * th;
    const float x = (float)(b.x0 + tx * kCullTile + (inside ? lane % tw : 0u)) + 0.5f;
    const float y = (float)(b.y0 + (ty * kCullTile + (inside ? lane / tw : 0u)) * b.ystep) + 0.5f;
    const float xn = x / (float)b.width * 2.0f - 1.0f, yn = 1.0f - y / (float)b.height * 2.0f;
    const float* P = b.inv_proj;
    const float* V = b.inv_view;
    float nr[4], fr[4];
    for (int c = 0; c < 4; ++c) {
        nr[c] = xn * P[c] + yn * P[4 + c] + P[12 + c];
        fr[c] = xn * P[c] + yn * P[4 + c] + P[8 + c] + P[12 + c];
    }
    float o[3], f[3];
    for (int c = 0; c < 3; ++c) {
        const float nx = nr[0] / nr[3], ny = nr[1] / nr[3], nz = nr[2] / nr[3];
        const float fx = fr[0] / fr[3], fy = fr[1] / fr[3], fz = fr[2] / fr[3];
        o[c] = nx * V[c] + ny * V[4 + c] + nz * V[8 + c] + V[12 + c];
        f[c] = fx * V[c] + fy * V[4 + c] + fz * V[8 + c] + V[12 + c];
    }
    float d[3] = {f[0] - o[0], f[1] - o[1], f[2] - o[2]};
    const float il = 1.0f / sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    d[0] *= il;
    d[1] *= il;
    d[2] *= il;
    for (uint32_t e = 0; e < n; ++e) {
        const uint32_t j = list[a0 + e];
        bool hit = false;
        for (uint32_t h = 0; h < 2u && inside; ++h) {
            const uint32_t kk = 2u * j + h;
            if (kk >= b.ntri) break;
            const float4_storage* tr = b.tris + (size_t)kk * kTriFloat4;
            const float e1[3] = {tr[0].w, tr[1].x, tr[1].y}, e2[3] = {tr[1].z, tr[1].w, tr[2].x};
            const float pv[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
            const float det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
            if (fabsf(det) < 1e-9f) continue;
            const float inv = 1.0f / det;
            const float tv[3] = {o[0] - tr[0].x, o[1] - tr[0].y, o[2] - tr[0].z};
            const float u = (tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2]) * inv;
            const float qv[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2], tv[0] * e1[1] - tv[1] * e1[0]};
            const float v = (d[0] * qv[0] + d[1] * qv[1] + d[2] * qv[2]) * inv;
            const float tt = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * inv;
            hit = hit || (u >= 0.0f && v >= 0.0f && u + v <= 1.0f && tt > 0.0f);
        }
        const uint32_t s = (uint32_t)__popcll(__ballot(hit));
        if (lane == 0) {
            sc[e] = s;
            ix[e] = j;
        }
    }
    __syncthreads();
    // rank by (score descending, position ascending): a permutation of [0, n)
    for (uint32_t e = lane; e < n; e += 64u) {
        const uint32_t s = sc[e];
        uint32_t r = 0;
        for (uint32_t q = 0; q < n; ++q) r += (sc[q] > s || (sc[q] == s && q < e)) ? 1u : 0u;
        list[a0 + r] = ix[e];
    }
}

// Per-pixel candidate masks over a tile's triangle list (round 6, kparams::pmask). A pixel's camera rays (its own
// jitter square) meet far fewer of the tile's candidates than the whole tile does — a streamed scene's silhouette
// and pole tiles hold long lists that every miss ray of the tile tests to the end. One wave per tile, lane = pixel in
// the tile's storage order; bit e of the lane's word w is set unless iq_interval.h proves that the reference's tests
// reject both triangles of list entry 32 w + e for every camera ray of the pixel (tri_culled, the tests the tile
// masks are built with). Skipping a cleared entry changes no result: the entry is rejected by that ray anyway, and
// the set entries keep the list's order. Tiles with more than kPixMaskMax entries are left without masks; a tile's
// words start at pmask_off[t] (64 per 32 entries, compact over the tiles). Also per pixel: whether one of its
// candidates accepts every camera ray of the pixel (tri_certain; certain[2 t], certain[2 t + 1]: the tile's 64-bit
// mask), for iqpt_anyhit_kernel.
__global__ __launch_bounds__(64) void iqpt_pixel_mask_kernel(const kbin b, const uint32_t* off_tri, const uint32_t* list,
                                                             const uint32_t* pmask_off, uint32_t* pmask,
                                                             uint32_t* certain) {
    const uint32_t t = blockIdx.x, lane = threadIdx.x;
    const uint32_t a = off_tri[t], n = off_tri[t + 1] - a;
    if (n > kPixMaskMax) {
        if (lane == 0) {
            certain[2 * (size_t)t] = 0u;
            certain[2 * (size_t)t + 1] = 0u;
        }
        return;
    }
    const uint32_t tx = t % b.ntx, ty = t / b.ntx;
    const uint32_t tw = min(kCullTile, b.ncols - tx * kCullTile), th = min(kCullTile, b.nrows - ty * kCullTile);
    const bool inside = lane < tw * th;
    iqiv::bundle bd;
    bd.ok = false;
    if (inside) {
        iqiv::camera_in ci;
        ci.width = b.width;
        ci.height = b.height;
        ci.rcp_width = 0.0f;
        ci.rcp_height = 0.0f;
        ci.inv_proj = b.inv_proj;
        ci.inv_view = b.inv_view;
        ci.cam_const = (int)b.cam_const;
        ci.near_rw = b.cam_near_rw;
        ci.far_rw = b.cam_far_rw;
        const uint32_t x = b.x0 + tx * kCullTile + lane % tw, y = b.y0 + (ty * kCullTile + lane / tw) * b.ystep;
        bd = iqiv::camera_bundle(ci, x, x, y, y);
    }
    uint32_t* out = pmask + pmask_off[t] + lane;
    bool sure = false;
    for (uint32_t w = 0; w * 32u < n; ++w) {
        uint32_t bits = 0u;
        for (uint32_t i = 0; i < 32u && inside; ++i) {
            const uint32_t e = w * 32u + i;
            if (e >= n) break;
            const uint32_t j = list[a + e];
            bool culled = bd.ok;
            for (uint32_t h = 0; h < 2u && culled; ++h) {
                const uint32_t k = 2u * j + h;
                if (k >= b.ntri) break;
                const float4_storage* tr = b.tris + (size_t)k * kTriFloat4;
                const float v0[3] = {tr[0].x, tr[0].y, tr[0].z};
                const float e1[3] = {tr[0].w, tr[1].x, tr[1].y};
                const float e2[3] = {tr[1].z, tr[1].w, tr[2].x};
                culled = iqiv::tri_culled(bd, v0, e1, e2);
                if (!culled && !sure) sure = iqiv::tri_certain(bd, v0, e1, e2);
            }
            if (!culled) bits |= 1u << i;
        }
        out[(size_t)w * 64u] = bits;
    }
    const uint64_t sm = __ballot(sure);
    if (lane == 0) {
        certain[2 * (size_t)t] = (uint32_t)sm;
        certain[2 * (size_t)t + 1] = (uint32_t)(sm >> 32);
    }
}

// Compact row-major <-> tile-major reorder of pixel-state planes (one thread per 32-bit word).
__global__ __launch_bounds__(256) void iqpt_relayout_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                            uint32_t ncols, uint32_t nrows, uint32_t words,
                                                            uint32_t planes, int to_compact) {
    const uint64_t npix = (uint64_t)ncols * nrows;
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= npix * words * planes) return;
    const uint64_t plane = i / (npix * words);
    const uint64_t e = i - plane * npix * words;
    const uint32_t c = (uint32_t)(e / words), k = (uint32_t)(e % words);   // compact pixel, word
    const uint32_t s = tile_store_index(c % ncols, c / ncols, ncols, nrows);
    const uint64_t ci = plane * npix * words + (uint64_t)c * words + k;
    const uint64_t si = plane * npix * words + (uint64_t)s * words + k;
    if (to_compact) dst[ci] = src[si];
    else dst[si] = src[ci];
}

// Multi-GPU frame assembly on the gather's root: the gathered buffer holds, per rank r <
// world, `stride` pixels of `words` words — rank r's rows b + r, b + r + S, ... of an S-way cyclic split in
// compact row-major order — and row k of rank r is row b + r + k S of the W x H frame (S = world and b = 0
// on a real node; a one-rank rehearsal of an S-way share, rank 0 owning rows b + k S, writes those rows
// only). One thread per gathered word.
__global__ __launch_bounds__(256) void iqpt_assemble_rows_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                                 uint32_t width, uint32_t height, uint32_t world,
                                                                 uint32_t split, uint32_t base, uint64_t stride,
                                                                 uint32_t words) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= (uint64_t)world * stride * words) return;
    const uint64_t blk = stride * words;
    const uint32_t r = (uint32_t)(i / blk);
    const uint64_t e = i - (uint64_t)r * blk;
    const uint64_t px = e / words;
    const uint32_t row = (uint32_t)(px / width), x = (uint32_t)(px - (uint64_t)row * width);
    const uint64_t y = (uint64_t)base + r + (uint64_t)row * split;
    if (y >= height) return;                          // padding past this rank's last row
    dst[(y * width + x) * words + (e - px * words)] = src[i];
}

// curand_init(seed, global pixel id, 0) per owned pixel (renderer_init_kernel, path_tracer.cu:36-46).
__global__ __launch_bounds__(256) void iqpt_rng_init_kernel(uint32_t width, uint32_t x0, uint32_t ncols,
                                                            uint32_t y0, uint32_t ystep, uint32_t nrows,
                                                            uint64_t seed, const uint32_t* __restrict__ tables,
                                                            uint32_t* __restrict__ rng) {
    const uint32_t npix = ncols * nrows;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;     // tile-major storage index
    if (p >= npix) return;
    uint32_t col, row;
    tile_decode(p, ncols, nrows, &col, &row);
    const uint32_t x = x0 + col;
    const uint32_t y = y0 + row * ystep;
    const uint64_t pid = (uint64_t)y * width + x;
    iq_xorwow_state s;
    iq_xorwow_seed(seed, &s);
    uint64_t sub = pid;
    for (int i = 0; i < 32 && sub; ++i, sub >>= 1) {
        if (sub & 1u) iq_gf2_matvec(tables + i * IQ_XORWOW_MAT_WORDS, s.v);
    }
    rng[p] = s.v[0];
    rng[(size_t)npix + p] = s.v[1];
    rng[2 * (size_t)npix + p] = s.v[2];
    rng[3 * (size_t)npix + p] = s.v[3];
    rng[4 * (size_t)npix + p] = s.v[4];
    rng[5 * (size_t)npix + p] = s.d;
}

// ---------------------------------------------------------------------------------------------
// kOptSplit: sample-parallel evaluation of a pixel's chain of samples.
//
// A pixel's samples are one sequential XORWOW stream (path_tracer.cu:339): sample k starts where
// sample k-1's draws ended, and a sample takes 2 draws (camera, random.cu:66-70 via camera.cu:24-25)
// plus 2 per Oren-Nayar scatter (random.cu:96-107). Every sample therefore starts at an EVEN offset
// of the stream, and what a sample does from offset 2j depends on j alone. Round 1 evaluates a
// sample at every even offset ("slot") j of a window [0, M) in parallel — a wave streams through one
// pixel's slots, one slot per lane, so its lanes trace nearly the same paths — recording the clamped
// colour and the slots consumed; the stitch then walks the chain 0 -> j + n_j -> ... in order,
// applying the running mean exactly as the plain kernel does. Slots off the chain (offsets inside
// some sample's scatter draws) are wasted work; a chain that leaves the window is finished by an
// anchored lane in round 2.
//
// The stitch: the chain of every split slot through its window, the running mean of
// path_tracer.cu:356-358 in sample order (the plain kernel's table values and mean_terms), the ray
// count (path_tracer.cu:252-318: a slot's rays are its slots consumed, or max_depth when it ended on
// a scatter at max_depth), and the RNG state where the chain stopped (the pixel's state before the
// launch advanced two draws per slot). Complete chains store the pixel as the plain kernel does; the
// others go to the leftover list for round 2. The walk reads the slot counts 16 at a time (one
// 16-byte load per 16 slots) and the colours of 8 chain samples at once, so the loads of a batch are
// in flight together.
// Before round 1: per split slot, heavy (no history, or >= heavy_rho slots per sample last launch) or
// light; a heavy pixel's window M (split_window), the RNG states at slots 0, R, 2R, ... < M (planes
// 0 ..) and at M (plane g_max); M = 0 marks a light pixel. A wave is one split tile (64 slots): it
// appends the tile's non-empty run chunks (r < ceil(max M / R)) to the round-1 chunk list.
__device__ __forceinline__ uint32_t split_prep_slot(const ksplit& s, uint32_t sp, uint32_t pix) {
    const uint32_t rho = s.sp_rho[sp];
    if (rho != 0u && rho < s.heavy_rho) {
        s.sp_win[sp] = 0u;
        return 0u;
    }
    const uint32_t M = split_window(rho, s.spp, s.m_cap), R = s.run_len;
    rng6 st = {s.rng[pix], s.rng[(size_t)s.npix + pix], s.rng[2 * (size_t)s.npix + pix],
               s.rng[3 * (size_t)s.npix + pix], s.rng[4 * (size_t)s.npix + pix], s.rng[5 * (size_t)s.npix + pix]};
    auto put = [&](uint32_t r) {
        const size_t pl = (size_t)r * 6u * s.ns_cap + sp;
        s.run_st[pl] = st.v0;
        s.run_st[pl + s.ns_cap] = st.v1;
        s.run_st[pl + 2 * (size_t)s.ns_cap] = st.v2;
        s.run_st[pl + 3 * (size_t)s.ns_cap] = st.v3;
        s.run_st[pl + 4 * (size_t)s.ns_cap] = st.v4;
        s.run_st[pl + 5 * (size_t)s.ns_cap] = st.d;
    };
    for (uint32_t j = 0; j < M; ++j) {
        if (j % R == 0u) put(j / R);
        (void)xorwow_next(st);
        (void)xorwow_next(st);
    }
    put(s.g_max);
    s.sp_win[sp] = M;
    return (M + R - 1u) / R;
}

__global__ __launch_bounds__(256) void iqpt_split_prep_kernel(const ksplit s) {
    const uint32_t sp = blockIdx.x * 256u + threadIdx.x;          // ns_cap is a multiple of 64
    const uint32_t pix = sp < s.ns_cap ? s.sp_pix[sp] : ~0u;
    uint32_t g = pix != ~0u ? split_prep_slot(s, sp, pix) : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) g = max(g, (uint32_t)__shfl_xor((int)g, off));
    uint32_t base = 0;
    if (__lane_id() == 0 && g) base = atomicAdd(s.chunk_count, g);
    base = (uint32_t)__shfl((int)base, 0);
    const uint32_t st = sp / kQueueChunk;
    for (uint32_t r = __lane_id(); r < g; r += 64u) {
        s.chunks[2 * (size_t)(base + r)] = s.split_tiles[st];
        s.chunks[2 * (size_t)(base + r) + 1] = st | (r << 23);
    }
}

template <int OPT>
__global__ __launch_bounds__(kStitchBlock) void iqpt_split_stitch_kernel(const ksplit s) {
    __shared__ float2 tab[kAccTableMax];
    __shared__ float tab_n[kAccTableMax];
    for (uint32_t k = threadIdx.x; k < s.spp; k += kStitchBlock) {
        const uint64_t n = s.frame0 + k + 1;
        tab[k] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
        tab_n[k] = (float)n;
    }
    __syncthreads();
    const uint32_t sp = blockIdx.x * kStitchBlock + threadIdx.x;
    uint32_t pix = ~0u;
    if (sp < s.ns_cap) pix = s.sp_pix[sp];
    unsigned long long rays = 0;
    const uint32_t M = pix != ~0u ? s.sp_win[sp] : 0u;   // 0: a light pixel, done in round 1
    if (M != 0u) {
        const float4_storage a = s.lin[pix];
        float ax = a.x, ay = a.y, az = a.z;
        uint32_t k = 0, j = 0;
        const float4* res = reinterpret_cast<const float4*>(s.res) + (size_t)sp * s.m_cap;
        const uint8_t* nr = s.nres + (size_t)sp * s.m_cap;     // m_cap is a multiple of 16
        uint32_t nbase = ~0u;
        uint4 nb = make_uint4(0u, 0u, 0u, 0u);
        constexpr int kBatch = 8;
        while (k < s.spp && j < M) {
            uint32_t cj[kBatch], cn[kBatch];
            int cnt = 0;
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                cj[b] = 0u;
                cn[b] = 0u;
                if (k + (uint32_t)b < s.spp && j < M) {
                    if ((j & ~15u) != nbase) {
                        nbase = j & ~15u;
                        nb = *reinterpret_cast<const uint4*>(nr + nbase);
                    }
                    const uint32_t o = j - nbase, w = o >> 2;
                    const uint32_t word = w == 0u ? nb.x : (w == 1u ? nb.y : (w == 2u ? nb.z : nb.w));
                    cj[b] = j;
                    cn[b] = (word >> ((o & 3u) * 8u)) & 0xffu;
                    j += cn[b];
                    cnt = b + 1;
                }
            }
            float4 v[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (b < cnt) v[b] = res[cj[b]];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                if (b < cnt) {
                    const float2 tv = tab[k];
                    float qx, qy, qz;
                    mean_terms<OPT>(v[b].x, v[b].y, v[b].z, tab_n[k], tv.x, s.mean_tiny, qx, qy, qz);
                    ax = qx + ax * tv.y;
                    ay = qy + ay * tv.y;
                    az = qz + az * tv.y;
                    rays += (cn[b] - 1u == (uint32_t)s.max_depth) ? (uint32_t)s.max_depth : cn[b];
                    ++k;
                }
            }
        }
        // the RNG state at slot j: from the nearest stored state at or below it
        uint32_t plane, steps;
        if (j >= M) {
            plane = s.g_max;
            steps = j - M;
        } else {
            plane = j / s.run_len;
            steps = j - plane * s.run_len;
        }
        const size_t pl = (size_t)plane * 6u * s.ns_cap + sp;
        rng6 st = {s.run_st[pl], s.run_st[pl + s.ns_cap], s.run_st[pl + 2 * (size_t)s.ns_cap],
                   s.run_st[pl + 3 * (size_t)s.ns_cap], s.run_st[pl + 4 * (size_t)s.ns_cap],
                   s.run_st[pl + 5 * (size_t)s.ns_cap]};
        for (uint32_t i = 0; i < steps; ++i) {
            (void)xorwow_next(st);
            (void)xorwow_next(st);
        }
        if (k == s.spp) {
            const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
            const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
            const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
            s.bgra[tile_to_compact(pix, s.ncols, s.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
            reinterpret_cast<float4*>(s.lin)[pix] = make_float4(ax, ay, az, 0.0f);
            s.rng[pix] = st.v0;
            s.rng[(size_t)s.npix + pix] = st.v1;
            s.rng[2 * (size_t)s.npix + pix] = st.v2;
            s.rng[3 * (size_t)s.npix + pix] = st.v3;
            s.rng[4 * (size_t)s.npix + pix] = st.v4;
            s.rng[5 * (size_t)s.npix + pix] = st.d;
            s.sp_rho[sp] = (uint32_t)(((uint64_t)j * 256u) / s.spp);
        } else {
            s.sp_st[sp] = st.v0;
            s.sp_st[(size_t)s.ns_cap + sp] = st.v1;
            s.sp_st[2 * (size_t)s.ns_cap + sp] = st.v2;
            s.sp_st[3 * (size_t)s.ns_cap + sp] = st.v3;
            s.sp_st[4 * (size_t)s.ns_cap + sp] = st.v4;
            s.sp_st[5 * (size_t)s.ns_cap + sp] = st.d;
            reinterpret_cast<float4*>(s.sp_acc)[sp] = make_float4(ax, ay, az, __uint_as_float(k));
            s.left[atomicAdd(s.left_count, 1u)] = sp;
            // the chain's rate so far (k >= 1: the window holds at least spp slots)
            s.sp_rho[sp] = (uint32_t)(((uint64_t)j * 256u) / (k ? k : 1u));
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
    if (__lane_id() == 0 && rays) add_rays(s.rays, rays);
}

// ------------------------------------------------------------------------------------------------
// Sample-parallel anchored tiles (iqpt_fan_kernel). A tile whose camera rays cannot
// reach a sphere (no sphere bit in its §3.3 mask) under the reference's materials (every triangle
// emissive, path_tracer.cu:248-249, 278) ends every path on its first ray: an emissive hit or the sky
// (path_tracer.cu:297-316). Every sample of such a pixel takes exactly the two jitter draws of
// camera::get_ray (camera.cu:24-25), so sample k starts at stream offset 2k with certainty, and the
// samples of a pixel are independent but for the ordered running mean (path_tracer.cu:356-358).
// One block = one 8x8 tile = four waves, lane = pixel in every wave: wave w evaluates a contiguous range
// of samples of each chunk of C <= 64 samples from the state 2 s draws into the pixel's stream (stepped
// there once per chunk), and leaves per sample a triangle-hit bit (a ballot) and the sky parameter
// a = (dir.y + 1) / 2 in LDS; wave 0 then folds the chunk in sample order with the plain kernel's table
// values and mean_terms. The ranges (fan_range) are sized so that wave 0's fold and the later waves'
// stream stepping even out the four waves' instruction counts. The pixel's chain is 16 samples per lane instead of 64, and no
// sample is evaluated that the pixel does not use. Same bits as the plain kernel: the same camera
// ray, the tile's mask pairs in index order (no sphere candidate: no sphere test), the same colour,
// clamp and mean, the state 2 spp draws on, spp rays per pixel.
constexpr uint32_t kFanBlock = 256;                    // four waves, one tile
constexpr uint32_t kFanChunk = 64;                     // samples per chunk (LDS: [chunk][pixel])

// First sample of wave w's range in a chunk of cn samples: 0, 20 %, 47 %, 73 % of the chunk (wave 0 also
// folds the chunk, about a twentieth of a sample per fold of a triangle hit; a later wave first steps 2 s
// draws, about 7 % of a sample per sample skipped), so that the four ranges cost about the same.
__device__ __forceinline__ uint32_t fan_range(uint32_t cn, uint32_t w) {
    return w == 0u ? 0u : (w == 1u ? (cn * 13u) / 64u : (w == 2u ? (cn * 30u) / 64u : (w == 3u ? (cn * 47u) / 64u : cn)));
}

__host__ __device__ inline uint32_t fan_lds_bytes(uint32_t ntri_pairs, uint32_t spp) {
    return ntri_pairs * kTriPairFloat4 * 16u + ((spp + 1u) & ~1u) * 8u + ((spp + 3u) & ~3u) * 4u + 16u * 4u +
           kFanChunk * 64u * 4u + kFanChunk * 8u;
}

template <int OPT>
__device__ __forceinline__ void fan_body(const kparams& p, uint32_t bid) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    float4* lds_tri = lds;
    float2* lds_tab = reinterpret_cast<float2*>(lds_tri + (size_t)p.ntri_pairs * kTriPairFloat4);
    float* lds_tab_n = reinterpret_cast<float*>(lds_tab + ((p.spp + 1u) & ~1u));
    uint32_t* lds_mask = reinterpret_cast<uint32_t*>(lds_tab_n + ((p.spp + 3u) & ~3u));   // the tile's words
    float* lds_sky = reinterpret_cast<float*>(lds_mask + 16);                             // [sample][lane]
    uint64_t* lds_hit = reinterpret_cast<uint64_t*>(lds_sky + kFanChunk * 64u);           // [sample]

    const uint32_t t = p.tile_order[bid];
    for (uint32_t i = threadIdx.x; i < p.ntri_pairs * kTriPairFloat4; i += kFanBlock)
        lds_tri[i] = reinterpret_cast<const float4*>(p.tri_pairs)[i];
    for (uint32_t s = threadIdx.x; s < p.spp; s += kFanBlock) {
        const uint64_t n = p.frame0 + s + 1;
        lds_tab[s] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
        lds_tab_n[s] = (float)n;
    }
    if (threadIdx.x < p.cull_wt) lds_mask[threadIdx.x] = p.cull[(size_t)t * p.cull_stride + threadIdx.x];
    __syncthreads();

    const uint32_t lane = __lane_id(), wave = threadIdx.x / 64u;
    const uint32_t tx = t % p.ntx, ty = t / p.ntx;
    const uint32_t th = min(kCullTile, p.nrows - ty * kCullTile), tw = min(kCullTile, p.ncols - tx * kCullTile);
    const uint32_t npt = tw * th;
    const bool inside = lane < npt;                     // partial tiles at the right / bottom edge
    // the pixels of this tile the fan kernel owns (chain launches: the others are the chain kernel's)
    const uint64_t own = p.fan_lanes ? p.fan_lanes[bid] : ~0ull;
    const bool has = inside && ((own >> lane) & 1ull);
    const uint32_t pix = ty * kCullTile * p.ncols + tx * kCullTile * th + (inside ? lane : 0u);
    const uint32_t px = p.x0 + tx * kCullTile + (inside ? lane % tw : 0u);
    const uint32_t py = p.y0 + (ty * kCullTile + (inside ? lane / tw : 0u)) * p.ystep;
    rng6 st = {p.rng[pix], p.rng[(size_t)p.npix + pix], p.rng[2 * (size_t)p.npix + pix],
               p.rng[3 * (size_t)p.npix + pix], p.rng[4 * (size_t)p.npix + pix], p.rng[5 * (size_t)p.npix + pix]};
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    if (wave == 0) {
        const float* a = reinterpret_cast<const float*>(p.lin + pix);
        ax = a[0];
        ay = a[1];
        az = a[2];
    }
    const uint64_t valid = (npt == 64u ? ~0ull : ((1ull << npt) - 1ull)) & own;
    const uint64_t cmask = p.certain != nullptr
                               ? ((uint64_t)p.certain[2 * (size_t)t] | ((uint64_t)p.certain[2 * (size_t)t + 1] << 32))
                               : 0ull;
    if ((cmask & valid) == valid) {
        // a certain tile (kparams::certain) — every pixel of it this kernel owns is certain (the others are the
        // sky kernel's): every sample takes the camera's two draws and ends on an emissive triangle, clamped
        // colour (1, 1, 1), whose mean term c / n is the table's RN(1 / n); wave 0 folds the launch's samples
        // in order, the other waves have nothing to do
        if (wave == 0 && has) {
            xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, 2u * p.spp);
            st.d += 2u * p.spp * IQ_XORWOW_WEYL;
            for (uint32_t k = 0; k < p.spp; ++k) {
                const float2 tv = lds_tab[k];
                ax = tv.x + ax * tv.y;
                ay = tv.x + ay * tv.y;
                az = tv.x + az * tv.y;
            }
            p.rng[pix] = st.v0;
            p.rng[(size_t)p.npix + pix] = st.v1;
            p.rng[2 * (size_t)p.npix + pix] = st.v2;
            p.rng[3 * (size_t)p.npix + pix] = st.v3;
            p.rng[4 * (size_t)p.npix + pix] = st.v4;
            p.rng[5 * (size_t)p.npix + pix] = st.d;
            const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
            const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
            const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
            p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
            reinterpret_cast<float4*>(p.lin)[pix] = make_float4(ax, ay, az, 0.0f);
        }
        if (threadIdx.x == 0)
            add_rays(p.rays, (unsigned long long)__popcll(own & (npt == 64u ? ~0ull : ((1ull << npt) - 1ull))) * p.spp);
        return;
    }
    const uint32_t tp = (p.ntri + 1) / 2;
    uint32_t pos = 0;                                   // samples whose draws this lane's state has passed

    for (uint32_t c0 = 0; c0 < p.spp; c0 += kFanChunk) {
        const uint32_t cn = min(kFanChunk, p.spp - c0);
        const uint32_t s0 = c0 + fan_range(cn, wave), s1 = c0 + fan_range(cn, wave + 1u);
        // to sample s0: 2 (s0 - pos) draws (d follows from the count)
        xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, 2u * (s0 - pos));
        st.d += 2u * (s0 - pos) * IQ_XORWOW_WEYL;
        for (uint32_t s = s0; s < s1; ++s) {
            ray3 ray;
            camera_ray<OPT>(p, px, py, st, ray);
            // the tile's candidate pairs in index order (path_tracer.cu:257-275); the lane's pixel has no
            // sphere candidate (its tile's mask, or its own bundle in chain launches), so no sphere test can
            // accept (iq_interval.h). Every triangle is emissive, so the sample's colour depends only on whether
            // some triangle is accepted, not on which (path_tracer.cu:278, material.cu:50-57): a lane stops at
            // its first accepted triangle (accepted against the initial closest, as the first acceptance of the
            // reference's loop is), the wave when every lane has one
            float closest = kTMax;
            int kind = kHitNone;
            uint32_t hidx = 0;
            for (uint32_t w = 0; w * 32u < tp; ++w) {
                uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_mask[w]);
                while (m && __any(kind != kHitTri)) {
                    const uint32_t j = w * 32u + (uint32_t)__builtin_ctz(m);
                    m &= m - 1u;
                    if (j >= tp) break;
                    if (kind != kHitTri) {
                        const float4* q = lds_tri + (size_t)j * kTriPairFloat4;
                        test_triangle_pair<OPT>(q[0], q[1], q[2], q[3], q[4], ray, closest, kind, hidx, 2 * j,
                                                2 * j + 1 < p.ntri);
                    }
                }
            }
            const uint64_t hit = __ballot(kind == kHitTri);
            if (lane == 0) lds_hit[s - c0] = hit;
            lds_sky[(s - c0) * 64u + lane] = (ray.dy + 1.0f) * 0.5f;   // sky gradient parameter (:308-313)
        }
        pos = s1;
        __syncthreads();
        if (wave == 0) {
            // the running mean in sample order (path_tracer.cu:341-358): an emissive hit is 10 clamped to 1
            for (uint32_t k = 0; k < cn; ++k) {
                const float2 tv = lds_tab[c0 + k];
                float qx, qy, qz;
                if ((lds_hit[k] >> lane) & 1ull) {
                    // c = (1, 1, 1): c / n = RN(1 / n), the table's rc, in every channel (mean_terms)
                    qx = tv.x;
                    qy = tv.x;
                    qz = tv.x;
                } else {
                    const float a = lds_sky[k * 64u + lane];
                    const float one_a = 1.0f - a;
                    float cx = one_a + a * 0.5f;
                    float cy = one_a + a * 0.7f;
                    float cz = one_a + a * 1.0f;
                    cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
                    cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
                    cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
                    mean_terms<OPT>(0.0f + cx, 0.0f + cy, 0.0f + cz, lds_tab_n[c0 + k], tv.x, p.mean_tiny, qx, qy, qz);
                }
                ax = qx + ax * tv.y;
                ay = qy + ay * tv.y;
                az = qz + az * tv.y;
            }
        }
        __syncthreads();
    }
    if (has) {
        if (pos == p.spp) {
            // the lane whose last sample is the launch's last: its state is 2 spp draws on
            p.rng[pix] = st.v0;
            p.rng[(size_t)p.npix + pix] = st.v1;
            p.rng[2 * (size_t)p.npix + pix] = st.v2;
            p.rng[3 * (size_t)p.npix + pix] = st.v3;
            p.rng[4 * (size_t)p.npix + pix] = st.v4;
            p.rng[5 * (size_t)p.npix + pix] = st.d;
        }
        if (wave == 0) {
            const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
            const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
            const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
            p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
            reinterpret_cast<float4*>(p.lin)[pix] = make_float4(ax, ay, az, 0.0f);
        }
    }
    if (threadIdx.x == 0)   // one query per sample
        add_rays(p.rays, (unsigned long long)__popcll(own & (npt == 64u ? ~0ull : ((1ull << npt) - 1ull))) * p.spp);
}

// ------------------------------------------------------------------------------------------------
// Slot-parallel sphere pixels (IQPT_SPLIT_SPEC). Only the pixels whose own camera-ray
// bundle may reach a sphere take more than one slot per sample, so only their chains need speculation.
// Sample k of a pixel starts where sample k - 1's draws ended (path_tracer.cu:339): 2 draws for the
// jitter (camera.cu:24-25) plus 2 per Oren-Nayar scatter (material.cu:10), and what a sample does from
// stream offset 2j ("slot" j) depends on j alone. One kernel, L = 8, 16, 32 or 64 lanes per sphere pixel
// (16 without a plan; a plan gives the pixels with the most work per lane more lanes, runtime):
//  * slots: the pixel's window of M slots (its last chain's slots per sample, spec_window) is cut into L
//    ranges; each lane steps its state to its range's first slot and traces the range's slots back to
//    back (the next slot's state is the one the current slot's camera draws leave), one ray per live lane
//    per iteration; colours go to HBM, the slot counts to LDS;
//  * walk: one lane per pixel follows the chain 0 -> j + n_j -> ... in LDS, a batch of chain samples at a
//    time; the pixel's lanes gather their colours, form the mean terms with the plain kernel's table
//    values and count each sample's rays (its slots, or max_depth when it ended on a scatter at
//    max_depth), and the walker folds the terms in sample order (path_tracer.cu:356-358); a chain that
//    leaves its window continues in a new window (another round).
// Same bits as the plain kernel: the same per-sample code, the same mean terms, the chain's own slots as
// rays, the state where the chain stops.
// Wave-synchronous step: every lane of the wave is past its earlier LDS writes before any reads after it
// (LDS operations of one wave complete in order; the fences keep the compiler from moving accesses across).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kSpecBlock = 256;
constexpr uint32_t kSpecLanes = 16;                    // lanes per sphere pixel without a plan
constexpr uint32_t kSpecPix = kSpecBlock / kSpecLanes; // sphere pixels per block without a plan
constexpr uint32_t kSpecMaxPix = 32;                   // pixels per block at 8 lanes each
constexpr uint32_t kSpecBatch = 512;                   // walk: chain samples gathered per block and batch
static_assert(kSpecPix == kSpecPixPerBlock && kSpecMaxPix == kSpecMaxPixPerBlock, "runtime and kernel agree on the spec block");

// Scatter records a spec lane keeps: one per bounce that continues (depth + 1 < max_depth); the last scatter
// ends the sample without a record. max_depth - 1 of them (not max_depth) keeps a C2 block at 31.9 KB of LDS,
// 5 blocks per CU instead of 4.
__host__ __device__ inline uint32_t spec_stack_depth(int max_depth) { return max_depth > 2 ? (uint32_t)(max_depth - 1) : 1u; }

__host__ __device__ inline uint32_t spec_lds_bytes(uint32_t ntri_pairs, uint32_t nsph_pairs, int max_depth, uint32_t spp,
                                                   uint32_t m_cap) {
    const uint32_t sp4 = (spp + 3u) & ~3u;
    return ntri_pairs * kTriPairFloat4 * 16u + nsph_pairs * kSphPairFloat4 * 16u + kSpecMaxPix * 16u +
           kSpecBatch * 16u + sp4 * 12u + spec_stack_depth(max_depth) * kSpecBlock * 4u +
           kSpecBlock * 20u + kSpecMaxPix * 64u + kSpecBatch * 2u + kSpecMaxPix * 8u + kSpecMaxPix * m_cap;
}

template <int MAXD, int OPT>
__device__ __forceinline__ void spec_body(const kparams& p, const kspec& s, uint32_t bid) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    const uint32_t sp4 = (p.spp + 3u) & ~3u;
    float4* lds_tri = lds;
    float4* lds_sph = lds_tri + (size_t)p.ntri_pairs * kTriPairFloat4;
    uint4* lds_cm = reinterpret_cast<uint4*>(lds_sph + (size_t)p.nsph_pairs * kSphPairFloat4);    // [pixel]
    float4* lds_c = reinterpret_cast<float4*>(lds_cm + kSpecMaxPix);                              // [pixel][batch]
    float2* tab = reinterpret_cast<float2*>(lds_c + kSpecBatch);
    float* tab_n = reinterpret_cast<float*>(tab + sp4);
    float* lds_stk = tab_n + sp4;                                                                  // [depth][thread]
    uint32_t* lds_st = reinterpret_cast<uint32_t*>(lds_stk + (size_t)spec_stack_depth(p.max_depth) * kSpecBlock);
    // per pixel: 0 the round's first slot (absolute), 1 its window, 2..6 the state there (v0..v4), 7 done,
    // and the walker's running mean (8..10), samples folded (11), storage index (13) — kept in
    // LDS across the slot loop, whose registers they would otherwise take
    uint32_t* lds_rd = lds_st + kSpecBlock * 5u;                                                    // [pixel][16]
    uint16_t* lds_pos = reinterpret_cast<uint16_t*>(lds_rd + kSpecMaxPix * 16u);                   // [pixel][batch]
    uint32_t* lds_w = reinterpret_cast<uint32_t*>(lds_pos + kSpecBatch);                           // [pixel][2]
    uint8_t* lds_n = reinterpret_cast<uint8_t*>(lds_w + 2u * kSpecMaxPix);                         // [pixel][slot]
    for (uint32_t i = threadIdx.x; i < p.ntri_pairs * kTriPairFloat4; i += kSpecBlock)
        lds_tri[i] = reinterpret_cast<const float4*>(p.tri_pairs)[i];
    for (uint32_t i = threadIdx.x; i < p.nsph_pairs * kSphPairFloat4; i += kSpecBlock)
        lds_sph[i] = reinterpret_cast<const float4*>(p.sph_pairs)[i];
    for (uint32_t k = threadIdx.x; k < p.spp; k += kSpecBlock) {
        const uint64_t n = p.frame0 + k + 1;
        tab[k] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
        tab_n[k] = (float)n;
    }
    if (OPT & kOptPrio) __builtin_amdgcn_s_setprio(3);   // these chains are the launch's longest

    // the block's pixels: a plan's block (s.blocks: first position in s.order, count | lanes per pixel << 8)
    // or the next 16 sphere pixels, 16 lanes each
    uint32_t first = bid * kSpecPix, cnt = min(kSpecPix, s.n - min(s.n, bid * kSpecPix)), L = kSpecLanes;
    if (s.blocks) {
        first = s.blocks[2 * bid];
        const uint32_t w = s.blocks[2 * bid + 1];
        cnt = w & 0xffu;
        L = w >> 8;                                        // lanes per pixel: 8, 16, 32 or 64
    }
    const uint32_t batch = min(64u, 2u * L);              // walk: chain samples per pixel and batch
    // pixel g of the block on lanes [g L, g L + L): L divides 64, so a pixel's lanes are one wave's, and each wave
    // runs its pixels' rounds on its own (round 5: no block barrier after the start; a wave that needs no
    // fix-up pass or second round does not wait for one that does)
    const uint32_t g = threadIdx.x / L, l = threadIdx.x - g * L;
    const uint32_t gw0 = (threadIdx.x & ~63u) / L;              // the wave's first pixel group
    const uint32_t gw1 = min(cnt, gw0 + 64u / L);                // ... and the end of its valid ones
    const bool valid = g < cnt, walker = valid && l == 0u;
    const uint32_t q = valid ? (s.order ? s.order[first + g] : first + g) : 0u;
    const uint32_t pix = valid ? s.pix[q] : 0u;
    uint8_t* ln = lds_n + (size_t)g * s.m_cap;
    uint32_t* lst = lds_st + (size_t)g * L * 5u;
    uint32_t* rd = lds_rd + g * 16u;
    uint32_t col = 0, row = 0;
    tile_decode(pix, p.ncols, p.nrows, &col, &row);
    const uint32_t px = p.x0 + col, py = p.y0 + row * p.ystep;
    if (l == 0u) {
        const uint32_t t = (row / kCullTile) * p.ntx + col / kCullTile;
        // (w: the pixel's column and row, read when a lane starts one of its slots)
        lds_cm[g] = make_uint4(p.cull[(size_t)t * p.cull_stride], p.cull[(size_t)t * p.cull_stride + p.cull_wt], t,
                               px | (py << 16));
    }
    if (walker) {
        // round 0: the launch's first slot, the window from the pixel's last chain, its state
        rd[0] = 0u;
        rd[1] = spec_window(s.rho[q] ? s.rho[q] : s.rho0, p.spp, s.m_cap, s.margin_div);
        rd[2] = p.rng[pix];
        rd[3] = p.rng[(size_t)p.npix + pix];
        rd[4] = p.rng[2 * (size_t)p.npix + pix];
        rd[5] = p.rng[3 * (size_t)p.npix + pix];
        rd[6] = p.rng[4 * (size_t)p.npix + pix];
        rd[7] = valid ? 0u : 1u;
        s.m[q] = rd[1];
        const uint32_t* a = reinterpret_cast<const uint32_t*>(p.lin + pix);
        rd[8] = a[0];
        rd[9] = a[1];
        rd[10] = a[2];
        rd[11] = 0u;
        rd[12] = q;
        rd[13] = pix;
        // parity pixel (round 0 traces the even slots first): its last chain took between s.parity_rho / 256 and
        // s.parity_hi / 256 slots per sample (two-slot samples: camera ray, sphere, scattered ray; above, the chain
        // has so many 3-slot samples that it lands on an odd slot early and the fix-up pass traces most odd slots
        // anyway, after a walk: r05 run 7); parity_rho 0 = every slot (round 4)
        const uint32_t r0 = s.rho[q] ? s.rho[q] : s.rho0;
        rd[14] = (s.parity_rho != 0u && r0 >= s.parity_rho && r0 <= s.parity_hi) ? 1u : 0u;
        rd[15] = 0u;
    } else if (!valid && l == 0u) {
        // no pixel (the grid's last block): an empty, finished record (every field is read by the rounds)
        for (uint32_t i = 0; i < 16u; ++i) rd[i] = 0u;
        rd[7] = 1u;
    }
    float4* res = reinterpret_cast<float4*>(s.res) + (size_t)q * s.m_cap;
    const bool rec = s.tl != nullptr && threadIdx.x == 0;   // measurement only
    const bool rec_w = s.tl != nullptr && (threadIdx.x & 63u) == 0u;
    uint64_t t_rec[3] = {rec ? __builtin_amdgcn_s_memrealtime() : 0ull, 0ull, 0ull};
    uint32_t rounds = 0, iters = 0;                          // measurement: this wave's slot-loop iterations
    uint32_t lane_rays = 0;                                  // rays of the chain samples this lane gathered
    __syncthreads();

    // Rounds: round 0 is the window; a chain that leaves it continues in a new window from its end
    // (never expected with the margins; bounded by spp rounds since each folds at least one sample)
    while (__any(rd[7] == 0u)) {
        const bool live = rd[7] == 0u;
        const uint32_t js = rd[0], M = rd[1];
        // ---- slot pass: slots [js + j0, js + j1) of this lane (relative slot indices j). Every slot of the
        // window, or (rd[14]: round 0 of a parity pixel) its even slots only: a pixel whose samples take two
        // slots each (camera ray, sphere, scattered ray) has a chain 0, 2, 4, ... of even slots, so the odd
        // ones (the scatters' draws) need tracing only from where the chain first lands on one (a sample of one
        // or three slots): the fix-up pass below, pooled over the block's lanes
        const uint32_t step = rd[14] != 0u ? 2u : 1u;
        const uint32_t ME = (M + step - 1u) / step;     // slots this pass traces
        auto start_of = [&](uint32_t k) { return step * (ME * k / L); };
        const uint32_t j0 = start_of(l), j1 = start_of(l + 1u);
        rng6 st = {rd[2], rd[3], rd[4], rd[5], rd[6], p.rng[5 * (size_t)p.npix + rd[13]] + 2u * (js + j0) * IQ_XORWOW_WEYL};
        xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, live ? 2u * j0 : 0u);
        lst[l * 5u] = st.v0;
        lst[l * 5u + 1u] = st.v1;
        lst[l * 5u + 2u] = st.v2;
        lst[l * 5u + 3u] = st.v3;
        lst[l * 5u + 4u] = st.v4;

        // The lane's slots: consecutive slots j, j + sp, ... < je of pixel group gg (its own in the slot pass;
        // in the fix-up pass a run of another pixel's odd slots, several runs in turn). Each slot is a whole
        // sample from its start state; the next one starts sp slots further (2 sp draws after this one's start:
        // the 2 camera draws then 2 (sp - 1) more).
        uint32_t gg = g, jc = j0, je = j1, sp = step;
        // (the slot's pixel coordinates, result row and slot counts are read or derived from gg where they are
        // used: registers for 5 fewer live values in the slot loop)
        bool active = live && j0 < j1;
        // fix-up pass: this lane's share [fa, fb) of the wave's pooled odd slots (pw: the prefix sums over the
        // wave's pixels of their fix-up slot counts, in the wave's own words of lds_w)
        uint32_t fa = 0, fb = 0;
        bool fix = false;
        ray3 ray = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        int depth = 0;
        rng6 base = st;
        // a slot's sample starts here: its camera ray, and the state its two draws leave (the next slot's)
        auto start_slot = [&]() {
            const uint32_t pxy = lds_cm[gg].w;
            camera_ray<OPT>(p, pxy & 0xffffu, pxy >> 16, st, ray);
            base = st;
            depth = 0;
        };
        // the next run of the fix-up share: pixel group gg holding pooled index fa, its odd slots from there on
        // (within [fa, fb)), the state at the first one stepped from the nearest slot-pass start state below it
        uint32_t* const pw = lds_w + 2u * gw0;
        auto next_run = [&]() -> bool {
            if (fa >= fb) return false;
            uint32_t i = 0;
            while (gw0 + i + 1u < gw1 && pw[i + 1u] <= fa) ++i;
            const uint32_t h = gw0 + i;
            const uint32_t* rh = lds_rd + h * 16u;
            const uint32_t Mh = rh[1], jsh = rh[0], ph = rh[13];
            const uint32_t n_here = min(fb, pw[i + 1u]) - fa;
            jc = rh[15] + 2u * (fa - pw[i]);              // an odd slot at or after where the chain got stuck
            je = jc + 2u * n_here;
            fa += n_here;
            gg = h;
            sp = 2u;
            // the pass-0 ranges of pixel h (even starts: 2 (ME_h k / L))
            const uint32_t MEh = (Mh + 1u) / 2u;
            uint32_t kk = L - 1u;
            while (kk > 0u && 2u * (MEh * kk / L) > jc) --kk;
            const uint32_t jk = 2u * (MEh * kk / L);
            const uint32_t* lh = lds_st + (size_t)h * L * 5u + kk * 5u;
            st = {lh[0], lh[1], lh[2], lh[3], lh[4], p.rng[5 * (size_t)p.npix + ph] + 2u * (jsh + jc) * IQ_XORWOW_WEYL};
            xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, 2u * (jc - jk));
            (void)Mh;
            return true;
        };
        auto trace = [&]() {
            if (active) start_slot();
            while (__any(active)) {
                if (rec_w) ++iters;
                // closest hit (path_tracer.cu:253-295): camera rays over their tile's mask pairs in index order
                float closest = kTMax;
                int kind = kHitNone;
                uint32_t hidx = 0;
                {
                    const bool cull = !__any(active && depth != 0);
                    uint4 cm = lds_cm[gg];
                    const uint32_t* lane_mask = (cull && active) ? p.cull + (size_t)cm.z * p.cull_stride : nullptr;
                    const uint64_t act = __ballot(active);
                    const uint32_t first = (uint32_t)__builtin_ctzll(act);
                    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)cm.z, (int)first);
                    const bool uni = cull && __ballot(active && cm.z != t0) == 0ull;
                    if (uni) {
                        cm.x = (uint32_t)__builtin_amdgcn_readlane((int)cm.x, (int)first);
                        cm.y = (uint32_t)__builtin_amdgcn_readlane((int)cm.y, (int)first);
                    }
                    const uint32_t* uni_mask = uni ? p.cull + (size_t)t0 * p.cull_stride : nullptr;
                    intersect_culled<OPT>(lds_tri, p.ntri, lds_sph, p.nsph, lane_mask, cm.x, cm.y, !cull, active, ray,
                                          closest, kind, hidx, p.cull_wt, uni_mask);
                }
                if (active) {
                    // shade (path_tracer.cu:297-316) under the reference's materials
                    bool term = false;
                    uint32_t md_end = 0;
                    float Lx = 0.0f, Ly = 0.0f, Lz = 0.0f;
                    if (kind == kHitSphere) {
                        const float* sq = reinterpret_cast<const float*>(lds_sph + (size_t)(hidx >> 1) * kSphPairFloat4) + (hidx & 1u);
                        const float sc = oren_nayar_scatter<OPT>(make_float4(sq[0], sq[2], sq[4], sq[6]), closest, ray, st);
                        if (depth + 1 >= p.max_depth) {
                            term = true;                 // the last record is this scatter (biased, :252)
                            md_end = 1;
                            Lx = sc;
                            Ly = sc;
                            Lz = sc;
                        } else {
                            lds_stk[(uint32_t)depth * kSpecBlock + threadIdx.x] = sc;
                            ++depth;
                        }
                    } else if (kind == kHitTri) {
                        term = true;                     // emissive(1, 10)
                        Lx = 10.0f;
                        Ly = 10.0f;
                        Lz = 10.0f;
                    } else {
                        term = true;                     // sky gradient, :308-313
                        const float a = (ray.dy + 1.0f) * 0.5f;
                        const float one_a = 1.0f - a;
                        Lx = one_a + a * 0.5f;
                        Ly = one_a + a * 0.7f;
                        Lz = one_a + a * 1.0f;
                    }
                    if (term) {
                        // backward product (:321-324), clamp (:345-347), 0 + colour (:341, 348)
                        float cx = Lx, cy = Ly, cz = Lz;
                        for (int i = depth - 1; i >= 0; --i) {
                            const float rr = lds_stk[(uint32_t)i * kSpecBlock + threadIdx.x];
                            cx = cx * rr;
                            cy = cy * rr;
                            cz = cz * rr;
                        }
                        cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
                        cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
                        cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
                        reinterpret_cast<float4*>(s.res)[(size_t)lds_rd[gg * 16u + 12u] * s.m_cap + jc] =
                            make_float4(0.0f + cx, 0.0f + cy, 0.0f + cz, 0.0f);
                        uint8_t* cln = lds_n + (size_t)gg * s.m_cap;
                        cln[jc] = (uint8_t)((uint32_t)depth + 1u + md_end);   // slots: 1 + its scatters
                        // slot pass over even slots: the odd slot after this one is untraced (0: the walk stops there)
                        if (!fix && sp == 2u && jc + 1u < M) cln[jc + 1u] = 0u;
                        jc += sp;
                        if (jc < je) {
                            st = base;                   // slot jc starts where slot jc - 1's camera draws ended ...
                            if (sp == 2u) {              // ... or two draws after that
                                (void)xorwow_next(st);
                                (void)xorwow_next(st);
                            }
                            start_slot();
                        } else if (next_run()) {
                            start_slot();
                        } else {
                            active = false;
                        }
                    }
                }
            }
        };
        uint32_t jw = 0;                                 // walker: the chain's next relative slot
        uint16_t* lp = lds_pos + g * batch;
        float ax = __uint_as_float(rd[8]), ay = __uint_as_float(rd[9]), az = __uint_as_float(rd[10]);
        uint32_t k = rd[11];
        // batches of chain samples up to the window's end, the launch's spp, or a slot not traced yet (an odd
        // slot of a parity pixel before the fix-up pass), while some walker of the wave can go on
        auto walk = [&]() {
            while (true) {
                const bool more = walker && live && k < p.spp && jw < M && ln[jw] != 0u;
                if (!__any(more)) break;
                if (walker) {
                    uint32_t c = 0;
                    while (more && c < batch && k + c < p.spp && jw < M) {
                        const uint32_t nj = ln[jw];
                        if (nj == 0u) break;
                        lp[c++] = (uint16_t)jw;
                        jw += nj;
                    }
                    lds_w[2 * g] = c;
                }
                wave_sync();
                const uint32_t cw = (valid && live) ? lds_w[2 * g] : 0u;
                // the pixel's lanes gather the chain samples' colours and form their mean terms c / n and
                // (n - 1) / n (sample k of the launch), and count their rays: the walker is left the
                // multiply-add chain of the running mean alone
                for (uint32_t i = l; i < cw; i += L) {
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(res + lp[i]);
                    const float cx = __uint_as_float(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    const float cy = __uint_as_float(__hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    const float cz = __uint_as_float(__hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    const float2 tv = tab[k + i];
                    float qx, qy, qz;
                    mean_terms<OPT>(cx, cy, cz, tab_n[k + i], tv.x, p.mean_tiny, qx, qy, qz);
                    lds_c[g * batch + i] = make_float4(qx, qy, qz, tv.y);
                    const uint32_t n = ln[lp[i]];
                    lane_rays += (n - 1u == (uint32_t)p.max_depth) ? (uint32_t)p.max_depth : n;
                }
                wave_sync();
                if (walker && live)
#pragma unroll 4
                    for (uint32_t i = 0; i < cw; ++i) {
                        const float4 v = lds_c[g * batch + i];
                        ax = v.x + ax * v.w;
                        ay = v.y + ay * v.w;
                        az = v.z + az * v.w;
                    }
                k += cw;
                wave_sync();
            }
        };
        // the slot pass and its walk, then (parity pixels whose chain landed on an odd slot at jw, if any in the
        // wave) the fix-up pass — every odd slot from there to the window's end, the even ones being traced, so
        // the walk then runs to the window's end — and the walk again. The wave's fix-up slots are pooled and
        // shared evenly by its 64 lanes: a few chains need them, most do not.
        for (uint32_t pass = 0;; ++pass) {
            trace();
            // walk: the colours are this wave's own stores (complete: vmcnt 0), read back from L2; the walk (and
            // a fix-up pass) ends the wave's pixels: the highest priority
            __builtin_amdgcn_s_waitcnt(0);
            wave_sync();
            if (rec && rounds == 0u && pass == 0u) t_rec[1] = __builtin_amdgcn_s_memrealtime();
            walk();
            if (pass == 1u) break;
            const bool stuck = walker && live && k < p.spp && jw < M && ln[jw] == 0u;
            if (!__any(stuck)) break;
            if (walker) rd[15] = stuck ? jw : M;
            if (stuck) atomicAdd(s.run_count, 1u);       // statistics: chains that needed the fix-up pass
            wave_sync();
            if (__lane_id() == 0u) {
                uint32_t acc = 0;
                for (uint32_t h = gw0; h < gw1; ++h) {
                    pw[h - gw0] = acc;
                    const uint32_t* rh = lds_rd + h * 16u;
                    if (rh[7] == 0u && rh[15] < rh[1]) acc += (rh[1] - rh[15] + 1u) / 2u;
                }
                pw[gw1 > gw0 ? gw1 - gw0 : 0u] = acc;
            }
            wave_sync();
            const uint32_t F = pw[gw1 > gw0 ? gw1 - gw0 : 0u];
            fa = (uint32_t)(((uint64_t)F * __lane_id()) / 64u);
            fb = (uint32_t)(((uint64_t)F * (__lane_id() + 1u)) / 64u);
            fix = true;
            active = next_run();
        }
        if (walker && live) {
            rd[8] = __float_as_uint(ax);
            rd[9] = __float_as_uint(ay);
            rd[10] = __float_as_uint(az);
            rd[11] = k;
            const uint32_t pix = rd[13];
            // the state at the chain's end, slot js + jw: from the start of the last range at or below it
            // (the lanes' start slots, as in the slot pass)
            uint32_t kk = L - 1u;
            while (kk > 0u && start_of(kk) > jw) --kk;
            const uint32_t jk = start_of(kk);
            uint32_t v0 = lst[kk * 5u], v1 = lst[kk * 5u + 1u], v2 = lst[kk * 5u + 2u], v3 = lst[kk * 5u + 3u],
                     v4 = lst[kk * 5u + 4u];
            xorwow_skip_v(v0, v1, v2, v3, v4, 2u * (jw - jk));
            rd[0] = js + jw;
            rd[2] = v0;
            rd[3] = v1;
            rd[4] = v2;
            rd[5] = v3;
            rd[6] = v4;
            if (k == p.spp) {
                rd[7] = 1u;
                const uint32_t jt = js + jw;
                const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
                const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
                const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
                p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
                reinterpret_cast<float4*>(p.lin)[pix] = make_float4(ax, ay, az, 0.0f);
                p.rng[pix] = v0;
                p.rng[(size_t)p.npix + pix] = v1;
                p.rng[2 * (size_t)p.npix + pix] = v2;
                p.rng[3 * (size_t)p.npix + pix] = v3;
                p.rng[4 * (size_t)p.npix + pix] = v4;
                p.rng[5 * (size_t)p.npix + pix] = p.rng[5 * (size_t)p.npix + pix] + 2u * jt * IQ_XORWOW_WEYL;
                s.rho[q] = (uint32_t)(((uint64_t)jt * 256u) / p.spp);
            } else {
                // the chain left its window: a new one from its end, sized for the remaining samples, every
                // slot traced
                atomicAdd(s.run_count + 1, 1u);
                const uint32_t rem = p.spp - k;
                rd[1] = min(s.m_cap, max(16u, 3u * rem + 4u));
                rd[14] = 0u;
            }
        }
        if (rec && rounds == 0u) t_rec[2] = __builtin_amdgcn_s_memrealtime();
        ++rounds;
        wave_sync();                                       // the walkers' records before the loop test
    }
    if (rec) {
        unsigned long long* o = s.tl + 8 * (size_t)bid;
        o[0] = t_rec[0];
        o[1] = t_rec[1];
        o[2] = t_rec[2];
    }
    // per wave: its end (48 bits) | its slot-loop iterations << 48 (the block's end: the latest of its waves)
    if (rec_w)
        s.tl[8 * (size_t)bid + 4 + threadIdx.x / 64u] =
            (__builtin_amdgcn_s_memrealtime() & 0xffffffffffffull) | ((unsigned long long)min(iters, 0xffffu) << 48);
    if (rec) s.tl[8 * (size_t)bid + 3] = (unsigned long long)rounds << 48;
    unsigned long long rays = lane_rays;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
    if (__lane_id() == 0 && rays) add_rays(p.rays, rays);
}

// ------------------------------------------------------------------------------------------------
// Certain-miss pixels. A pixel whose own camera-ray bundle (its jitter square, iq_interval.h)
// is proven to miss every primitive ends every sample on its camera ray with the sky gradient
// (path_tracer.cu:307-316), after exactly the camera's two jitter draws (camera.cu:24-25): one ray per sample,
// no intersection test, no scatter. Lane = pixel, one wave per tile of such pixels (kparams::miss), one tile
// per block; each lane runs its samples in order — camera ray, sky colour, clamp, running mean with the plain
// kernel's table values and mean terms — the plain kernel's own operations for that path, so the same bits,
// at a fraction of its per-iteration cost (no mask, no closest-hit loop, no refill or path bookkeeping).
// one tile per block: the blocks slot into the CUs beside the plain kernel's waves one wave at a time (C2 N = 1:
// 0.840 -> 0.812 ms per step against four tiles per block, r06 run 47)
constexpr uint32_t kSkyBlock = 64;

template <int OPT>
__global__ __launch_bounds__(kSkyBlock) void iqpt_sky_kernel(const kparams p, const uint32_t* __restrict__ tiles,
                                                             uint32_t ntiles) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    float2* tab = reinterpret_cast<float2*>(lds);
    float* tab_n = reinterpret_cast<float*>(tab + ((p.spp + 1u) & ~1u));
    for (uint32_t k = threadIdx.x; k < p.spp; k += kSkyBlock) {
        const uint64_t n = p.frame0 + k + 1;
        tab[k] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
        tab_n[k] = (float)n;
    }
    __syncthreads();
    const uint32_t w = blockIdx.x * (kSkyBlock / 64u) + threadIdx.x / 64u;
    if (w >= ntiles) return;
    const uint32_t lane = __lane_id();
    const uint32_t t = tiles[w];
    const uint64_t miss = (uint64_t)p.miss[2 * (size_t)t] | ((uint64_t)p.miss[2 * (size_t)t + 1] << 32);
    if ((miss >> lane) & 1ull) {
        const uint32_t tx = t % p.ntx, ty = t / p.ntx;
        const uint32_t th = min(kCullTile, p.nrows - ty * kCullTile);
        const uint32_t pix = ty * kCullTile * p.ncols + tx * kCullTile * th + lane;   // tile-major storage
        uint32_t col, row;
        tile_decode(pix, p.ncols, p.nrows, &col, &row);
        const uint32_t px = p.x0 + col, py = p.y0 + row * p.ystep;
        rng6 st = {p.rng[pix], p.rng[(size_t)p.npix + pix], p.rng[2 * (size_t)p.npix + pix],
                   p.rng[3 * (size_t)p.npix + pix], p.rng[4 * (size_t)p.npix + pix], p.rng[5 * (size_t)p.npix + pix]};
        const float4 a0 = reinterpret_cast<const float4*>(p.lin)[pix];
        float ax = a0.x, ay = a0.y, az = a0.z;
        for (uint32_t k = 0; k < p.spp; ++k) {
            ray3 ray;
            camera_ray<OPT>(p, px, py, st, ray);
            // sky gradient (:308-313), no records: the colour itself, clamped (:345-347), 0 + colour (:341, 348)
            const float a = (ray.dy + 1.0f) * 0.5f;
            const float one_a = 1.0f - a;
            float cx = one_a + a * 0.5f, cy = one_a + a * 0.7f, cz = one_a + a * 1.0f;
            cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
            cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
            cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
            cx = 0.0f + cx;
            cy = 0.0f + cy;
            cz = 0.0f + cz;
            // running mean (:356-358) with the launch table's RN(1 / n), (n - 1) / n and (float) n
            const float2 tv = tab[k];
            float qx, qy, qz;
            mean_terms<OPT>(cx, cy, cz, tab_n[k], tv.x, p.mean_tiny, qx, qy, qz);
            ax = qx + ax * tv.y;
            ay = qy + ay * tv.y;
            az = qz + az * tv.y;
        }
        const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
        const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
        const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
        p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
        reinterpret_cast<float4*>(p.lin)[pix] = make_float4(ax, ay, az, 0.0f);
        p.rng[pix] = st.v0;
        p.rng[(size_t)p.npix + pix] = st.v1;
        p.rng[2 * (size_t)p.npix + pix] = st.v2;
        p.rng[3 * (size_t)p.npix + pix] = st.v3;
        p.rng[4 * (size_t)p.npix + pix] = st.v4;
        p.rng[5 * (size_t)p.npix + pix] = st.d;
    }
    // one closest-hit query per sample (path_tracer.cu:252-318: the miss ends the loop at crt_depth 1)
    const uint32_t nm = (uint32_t)__popcll(miss);
    if (lane == 0 && nm) add_rays(p.rays, (unsigned long long)nm * p.spp);
}

// ------------------------------------------------------------------------------------------------
// Any-hit scenes (kparams::anyhit: no sphere, every triangle emissive, the reference's materials) whose every tile
// list has per-pixel masks (kparams::pmask), round 6. A sample of such a scene is one camera ray (the camera's two
// jitter draws, camera.cu:24-25) that either meets some triangle — emissive, colour (10, 10, 10) clamped to (1, 1, 1)
// (path_tracer.cu:278, 341-348), whichever triangle it is — or misses everything and takes the sky gradient
// (:307-316). Lane = pixel, one wave per tile (in the cost order), four tiles per block: the tile's candidate list
// in LDS, the lane's mask words in registers for all of its samples; per sample the lane tests its own candidates in
// list order with the reference's Möller–Trumbore (test_triangle_pair) until one accepts the ray. The plain kernel's
// operations for these paths — camera ray, tests, clamp, running mean with the launch table — so the same bits,
// without its queue, refill, batches and path bookkeeping, and with no pixel waiting on another tile's list.
constexpr uint32_t kAnyBlock = 256;
#ifndef IQPT_ANY_BATCH
#define IQPT_ANY_BATCH 2
#endif
constexpr uint32_t kAnyBatch = IQPT_ANY_BATCH;          // samples traced together per lane

template <int OPT>
__global__ __launch_bounds__(kAnyBlock) void iqpt_anyhit_kernel(const kparams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    float2* tab = reinterpret_cast<float2*>(lds);
    float* tab_n = reinterpret_cast<float*>(tab + ((p.spp + 1u) & ~1u));
    uint32_t* lists = reinterpret_cast<uint32_t*>(tab_n + ((p.spp + 3u) & ~3u));
    for (uint32_t k = threadIdx.x; k < p.spp; k += kAnyBlock) {
        const uint64_t n = p.frame0 + k + 1;
        tab[k] = make_float2(1.0f / (float)n, (float)(n - 1) / (float)n);
        tab_n[k] = (float)n;
    }
    const uint32_t wv = threadIdx.x / 64u, lane = __lane_id();
    const uint32_t q = blockIdx.x * (kAnyBlock / 64u) + wv;
    const bool live = q < p.ntiles;
    const uint32_t t = live ? (p.tile_order ? p.tile_order[q] : q) : 0u;
    const uint32_t la = live ? p.list_off_tri[t] : 0u, n = live ? p.list_off_tri[t + 1] - la : 0u;
    uint32_t* wl = lists + wv * kAnyMaxEntries;
    for (uint32_t e = lane; e < n; e += 64u) wl[e] = p.list[la + e];
    __syncthreads();
    if (!live) return;
    const uint32_t tx = t % p.ntx, ty = t / p.ntx;
    const uint32_t th = min(kCullTile, p.nrows - ty * kCullTile), tw = min(kCullTile, p.ncols - tx * kCullTile);
    if (lane < tw * th) {
        const uint32_t pix = ty * kCullTile * p.ncols + tx * kCullTile * th + lane;   // tile-major storage
        uint32_t col, row;
        tile_decode(pix, p.ncols, p.nrows, &col, &row);
        const uint32_t px = p.x0 + col, py = p.y0 + row * p.ystep;
        rng6 st = {p.rng[pix], p.rng[(size_t)p.npix + pix], p.rng[2 * (size_t)p.npix + pix],
                   p.rng[3 * (size_t)p.npix + pix], p.rng[4 * (size_t)p.npix + pix], p.rng[5 * (size_t)p.npix + pix]};
        const float4 a0 = reinterpret_cast<const float4*>(p.lin)[pix];
        float ax = a0.x, ay = a0.y, az = a0.z;
        // a certain pixel: every sample takes the camera's two draws and ends on a triangle, colour (1, 1, 1), whose
        // mean term c / n is the table's RN(1 / n) (the plain kernel's certain fold)
        const bool sure = (p.pmask_certain[2 * (size_t)t + lane / 32u] >> (lane % 32u)) & 1u;
        const uint32_t nk = sure ? 0u : p.spp;
        if (sure) {
            xorwow_skip_v(st.v0, st.v1, st.v2, st.v3, st.v4, 2u * p.spp);
            st.d += 2u * p.spp * IQ_XORWOW_WEYL;
            for (uint32_t k = 0; k < p.spp; ++k) {
                const float2 tv = tab[k];
                ax = tv.x + ax * tv.y;
                ay = tv.x + ay * tv.y;
                az = tv.x + az * tv.y;
            }
        }
        constexpr uint32_t kW = kAnyMaxEntries / 32u;
        uint32_t wm[kW];
        const uint32_t* pm = p.pmask + p.pmask_off[t] + lane;
#pragma unroll
        for (uint32_t w = 0; w < kW; ++w) wm[w] = w * 32u < n ? pm[(size_t)w * 64u] : 0u;
        const float4* __restrict__ gp = reinterpret_cast<const float4*>(p.tri_pairs);
        // kAnyBatch samples at a time: a sample's draws are its camera's two, whatever it meets, so the batch's rays
        // are made in sample order up front; each candidate pair is loaded once for the batch and tested against
        // every ray of it not yet accepted (the rays' own operations, so the same bits); the colours fold in order
        for (uint32_t k0 = 0; k0 < nk; k0 += kAnyBatch) {
            ray3 rs[kAnyBatch];
            float cl[kAnyBatch];
            int kd[kAnyBatch];
            uint32_t live = 0u;                                  // bit r: ray r not yet accepted
#pragma unroll
            for (uint32_t r = 0; r < kAnyBatch; ++r) {
                cl[r] = kTMax;
                kd[r] = kHitNone;
                if (k0 + r < nk) {
                    camera_ray<OPT>(p, px, py, st, rs[r]);
                    live |= 1u << r;
                } else {
                    rs[r] = rs[0];
                }
            }
#pragma unroll
            for (uint32_t w = 0; w < kW; ++w) {
                uint32_t m = wm[w];
                while (m != 0u && live != 0u) {
                    const uint32_t j = wl[w * 32u + (uint32_t)__builtin_ctz(m)];
                    m &= m - 1u;
                    const float4* qq = gp + (size_t)j * kTriPairFloat4;
                    const float4 q0 = qq[0], q1 = qq[1], q2 = qq[2], q3 = qq[3], q4 = qq[4];
#pragma unroll
                    for (uint32_t r = 0; r < kAnyBatch; ++r)
                        if ((live >> r) & 1u) {
                            uint32_t hidx = 0;
                            test_triangle_pair<OPT>(q0, q1, q2, q3, q4, rs[r], cl[r], kd[r], hidx, 2 * j,
                                                    2 * j + 1 < p.ntri);
                            if (kd[r] == kHitTri) live &= ~(1u << r);
                        }
                }
            }
#pragma unroll
            for (uint32_t r = 0; r < kAnyBatch; ++r) {
                if (k0 + r >= nk) break;
                float cx, cy, cz;
                if (kd[r] == kHitTri) {
                    cx = 1.0f;                                   // emissive (1, 10): 10 clamped (:345-347)
                    cy = 1.0f;
                    cz = 1.0f;
                } else {
                    const float a = (rs[r].dy + 1.0f) * 0.5f;    // sky gradient (:308-313)
                    const float one_a = 1.0f - a;
                    cx = one_a + a * 0.5f;
                    cy = one_a + a * 0.7f;
                    cz = one_a + a * 1.0f;
                    cx = cx > 1.0f ? 1.0f : (cx < 0.0f ? 0.0f : cx);
                    cy = cy > 1.0f ? 1.0f : (cy < 0.0f ? 0.0f : cy);
                    cz = cz > 1.0f ? 1.0f : (cz < 0.0f ? 0.0f : cz);
                }
                const float2 tv = tab[k0 + r];
                float qx, qy, qz;
                mean_terms<OPT>(0.0f + cx, 0.0f + cy, 0.0f + cz, tab_n[k0 + r], tv.x, p.mean_tiny, qx, qy, qz);
                ax = qx + ax * tv.y;
                ay = qy + ay * tv.y;
                az = qz + az * tv.y;
            }
        }
        const uint32_t r8 = to_u8(255.0f * iq_sqrtf(ax));
        const uint32_t g8 = to_u8(255.0f * iq_sqrtf(ay));
        const uint32_t b8 = to_u8(255.0f * iq_sqrtf(az));
        p.bgra[tile_to_compact(pix, p.ncols, p.nrows)] = b8 | (g8 << 8) | (r8 << 16) | (255u << 24);
        reinterpret_cast<float4*>(p.lin)[pix] = make_float4(ax, ay, az, 0.0f);
        p.rng[pix] = st.v0;
        p.rng[(size_t)p.npix + pix] = st.v1;
        p.rng[2 * (size_t)p.npix + pix] = st.v2;
        p.rng[3 * (size_t)p.npix + pix] = st.v3;
        p.rng[4 * (size_t)p.npix + pix] = st.v4;
        p.rng[5 * (size_t)p.npix + pix] = st.d;
    }
    // one closest-hit query per sample (the hit or the miss ends the path at crt_depth 1)
    if (lane == 0) add_rays(p.rays, (unsigned long long)(tw * th) * p.spp);
}

template <int OPT>
__global__ __launch_bounds__(kFanBlock, 2) void iqpt_fan_kernel(const kparams p) {
    fan_body<OPT>(p, blockIdx.x);
}

template <int MAXD, int OPT>
__global__ __launch_bounds__(kSpecBlock, 4) void iqpt_spec_kernel(const kparams p, const kspec s) {
    spec_body<MAXD, OPT>(p, s, blockIdx.x);
}

// Events bound to the next kernel launch (bind_launch_events): recorded by the dispatch itself
// (hipExtLaunchKernel) instead of as marker packets of their own between two kernels on the stream.
namespace {
thread_local hipEvent_t tl_ev_start = nullptr, tl_ev_stop = nullptr;
template <typename F, typename... Args>
void dispatch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t stream, Args... args) {
    const hipEvent_t a = tl_ev_start, z = tl_ev_stop;
    tl_ev_start = tl_ev_stop = nullptr;
    if (a || z)
        hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, a, z, 0u, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
}
}  // namespace

template <int MAXD, bool STREAM, int OPT>
int launch_t(hipStream_t stream, const kparams& p, uint32_t grid, uint32_t lds) {
    dispatch(iqpt_render_kernel<MAXD, STREAM, OPT>, dim3(grid), dim3(kRenderBlock), lds, stream, p);
    return (int)hipGetLastError();
}
template <int MAXD, bool STREAM, int OPT>
int occ_t(uint32_t lds, int* blocks) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, iqpt_render_kernel<MAXD, STREAM, OPT>,
                                                             kRenderBlock, lds);
}

// Variant table: the production option set for every (MAXD, STREAM), plus (IQPT_STATS_VARIANTS builds)
// the instrumented kOptStats variants.
struct variant {
    int maxd;
    bool stream;
    int opt;
    int (*launch)(hipStream_t, const kparams&, uint32_t, uint32_t);
    int (*occ)(uint32_t, int*);
};
#define IQPT_V(M, S, O) {M, S, O, launch_t<M, S, O>, occ_t<M, S, O>}
const variant kVariants[] = {
    // MAXD 16 (max_depth 9-16) differs only in the LDS stack size the runtime reserves. Streamed
    // scenes with LDS batches run without the 5-wave bound (4 waves/SIMD); the batch-free BVH-primary
    // variants keep it (5 waves measured 2.5 % faster on C5 than 4, 6 slower: profiles/ab/r01_ab72).
    // Streamed scenes also get the kOptBvhPrimary form (camera rays through the BVH), chosen per
    // packet by timing (iqpt_runtime.cpp).
    // Resident variants carry kOptPrio (waves holding scatter-heavy tiles win VALU arbitration: the
    // launch ends with the longest chains, profiles/r02/ab_prio.json); the runtime adds the bit.
#define IQPT_PROD(O) IQPT_V(8, false, (O) | kOptPrio), IQPT_V(16, false, (O) | kOptPrio), IQPT_V(8, true, (O) & ~kOptLB5), \
                     IQPT_V(16, true, (O) & ~kOptLB5), IQPT_V(8, true, (O) | kOptBvhPrimary), \
                     IQPT_V(16, true, (O) | kOptBvhPrimary)
    IQPT_PROD(kOptDefault),
    // BVH-primary at 4 waves per SIMD (128 VGPRs, no spills): the runtime's choice above 4 samples per launch
    // (C5 16 spp -5 %, 1 spp +7 % against the 5-wave form, r06 run 36)
    IQPT_V(8, true, (kOptDefault | kOptBvhPrimary) & ~kOptLB5), IQPT_V(16, true, (kOptDefault | kOptBvhPrimary) & ~kOptLB5),
    // streamed any-hit scenes (kOptAnyHit: no sphere, reference materials; C4): the first accepted triangle ends
    // a ray's traversal. Variants of their own: the exits cost the other streamed scenes registers (C5 58.6-60.3
    // against 56.6-56.7 ms per launch with them compiled in, r05 run 16)
    IQPT_V(8, true, (kOptDefault | kOptAnyHit) & ~kOptLB5), IQPT_V(16, true, (kOptDefault | kOptAnyHit) & ~kOptLB5),
    IQPT_V(8, true, kOptDefault | kOptAnyHit | kOptBvhPrimary), IQPT_V(16, true, kOptDefault | kOptAnyHit | kOptBvhPrimary),
    IQPT_V(8, true, ((kOptDefault & ~kOptFastDiv) | kOptAnyHit) & ~kOptLB5),
    IQPT_V(8, true, (kOptDefault & ~kOptFastDiv) | kOptAnyHit | kOptBvhPrimary),
    // pitch-only cameras (kOptCamAxis), resident scenes: 10.5 % fewer VALU instructions on C2; chosen by the
    // runtime wherever the camera qualifies (round 1 measured no gain; after kOptPrio / kOptScatter2 and
    // with overlapped launches it is -12..-14 %)
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio), IQPT_V(16, false, kOptDefault | kOptCamAxis | kOptPrio),
    IQPT_V(8, false, kOptDefault | kOptMaterials | kOptCamAxis | kOptPrio),
    IQPT_PROD(kOptDefault & ~kOptFastDiv),                  // packets outside the kOptFastDiv range
    IQPT_PROD(kOptDefault | kOptMaterials),                 // packets with a material table
    IQPT_PROD((kOptDefault & ~kOptFastDiv) | kOptMaterials),
    // overlapped launches (kOptOverlap), resident scenes
    IQPT_V(8, false, kOptDefault | kOptPrio | kOptOverlap), IQPT_V(16, false, kOptDefault | kOptPrio | kOptOverlap),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptPrio | kOptOverlap),
    IQPT_V(8, false, kOptDefault | kOptMaterials | kOptPrio | kOptOverlap),
    // overlapped launches of pitch-only cameras take the short camera transform (kOptCamAxis): with the
    // chip kept full by the overlap, its 10.5 % fewer VALU instructions shorten C2 by 14 % (profiles/r02/
    // ab_camaxis_overlap.json); without the overlap they did not
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap),
    IQPT_V(16, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap),
    IQPT_V(8, false, kOptDefault | kOptMaterials | kOptCamAxis | kOptPrio | kOptOverlap),
    // two rays per lane (kOptPipe): resident scenes under the reference's materials
    IQPT_V(8, false, kOptDefault | kOptPrio | kOptPipe), IQPT_V(16, false, kOptDefault | kOptPrio | kOptPipe),
    IQPT_V(8, false, kOptDefault | kOptPrio | kOptOverlap | kOptPipe),
    IQPT_V(16, false, kOptDefault | kOptPrio | kOptOverlap | kOptPipe),
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio | kOptPipe),
    IQPT_V(16, false, kOptDefault | kOptCamAxis | kOptPrio | kOptPipe),
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap | kOptPipe),
    IQPT_V(16, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap | kOptPipe),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptPrio | kOptPipe),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptPrio | kOptOverlap | kOptPipe),
    // sample-parallel chains (kOptSplit), resident scenes
    IQPT_V(8, false, kOptDefault | kOptSplit | kOptPrio), IQPT_V(16, false, kOptDefault | kOptSplit | kOptPrio),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptSplit | kOptPrio),
    IQPT_V(8, false, kOptDefault | kOptMaterials | kOptSplit | kOptPrio),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptMaterials | kOptSplit | kOptPrio),
#undef IQPT_PROD
#if defined(IQPT_STATS_VARIANTS)
    // instrumented build (libiqpt_stats.so, tools/work_counters.py and the wave timelines of tools/):
    // kOptStats counts the primitive and node tests each query executes (the executed-work roofline)
    IQPT_V(8, false, kOptDefault | kOptStats),
    IQPT_V(8, false, kOptDefault | kOptPrio | kOptStats),
    IQPT_V(8, false, kOptDefault | kOptPrio | kOptStats | kOptPipe),
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap | kOptStats),
    IQPT_V(8, false, kOptDefault | kOptCamAxis | kOptPrio | kOptOverlap | kOptStats | kOptPipe),
    IQPT_V(8, false, (kOptDefault & ~kOptFastDiv) | kOptStats),
    IQPT_V(8, true, (kOptDefault | kOptStats) & ~kOptLB5),
    IQPT_V(8, true, kOptDefault | kOptStats | kOptBvhPrimary),
    IQPT_V(8, true, (kOptDefault | kOptStats | kOptBvhPrimary) & ~kOptLB5),
    IQPT_V(8, false, kOptDefault | kOptSplit | kOptStats),
    IQPT_V(8, true, (kOptDefault | kOptStats | kOptAnyHit) & ~kOptLB5),
    IQPT_V(8, true, kOptDefault | kOptStats | kOptBvhPrimary | kOptAnyHit),
    IQPT_V(8, true, (kOptDefault | kOptStats | kOptBvhPrimary | kOptAnyHit) & ~kOptLB5),
#endif
};
#undef IQPT_V

const variant* find_variant(int max_depth, bool stream, int opt) {
    const int maxd = max_depth <= 8 ? 8 : 16;
    for (const variant& v : kVariants)
        if (v.maxd == maxd && v.stream == stream && v.opt == opt) return &v;
    return nullptr;
}

}  // namespace

void take_launch_events(void** start, void** stop) {
    *start = tl_ev_start;
    *stop = tl_ev_stop;
    tl_ev_start = tl_ev_stop = nullptr;
}

void bind_launch_events(void* start, void* stop) {
    tl_ev_start = (hipEvent_t)start;
    tl_ev_stop = (hipEvent_t)stop;
}

int launch_rng_init(void* stream, uint32_t width, uint32_t x0, uint32_t ncols, uint32_t y0, uint32_t ystep,
                    uint32_t nrows, uint64_t seed, const uint32_t* tables, uint32_t* rng) {
    const uint32_t npix = ncols * nrows;
    if (npix == 0) return 0;
    const uint32_t grid = (npix + 255) / 256;
    hipLaunchKernelGGL(iqpt_rng_init_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, width, x0, ncols,
                       y0, ystep, nrows, seed, tables, rng);
    return (int)hipGetLastError();
}

int launch_relayout(void* stream, const uint32_t* src, uint32_t* dst, uint32_t ncols, uint32_t nrows, uint32_t words,
                    uint32_t planes, bool to_compact) {
    const uint64_t n = (uint64_t)ncols * nrows * words * planes;
    if (n == 0) return 0;
    hipLaunchKernelGGL(iqpt_relayout_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       src, dst, ncols, nrows, words, planes, to_compact ? 1 : 0);
    return (int)hipGetLastError();
}

int launch_assemble_rows(void* stream, const uint32_t* src, uint32_t* dst, uint32_t width, uint32_t height,
                         uint32_t world, uint32_t split, uint32_t base, uint64_t stride, uint32_t words) {
    const uint64_t n = (uint64_t)world * stride * words;
    if (n == 0) return 0;
    hipLaunchKernelGGL(iqpt_assemble_rows_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       src, dst, width, height, world, split, base, stride, words);
    return (int)hipGetLastError();
}

int launch_lds_poison(void* stream, uint32_t pattern, uint32_t lds_bytes, uint32_t blocks) {
    if (blocks == 0 || lds_bytes < 4) return 0;
    hipLaunchKernelGGL(iqpt_lds_poison_kernel, dim3(blocks), dim3(256), lds_bytes, (hipStream_t)stream, pattern,
                       lds_bytes / 4u);
    return (int)hipGetLastError();
}

int launch_libm(void* stream, int fn, const float* a, const float* b, float* out, uint32_t n) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(iqpt_libm_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, a, b, out, n);
    return (int)hipGetLastError();
}

int launch_camera_probe(void* stream, const kparams& p, const float* ndc, float* gen, float* axis, uint32_t n,
                        bool do_axis) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(iqpt_camera_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, p, ndc,
                       gen, axis, n, do_axis ? 1 : 0);
    return (int)hipGetLastError();
}

int launch_bin(void* stream, const kbin& b) {
    const uint64_t n = (uint64_t)b.ntx * b.nty * b.stride;
    if (n == 0) return 0;
    if (n > 0xffffffffull * 256ull) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(iqpt_bin_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, b);
    return (int)hipGetLastError();
}

int launch_certain(void* stream, const kbin& b, uint32_t* certain) {
    const uint32_t ntiles = b.ntx * b.nty;
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(iqpt_certain_kernel, dim3(ntiles), dim3(64), 0, (hipStream_t)stream, b, certain);
    return (int)hipGetLastError();
}

int launch_tile_list_order(void* stream, const kbin& b, const uint32_t* off_tri, uint32_t* list) {
    const uint32_t ntiles = b.ntx * b.nty;
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(iqpt_tile_list_order_kernel, dim3(ntiles), dim3(64), 0, (hipStream_t)stream, b, off_tri, list);
    return (int)hipGetLastError();
}

int launch_pixel_mask(void* stream, const kbin& b, const uint32_t* off_tri, const uint32_t* list,
                      const uint32_t* pmask_off, uint32_t* pmask, uint32_t* certain) {
    const uint32_t ntiles = b.ntx * b.nty;
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(iqpt_pixel_mask_kernel, dim3(ntiles), dim3(64), 0, (hipStream_t)stream, b, off_tri, list,
                       pmask_off, pmask, certain);
    return (int)hipGetLastError();
}

int launch_tile_count(void* stream, const uint32_t* cull, uint32_t ntiles, uint32_t wt, uint32_t stride,
                      uint32_t* cnt_tri, uint32_t* cnt_sph) {
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(iqpt_tile_count_kernel, dim3((ntiles + 255) / 256), dim3(256), 0, (hipStream_t)stream, cull,
                       ntiles, wt, stride, cnt_tri, cnt_sph);
    return (int)hipGetLastError();
}

int launch_tile_list(void* stream, const uint32_t* cull, uint32_t ntiles, uint32_t wt, uint32_t stride,
                     const uint32_t* off_tri, const uint32_t* off_sph, uint32_t* list) {
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(iqpt_tile_list_kernel, dim3((ntiles + 255) / 256), dim3(256), 0, (hipStream_t)stream, cull,
                       ntiles, wt, stride, off_tri, off_sph, list);
    return (int)hipGetLastError();
}

int launch_render(void* stream, const kparams& p, uint32_t grid, uint32_t lds, bool stream_batches, int opt) {
    const variant* v = find_variant(p.max_depth, stream_batches, opt);
    if (!v) return (int)hipErrorInvalidDeviceFunction;
    return v->launch((hipStream_t)stream, p, grid, lds);
}

int render_occupancy(int max_depth, bool stream_batches, int opt, uint32_t lds, int* blocks) {
    const variant* v = find_variant(max_depth, stream_batches, opt);
    if (!v) return (int)hipErrorInvalidDeviceFunction;
    return v->occ(lds, blocks);
}

bool render_variant_exists(int max_depth, bool stream_batches, int opt) {
    return find_variant(max_depth, stream_batches, opt) != nullptr;
}

const char* render_kernel_name() { return "iqpt_render_kernel"; }

int launch_split_prep(void* stream, const ksplit& s) {
    if (s.ns_cap == 0) return 0;
    hipLaunchKernelGGL(iqpt_split_prep_kernel, dim3((s.ns_cap + 255) / 256), dim3(256), 0, (hipStream_t)stream, s);
    return (int)hipGetLastError();
}

int launch_split_stitch(void* stream, const ksplit& s, bool fastdiv) {
    if (s.ns_cap == 0) return 0;
    if (s.spp > kAccTableMax) return (int)hipErrorInvalidValue;
    const dim3 grid((s.ns_cap + kStitchBlock - 1) / kStitchBlock);
    if (fastdiv)
        hipLaunchKernelGGL(iqpt_split_stitch_kernel<kOptDefault>, grid, dim3(kStitchBlock), 0, (hipStream_t)stream, s);
    else
        hipLaunchKernelGGL(iqpt_split_stitch_kernel<(kOptDefault & ~kOptFastDiv)>, grid, dim3(kStitchBlock), 0,
                           (hipStream_t)stream, s);
    return (int)hipGetLastError();
}


// iqpt_fan_kernel launches: the option bits it depends on are the camera form and the division forms
namespace {
template <int OPT>
int fan_launch_t(hipStream_t stream, const kparams& p, uint32_t grid, uint32_t lds) {
    dispatch(iqpt_fan_kernel<OPT>, dim3(grid), dim3(kFanBlock), lds, stream, p);
    return (int)hipGetLastError();
}
struct fan_variant {
    int key;
    int (*launch)(hipStream_t, const kparams&, uint32_t, uint32_t);
};
constexpr int kFanKeyBits = kOptFastDiv | kOptCamAxis;
const fan_variant kFanVariants[] = {
    {kOptFastDiv, fan_launch_t<kOptDefault>},
    {0, fan_launch_t<kOptDefault & ~kOptFastDiv>},
    {kOptFastDiv | kOptCamAxis, fan_launch_t<kOptDefault | kOptCamAxis>},
};
const fan_variant* find_fan(int opt) {
    // the production option sets differ from kOptDefault only in these bits (and in bits the fan
    // kernel does not read: priority, overlap, split)
    if ((opt & (kOptPair | kOptCull | kOptAccTable | kOptCamConst)) !=
            (kOptPair | kOptCull | kOptAccTable | kOptCamConst) || (opt & (kOptMaterials | kOptStats)))
        return nullptr;
    for (const fan_variant& v : kFanVariants)
        if (v.key == (opt & kFanKeyBits)) return &v;
    return nullptr;
}
}  // namespace

bool fan_variant_exists(int opt) { return find_fan(opt) != nullptr; }

// iqpt_sky_kernel launches: keyed like the fan kernel (camera form, division forms)
namespace {
template <int OPT>
int sky_launch_t(hipStream_t stream, const kparams& p, const uint32_t* tiles, uint32_t ntiles, uint32_t lds) {
    dispatch(iqpt_sky_kernel<OPT>, dim3((ntiles + kSkyBlock / 64u - 1u) / (kSkyBlock / 64u)), dim3(kSkyBlock), lds,
             stream, p, tiles, ntiles);
    return (int)hipGetLastError();
}
struct sky_variant {
    int key;
    int (*launch)(hipStream_t, const kparams&, const uint32_t*, uint32_t, uint32_t);
};
const sky_variant kSkyVariants[] = {
    {kOptFastDiv, sky_launch_t<kOptDefault>},
    {0, sky_launch_t<kOptDefault & ~kOptFastDiv>},
    {kOptFastDiv | kOptCamAxis, sky_launch_t<kOptDefault | kOptCamAxis>},
};
const sky_variant* find_sky(int opt) {
    // (kOptStats launches keep the sky kernel: it runs no intersection test, and the instrumented plain kernel
    // beside it then counts the tests of the pixels it renders in production, tools/work_counters.py)
    if ((opt & (kOptAccTable | kOptCamConst)) != (kOptAccTable | kOptCamConst) || (opt & kOptMaterials))
        return nullptr;
    for (const sky_variant& v : kSkyVariants)
        if (v.key == (opt & kFanKeyBits)) return &v;
    return nullptr;
}
}  // namespace

bool sky_variant_exists(int opt) { return find_sky(opt) != nullptr; }

int launch_sky(void* stream, const kparams& p, const uint32_t* tiles, uint32_t ntiles, int opt) {
    const sky_variant* v = find_sky(opt);
    if (!v || p.spp > kAccTableMax || p.miss == nullptr || tiles == nullptr) return (int)hipErrorInvalidDeviceFunction;
    if (ntiles == 0 || p.spp == 0) return 0;
    return v->launch((hipStream_t)stream, p, tiles, ntiles, ((p.spp + 1u) & ~1u) * 8u + ((p.spp + 3u) & ~3u) * 4u);
}

// iqpt_anyhit_kernel launches: keyed like the sky kernel (camera form, division forms)
namespace {
template <int OPT>
int anyhit_launch_t(hipStream_t stream, const kparams& p, uint32_t lds) {
    dispatch(iqpt_anyhit_kernel<OPT>, dim3((p.ntiles + kAnyBlock / 64u - 1u) / (kAnyBlock / 64u)), dim3(kAnyBlock),
             lds, stream, p);
    return (int)hipGetLastError();
}
struct anyhit_variant {
    int key;
    int (*launch)(hipStream_t, const kparams&, uint32_t);
};
const anyhit_variant kAnyVariants[] = {
    {kOptFastDiv, anyhit_launch_t<kOptDefault>},
    {0, anyhit_launch_t<kOptDefault & ~kOptFastDiv>},
    {kOptFastDiv | kOptCamAxis, anyhit_launch_t<kOptDefault | kOptCamAxis>},
};
const anyhit_variant* find_anyhit(int opt) {
    if ((opt & (kOptAccTable | kOptCamConst | kOptPair)) != (kOptAccTable | kOptCamConst | kOptPair) ||
        (opt & (kOptMaterials | kOptStats)))
        return nullptr;
    for (const anyhit_variant& v : kAnyVariants)
        if (v.key == (opt & kFanKeyBits)) return &v;
    return nullptr;
}
}  // namespace

bool anyhit_variant_exists(int opt) { return find_anyhit(opt) != nullptr; }

int launch_anyhit(void* stream, const kparams& p, int opt) {
    const anyhit_variant* v = find_anyhit(opt);
    if (!v || p.spp > kAccTableMax || !p.list || !p.list_off_tri || !p.pmask || !p.pmask_off || !p.pmask_certain ||
        !p.anyhit)
        return (int)hipErrorInvalidDeviceFunction;
    if (p.ntiles == 0 || p.spp == 0) return 0;
    return v->launch((hipStream_t)stream, p,
                     ((p.spp + 1u) & ~1u) * 8u + ((p.spp + 3u) & ~3u) * 4u + (kAnyBlock / 64u) * kAnyMaxEntries * 4u);
}

uint32_t fan_lds(const kparams& p) { return fan_lds_bytes(p.ntri_pairs, p.spp); }

int launch_fan(void* stream, const kparams& p, uint32_t ntiles, int opt) {
    const fan_variant* v = find_fan(opt);
    if (!v || p.spp > kAccTableMax || p.cull == nullptr || p.cull_wt > 16u || p.tile_order == nullptr)
        return (int)hipErrorInvalidDeviceFunction;
    if (ntiles == 0 || p.spp == 0) return 0;
    return v->launch((hipStream_t)stream, p, ntiles, fan_lds(p));
}

// Slot-parallel sphere pixels (IQPT_SPLIT_SPEC): the resident production option sets, reference materials
namespace {
template <int MAXD, int OPT>
int spec_launch_t(hipStream_t stream, const kparams& p, const kspec& s, uint32_t lds) {
    dispatch(iqpt_spec_kernel<MAXD, OPT>, dim3(s.blocks ? s.nblocks : (s.n + kSpecPix - 1u) / kSpecPix),
             dim3(kSpecBlock), lds, stream, p, s);
    return (int)hipGetLastError();
}
template <int MAXD, int OPT>
int spec_occ_t(uint32_t lds, int* blocks) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, iqpt_spec_kernel<MAXD, OPT>, kSpecBlock, lds);
}
struct spec_variant {
    int maxd, opt;
    int (*launch)(hipStream_t, const kparams&, const kspec&, uint32_t);
    int (*occ)(uint32_t, int*);
};
#define IQPT_SV(M, O) {M, O, spec_launch_t<M, O>, spec_occ_t<M, O>}
#define IQPT_SV2(O) IQPT_SV(8, O), IQPT_SV(16, O)
const spec_variant kSpecVariants[] = {
    IQPT_SV2(kOptDefault | kOptPrio),
    IQPT_SV2((kOptDefault & ~kOptFastDiv) | kOptPrio),
    IQPT_SV2(kOptDefault | kOptCamAxis | kOptPrio),
};
#undef IQPT_SV2
#undef IQPT_SV
const spec_variant* find_spec(int max_depth, int opt) {
    const int maxd = max_depth <= 8 ? 8 : 16;
    for (const spec_variant& v : kSpecVariants)
        if (v.maxd == maxd && v.opt == ((opt | kOptPrio) & ~(kOptOverlap | kOptSplit))) return &v;
    return nullptr;
}
}  // namespace

bool spec_variant_exists(int max_depth, int opt) { return max_depth <= 16 && find_spec(max_depth, opt) != nullptr; }

uint32_t spec_lds(const kparams& p, const kspec& s) {
    return spec_lds_bytes(p.ntri_pairs, p.nsph_pairs, p.max_depth, p.spp, s.m_cap);
}

int launch_spec(void* stream, const kparams& p, const kspec& s, int opt) {
    const spec_variant* v = find_spec(p.max_depth, opt);
    if (!v || p.max_depth > 16 || p.cull == nullptr || p.spp > kAccTableMax || s.m_cap > 65535u)
        return (int)hipErrorInvalidDeviceFunction;
    if (s.n == 0) return 0;
    return v->launch((hipStream_t)stream, p, s, spec_lds(p, s));
}

int spec_occupancy(const kparams& p, const kspec& s, int opt, int* blocks) {
    const spec_variant* v = find_spec(p.max_depth, opt);
    if (!v) return (int)hipErrorInvalidDeviceFunction;
    return v->occ(spec_lds(p, s), blocks);
}

}  // namespace iqpt
