// iq_bvh.hpp — exact BVH for secondary rays, host side: error bounds + builder.
//
// The closest hit must be the one the reference's brute-force loop finds (path_tracer.cu:257-295):
// over triangles, the accepted hit with the smallest computed t, the LAST one in packet order among
// equal t (t_max < t rejects, t == closest is accepted). That is order-free — (min t, max index) —
// so a BVH can visit triangles in any order, provided it never skips a triangle whose own
// Möller–Trumbore test (shape.cu:62-103, in binary32 round-to-nearest as the kernel evaluates it)
// would accept the ray with t <= closest. Skipping is decided with boxes, so the boxes must contain
// every point where the float test can accept — not just the triangle:
//
//   With u = 2^-24, gamma_n = n u / (1 - n u), |d_i| <= M_d, |e1_i| <= M1, |e2_i| <= M2, |s_i| <= S
//   (s = o - v0) and the computed determinant |det^| >= 1e-6 (smaller ones are rejected), forward
//   error analysis of the kernel's operation sequence gives (P = 2 M_d M2, Q = 2 S M1):
//     |det^ - det|        <= E_det = 3 M1 [gamma_3 (P + dP) + dP],          dP = gamma_2 P
//     |N_u^ - s.p|        <= E_u   = 3 S (1+u) [gamma_3 (P + dP) + u (P + dP) + dP]
//     |N_v^ - d.q|        <= E_v   = 3 M_d [gamma_3 (Q + dQ) + dQ],          dQ = (gamma_2 + 2u) Q
//     |N_t^ - e2.q|       <= E_t   = 3 M2 [gamma_3 (Q + dQ) + dQ]
//   and with R = E_det / 1e-6 < 1, the exact barycentrics of an accepted hit satisfy
//     |u^ - u| <= Du = (E_u / 1e-6 + R + 2 gamma_2) / (1 - R)     (|u^| <= 1), likewise Dv,
//     |t^ - t| <= (E_t / 1e-6 + R |t| + 2 gamma_2 |t^|) / (1 - R).
//   The exact line point o + t d = v0 + u e1 + v e2 (det != 0: |det^ - det| < 1e-6 <= |det^|) has
//   u >= -Du, v >= -Dv, u + v <= 1 + Du + Dv + 4u; moving it into the triangle shifts u by at most
//   3 Du + 2 Dv + 4u and v by at most 2 Du + 3 Dv + 4u, so it lies in the triangle's box grown by
//   delta = 3 (Du + Dv + 4u) (M1 + M2) per axis, at a parameter within Dt of the accepted t^.
//   Every term is linear in S = max_i |o_i - v0_i| (the ray origin's distance to the triangle):
//   delta = gA + gB S and |t^ - t| <= tA S + tB |t|. A node stores its triangles' tight vertex box
//   and the maxima of (gA, gB, tA, tB) over them; traversal bounds S for the node from the ray
//   origin and the tight box, grows the box by gA + gB S (rounded up) and widens the ray segment
//   by tA S + tB closest. The bound therefore tightens near the ray origin, where secondary rays
//   find their hits, instead of being priced at the scene's diameter. Rays with |d_i| > M_d or a
//   non-finite origin test every triangle.
//
// Triangles whose R exceeds 1/4 (large triangles: the 1e-6 determinant threshold is tiny against
// |e1| |e2|, so grazing hits are poorly conditioned) are not put in the BVH; they stay on an
// "always test" list. Every bound is multiplied by a safety factor of 2 and box corners are rounded
// outward. tests/test_bvh.py checks the bound against the oracle on adversarial rays (grazing
// directions near the determinant threshold, hits on edges and vertices, origins near and far).
#pragma once

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace iqbvh {

constexpr double kU = 5.9604644775390625e-8;   // 2^-24
constexpr double kDetMin = 1e-6;               // |det| threshold of the reject test (as float 0.000001f)
constexpr double kSafety = 2.0;

inline double gamma_n(int n) { return n * kU / (1.0 - n * kU); }

struct tri_coeffs {
    bool eligible;        // R <= 1/4: may go into the BVH
    double gA, gB;        // per-axis growth of the triangle's box: gA + gB S (= gR + gC + gB S)
    double gR, gC;        // the parts of gA that scale with 1/D (normal cones) and that do not
    double tA, tB;        // |t^ - t| <= tA S + tB |t|   (t <= closest during traversal)
    double edet;          // safety x E_det: |det^ - det| (normal cones, below)
};

// e1, e2: the kernel's world-space edges; Md: bound on |d_i| (normalized directions: 1 + a few ulp).
inline tri_coeffs triangle_coeffs(const float e1[3], const float e2[3], double Md) {
    const double M1 = std::max({std::fabs((double)e1[0]), std::fabs((double)e1[1]), std::fabs((double)e1[2])});
    const double M2 = std::max({std::fabs((double)e2[0]), std::fabs((double)e2[1]), std::fabs((double)e2[2])});
    const double g2 = gamma_n(2), g3 = gamma_n(3);
    const double P = 2.0 * Md * M2, dP = g2 * P;
    const double Q1 = 2.0 * M1, dQ1 = (g2 + 2.0 * kU) * Q1;               // Q = S Q1
    const double E_det = 3.0 * M1 * (g3 * (P + dP) + dP);
    const double E_u1 = 3.0 * (1.0 + kU) * (g3 * (P + dP) + kU * (P + dP) + dP);   // E_u = S E_u1
    const double E_v1 = 3.0 * Md * (g3 * (Q1 + dQ1) + dQ1);                         // E_v = S E_v1
    const double E_t1 = 3.0 * M2 * (g3 * (Q1 + dQ1) + dQ1);                         // E_t = S E_t1
    const double R = kSafety * E_det / kDetMin;
    tri_coeffs c;
    c.eligible = std::isfinite(R) && R <= 0.25 && std::isfinite(M1) && std::isfinite(M2);
    if (!c.eligible) {
        c.gA = c.gB = c.gR = c.gC = c.tA = c.tB = INFINITY;
        return c;
    }
    // Du = du0 + du1 S, Dv = dv0 + dv1 S; delta = 3 (Du + Dv + 4u) (M1 + M2)
    const double d0 = kSafety * (R + 2.0 * g2) / (1.0 - R);
    const double du1 = kSafety * (E_u1 / kDetMin) / (1.0 - R), dv1 = kSafety * (E_v1 / kDetMin) / (1.0 - R);
    c.gA = 3.0 * (2.0 * d0 + 4.0 * kU) * (M1 + M2);
    c.gR = 3.0 * (2.0 * kSafety * R / (1.0 - R)) * (M1 + M2);
    c.gC = 3.0 * (4.0 * kSafety * g2 / (1.0 - R) + 4.0 * kU) * (M1 + M2);
    c.gB = 3.0 * (du1 + dv1) * (M1 + M2);
    c.tA = kSafety * (E_t1 / kDetMin) / (1.0 - R);
    c.tB = kSafety * (R + 4.0 * g2) / (1.0 - R);
    c.edet = kSafety * E_det;
    return c;
}

// Normal cones (tightening for non-grazing rays). Every bound above divides an error by the smallest
// determinant an accepted hit can have, priced at the reject threshold 1e-6. For a given ray a larger
// lower bound D is often known: det = e1 . (d x e2) = -d . n with n = e1 x e2, so if the normals of a
// node's triangles lie (as lines) within angle beta of an axis a and |n| >= Nmin, then
// |det^| >= Nmin |d| cos(theta + beta) - E_det with theta = angle(d, a) (when theta + beta < 90 deg).
// With lambda = 1e-6 / max(1e-6, D) <= 1 the bounds become
//   growth <= lambda (gR + gB S) + gC,   |t^ - t| <= lambda tA S + tB |t|
// (R, Du, Dv and the t error scale with 1/D; gC and tB hold the D-independent remainders — gC is a
// few ulp of the triangle size and is applied as one scene-wide maximum).
// Triangles that no ray can accept (|n| sqrt(3) Md + E_det < 1e-6) do not constrain a cone.
struct tri_normal {
    double n[3];          // e1 x e2 (exact in double up to one rounding per component)
    double len;           // |n|
    bool hittable;
};

inline tri_normal triangle_normal(const float e1[3], const float e2[3], double Md, double edet) {
    tri_normal t;
    t.n[0] = (double)e1[1] * e2[2] - (double)e1[2] * e2[1];
    t.n[1] = (double)e1[2] * e2[0] - (double)e1[0] * e2[2];
    t.n[2] = (double)e1[0] * e2[1] - (double)e1[1] * e2[0];
    t.len = std::sqrt(t.n[0] * t.n[0] + t.n[1] * t.n[1] + t.n[2] * t.n[2]);
    t.hittable = t.len * std::sqrt(3.0) * Md + edet >= kDetMin;
    return t;
}

// Node of the stackless (threaded) BVH, DFS preorder: a box and the index of the next node after the
// subtree (`skip`); leaves hold [first, first + count) of the leaf-ordered triangle pairs.
struct node {
    float bmin[3];          // tight box of the subtree's vertices (rounded outward)
    uint32_t skip;
    float bmax[3];
    uint32_t first_count;   // leaf: first pair << 8 | pair count (count 1..255); inner: 0
    float gR, gB, tA, tB;   // maxima of the subtree's triangle coefficients (rounded up)
    float axis[3];          // normal cone of the hittable triangles (float axis, |axis| ~ 1)
    float cos_beta;         // rounded down; 0 = no useful cone
    float sin_beta;         // rounded up
    float nmin;             // min |e1 x e2| over hittable triangles, rounded down
    float edet;             // max safety x E_det, rounded up
    float pad;
};
static_assert(sizeof(node) == 80, "host-side node (the device node is 64 bytes, iqpt_runtime.cpp)");

struct build_input {
    std::vector<float> lo, hi;       // 3 per triangle: tight vertex box, rounded outward
    std::vector<float> centroid;     // 3 per triangle
    std::vector<float> coeff;        // 4 per triangle: gR, gB, tA, tB rounded up
    std::vector<tri_normal> normal;  // per triangle
    std::vector<double> edet;        // per triangle
    std::vector<uint32_t> tris;      // triangle indices in the BVH (packet order)
};

struct build_output {
    std::vector<node> nodes;
    std::vector<uint32_t> order;     // BVH triangles in leaf order (packet indices), pairs padded by ~0u
};

inline float round_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -INFINITY);
    return f;
}
inline float round_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}
// bf16 bits (the high half of a float) rounded up, for v >= 0
inline uint32_t bf16_up_bits(float v) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    return (u & 0xffffu) ? (u >> 16) + 1u : (u >> 16);
}

// Binned surface-area-heuristic split of idx[b, e) (16 bins per axis over the centroid bounds; cost =
// area(left box) x left count + area(right box) x right count). Falls back to the median on the longest
// centroid axis when the centroids do not spread. Any split is exact: node boxes are computed from
// their members. cen(i) / lo(i) / hi(i) give primitive i's centroid and box (float[3]).
template <class Cen, class Lo, class Hi>
inline uint32_t sah_split(std::vector<uint32_t>& idx, uint32_t b, uint32_t e, Cen cen, Lo lo, Hi hi) {
    constexpr int kBins = 16;
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = b; i < e; ++i)
        for (int a = 0; a < 3; ++a) {
            cmin[a] = std::min(cmin[a], cen(idx[i])[a]);
            cmax[a] = std::max(cmax[a], cen(idx[i])[a]);
        }
    auto area = [](const double* l, const double* h) {
        if (!(l[0] <= h[0])) return 0.0;
        const double dx = h[0] - l[0], dy = h[1] - l[1], dz = h[2] - l[2];
        return dx * dy + dy * dz + dz * dx;
    };
    auto bin_of = [&](uint32_t t, int ax) {
        const double ext = (double)cmax[ax] - cmin[ax];
        const int k = (int)(((double)cen(t)[ax] - cmin[ax]) / ext * kBins);
        return std::min(kBins - 1, std::max(0, k));
    };
    double best = INFINITY;
    int best_ax = -1, best_bin = 0;
    for (int ax = 0; ax < 3; ++ax) {
        if (!(cmax[ax] > cmin[ax])) continue;
        uint32_t cnt[kBins] = {};
        double bl[kBins][3], bh[kBins][3];
        for (int k = 0; k < kBins; ++k)
            for (int a = 0; a < 3; ++a) {
                bl[k][a] = INFINITY;
                bh[k][a] = -INFINITY;
            }
        for (uint32_t i = b; i < e; ++i) {
            const uint32_t t = idx[i];
            const int k = bin_of(t, ax);
            ++cnt[k];
            for (int a = 0; a < 3; ++a) {
                bl[k][a] = std::min(bl[k][a], (double)lo(t)[a]);
                bh[k][a] = std::max(bh[k][a], (double)hi(t)[a]);
            }
        }
        double rarea[kBins];
        uint32_t rcnt[kBins];
        double l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t n = 0;
        for (int k = kBins - 1; k >= 1; --k) {
            for (int a = 0; a < 3; ++a) {
                l[a] = std::min(l[a], bl[k][a]);
                h[a] = std::max(h[a], bh[k][a]);
            }
            n += cnt[k];
            rarea[k] = area(l, h);
            rcnt[k] = n;
        }
        for (int a = 0; a < 3; ++a) {
            l[a] = INFINITY;
            h[a] = -INFINITY;
        }
        n = 0;
        for (int k = 1; k < kBins; ++k) {
            for (int a = 0; a < 3; ++a) {
                l[a] = std::min(l[a], bl[k - 1][a]);
                h[a] = std::max(h[a], bh[k - 1][a]);
            }
            n += cnt[k - 1];
            if (n == 0 || rcnt[k] == 0) continue;
            const double c = area(l, h) * n + rarea[k] * rcnt[k];
            if (c < best) {
                best = c;
                best_ax = ax;
                best_bin = k;
            }
        }
    }
    if (best_ax >= 0) {
        const auto it = std::stable_partition(idx.begin() + b, idx.begin() + e,
                                              [&](uint32_t t) { return bin_of(t, best_ax) < best_bin; });
        const uint32_t mid = (uint32_t)(it - idx.begin());
        if (mid > b && mid < e) return mid;
    }
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (cmax[a] - cmin[a] > cmax[ax] - cmin[ax]) ax = a;
    const uint32_t mid = b + (e - b) / 2;
    std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e, [&](uint32_t x, uint32_t y) {
        const float cx = cen(x)[ax], cy = cen(y)[ax];
        return cx < cy || (cx == cy && x < y);
    });
    return mid;
}

// Binned-SAH splits (sah_split), leaves of <= kLeafTris triangles (kept even by padding).
#ifndef IQPT_LEAF_TRIS
#define IQPT_LEAF_TRIS 4
#endif
constexpr uint32_t kLeafTris = IQPT_LEAF_TRIS;

inline void build(build_input& in, build_output& out) {
    out.nodes.clear();
    out.order.clear();
    if (in.tris.empty()) return;
    std::vector<uint32_t> idx(in.tris.size());
    for (uint32_t i = 0; i < idx.size(); ++i) idx[i] = i;
    // DFS preorder with an explicit stack; skip pointers patched when a subtree closes
    struct frame {
        uint32_t begin, end, node, stage, mid;
    };
    std::vector<frame> st;
    auto make = [&](uint32_t b, uint32_t e) {
        node n;
        n.bmin[0] = n.bmin[1] = n.bmin[2] = INFINITY;
        n.bmax[0] = n.bmax[1] = n.bmax[2] = -INFINITY;
        float co[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (uint32_t i = b; i < e; ++i) {
            const uint32_t t = idx[i];
            for (int a = 0; a < 3; ++a) {
                n.bmin[a] = std::min(n.bmin[a], in.lo[3 * t + a]);
                n.bmax[a] = std::max(n.bmax[a], in.hi[3 * t + a]);
            }
            for (int q = 0; q < 4; ++q) co[q] = std::max(co[q], in.coeff[4 * t + q]);
        }
        n.gR = co[0];
        n.gB = co[1];
        n.tA = co[2];
        n.tB = co[3];
        // normal cone (as lines) of the hittable triangles
        n.axis[0] = 1.0f;
        n.axis[1] = n.axis[2] = 0.0f;
        n.cos_beta = 0.0f;
        n.sin_beta = 1.0f;
        n.nmin = 0.0f;
        n.edet = 0.0f;
        n.pad = 0.0f;
        double sum[3] = {0.0, 0.0, 0.0}, ref[3] = {0.0, 0.0, 0.0}, nmin = INFINITY, edet = 0.0;
        bool have_ref = false;
        for (uint32_t i = b; i < e; ++i) {
            const uint32_t t = idx[i];
            edet = std::max(edet, in.edet[t]);
            const tri_normal& tn = in.normal[t];
            if (!tn.hittable) continue;
            nmin = std::min(nmin, tn.len);
            const double u[3] = {tn.n[0] / tn.len, tn.n[1] / tn.len, tn.n[2] / tn.len};
            if (!have_ref) {
                for (int a = 0; a < 3; ++a) ref[a] = u[a];
                have_ref = true;
            }
            const double sg = (u[0] * ref[0] + u[1] * ref[1] + u[2] * ref[2]) < 0.0 ? -1.0 : 1.0;
            for (int a = 0; a < 3; ++a) sum[a] += sg * u[a];
        }
        const double sl = std::sqrt(sum[0] * sum[0] + sum[1] * sum[1] + sum[2] * sum[2]);
        if (have_ref && sl > 1e-3 && std::isfinite(nmin)) {
            float af[3];
            for (int a = 0; a < 3; ++a) af[a] = (float)(sum[a] / sl);
            const double al = std::sqrt((double)af[0] * af[0] + (double)af[1] * af[1] + (double)af[2] * af[2]);
            double cmin = 1.0;
            for (uint32_t i = b; i < e; ++i) {
                const tri_normal& tn = in.normal[idx[i]];
                if (!tn.hittable) continue;
                const double c = std::fabs(tn.n[0] * af[0] + tn.n[1] * af[1] + tn.n[2] * af[2]) / (tn.len * al);
                cmin = std::min(cmin, c);
            }
            cmin = std::min(1.0, cmin * (1.0 - 1e-12)) - 1e-12;
            if (cmin > 0.0) {
                for (int a = 0; a < 3; ++a) n.axis[a] = af[a];
                n.cos_beta = round_down(cmin);
                n.sin_beta = round_up(std::min(1.0, std::sqrt(std::max(0.0, 1.0 - cmin * cmin)) * (1.0 + 1e-12) + 1e-12));
                n.nmin = round_down(nmin * (1.0 - 1e-12));
            }
        }
        n.edet = round_up(edet);
        n.skip = 0;
        n.first_count = 0;
        out.nodes.push_back(n);
        return (uint32_t)out.nodes.size() - 1;
    };
    st.push_back({0, (uint32_t)idx.size(), make(0, (uint32_t)idx.size()), 0, 0});
    while (!st.empty()) {
        frame& f = st.back();
        const uint32_t count = f.end - f.begin;
        if (count <= kLeafTris) {
            const uint32_t first_pair = (uint32_t)out.order.size() / 2;
            for (uint32_t i = f.begin; i < f.end; ++i) out.order.push_back(in.tris[idx[i]]);
            if (out.order.size() & 1u) out.order.push_back(~0u);
            const uint32_t pairs = (uint32_t)out.order.size() / 2 - first_pair;
            out.nodes[f.node].first_count = (first_pair << 8) | pairs;
            out.nodes[f.node].skip = (uint32_t)out.nodes.size();
            st.pop_back();
            continue;
        }
        if (f.stage == 0) {
            const uint32_t mid = sah_split(
                idx, f.begin, f.end, [&](uint32_t t) { return &in.centroid[3 * t]; },
                [&](uint32_t t) { return &in.lo[3 * t]; }, [&](uint32_t t) { return &in.hi[3 * t]; });
            f.mid = mid;
            f.stage = 1;
            const uint32_t b = f.begin;
            const uint32_t n = make(b, mid);
            st.push_back({b, mid, n, 0, 0});
        } else if (f.stage == 1) {
            f.stage = 2;
            const uint32_t mid = f.mid, e = f.end;
            const uint32_t n = make(mid, e);
            st.push_back({mid, e, n, 0, 0});
        } else {
            out.nodes[f.node].skip = (uint32_t)out.nodes.size();
            st.pop_back();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Sphere BVH (secondary rays in scenes with many spheres).
//
// The reference folds the spheres in packet order after the triangles (path_tracer.cu:283-295,
// shape.cu:13-46): for each sphere, delta = halfb^2 - cc < 0 rejects; t = halfb - sqrt(delta) is
// rejected if closest < t; if t < t_min the far root halfb + sqrt(delta) is taken WITHOUT the t_max
// test (rejected only below t_min). So a sphere is one of
//   * inert:   delta^ < 0 or t_far^ < t_min — never changes the state;
//   * normal:  t_near^ >= t_min — "closest = min(closest, t_near^)", the later sphere on ties;
//   * inside:  t_near^ < t_min <= t_far^ (the origin is inside or within ~1e-6 of it) — since
//              closest >= t_min always holds, it sets closest = t_far^ unconditionally.
// The fold is therefore order-free up to its LAST inside sphere j*: with none, the result is the
// smallest t_near^ over normal spheres (largest index among equal t, a sphere beating a triangle
// at equal t); with one, it is t_far^(j*) lowered by normal spheres of index > j* (same rule). A
// traversal may visit spheres in any order if it never skips a non-inert sphere.
//
// Bound. With u = 2^-24, w = c - o (exact) and its computed oc (|oc_i - w_i| <= u |w_i|), |d| within
// a few ulp of 1 (normalized, |d_i| <= 1.001), the kernel's delta^ differs from the exact
// Delta(oc) = (d.oc)^2 - |oc|^2 + r^2 by at most 13.2 u |oc|^2 + 3 u r^2 (first order, forward error
// of the operation sequence of shape.cu:16-25), and Delta(oc) = r^2 - |oc x d|^2 + |oc|^2 (|d|^2 - 1).
// So delta^ >= 0 implies that the ray line passes within rho <= sqrt(r^2 + K) + 2 u S of the
// centre, K = 12 u r^2 + 43 u S^2 (S >= |w|; the 2 u S covers oc's rounding). Each term is doubled
// (safety 2), and sqrt(r^2 + K) - r = K / (sqrt(r^2 + K) + r) is evaluated without cancellation:
//   growth(S) = K / (sqrt(r_min^2 + K) + r_min) + 4 u S + 8 u r_max,  K = 24 u r_max^2 + 86 u S^2
// is an upper bound over a node's spheres (decreasing in r_min). The sphere then lies in its box
// grown by growth(S). The computed roots are within 10 u S of the grown sphere's (the root error is
// in |halfb^ - d.w| <= 4 u S and the square root of the already bounded delta), so a non-inert
// sphere has t_far^ >= t_min and hence meets the half-line s >= t_min - 20 u S, and its t_near^ is
// at least the grown box's entry minus 20 u S: a node whose entry exceeds the running closest by
// more than that holds neither a better normal sphere nor an inside one (inside spheres have
// t_near^ < t_min <= closest). Scenes with |c_i| or r above 2^60 get no sphere BVH (the bound
// assumes no overflow; ray origins are bounded by bvh_ray_ok), and spheres much larger than the
// median stay on an "always" list tested by every ray (their boxes would cover every node).
struct sph_node {
    float bmin[3];          // box of the subtree's spheres, centre -/+ radius (rounded outward)
    uint32_t skip;
    float bmax[3];
    uint32_t first_count;   // leaf: first sphere slot << 8 | count (1..255); inner: 0
    float rmin, rmax;       // radii of the subtree (rmin rounded down, rmax up)
    float pad0, pad1;
};
static_assert(sizeof(sph_node) == 48, "sphere node is three float4");

// growth(S) of the bound above in double (tests/test_sphere_bvh.py; the kernel evaluates the same
// expression in float with upward rounding)
inline double sphere_growth(double rmin, double rmax, double S) {
    const double K = 24.0 * kU * rmax * rmax + 86.0 * kU * S * S;
    return K / (std::sqrt(rmin * rmin + K) + rmin) + 4.0 * kU * S + 8.0 * kU * rmax;
}

#ifndef IQPT_LEAF_SPHERES
#define IQPT_LEAF_SPHERES 4
#endif
constexpr uint32_t kLeafSpheres = IQPT_LEAF_SPHERES;

// centres/radii: float per sphere (c.xyz, r) in packet order; bvh: indices (packet order) of the
// spheres put in the BVH. Median split on the longest centre axis. Fills the nodes (DFS preorder with
// skip pointers) and the leaf order (packet indices).
inline void build_spheres(const std::vector<float>& sph4, const std::vector<uint32_t>& ids,
                          std::vector<sph_node>& nodes, std::vector<uint32_t>& order) {
    nodes.clear();
    order.clear();
    if (ids.empty()) return;
    std::vector<uint32_t> idx(ids);
    std::vector<float> slo(sph4.size() / 4 * 3), shi(sph4.size() / 4 * 3);   // sphere boxes (SAH)
    for (size_t k = 0; k < sph4.size() / 4; ++k)
        for (int a = 0; a < 3; ++a) {
            const float r = std::fabs(sph4[4 * k + 3]);
            slo[3 * k + a] = sph4[4 * k + a] - r;
            shi[3 * k + a] = sph4[4 * k + a] + r;
        }
    struct frame {
        uint32_t begin, end, node, stage, mid;
    };
    std::vector<frame> st;
    auto make = [&](uint32_t b, uint32_t e) {
        sph_node n;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double rmin = INFINITY, rmax = 0.0;
        for (uint32_t i = b; i < e; ++i) {
            const float* s4 = &sph4[4 * (size_t)idx[i]];
            const double r = std::fabs((double)s4[3]);
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], (double)s4[a] - r);
                hi[a] = std::max(hi[a], (double)s4[a] + r);
            }
            rmin = std::min(rmin, r);
            rmax = std::max(rmax, r);
        }
        for (int a = 0; a < 3; ++a) {
            n.bmin[a] = round_down(lo[a]);
            n.bmax[a] = round_up(hi[a]);
        }
        n.rmin = round_down(rmin);
        n.rmax = round_up(rmax);
        n.pad0 = n.pad1 = 0.0f;
        n.skip = 0;
        n.first_count = 0;
        nodes.push_back(n);
        return (uint32_t)nodes.size() - 1;
    };
    st.push_back({0, (uint32_t)idx.size(), make(0, (uint32_t)idx.size()), 0, 0});
    while (!st.empty()) {
        frame& f = st.back();
        const uint32_t count = f.end - f.begin;
        if (count <= kLeafSpheres) {
            const uint32_t first = (uint32_t)order.size();
            for (uint32_t i = f.begin; i < f.end; ++i) order.push_back(idx[i]);
            nodes[f.node].first_count = (first << 8) | count;
            nodes[f.node].skip = (uint32_t)nodes.size();
            st.pop_back();
            continue;
        }
        if (f.stage == 0) {
            const uint32_t mid = sah_split(
                idx, f.begin, f.end, [&](uint32_t t) { return &sph4[4 * (size_t)t]; },
                [&](uint32_t t) { return &slo[3 * (size_t)t]; }, [&](uint32_t t) { return &shi[3 * (size_t)t]; });
            f.mid = mid;
            f.stage = 1;
            const uint32_t b = f.begin;
            const uint32_t n = make(b, mid);
            st.push_back({b, mid, n, 0, 0});
        } else if (f.stage == 1) {
            f.stage = 2;
            const uint32_t mid = f.mid, e = f.end;
            const uint32_t n = make(mid, e);
            st.push_back({mid, e, n, 0, 0});
        } else {
            nodes[f.node].skip = (uint32_t)nodes.size();
            st.pop_back();
        }
    }
}

}  // namespace iqbvh
