/*
 * iqpt_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the IoniqRE path-tracing hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the CPU baseline. The product (libiqpt.so) never links or calls it.
 *
 * What it restates (reference = GionutN/path-tracer-and-rasterizer-engine @ 2025-12-05):
 *   render_kernel            IoniqRE/path_tracer.cu:330-366
 *   path_tracer::ray_color   IoniqRE/path_tracer.cu:231-328
 *   camera::get_ray          IoniqRE/camera.cu:20-43
 *   triangle::intersect      IoniqRE/shape.cu:62-103  (MOLLER_TRUMBORE 1)
 *   sphere::intersect        IoniqRE/shape.cu:13-46
 *   oren_nayar::scatter/pdf  IoniqRE/material.cu:5-48
 *   emissive::scatter        IoniqRE/material.cu:50-57
 *   onb                      IoniqRE/onb.h:5-25
 *   random::real / cosine_weighted (device) IoniqRE/random.cu:66-70, 96-107
 *   iqvec / iqmat / mat3x3   IoniqRE/vector.h, IoniqRE/matrix.cu
 *   curand_init / curand     cuRAND XORWOW (CUDA 12.6, un-vendored; see csrc/iq_xorwow.h)
 *
 * It deliberately keeps the reference's structure and per-ray work: the AoS gpu_packet, the
 * per-drawcall normal-matrix inverse, the six per-ray vertex/normal transforms, the virtual
 * material dispatch (as a switch) and the scatter_record stack evaluated backwards. That makes it
 * both the parity oracle and the "reference kernel as a host-side loop" CPU baseline
 * (BASELINE.md §3). OpenMP over 16x16 pixel tiles, dynamic schedule; per-pixel results do not
 * depend on the thread count.
 *
 * Parity status: the reference cannot be compiled in this environment (its sources include
 * <cuda.h>/<cuda_runtime.h>/<curand_kernel.h>/<d3d11.h>, which the image lacks, and stand-in
 * headers are not allowed), and it ships no tests or golden outputs (IoniqRE/image.ppm is 0
 * bytes). PARITY UNPINNED against the reference binary: this file is pinned only by
 * known-answer tests of its parts (tests/test_oracle_units.py, tests/test_xorwow.py) and by the
 * golden fixtures it generated (tests/golden/), which guard it against regressions.
 *
 * Floating point: compiled with -ffp-contract=off (no FMA contraction), IEEE division/sqrt, and
 * the shared transcendentals of csrc/iq_fp.h (flavour B of SURVEY.md §8c). Building with
 * -DIQO_GLIBC_LIBM swaps in glibc sinf/cosf/tanf/acosf/atan2f (flavour A, informational).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "iqpt.h"
#include "iq_fp.h"
#include "iq_xorwow.h"

#ifdef IQO_GLIBC_LIBM
#define O_SINF sinf
#define O_COSF cosf
#define O_TANF tanf
#define O_ACOSF acosf
#define O_ATAN2F atan2f
#else
#define O_SINF iq_sinf
#define O_COSF iq_cosf
#define O_TANF iq_tanf
#define O_ACOSF iq_acosf
#define O_ATAN2F iq_atan2f
#endif
#define O_FMAXF iq_fmaxf
#define O_FMINF iq_fminf

/* ------------------------------------------------------------------ iqvec (vector.h:30-395) */
typedef struct { float x, y, z, w; } vec4;

static inline vec4 V(float x, float y, float z, float w) { vec4 r = {x, y, z, w}; return r; }
static inline vec4 vsplat(float s) { return V(s, s, s, s); }                      /* vector.h:44 */
static inline vec4 vneg(vec4 a) { return V(-a.x, -a.y, -a.z, -a.w); }             /* :76-78 */
static inline vec4 vsub(vec4 a, vec4 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline vec4 vadd(vec4 a, vec4 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline vec4 vmul(vec4 a, float s) { return V(a.x * s, a.y * s, a.z * s, a.w * s); } /* :91-96 */
static inline vec4 vdiv(vec4 a, float s) { const float inv = 1 / s; return vmul(a, inv); }  /* :100-103 */
static inline vec4 vhad(vec4 a, vec4 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static inline float dot3(vec4 a, vec4 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* :194-196 */
static inline float dot4(vec4 a, vec4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
static inline float length3(vec4 a) { return sqrtf(dot3(a, a)); }
static inline vec4 cross3(vec4 a, vec4 o) {                                        /* :219-224 */
    return V(a.y * o.z - a.z * o.y, a.z * o.x - a.x * o.z, a.x * o.y - a.y * o.x, 0.0f);
}
static inline int is_null3(vec4 a) {                                              /* :225-232 */
    const float eps = 0.00001f;
    return fabsf(a.x - 0.0f) < eps && fabsf(a.y - 0.0f) < eps && fabsf(a.z - 0.0f) < eps;
}
static inline vec4 normalized3(vec4 a) {                                          /* :239-244 */
    if (is_null3(a)) return vsplat(0.0f);
    return vdiv(a, length3(a));
}

/* ------------------------------------------------------------------ iqmat (matrix.h, matrix.cu) */
typedef struct { float m[4][4]; } mat4;
typedef struct { float m[3][4]; } mat3;

static inline vec4 col_to_vec(const mat4* M, int c) {                             /* matrix.cu:33-35 */
    return V(M->m[0][c], M->m[1][c], M->m[2][c], M->m[3][c]);
}
enum { USAGE_DIRECTION = 0, USAGE_POINT = 1, USAGE_MISC = 2 };                   /* vector.h:33-40 */
/* iqvec::transformed (vector.h:371-383) */
static inline vec4 transformed(vec4 v, const mat4* M, int usage) {
    vec4 aux = v, r;
    if (usage == USAGE_POINT) aux.w = 1.0f;
    else if (usage == USAGE_DIRECTION) aux.w = 0.0f;
    r.x = dot4(aux, col_to_vec(M, 0));
    r.y = dot4(aux, col_to_vec(M, 1));
    r.z = dot4(aux, col_to_vec(M, 2));
    r.w = dot4(aux, col_to_vec(M, 3));
    return r;
}
/* iqvec::load(vec3, usage) (vector.h:48-50) */
static inline vec4 load3(const float* p, int usage) { return V(p[0], p[1], p[2], (float)usage); }

static mat3 mat3_ident(float val) {                                               /* matrix.cu:441-450 */
    mat3 r;
    memset(&r, 0, sizeof r);
    r.m[0][0] = r.m[1][1] = r.m[2][2] = val;
    return r;
}
static mat3 store3x3(const mat4* M) {                                             /* matrix.cu:50-60 */
    mat3 r = mat3_ident(1.0f);
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) r.m[i][j] = M->m[i][j];
    return r;
}
static mat3 mat3_transposed(const mat3* a) {                                      /* matrix.cu:488-498 */
    mat3 r = mat3_ident(1.0f);
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) r.m[j][i] = a->m[i][j];
    return r;
}
static float mat3_det(const mat3* a) {                                            /* matrix.cu:452-457 */
    const float (*m)[4] = a->m;
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
           m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
           m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
}
static mat3 mat3_inversed(const mat3* a) {                                        /* matrix.cu:459-480 */
    float det = mat3_det(a);
    if (fabsf(det) < 0.00001f) return mat3_ident(INFINITY);
    const float (*m)[4] = a->m;
    mat3 inv = mat3_ident(1.0f);
    inv.m[0][0] = (m[1][1] * m[2][2] - m[1][2] * m[2][1]) / det;
    inv.m[0][1] = -(m[0][1] * m[2][2] - m[0][2] * m[2][1]) / det;
    inv.m[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) / det;
    inv.m[1][0] = -(m[1][0] * m[2][2] - m[1][2] * m[2][0]) / det;
    inv.m[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) / det;
    inv.m[1][2] = -(m[0][0] * m[1][2] - m[0][2] * m[1][0]) / det;
    inv.m[2][0] = (m[1][0] * m[2][1] - m[1][1] * m[2][0]) / det;
    inv.m[2][1] = -(m[0][0] * m[2][1] - m[0][1] * m[2][0]) / det;
    inv.m[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) / det;
    return inv;
}
static mat4 load3x3(const mat3* a, float val) {                                   /* matrix.cu:37-48 */
    mat4 r;
    memset(&r, 0, sizeof r);
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0f;                         /* iqmat() */
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) r.m[i][j] = a->m[i][j];
    r.m[3][3] = val;
    return r;
}

/* ------------------------------------------------------------------ rng (random.cu:66-107) */
static inline float rand_real(iq_xorwow_state* s, float lo, float hi) {          /* random.cu:66-70 */
    float t = (float)iq_xorwow_next(s) / (float)UINT32_MAX;
    return t * (hi - lo) + lo;
}
static inline vec4 cosine_weighted(iq_xorwow_state* s) {                         /* random.cu:96-107 */
    const float u1 = rand_real(s, 0.0f, 1.0f);
    const float u2 = rand_real(s, 0.0f, 1.0f);
    float phi = 2 * IQ_PI * u1;
    float x = O_COSF(phi) * sqrtf(u2);
    float y = O_SINF(phi) * sqrtf(u2);
    float z = sqrtf(1.0f - u2);
    return V(x, y, z, 0.0f);
}

/* ------------------------------------------------------------------ geometry (shape.cu) */
typedef struct { vec4 o, d; } ray_t;                                              /* ray.h:5-19 */
static inline vec4 ray_at(const ray_t* r, float t) { return vadd(r->o, vmul(r->d, t)); }

enum { MAT_NONE = 0, MAT_EMISSIVE = 1, MAT_OREN_NAYAR = 2 };
/* mat: MAT_*; albedo / param of the hit primitive's material (param: emissive strength or the
 * clamped Oren-Nayar sigma) */
typedef struct { vec4 p, n; float t; int front_face; int mat; vec4 albedo; float param; } hit_record;  /* shape.h:7-14 */

static int triangle_intersect(vec4 v0, vec4 v1, vec4 v2, vec4 n0, vec4 n1, vec4 n2,
                              const ray_t* r, float t_min, float t_max, hit_record* hr) {
    const vec4 v0v1 = vsub(v1, v0);                                               /* shape.cu:65-103 */
    const vec4 v0v2 = vsub(v2, v0);
    const vec4 pvec = cross3(r->d, v0v2);
    float det = dot3(v0v1, pvec);
    if (fabsf(fabsf(det)) < 0.000001f) return 0;                                  /* is_zero, iqmath.h:28-31 */
    det = 1 / det;
    vec4 tvec = vsub(r->o, v0);
    const float u = dot3(tvec, pvec) * det;
    if (u < 0.0f || u > 1.0f) return 0;
    vec4 qvec = cross3(tvec, v0v1);
    const float v = dot3(r->d, qvec) * det;
    if (v < 0.0f || u + v > 1.0f) return 0;
    const float t = dot3(v0v2, qvec) * det;
    if (t < t_min || t_max < t) return 0;
    hr->t = t;
    hr->p = ray_at(r, t);
    hr->n = vadd(vadd(vmul(n0, 1.0f - u - v), vmul(n1, u)), vmul(n2, v));
    hr->n = normalized3(hr->n);
    hr->front_face = dot3(r->d, cross3(v0v1, v0v2)) < 0.0f;
    if (!hr->front_face) hr->n = vneg(hr->n);
    return 1;
}

static int sphere_intersect(vec4 c, float radius, const ray_t* r, float t_min, float t_max,
                            hit_record* hr) {
    const vec4 oc = vsub(c, r->o);                                                /* shape.cu:13-46 */
    const float halfb = dot3(r->d, oc);
    const float cc = dot3(oc, oc) - radius * radius;
    const float delta = halfb * halfb - cc;
    if (delta < 0.0f) return 0;
    float t = halfb - sqrtf(delta);
    if (t_max < t) return 0;
    if (t < t_min) {
        t = halfb + sqrtf(delta);
        if (t < t_min) return 0;
    }
    hr->t = t;
    hr->p = ray_at(r, t);
    hr->n = vdiv(vsub(hr->p, c), radius);
    hr->front_face = dot3(r->d, hr->n) < 0.0f;
    if (!hr->front_face) hr->n = vneg(hr->n);
    return 1;
}

/* ------------------------------------------------------------------ materials (material.cu) */
typedef struct { vec4 attenuation; float pdf_val; float cos_law_weight; } scatter_record;

typedef struct { vec4 w_[3]; } onb_t;                                             /* onb.h:5-25 */
static onb_t onb_make(vec4 n) {
    onb_t b;
    b.w_[2] = normalized3(n);
    vec4 a = (fabsf(b.w_[2].x) > 0.9f) ? V(0.0f, 1.0f, 0.0f, 0.0f) : V(1.0f, 0.0f, 0.0f, 0.0f);
    b.w_[1] = normalized3(cross3(b.w_[2], a));
    b.w_[0] = cross3(b.w_[1], b.w_[2]);
    return b;
}
static vec4 onb_to_world(const onb_t* b, vec4 v) {
    return vadd(vadd(vmul(b->w_[0], v.x), vmul(b->w_[1], v.y)), vmul(b->w_[2], v.z));
}

/* The reference's materials (path_tracer.cu:248-249): oren_nayar(iqvec(.5,.5,.5,0), 1.0) on every
 * sphere, emissive(iqvec(1.0f), 10.0f) on every triangle. A packet may carry a material table instead
 * (iqpt.h). */
static const vec4 ON_ALBEDO = {0.5f, 0.5f, 0.5f, 0.0f};
static const float ON_SIGMA = 1.0f;
static const vec4 EM_ALBEDO = {1.0f, 1.0f, 1.0f, 1.0f};
static const float EM_STRENGTH = 10.0f;

/* oren_nayar::oren_nayar clamps the roughness to [0, 1] (material.h:25-29) */
static float clamp_sigma(float r) { return r < 0.0f ? 0.0f : (r > 1.0f ? 1.0f : r); }

/* material of drawcall i of the given kind, into the hit record */
static void set_material(hit_record* hr, const iqpt_packet_desc* pk, int kind, uint32_t i) {
    if (!pk->materials) {
        hr->mat = kind == IQPT_MESH_TRIANGLES ? MAT_EMISSIVE : MAT_OREN_NAYAR;
        hr->albedo = kind == IQPT_MESH_TRIANGLES ? EM_ALBEDO : ON_ALBEDO;
        hr->param = kind == IQPT_MESH_TRIANGLES ? EM_STRENGTH : ON_SIGMA;
        return;
    }
    const uint32_t k = kind == IQPT_MESH_TRIANGLES ? pk->tri_dc_material[i] : pk->sphere_dc_material[i];
    const iqpt_material* m = &pk->materials[k];
    memcpy(&hr->albedo, m->albedo, sizeof hr->albedo);
    if (m->type == IQPT_MAT_EMISSIVE) {
        hr->mat = MAT_EMISSIVE;
        hr->param = m->param;
    } else {
        hr->mat = MAT_OREN_NAYAR;
        hr->param = clamp_sigma(m->param);
    }
}

static int oren_nayar_scatter(const ray_t* r_in, const hit_record* hr, scatter_record* srec,
                              ray_t* r_out, iq_xorwow_state* st) {
    onb_t uvw = onb_make(hr->n);                                                  /* material.cu:5-43 */
    const vec4 wo = vneg(r_in->d);
    r_out->o = vadd(hr->p, vmul(hr->n, 0.0001f));
    r_out->d = onb_to_world(&uvw, cosine_weighted(st));
    srec->pdf_val = dot3(hr->n, r_out->d) / IQ_PI;                                /* pdf, :45-48 */
    if (srec->pdf_val < 0.00001f) {
        r_out->o = vadd(hr->p, vmul(hr->n, 0.0001f));
        r_out->d = hr->n;
        srec->pdf_val = 1 / IQ_PI;
    }
    srec->cos_law_weight = O_FMAXF(0.0f, dot3(hr->n, r_out->d));
    const vec4 wi = r_out->d;
    const float sigma2 = hr->param * hr->param;
    const float A = 1.0f - 0.5f * sigma2 / (sigma2 + 0.33f);
    const float B = 0.45f * sigma2 / (sigma2 + 0.09f);
    const float phi_o = O_ATAN2F(wo.y, wo.x);
    const float phi_i = O_ATAN2F(wi.y, wi.x);
    const float costheta_o = O_FMAXF(0.0f, dot3(wo, hr->n));
    const float theta_o = costheta_o > 1.0f ? 0.0f : O_ACOSF(costheta_o);
    const float costheta_i = O_FMAXF(0.0f, dot3(wi, hr->n));
    const float theta_i = costheta_i > 1.0f ? 0.0f : O_ACOSF(costheta_i);
    const float alpha = O_FMAXF(theta_i, theta_o);
    const float beta = O_FMINF(theta_i, theta_o);
    const float coeff = A + B * O_COSF(phi_i - phi_o) * O_SINF(alpha) * O_TANF(beta);
    srec->attenuation = vdiv(vmul(hr->albedo, coeff), IQ_PI);
    return 1;
}

/* emissive::scatter (material.cu:50-57): m_strength * m_albedo */
static int emissive_scatter(const hit_record* hr, scatter_record* srec) {
    srec->attenuation = vmul(hr->albedo, hr->param);
    srec->cos_law_weight = 1.0f;
    srec->pdf_val = 1.0f;
    return 0;
}

/* ------------------------------------------------------------------ camera::get_ray (camera.cu:20-43) */
static ray_t camera_get_ray(const iqpt_camera* cam, uint32_t x, uint32_t y, iq_xorwow_state* st) {
    const mat4* inv_proj = (const mat4*)cam->inv_proj;
    const mat4* inv_view = (const mat4*)cam->inv_view;
    const float x_ndc = (((float)(uint16_t)x + rand_real(st, -0.5f, 0.5f)) / (float)cam->width) * 2 - 1;
    const float y_ndc = 1 - (((float)(uint16_t)y + rand_real(st, -0.5f, 0.5f)) / (float)cam->height) * 2;
    const vec4 p_ndc_near = V(x_ndc, y_ndc, 0.0f, 1.0f);
    const vec4 p_ndc_far = V(x_ndc, y_ndc, 1.0f, 1.0f);
    vec4 p_view_near = transformed(p_ndc_near, inv_proj, USAGE_POINT);
    p_view_near = vdiv(p_view_near, p_view_near.w);
    vec4 p_view_far = transformed(p_ndc_far, inv_proj, USAGE_POINT);
    p_view_far = vdiv(p_view_far, p_view_far.w);
    vec4 p_world_near = transformed(p_view_near, inv_view, USAGE_POINT);
    vec4 p_world_far = transformed(p_view_far, inv_view, USAGE_POINT);
    const vec4 dir = vsub(p_world_far, p_world_near);
    ray_t r;
    r.o = p_world_near;
    r.d = normalized3(dir);
    return r;
}

/* ------------------------------------------------------------------ ray_color (path_tracer.cu:231-328) */
#define ORACLE_MAX_DEPTH 64

static vec4 ray_color(const ray_t* r0, const iqpt_packet_desc* pk, const mat4* normal_mats,
                      int max_depth, iq_xorwow_state* st, int* rays_out) {
    const float t_min = 0.000001f, t_max = 999.99f;
    scatter_record ray_stack[ORACLE_MAX_DEPTH];
    memset(ray_stack, 0, sizeof(scatter_record) * (size_t)max_depth);
    ray_t crt_ray = *r0;
    int crt_depth;
    for (crt_depth = 0; crt_depth < max_depth; crt_depth++) {
        hit_record final_hr;
        memset(&final_hr, 0, sizeof final_hr);
        float closest_hit = t_max;
        int hit = 0;
        for (uint32_t i = 0; i < pk->num_drawcalls[IQPT_MESH_TRIANGLES]; i++) {
            const uint32_t mesh_id = pk->tri_mesh_dcs[i].mesh_id;
            const mat4* transform = (const mat4*)pk->tri_mesh_dcs[i].transform;
            const mat4* normal_matrix = &normal_mats[i];   /* load3x3(transpose(3x3).inverse()), :260 */
            const iqpt_tri_mesh* m = &pk->tri_meshes[mesh_id];
            for (uint32_t j = 0; j < m->num_indices; j += 3) {
                const iqpt_vertex* a = &m->vertices[m->indices[j + 0]];
                const iqpt_vertex* b = &m->vertices[m->indices[j + 1]];
                const iqpt_vertex* c = &m->vertices[m->indices[j + 2]];
                vec4 v0 = transformed(load3(a->pos, USAGE_POINT), transform, USAGE_MISC);
                vec4 v1 = transformed(load3(b->pos, USAGE_POINT), transform, USAGE_MISC);
                vec4 v2 = transformed(load3(c->pos, USAGE_POINT), transform, USAGE_MISC);
                vec4 n0 = transformed(load3(a->normal, USAGE_DIRECTION), normal_matrix, USAGE_MISC);
                vec4 n1 = transformed(load3(b->normal, USAGE_DIRECTION), normal_matrix, USAGE_MISC);
                vec4 n2 = transformed(load3(c->normal, USAGE_DIRECTION), normal_matrix, USAGE_MISC);
                hit_record hr;
                if (triangle_intersect(v0, v1, v2, n0, n1, n2, &crt_ray, t_min, closest_hit, &hr)) {
                    closest_hit = hr.t;
                    final_hr = hr;
                    set_material(&final_hr, pk, IQPT_MESH_TRIANGLES, i);
                    hit = 1;
                }
            }
        }
        for (uint32_t i = 0; i < pk->num_drawcalls[IQPT_MESH_SPHERES]; i++) {
            vec4 center;
            memcpy(&center, pk->sphere_dcs[i].center, sizeof center);
            hit_record hr;
            if (sphere_intersect(center, pk->sphere_dcs[i].radius, &crt_ray, t_min, closest_hit, &hr)) {
                closest_hit = hr.t;
                final_hr = hr;
                set_material(&final_hr, pk, IQPT_MESH_SPHERES, i);
                hit = 1;
            }
        }
        if (hit) {
            ray_t r_out;
            int cont = final_hr.mat == MAT_OREN_NAYAR
                           ? oren_nayar_scatter(&crt_ray, &final_hr, &ray_stack[crt_depth], &r_out, st)
                           : emissive_scatter(&final_hr, &ray_stack[crt_depth]);
            if (cont) {
                crt_ray = r_out;
            } else {
                crt_depth++;
                break;
            }
        } else {
            vec4 dir = crt_ray.d;
            const float a = (dir.y + 1.0f) * 0.5f;
            ray_stack[crt_depth].attenuation =
                vadd(vmul(vsplat(1.0f), 1.0f - a), vmul(V(0.5f, 0.7f, 1.0f, 0.0f), a));
            ray_stack[crt_depth].pdf_val = 1.0f;
            ray_stack[crt_depth].cos_law_weight = 1.0f;
            crt_depth++;
            break;
        }
    }
    *rays_out = crt_depth;
    const scatter_record* last = &ray_stack[crt_depth - 1];
    vec4 final_color = vmul(last->attenuation, last->cos_law_weight / last->pdf_val);
    for (int depth = crt_depth - 2; depth >= 0; depth--) {
        final_color = vhad(final_color,
                           vmul(ray_stack[depth].attenuation,
                                ray_stack[depth].cos_law_weight / ray_stack[depth].pdf_val));
    }
    return final_color;
}

/* uint8_t conversion of CUDA: NaN -> 0, saturate to [0, 255], truncate toward zero. */
static inline uint8_t to_u8(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}

/* ------------------------------------------------------------------ exported API (ctypes) */

static int check_packet(const iqpt_packet_desc* pk) {
    if (!pk) return IQPT_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < pk->num_drawcalls[IQPT_MESH_TRIANGLES]; i++) {
        uint32_t id = pk->tri_mesh_dcs[i].mesh_id;
        if (id >= pk->num_tri_meshes) return IQPT_ERR_INVALID_ARG;
        const iqpt_tri_mesh* m = &pk->tri_meshes[id];
        if (m->num_indices % 3) return IQPT_ERR_INVALID_ARG;
        for (uint32_t j = 0; j < m->num_indices; j++)
            if (m->indices[j] >= m->num_vertices) return IQPT_ERR_INVALID_ARG;
    }
    if (pk->materials) {
        for (int kind = 0; kind < 2; ++kind) {
            const uint32_t* idx = kind == IQPT_MESH_TRIANGLES ? pk->tri_dc_material : pk->sphere_dc_material;
            if (pk->num_drawcalls[kind] && !idx) return IQPT_ERR_INVALID_ARG;
            for (uint32_t i = 0; i < pk->num_drawcalls[kind]; i++)
                if (idx[i] >= pk->num_materials) return IQPT_ERR_INVALID_ARG;
        }
        for (uint32_t k = 0; k < pk->num_materials; k++)
            if (pk->materials[k].type != IQPT_MAT_EMISSIVE && pk->materials[k].type != IQPT_MAT_OREN_NAYAR)
                return IQPT_ERR_INVALID_ARG;
    }
    return IQPT_OK;
}

/* curand_init(seed, global pixel id, 0) for every pixel of the set; states: [npix][6] (v0..v4, d). */
int iqo_rng_init(uint32_t width, const iqpt_pixel_set* ps, uint64_t seed, uint32_t* states) {
    static uint32_t tables[32 * IQ_XORWOW_MAT_WORDS];
    static int have_tables = 0;
    if (!have_tables) {
        iq_xorwow_subseq_tables(tables, 32);
        have_tables = 1;
    }
    const uint32_t ncols = ps->x1 - ps->x0;
    const int64_t npix = (int64_t)ncols * ps->nrows;
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < npix; ++p) {
        uint32_t x = ps->x0 + (uint32_t)(p % ncols);
        uint32_t y = ps->y0 + (uint32_t)(p / ncols) * ps->ystep;
        uint64_t pid = (uint64_t)y * width + x;
        iq_xorwow_state s;
        iq_xorwow_init(seed, pid, tables, 32, &s);
        for (int k = 0; k < 5; ++k) states[p * 6 + k] = s.v[k];
        states[p * 6 + 5] = s.d;
    }
    return IQPT_OK;
}

/* Renders spp consecutive reference launches (frames frame0+1 .. frame0+spp) over the pixel set.
 * lin: [npix][4] float (in/out), bgra: [npix][4] (out), states: [npix][6] (in/out),
 * rays: [npix] (out, optional) closest-hit queries per pixel. Returns an iqpt_status. */
int iqo_render(const iqpt_packet_desc* pk, const iqpt_camera* cam, int max_depth,
               const iqpt_pixel_set* ps, uint64_t frame0, uint32_t spp,
               uint32_t* states, float* lin, uint8_t* bgra, uint64_t* rays, int nthreads) {
    if (!pk || !cam || !ps || !states || !lin || !bgra) return IQPT_ERR_INVALID_ARG;
    if (max_depth < 1 || max_depth > ORACLE_MAX_DEPTH) return IQPT_ERR_UNSUPPORTED;
    int st = check_packet(pk);
    if (st) return st;
    const uint32_t ntdc = pk->num_drawcalls[IQPT_MESH_TRIANGLES];
    mat4* normal_mats = (mat4*)malloc(sizeof(mat4) * (ntdc ? ntdc : 1));
    for (uint32_t i = 0; i < ntdc; i++) {
        mat3 s = store3x3((const mat4*)pk->tri_mesh_dcs[i].transform);
        mat3 t = mat3_transposed(&s);
        mat3 inv = mat3_inversed(&t);
        normal_mats[i] = load3x3(&inv, 1.0f);
    }
    const uint32_t ncols = ps->x1 - ps->x0;
    const uint32_t tiles_x = (ncols + 15) / 16, tiles_y = (ps->nrows + 15) / 16;
    const int64_t ntiles = (int64_t)tiles_x * tiles_y;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tile = 0; tile < ntiles; ++tile) {
        const uint32_t tx = (uint32_t)(tile % tiles_x), ty = (uint32_t)(tile / tiles_x);
        for (uint32_t k = ty * 16; k < ty * 16 + 16 && k < ps->nrows; ++k) {
            for (uint32_t c = tx * 16; c < tx * 16 + 16 && c < ncols; ++c) {
                const uint64_t p = (uint64_t)k * ncols + c;
                const uint32_t x = ps->x0 + c, y = ps->y0 + k * ps->ystep;
                iq_xorwow_state s;
                for (int q = 0; q < 5; ++q) s.v[q] = states[p * 6 + q];
                s.d = states[p * 6 + 5];
                vec4 lf = V(lin[p * 4 + 0], lin[p * 4 + 1], lin[p * 4 + 2], lin[p * 4 + 3]);
                uint64_t nrays = 0;
                for (uint32_t sidx = 0; sidx < spp; ++sidx) {
                    const uint64_t num_frame = frame0 + sidx + 1;            /* path_tracer.cu:401 */
                    vec4 path_color = vsplat(0.0f);                           /* :341 */
                    ray_t r = camera_get_ray(cam, x, y, &s);                  /* :342 */
                    int nr = 0;
                    vec4 color = ray_color(&r, pk, normal_mats, max_depth, &s, &nr);
                    nrays += (uint64_t)nr;
                    color.x = color.x > 1.0f ? 1.0f : (color.x < 0.0f ? 0.0f : color.x);
                    color.y = color.y > 1.0f ? 1.0f : (color.y < 0.0f ? 0.0f : color.y);
                    color.z = color.z > 1.0f ? 1.0f : (color.z < 0.0f ? 0.0f : color.z);
                    path_color = vadd(path_color, color);                     /* :348 */
                    lf.x = path_color.x / (float)num_frame + lf.x * ((float)(num_frame - 1) / (float)num_frame);
                    lf.y = path_color.y / (float)num_frame + lf.y * ((float)(num_frame - 1) / (float)num_frame);
                    lf.z = path_color.z / (float)num_frame + lf.z * ((float)(num_frame - 1) / (float)num_frame);
                }
                lin[p * 4 + 0] = lf.x;
                lin[p * 4 + 1] = lf.y;
                lin[p * 4 + 2] = lf.z;
                lin[p * 4 + 3] = lf.w;
                if (spp > 0) {                                                /* :360-365 */
                    bgra[p * 4 + 0] = to_u8(255.0f * sqrtf(lf.z));
                    bgra[p * 4 + 1] = to_u8(255.0f * sqrtf(lf.y));
                    bgra[p * 4 + 2] = to_u8(255.0f * sqrtf(lf.x));
                    bgra[p * 4 + 3] = 255;
                }
                for (int q = 0; q < 5; ++q) states[p * 6 + q] = s.v[q];
                states[p * 6 + 5] = s.d;
                if (rays) rays[p] = nrays;
            }
        }
    }
    free(normal_mats);
    return IQPT_OK;
}

/* ------------------------------------------------------------------ unit hooks for the tests */
void iqo_get_ray(const iqpt_camera* cam, uint32_t x, uint32_t y, uint32_t* state6, float* o4, float* d4) {
    iq_xorwow_state s;
    for (int q = 0; q < 5; ++q) s.v[q] = state6[q];
    s.d = state6[5];
    ray_t r = camera_get_ray(cam, x, y, &s);
    memcpy(o4, &r.o, 16);
    memcpy(d4, &r.d, 16);
    for (int q = 0; q < 5; ++q) state6[q] = s.v[q];
    state6[5] = s.d;
}
int iqo_triangle_intersect(const float* v0, const float* v1, const float* v2, const float* n0,
                           const float* n1, const float* n2, const float* o, const float* d,
                           float t_min, float t_max, float* t_out, float* p4, float* n4, int* front) {
    ray_t r;
    memcpy(&r.o, o, 16);
    memcpy(&r.d, d, 16);
    vec4 a, b, c, na, nb, nc;
    memcpy(&a, v0, 16); memcpy(&b, v1, 16); memcpy(&c, v2, 16);
    memcpy(&na, n0, 16); memcpy(&nb, n1, 16); memcpy(&nc, n2, 16);
    hit_record hr;
    int hit = triangle_intersect(a, b, c, na, nb, nc, &r, t_min, t_max, &hr);
    if (hit) { *t_out = hr.t; memcpy(p4, &hr.p, 16); memcpy(n4, &hr.n, 16); *front = hr.front_face; }
    return hit;
}
int iqo_sphere_intersect(const float* c4, float radius, const float* o, const float* d, float t_min,
                         float t_max, float* t_out, float* p4, float* n4, int* front) {
    ray_t r;
    memcpy(&r.o, o, 16);
    memcpy(&r.d, d, 16);
    vec4 c;
    memcpy(&c, c4, 16);
    hit_record hr;
    int hit = sphere_intersect(c, radius, &r, t_min, t_max, &hr);
    if (hit) { *t_out = hr.t; memcpy(p4, &hr.p, 16); memcpy(n4, &hr.n, 16); *front = hr.front_face; }
    return hit;
}
void iqo_onb(const float* n4, float* u4, float* v4, float* w4) {
    vec4 n;
    memcpy(&n, n4, 16);
    onb_t b = onb_make(n);
    memcpy(u4, &b.w_[0], 16);
    memcpy(v4, &b.w_[1], 16);
    memcpy(w4, &b.w_[2], 16);
}
void iqo_cosine_weighted(uint32_t* state6, float* out4) {
    iq_xorwow_state s;
    for (int q = 0; q < 5; ++q) s.v[q] = state6[q];
    s.d = state6[5];
    vec4 v = cosine_weighted(&s);
    memcpy(out4, &v, 16);
    for (int q = 0; q < 5; ++q) state6[q] = s.v[q];
    state6[5] = s.d;
}
/* One Oren-Nayar scatter; returns pdf, cos weight and attenuation.x and the outgoing ray. */
void iqo_oren_nayar(const float* p4, const float* n4, const float* din4, uint32_t* state6,
                    float* att4, float* pdf, float* cosw, float* ro4, float* rd4) {
    ray_t rin, rout;
    memset(&rin, 0, sizeof rin);
    memcpy(&rin.d, din4, 16);
    hit_record hr;
    memset(&hr, 0, sizeof hr);
    memcpy(&hr.p, p4, 16);
    memcpy(&hr.n, n4, 16);
    hr.mat = MAT_OREN_NAYAR;
    hr.albedo = ON_ALBEDO;
    hr.param = ON_SIGMA;
    iq_xorwow_state s;
    for (int q = 0; q < 5; ++q) s.v[q] = state6[q];
    s.d = state6[5];
    scatter_record sr;
    oren_nayar_scatter(&rin, &hr, &sr, &rout, &s);
    memcpy(att4, &sr.attenuation, 16);
    *pdf = sr.pdf_val;
    *cosw = sr.cos_law_weight;
    memcpy(ro4, &rout.o, 16);
    memcpy(rd4, &rout.d, 16);
    for (int q = 0; q < 5; ++q) state6[q] = s.v[q];
    state6[5] = s.d;
}
void iqo_normal_matrix(const float* transform16, float* out16) {
    mat3 s = store3x3((const mat4*)transform16);
    mat3 t = mat3_transposed(&s);
    mat3 inv = mat3_inversed(&t);
    mat4 r = load3x3(&inv, 1.0f);
    memcpy(out16, &r, 64);
}
void iqo_transform_point(const float* p3, const float* m16, float* out4) {
    vec4 r = transformed(load3(p3, USAGE_POINT), (const mat4*)m16, USAGE_MISC);
    memcpy(out4, &r, 16);
}
/* libm hooks (shared FP policy) for tests/test_libm.py */
float iqo_sinf(float x) { return O_SINF(x); }
float iqo_cosf(float x) { return O_COSF(x); }
float iqo_tanf(float x) { return O_TANF(x); }
float iqo_acosf(float x) { return O_ACOSF(x); }
float iqo_asinf(float x) { return iq_asinf(x); }
float iqo_atan2f(float y, float x) { return O_ATAN2F(y, x); }
void iqo_libm_batch(int fn, const float* a, const float* b, float* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = O_SINF(a[i]); break;
        case 1: out[i] = O_COSF(a[i]); break;
        case 2: out[i] = O_TANF(a[i]); break;
        case 3: out[i] = O_ACOSF(a[i]); break;
        case 4: out[i] = O_ATAN2F(a[i], b[i]); break;
        case 5: out[i] = iq_asinf(a[i]); break;
        case 6: out[i] = iq_atanf(a[i]); break;
        default: out[i] = 0.0f;
        }
    }
}
int iqo_xorwow_tables(uint32_t* out, int count) { iq_xorwow_subseq_tables(out, count); return 0; }
void iqo_xorwow_seed(uint64_t seed, uint32_t* state6) {
    iq_xorwow_state s;
    iq_xorwow_seed(seed, &s);
    for (int q = 0; q < 5; ++q) state6[q] = s.v[q];
    state6[5] = s.d;
}
uint32_t iqo_xorwow_next(uint32_t* state6) {
    iq_xorwow_state s;
    for (int q = 0; q < 5; ++q) s.v[q] = state6[q];
    s.d = state6[5];
    uint32_t r = iq_xorwow_next(&s);
    for (int q = 0; q < 5; ++q) state6[q] = s.v[q];
    state6[5] = s.d;
    return r;
}
int iqo_has_glibc_libm(void) {
#ifdef IQO_GLIBC_LIBM
    return 1;
#else
    return 0;
#endif
}
