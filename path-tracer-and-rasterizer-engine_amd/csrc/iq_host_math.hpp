// iq_host_math.hpp — host-side vector/matrix arithmetic with the reference's operation order.
//
// Used by the packet relayout (world-space precompute), the camera constructor and the scene
// builder. Every function cites the reference routine whose rounding sequence it reproduces
// (IoniqRE/vector.h, IoniqRE/matrix.cu); compiled with -ffp-contract=off like the kernel.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#include "iq_fp.h"

namespace iq {

struct vec4 {
    float x = 0.0f, y = 0.0f, z = 0.0f, w = 0.0f;
    vec4() = default;
    vec4(float x_, float y_, float z_, float w_) : x(x_), y(y_), z(z_), w(w_) {}
    explicit vec4(float s) : x(s), y(s), z(s), w(s) {}                      // vector.h:44
};

inline vec4 operator-(const vec4& a) { return {-a.x, -a.y, -a.z, -a.w}; }
inline vec4 operator+(const vec4& a, const vec4& b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline vec4 operator-(const vec4& a, const vec4& b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline vec4 operator*(const vec4& a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }  // vector.h:91-96
inline vec4 operator/(const vec4& a, float s) { const float inv = 1 / s; return a * inv; }      // vector.h:100-103
inline float dot3(const vec4& a, const vec4& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // vector.h:194
inline float dot4(const vec4& a, const vec4& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
inline vec4 cross3(const vec4& a, const vec4& o) {                                              // vector.h:219
    return {a.y * o.z - a.z * o.y, a.z * o.x - a.x * o.z, a.x * o.y - a.y * o.x, 0.0f};
}
inline vec4 normalized3(const vec4& a) {                                                        // vector.h:239
    const float eps = 0.00001f;
    if (std::fabs(a.x - 0.0f) < eps && std::fabs(a.y - 0.0f) < eps && std::fabs(a.z - 0.0f) < eps)
        return vec4();
    return a / std::sqrt(dot3(a, a));
}

enum class usage { DIRECTION = 0, POINT = 1, MISCELLANEOUS = 2 };                              // vector.h:33

struct mat4 {
    float m[4][4];
    explicit mat4(float val = 1.0f) {                                                           // matrix.cu:21-29
        std::memset(m, 0, sizeof m);
        m[0][0] = m[1][1] = m[2][2] = m[3][3] = val;
    }
    static mat4 from(const float* d) { mat4 r; std::memcpy(r.m, d, sizeof r.m); return r; }
    vec4 row(int r) const { return {m[r][0], m[r][1], m[r][2], m[r][3]}; }
    vec4 col(int c) const { return {m[0][c], m[1][c], m[2][c], m[3][c]}; }
};

struct mat3 {
    float m[3][4];
    explicit mat3(float val = 1.0f) {                                                           // matrix.cu:441-450
        std::memset(m, 0, sizeof m);
        m[0][0] = m[1][1] = m[2][2] = val;
    }
};

// iqvec::transformed (vector.h:371-383)
inline vec4 transformed(const vec4& v, const mat4& M, usage u = usage::MISCELLANEOUS) {
    vec4 aux = v;
    if (u == usage::POINT) aux.w = 1.0f;
    else if (u == usage::DIRECTION) aux.w = 0.0f;
    return {dot4(aux, M.col(0)), dot4(aux, M.col(1)), dot4(aux, M.col(2)), dot4(aux, M.col(3))};
}
// iqvec::load(vec3, usage) (vector.h:48-50)
inline vec4 load3(const float* p, usage u) { return {p[0], p[1], p[2], (float)(int)u}; }

// iqmat::operator*(iqmat) (matrix.cu:62-82)
inline mat4 operator*(const mat4& a, const mat4& b) {
    mat4 r(0.0f);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = dot4(a.row(i), b.col(j));
    return r;
}

// iqmat::determinant (matrix.cu:125-139) — the 24-term expansion, evaluated left to right.
inline float determinant(const mat4& A) {
    const float (*m)[4] = A.m;
    return m[0][3] * m[1][2] * m[2][1] * m[3][0] - m[0][2] * m[1][3] * m[2][1] * m[3][0] -
           m[0][3] * m[1][1] * m[2][2] * m[3][0] + m[0][1] * m[1][3] * m[2][2] * m[3][0] +
           m[0][2] * m[1][1] * m[2][3] * m[3][0] - m[0][1] * m[1][2] * m[2][3] * m[3][0] -
           m[0][3] * m[1][2] * m[2][0] * m[3][1] + m[0][2] * m[1][3] * m[2][0] * m[3][1] +
           m[0][3] * m[1][0] * m[2][2] * m[3][1] - m[0][0] * m[1][3] * m[2][2] * m[3][1] -
           m[0][2] * m[1][0] * m[2][3] * m[3][1] + m[0][0] * m[1][2] * m[2][3] * m[3][1] +
           m[0][3] * m[1][1] * m[2][0] * m[3][2] - m[0][1] * m[1][3] * m[2][0] * m[3][2] -
           m[0][3] * m[1][0] * m[2][1] * m[3][2] + m[0][0] * m[1][3] * m[2][1] * m[3][2] +
           m[0][1] * m[1][0] * m[2][3] * m[3][2] - m[0][0] * m[1][1] * m[2][3] * m[3][2] -
           m[0][2] * m[1][1] * m[2][0] * m[3][3] + m[0][1] * m[1][2] * m[2][0] * m[3][3] +
           m[0][2] * m[1][0] * m[2][1] * m[3][3] - m[0][0] * m[1][2] * m[2][1] * m[3][3] -
           m[0][1] * m[1][0] * m[2][2] * m[3][3] + m[0][0] * m[1][1] * m[2][2] * m[3][3];
}

// iqmat::inversed (matrix.cu:141-271): cofactor expansion on the flat copy, then * (1/det).
inline mat4 inversed(const mat4& A) {
    float det = determinant(A);
    if (std::fabs(det) < 0.00001f) return mat4(INFINITY);
    float m[16], inv[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) m[i * 4 + j] = A.m[i][j];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    det = 1 / det;
    for (int i = 0; i < 16; ++i) inv[i] *= det;
    return mat4::from(inv);
}

// matrix.cu:50-60, 488-498, 452-457, 459-480, 37-48: the normal matrix of path_tracer.cu:260,
// load3x3(transform.store3x3().transpose().inverse()).
inline mat3 store3x3(const mat4& a) {
    mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j];
    return r;
}
inline mat3 transposed(const mat3& a) {
    mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[j][i] = a.m[i][j];
    return r;
}
inline float determinant(const mat3& a) {
    const float (*m)[4] = a.m;
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
           m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
           m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
}
inline mat3 inversed(const mat3& a) {
    const float det = determinant(a);
    if (std::fabs(det) < 0.00001f) return mat3(INFINITY);
    const float (*m)[4] = a.m;
    mat3 inv;
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
inline mat4 load3x3(const mat3& a, float val = 1.0f) {
    mat4 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j];
    r.m[3][3] = val;
    return r;
}
inline mat4 normal_matrix(const mat4& transform) {
    return load3x3(inversed(transposed(store3x3(transform))));
}

// Transform builders of matrix.cu:315-423. Transcendentals come from iq_fp.h so the host side is
// reproducible on every machine (the reference used the MSVC CRT).
inline mat4 look_at(const vec4& eye, const vec4& focus) {                                    // :315-324
    const vec4 aux(0.0f, 1.0f, 0.0f, 0.0f);
    vec4 forward = normalized3(focus - eye);
    vec4 right = cross3(aux, forward);
    vec4 up = cross3(forward, right);
    mat4 r(0.0f);
    const float v[16] = {right.x, up.x, forward.x, 0.0f,
                         right.y, up.y, forward.y, 0.0f,
                         right.z, up.z, forward.z, 0.0f,
                         -dot3(right, eye), -dot3(up, eye), -dot3(forward, eye), 1.0f};
    std::memcpy(r.m, v, sizeof v);
    return r;
}
inline mat4 perspective(float aspect_ratio, float fovh, float znear, float zfar) {          // :342-357
    if (znear < 0.0f || zfar < 0.0f || std::fabs(znear - zfar) < 0.00001f) return mat4(INFINITY);
    const float y_scale = 1.0f / iq_tanf((float)(fovh * 0.5));
    const float x_scale = y_scale / aspect_ratio;
    mat4 r(0.0f);
    r.m[0][0] = x_scale;
    r.m[1][1] = y_scale;
    r.m[2][2] = zfar / (zfar - znear);
    r.m[2][3] = 1.0f;
    r.m[3][2] = -znear * zfar / (zfar - znear);
    return r;
}
inline mat4 scale(const vec4& f) { mat4 r; r.m[0][0] = f.x; r.m[1][1] = f.y; r.m[2][2] = f.z; return r; }
inline mat4 translate(const vec4& o) { mat4 r; r.m[3][0] = o.x; r.m[3][1] = o.y; r.m[3][2] = o.z; return r; }
inline mat4 rotation_x(float a) {                                                            // :373-383
    mat4 r; const float s = iq_sinf(a), c = iq_cosf(a);
    r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = -s; r.m[2][2] = c; return r;
}
inline mat4 rotation_y(float a) {                                                            // :384-394
    mat4 r; const float s = iq_sinf(a), c = iq_cosf(a);
    r.m[0][0] = c; r.m[0][2] = -s; r.m[2][0] = s; r.m[2][2] = c; return r;
}
inline mat4 rotation_z(float a) {                                                            // :395-405
    mat4 r; const float s = iq_sinf(a), c = iq_cosf(a);
    r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = -s; r.m[1][1] = c; return r;
}
inline float to_radians(float angle) { return angle * IQ_PI / 180.0f; }                     // iqmath.h:17-20

}  // namespace iq
