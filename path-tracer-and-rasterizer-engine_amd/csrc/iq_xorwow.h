/*
 * iq_xorwow.h — cuRAND-compatible XORWOW generator (host + device), written from the published
 * algorithm, no cuRAND / rocRAND code.
 *
 * The reference draws every random number through cuRAND's default generator
 * (curandState = XORWOW; IoniqRE/path_tracer.h:3, random.cu:66-70): per pixel
 * curand_init(1984, pixelid, 0, &state) (path_tracer.cu:45) and curand() per draw.
 * cuRAND (CUDA 12.6, IoniqRE.vcxproj:34) is an un-vendored NVIDIA dependency; its published
 * algorithm is restated here:
 *   - step (Marsaglia 2003 "xorwow"): t = v0 ^ (v0 >> 2); v0..v3 <- v1..v4;
 *     v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1)); d += 362437; return v4 + d
 *   - seeding: s0 = lo32(seed) ^ 0xaad26b49, s1 = hi32(seed) ^ 0xf7dcefdd,
 *     t0 = 1099087573 * s0, t1 = 2591861531 * s1, d = 6615241 + t1 + t0,
 *     v = {123456789 + t0, 362436069 ^ t0, 521288629 + t1, 88675123 ^ t1, 5783321 + t0}
 *   - subsequence k starts 2^67 * k draws later: v <- A^(k * 2^67) v over GF(2) (d is unchanged,
 *     2^67 * 362437 = 0 mod 2^32).
 * The jump matrices are computed here by GF(2) squaring of the one-step matrix A;
 * tests/test_xorwow.py checks A^(2^67) and A^(4*2^67) against the independent tables that ROCm
 * ships in rocrand_xorwow_precomputed.h. The seeding constants cannot be checked against cuRAND
 * in this environment: RNG parity with real cuRAND streams is unpinned.
 *
 * Matrix layout (same as rocRAND's, so the tables are directly comparable): a 160x160 GF(2)
 * matrix is stored as 160 columns of 5 words; column c = 32*i + j (input word i, bit j) lives at
 * m[c*5 .. c*5+4], and y = M x is the XOR of the columns of the set bits of x.
 */
#ifndef IQ_XORWOW_H
#define IQ_XORWOW_H

#include "iq_fp.h"

#define IQ_XORWOW_WORDS 5
#define IQ_XORWOW_MAT_WORDS (160 * 5)
#define IQ_XORWOW_WEYL 362437u

typedef struct iq_xorwow_state {
    uint32_t v[5];
    uint32_t d;
} iq_xorwow_state;

IQ_INLINE uint32_t iq_xorwow_next(iq_xorwow_state* s) {
    uint32_t t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1];
    s->v[1] = s->v[2];
    s->v[2] = s->v[3];
    s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += IQ_XORWOW_WEYL;
    return s->v[4] + s->d;
}

/* curand_init(seed, 0, 0): the seed scramble only. */
IQ_INLINE void iq_xorwow_seed(uint64_t seed, iq_xorwow_state* s) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
}

/* y = M x in place (x = 5 words). */
IQ_INLINE void iq_gf2_matvec(const uint32_t* m, uint32_t* x) {
    uint32_t r[5] = {0u, 0u, 0u, 0u, 0u};
    for (int i = 0; i < 5; ++i) {
        uint32_t w = x[i];
        for (int j = 0; j < 32; ++j) {
            uint32_t mask = 0u - ((w >> j) & 1u);
            const uint32_t* col = m + (i * 32 + j) * 5;
            r[0] ^= mask & col[0];
            r[1] ^= mask & col[1];
            r[2] ^= mask & col[2];
            r[3] ^= mask & col[3];
            r[4] ^= mask & col[4];
        }
    }
    for (int k = 0; k < 5; ++k) x[k] = r[k];
}

/* Host-side construction of the jump tables (host functions: never called from a kernel) ------ */

/* One-step matrix A: column c is the image of the unit state e_c under one xorwow step. */
static inline void iq_xorwow_step_matrix(uint32_t* a) {
    for (int c = 0; c < 160; ++c) {
        iq_xorwow_state s;
        for (int k = 0; k < 5; ++k) s.v[k] = 0u;
        s.v[c / 32] = 1u << (c % 32);
        s.d = 0u;
        iq_xorwow_next(&s);
        for (int k = 0; k < 5; ++k) a[c * 5 + k] = s.v[k];
    }
}

/* out = a * b (GF(2)); out may not alias a or b. Column c of a*b = a * (column c of b). */
static inline void iq_gf2_matmul(const uint32_t* a, const uint32_t* b, uint32_t* out) {
    for (int c = 0; c < 160; ++c) {
        uint32_t x[5];
        for (int k = 0; k < 5; ++k) x[k] = b[c * 5 + k];
        iq_gf2_matvec(a, x);
        for (int k = 0; k < 5; ++k) out[c * 5 + k] = x[k];
    }
}

/* tables[i] = A^(2^(67+i)) for i in [0, count): the per-bit subsequence jumps. */
static inline void iq_xorwow_subseq_tables(uint32_t* tables, int count) {
    uint32_t cur[IQ_XORWOW_MAT_WORDS], tmp[IQ_XORWOW_MAT_WORDS];
    iq_xorwow_step_matrix(cur);
    for (int i = 0; i < 67; ++i) {
        iq_gf2_matmul(cur, cur, tmp);
        for (int k = 0; k < IQ_XORWOW_MAT_WORDS; ++k) cur[k] = tmp[k];
    }
    for (int t = 0; t < count; ++t) {
        for (int k = 0; k < IQ_XORWOW_MAT_WORDS; ++k) tables[t * IQ_XORWOW_MAT_WORDS + k] = cur[k];
        iq_gf2_matmul(cur, cur, tmp);
        for (int k = 0; k < IQ_XORWOW_MAT_WORDS; ++k) cur[k] = tmp[k];
    }
}

/* curand_init(seed, subsequence, 0) given the per-bit tables (A^(2^(67+i)), i < nbits). */
IQ_INLINE void iq_xorwow_init(uint64_t seed, uint64_t subsequence, const uint32_t* tables,
                              int nbits, iq_xorwow_state* s) {
    iq_xorwow_seed(seed, s);
    for (int i = 0; i < nbits && subsequence; ++i, subsequence >>= 1) {
        if (subsequence & 1u) iq_gf2_matvec(tables + i * IQ_XORWOW_MAT_WORDS, s->v);
    }
}

/* random::real(state) of IoniqRE/random.cu:66-70: curand(state) / (float)UINT32_MAX.
 * (float)UINT32_MAX rounds to 4294967296.0f = 2^32, so the division is an exact power-of-two
 * scaling and equals the multiplication below bit for bit; u can be exactly 1.0f. */
IQ_INLINE float iq_u32_to_unit(uint32_t r) { return (float)r * 2.3283064365386963e-10f; }

#endif /* IQ_XORWOW_H */
