/*
 * oracle/gl.h — Goldilocks field + quadratic extension, CPU restatement.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by,
 * or called from the product path (libqpgpu.so).  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() use it, as the checker.
 *
 * Restates qp-plonky2-field 1.1.1 (Cargo.lock:514-530, not vendored; upstream
 * plonky2 field/src/goldilocks_field.rs, field/src/goldilocks_extensions.rs):
 *   p = 2^64 - 2^32 + 1, canonical u64 representation.
 *   multiplicative generator g = 0xc65c18b67785d900 ([FIX] common.bin k_is,
 *   SURVEY.md A.1); 2-adic generator w_{2^32} = 7277203076849721926.
 *   Quadratic extension F[X]/(X^2 - 7).
 */
#ifndef QP_ORACLE_GL_H
#define QP_ORACLE_GL_H
#include <stdint.h>
#include <stddef.h>

typedef uint64_t gl_t;
typedef struct { gl_t c0, c1; } glx_t;

#define GL_P 0xFFFFFFFF00000001ULL
#define GL_EPS 0xFFFFFFFFULL /* 2^64 mod p */
#define GL_GEN 0xc65c18b67785d900ULL
#define GL_TWO_ADIC_GEN 7277203076849721926ULL
#define GL_TWO_ADICITY 32
#define GL_W 7ULL /* extension non-residue */

static inline gl_t gl_reduce(gl_t x) { return x >= GL_P ? x - GL_P : x; }

static inline gl_t gl_add(gl_t a, gl_t b) {
    unsigned __int128 s = (unsigned __int128)a + b;
    if (s >= GL_P) s -= GL_P;
    return (gl_t)s;
}
static inline gl_t gl_sub(gl_t a, gl_t b) { return a >= b ? a - b : a + (GL_P - b); }
static inline gl_t gl_neg(gl_t a) { return a ? GL_P - a : 0; }

/* reduce a 128-bit product: x = lo + 2^64 hi = lo + 2^64 (hh 2^32 + hl)
 * 2^64 = 2^32 - 1, 2^96 = -1  =>  x = lo - hh + hl (2^32 - 1)            */
static inline gl_t gl_reduce128(unsigned __int128 x) {
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    uint64_t hh = hi >> 32, hl = hi & 0xFFFFFFFFULL;
    uint64_t t0 = lo - hh;
    if (lo < hh) t0 -= GL_EPS; /* borrow: add p == subtract eps mod 2^64 */
    uint64_t t1 = hl * GL_EPS;
    uint64_t r = t0 + t1;
    if (r < t1) r += GL_EPS; /* carry: 2^64 = eps */
    return gl_reduce(r);
}
static inline gl_t gl_mul(gl_t a, gl_t b) { return gl_reduce128((unsigned __int128)a * b); }
static inline gl_t gl_sqr(gl_t a) { return gl_mul(a, a); }
static inline gl_t gl_pow(gl_t a, uint64_t e) {
    gl_t r = 1;
    while (e) { if (e & 1) r = gl_mul(r, a); a = gl_mul(a, a); e >>= 1; }
    return r;
}
static inline gl_t gl_inv(gl_t a) { return gl_pow(a, GL_P - 2); }
static inline gl_t gl_from_u64(uint64_t x) { return gl_reduce(x); }

/* primitive 2^k-th root of unity, upstream Field::primitive_root_of_unity */
static inline gl_t gl_root_of_unity(unsigned k) {
    gl_t r = GL_TWO_ADIC_GEN;
    for (unsigned i = k; i < GL_TWO_ADICITY; i++) r = gl_sqr(r);
    return r;
}

/* ---------------- quadratic extension ---------------- */
static inline glx_t glx(gl_t a, gl_t b) { glx_t r = {a, b}; return r; }
static inline glx_t glx_from(gl_t a) { return glx(a, 0); }
static inline glx_t glx_add(glx_t a, glx_t b) { return glx(gl_add(a.c0, b.c0), gl_add(a.c1, b.c1)); }
static inline glx_t glx_sub(glx_t a, glx_t b) { return glx(gl_sub(a.c0, b.c0), gl_sub(a.c1, b.c1)); }
static inline glx_t glx_neg(glx_t a) { return glx(gl_neg(a.c0), gl_neg(a.c1)); }
static inline glx_t glx_mul(glx_t a, glx_t b) {
    gl_t c0 = gl_add(gl_mul(a.c0, b.c0), gl_mul(GL_W, gl_mul(a.c1, b.c1)));
    gl_t c1 = gl_add(gl_mul(a.c0, b.c1), gl_mul(a.c1, b.c0));
    return glx(c0, c1);
}
static inline glx_t glx_scale(glx_t a, gl_t s) { return glx(gl_mul(a.c0, s), gl_mul(a.c1, s)); }
static inline int glx_eq(glx_t a, glx_t b) { return a.c0 == b.c0 && a.c1 == b.c1; }
static inline int glx_is_zero(glx_t a) { return a.c0 == 0 && a.c1 == 0; }
static inline glx_t glx_inv(glx_t a) {
    /* (a0 - a1 X) / (a0^2 - 7 a1^2) */
    gl_t n = gl_sub(gl_sqr(a.c0), gl_mul(GL_W, gl_sqr(a.c1)));
    gl_t ni = gl_inv(n);
    return glx(gl_mul(a.c0, ni), gl_mul(gl_neg(a.c1), ni));
}
static inline glx_t glx_pow(glx_t a, uint64_t e) {
    glx_t r = glx(1, 0);
    while (e) { if (e & 1) r = glx_mul(r, a); a = glx_mul(a, a); e >>= 1; }
    return r;
}
static inline glx_t glx_exp_power_of_2(glx_t a, unsigned k) {
    for (unsigned i = 0; i < k; i++) a = glx_mul(a, a);
    return a;
}

static inline uint64_t rev_bits(uint64_t x, unsigned bits) {
    uint64_t r = 0;
    for (unsigned i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

#endif
