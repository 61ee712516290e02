/* layout_sparse.c — development tool next to layout_probe.c: sparse-difference
 * tests of a preprocessed column against the reference's evaluations of it.
 *
 * A column f over H = <w> (n = 2^log_n) evaluated at x not in H is
 *   f(x) = (x^n - 1)/n * sum_r f_r w^r / (x - w^r),
 * so for D = ref - ours, R(x) = D(x) n / (x^n - 1) is a rational function whose
 * denominator is prod_{r in S} (x - w^r), S = rows where the columns differ.
 * ls_rational_fit finds the smallest |S| <= s_max consistent with R at the
 * sample points (Berlekamp-Welch style linear system) and the rows it names.
 * ls_shift_evals gives ours(w^-d x) for all d at once (one NTT per point), so a
 * rotated copy of a column can be tested the same way.
 * Not shipped; built by tools/layout_sparse.py with gcc.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../oracle/gl.h"

int lp_solve(const gl_t *A_in, const gl_t *b_in, size_t m, size_t u, gl_t *d);

static void ntt(gl_t *a, unsigned log_n, gl_t w) {
    size_t n = (size_t)1 << log_n;
    for (size_t i = 1, j = 0; i < n; i++) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { gl_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        gl_t wl = gl_pow(w, n / len);
        for (size_t i = 0; i < n; i += len) {
            gl_t x = 1;
            for (size_t j = 0; j < len / 2; j++) {
                gl_t u = a[i + j], v = gl_mul(a[i + j + len / 2], x);
                a[i + j] = gl_add(u, v);
                a[i + j + len / 2] = gl_sub(u, v);
                x = gl_mul(x, wl);
            }
        }
    }
}

/* coefficients of the column (values over H in natural order) */
void ls_coeffs(const gl_t *vals, unsigned log_n, gl_t *coeffs) {
    size_t n = (size_t)1 << log_n;
    memcpy(coeffs, vals, n * 8);
    ntt(coeffs, log_n, gl_inv(gl_root_of_unity(log_n)));
    gl_t ninv = gl_inv((gl_t)n);
    for (size_t i = 0; i < n; i++) coeffs[i] = gl_mul(coeffs[i], ninv);
}

/* out[k*n + d] = f(w^-d * xs[k]) where f has the given coefficients */
void ls_shift_evals(const gl_t *coeffs, unsigned log_n, const gl_t *xs, size_t nx, gl_t *out) {
    size_t n = (size_t)1 << log_n;
    gl_t winv = gl_inv(gl_root_of_unity(log_n));
    for (size_t k = 0; k < nx; k++) {
        gl_t *a = out + k * n, xp = 1;
        for (size_t j = 0; j < n; j++) { a[j] = gl_mul(coeffs[j], xp); xp = gl_mul(xp, xs[k]); }
        ntt(a, log_n, winv);  /* a[d] = sum_j c_j x^j w^-dj */
    }
}

/* Smallest s <= s_max with R(x_k) = N(x_k)/Q(x_k), deg N < s, Q monic of
 * degree s.  Returns s (Q in q[0..s], q[s] = 1), 0 if R == 0, -1 if none. */
int ls_rational_fit(const gl_t *xs, const gl_t *R, size_t m, unsigned s_max, gl_t *q) {
    size_t k;
    for (k = 0; k < m && R[k] == 0; k++) {}
    if (k == m) return 0;
    for (unsigned s = 1; s <= s_max && 2 * s < m; s++) {
        size_t u = 2 * s;
        gl_t *A = malloc(m * u * 8), *b = malloc(m * 8), *d = malloc(u * 8);
        /* N(x) - R Q(x) = 0:  sum_{i<s} n_i x^i - R sum_{i<s} q_i x^i = R x^s */
        for (size_t r = 0; r < m; r++) {
            gl_t xp = 1;
            for (unsigned i = 0; i < s; i++) {
                A[r * u + i] = xp;
                A[r * u + s + i] = gl_neg(gl_mul(R[r], xp));
                xp = gl_mul(xp, xs[r]);
            }
            b[r] = gl_mul(R[r], xp);
        }
        int ok = lp_solve(A, b, m, u, d);
        if (ok == 1) {
            for (unsigned i = 0; i < s; i++) q[i] = d[s + i];
            q[s] = 1;
            free(A); free(b); free(d);
            return (int)s;
        }
        free(A); free(b); free(d);
    }
    return -1;
}

/* rows r in [0,n) with Q(w^r) = 0 */
long ls_roots(const gl_t *q, unsigned s, unsigned log_n, uint32_t *rows, size_t maxr) {
    size_t n = (size_t)1 << log_n, nr = 0;
    gl_t w = gl_root_of_unity(log_n), x = 1;
    for (size_t r = 0; r < n; r++) {
        gl_t v = 0;
        for (unsigned i = s + 1; i-- > 0;) v = gl_add(gl_mul(v, x), q[i]);
        if (v == 0 && nr < maxr) rows[nr++] = (uint32_t)r;
        x = gl_mul(x, w);
    }
    return (long)nr;
}
