/* layout_scan.c — development tool (not shipped): scans the position of a
 * known block of rows against evaluations of a preprocessed column
 * combination at the fixture's LDE points.
 *
 * For every candidate start r0, the hypothesis column is
 *   h[r] = head for r < r0,  h[r0 + k] = tail[k] (k < ntail),  0 after,
 * and the residual (meas - h)(x) is tested for sparsity with
 * ls_rational_fit (layout_sparse.c).  Prints r0 and the sparse rows of every
 * candidate whose residual is at most s_max-sparse.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "../oracle/gl.h"

int ls_rational_fit(const gl_t *xs, const gl_t *R, size_t m, unsigned s_max, gl_t *q);
long ls_roots(const gl_t *q, unsigned s, unsigned log_n, uint32_t *rows, size_t maxr);

/* Lagrange basis L_r(x) = (x^n - 1)/n * w^r / (x - w^r), table [r][k] */
static gl_t *lagrange_table(const gl_t *xs, size_t m, unsigned log_n) {
    size_t n = (size_t)1 << log_n;
    gl_t *T = malloc(n * m * 8);
    gl_t w = gl_root_of_unity(log_n), ninv = gl_inv((gl_t)n);
    for (size_t k = 0; k < m; k++) {
        gl_t c = gl_mul(gl_sub(gl_pow(xs[k], n), 1), ninv), wr = 1;
        for (size_t r = 0; r < n; r++) {
            T[r * m + k] = gl_mul(c, gl_mul(wr, gl_inv(gl_sub(xs[k], wr))));
            wr = gl_mul(wr, w);
        }
    }
    return T;
}

/* meas[k]: measured combination at xs[k].  Returns number of hits. */
long ls_block_scan(const gl_t *xs, const gl_t *meas, size_t m, unsigned log_n, gl_t head, const gl_t *tail,
                   size_t ntail, unsigned s_max, uint32_t r0_lo, uint32_t r0_hi, uint32_t *hits, int32_t *hit_s,
                   uint32_t *hit_rows, size_t max_hits) {
    size_t n = (size_t)1 << log_n;
    gl_t *T = lagrange_table(xs, m, log_n);
    gl_t *pre = calloc((n + 1) * m, 8); /* pre[r][k] = sum_{i<r} L_i(x_k) */
    for (size_t r = 0; r < n; r++)
        for (size_t k = 0; k < m; k++) pre[(r + 1) * m + k] = gl_add(pre[r * m + k], T[r * m + k]);
    gl_t *R = malloc(m * 8), *q = malloc((s_max + 1) * 8);
    gl_t *xn = malloc(m * 8);
    for (size_t k = 0; k < m; k++) xn[k] = gl_mul((gl_t)n, gl_inv(gl_sub(gl_pow(xs[k], n), 1)));
    long nh = 0;
    for (uint32_t r0 = r0_lo; r0 < r0_hi && r0 + ntail <= n; r0++) {
        for (size_t k = 0; k < m; k++) {
            gl_t h = gl_mul(head, pre[r0 * m + k]);
            for (size_t t = 0; t < ntail; t++) h = gl_add(h, gl_mul(tail[t], T[(r0 + t) * m + k]));
            R[k] = gl_mul(gl_sub(meas[k], h), xn[k]);
        }
        int s = ls_rational_fit(xs, R, m, s_max, q);
        if (s < 0) continue;
        if ((size_t)nh < max_hits) {
            hits[nh] = r0;
            hit_s[nh] = s;
            uint32_t rows[64] = {0};
            long nr = s ? ls_roots(q, (unsigned)s, log_n, rows, 64) : 0;
            for (long i = 0; i < 16; i++) hit_rows[nh * 16 + i] = i < nr ? rows[i] : 0xFFFFFFFFu;
        }
        nh++;
    }
    free(T); free(pre); free(R); free(q); free(xn);
    return nh;
}

/* evaluations of the Lagrange basis for callers: out[r*m+k] */
void ls_lagrange(const gl_t *xs, size_t m, unsigned log_n, gl_t *out) {
    size_t n = (size_t)1 << log_n;
    gl_t *T = lagrange_table(xs, m, log_n);
    for (size_t i = 0; i < n * m; i++) out[i] = T[i];
    free(T);
}
