/* layout_probe.c — development tool: localise where a preprocessed or witness
 * column of the native circuit differs from the reference's, given the
 * reference's evaluations of that column at a few points (the query leaves and
 * openings of tests/golden/dummy_proof*.bin).
 *
 * A column f over H = <w> (n = 2^log_n) evaluates at x not in H as
 *   f(x) = sum_r f_r L_r(x),  L_r(x) = (x^n - 1)/n * w^r / (x - w^r).
 * With D(x) = ref(x) - ours(x), a hypothesis "the columns differ only on rows
 * S" is an overdetermined linear system in the |S| unknown row differences.
 * Not shipped; built by tools/layout_probe.py with gcc.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../oracle/gl.h"

static gl_t *g_wpow = NULL;
static unsigned g_log_n = 0;

static void ensure_wpow(unsigned log_n) {
    if (g_wpow && g_log_n == log_n) return;
    free(g_wpow);
    size_t n = (size_t)1 << log_n;
    g_wpow = malloc(n * 8);
    gl_t w = gl_root_of_unity(log_n), x = 1;
    for (size_t i = 0; i < n; i++) { g_wpow[i] = x; x = gl_mul(x, w); }
    g_log_n = log_n;
}

/* out[k*nr + j] = L_{rows[j]}(xs[k]) */
void lp_lagrange(const gl_t *xs, size_t nx, unsigned log_n, const uint32_t *rows, size_t nr, gl_t *out) {
    ensure_wpow(log_n);
    gl_t ninv = gl_inv((gl_t)1 << log_n);
    for (size_t k = 0; k < nx; k++) {
        gl_t zh = gl_mul(gl_sub(gl_pow(xs[k], (uint64_t)1 << log_n), 1), ninv);
        for (size_t j = 0; j < nr; j++) {
            gl_t wr = g_wpow[rows[j]];
            out[k * nr + j] = gl_mul(zh, gl_mul(wr, gl_inv(gl_sub(xs[k], wr))));
        }
    }
}

/* barycentric evaluation of ncols columns [ncols][n] at nx points: out[c*nx + k] */
void lp_eval(const gl_t *vals, size_t ncols, unsigned log_n, const gl_t *xs, size_t nx, gl_t *out) {
    ensure_wpow(log_n);
    size_t n = (size_t)1 << log_n;
    gl_t ninv = gl_inv((gl_t)n);
    gl_t *lag = malloc(n * 8);
    for (size_t k = 0; k < nx; k++) {
        gl_t zh = gl_mul(gl_sub(gl_pow(xs[k], n), 1), ninv);
        /* batch inversion of (x - w^r) */
        gl_t *pre = malloc(n * 8);
        gl_t acc = 1;
        for (size_t r = 0; r < n; r++) { pre[r] = acc; acc = gl_mul(acc, gl_sub(xs[k], g_wpow[r])); }
        gl_t inv = gl_inv(acc);
        for (size_t r = n; r-- > 0;) {
            gl_t d = gl_sub(xs[k], g_wpow[r]);
            lag[r] = gl_mul(zh, gl_mul(g_wpow[r], gl_mul(inv, pre[r])));
            inv = gl_mul(inv, d);
        }
        free(pre);
        for (size_t c = 0; c < ncols; c++) {
            const gl_t *v = vals + c * n;
            unsigned __int128 s = 0;
            gl_t t = 0;
            for (size_t r = 0; r < n; r++) {
                if (!v[r]) continue;
                t = gl_add(t, gl_mul(v[r], lag[r]));
            }
            (void)s;
            out[c * nx + k] = t;
        }
    }
    free(lag);
}

/* Solve A d = b (m equations, u unknowns, m >= u) over GF(p): uses Gaussian
 * elimination with the first independent equations, then checks the rest.
 * Returns 1 if consistent (d filled), 0 if inconsistent, -1 if rank < u. */
int lp_solve(const gl_t *A_in, const gl_t *b_in, size_t m, size_t u, gl_t *d) {
    gl_t *A = malloc(m * (u + 1) * 8);
    for (size_t i = 0; i < m; i++) {
        memcpy(A + i * (u + 1), A_in + i * u, u * 8);
        A[i * (u + 1) + u] = b_in[i];
    }
    size_t row = 0;
    int full = 1;
    for (size_t col = 0; col < u; col++) {
        size_t piv = row;
        while (piv < m && A[piv * (u + 1) + col] == 0) piv++;
        if (piv == m) { full = 0; continue; }
        if (piv != row)
            for (size_t j = 0; j <= u; j++) {
                gl_t t = A[row * (u + 1) + j];
                A[row * (u + 1) + j] = A[piv * (u + 1) + j];
                A[piv * (u + 1) + j] = t;
            }
        gl_t inv = gl_inv(A[row * (u + 1) + col]);
        for (size_t j = col; j <= u; j++) A[row * (u + 1) + j] = gl_mul(A[row * (u + 1) + j], inv);
        for (size_t i = 0; i < m; i++) {
            if (i == row) continue;
            gl_t f = A[i * (u + 1) + col];
            if (!f) continue;
            for (size_t j = col; j <= u; j++)
                A[i * (u + 1) + j] = gl_sub(A[i * (u + 1) + j], gl_mul(f, A[row * (u + 1) + j]));
        }
        row++;
    }
    int ok = 1;
    for (size_t i = row; i < m; i++)
        if (A[i * (u + 1) + u]) { ok = 0; break; }
    if (ok && d) {
        /* read back solution (pivot columns in order) */
        size_t r = 0;
        for (size_t col = 0; col < u && r < row; col++) {
            if (A[r * (u + 1) + col] == 1) { d[col] = A[r * (u + 1) + u]; r++; }
            else d[col] = 0;
        }
    }
    free(A);
    if (!full) return ok ? -1 : 0;
    return ok;
}

/* For each window [a, a+w) (a in [a0,a1) step s), test whether D is explained
 * by differences on those rows only.  hits[] receives consistent starts. */
/* Lfull: [nx][n] Lagrange matrix from lp_lagrange over all rows */
long lp_window_scan(const gl_t *D, const gl_t *Lfull, size_t nx, unsigned log_n, unsigned w, unsigned a0,
                    unsigned a1, unsigned step, uint32_t *hits, size_t maxhits) {
    size_t nh = 0, n = (size_t)1 << log_n;
    gl_t *A = malloc(nx * w * 8);
    for (unsigned a = a0; a < a1 && nh < maxhits; a += step) {
        for (size_t k = 0; k < nx; k++)
            for (unsigned j = 0; j < w; j++) A[k * w + j] = Lfull[k * n + ((a + j) & (n - 1))];
        if (lp_solve(A, D, nx, w, NULL) == 1) hits[nh++] = a;
    }
    free(A);
    return (long)nh;
}

/* Two-segment shift model for an indicator column: rows of S below a stay,
 * rows of S at or above a move by delta.  target[k] = sum_{r in S'} L_r(x_k).
 * Reports (a, delta) pairs that reproduce target exactly. */
long lp_shift_scan(const gl_t *target, const gl_t *xs, size_t nx, unsigned log_n, const uint8_t *inS, int dmin,
                   int dmax, int32_t *hits, size_t maxhits) {
    ensure_wpow(log_n);
    size_t n = (size_t)1 << log_n, nh = 0;
    gl_t ninv = gl_inv((gl_t)n);
    gl_t *pre0 = malloc((n + 1) * nx * 8), *suf = malloc((n + 1) * nx * 8), *lag = malloc(n * 8);
    /* prefix sums of unshifted */
    for (size_t k = 0; k < nx; k++) {
        gl_t zh = gl_mul(gl_sub(gl_pow(xs[k], n), 1), ninv);
        gl_t acc = 0;
        for (size_t r = 0; r < n; r++) {
            pre0[r * nx + k] = acc;
            if (inS[r]) acc = gl_add(acc, gl_mul(zh, gl_mul(g_wpow[r], gl_inv(gl_sub(xs[k], g_wpow[r])))));
        }
        pre0[n * nx + k] = acc;
    }
    for (int d = dmin; d <= dmax; d++) {
        for (size_t k = 0; k < nx; k++) {
            gl_t zh = gl_mul(gl_sub(gl_pow(xs[k], n), 1), ninv);
            gl_t acc = 0;
            suf[n * nx + k] = 0;
            for (size_t r = n; r-- > 0;) {
                if (inS[r]) {
                    size_t rr = (size_t)(((long)r + d) & (long)(n - 1));
                    acc = gl_add(acc, gl_mul(zh, gl_mul(g_wpow[rr], gl_inv(gl_sub(xs[k], g_wpow[rr])))));
                }
                suf[r * nx + k] = acc;
            }
        }
        for (size_t a = 0; a <= n && nh < maxhits; a++) {
            size_t k = 0;
            for (; k < nx; k++)
                if (gl_add(pre0[a * nx + k], a < n ? suf[a * nx + k] : 0) != target[k]) break;
            if (k == nx) { hits[2 * nh] = (int32_t)a; hits[2 * nh + 1] = d; nh++; }
        }
    }
    free(pre0); free(suf); free(lag);
    return (long)nh;
}

/* out[k*ncols + c] = sum_r L[k*n + r] * vals[c*n + r]  (column evaluation at nx points) */
void lp_matvec(const gl_t *L, size_t nx, size_t n, const gl_t *vals, size_t ncols, gl_t *out) {
    for (size_t c = 0; c < ncols; c++) {
        const gl_t *v = vals + c * n;
        for (size_t k = 0; k < nx; k++) {
            const gl_t *l = L + k * n;
            gl_t t = 0;
            for (size_t r = 0; r < n; r++)
                if (v[r]) t = gl_add(t, gl_mul(v[r], l[r]));
            out[k * ncols + c] = t;
        }
    }
}
