/* oracle/fft.c — see fft.h.  TEST INFRASTRUCTURE ONLY. */
#include "fft.h"
#include <stdlib.h>
#include <string.h>

void or_reverse_index_bits(gl_t *a, unsigned log_n) {
    size_t n = (size_t)1 << log_n;
    for (size_t i = 0; i < n; i++) {
        size_t j = rev_bits(i, log_n);
        if (j > i) { gl_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
}

static void ntt_core(gl_t *a, unsigned log_n, gl_t root) {
    size_t n = (size_t)1 << log_n;
    or_reverse_index_bits(a, log_n);
    for (unsigned s = 1; s <= log_n; s++) {
        size_t m = (size_t)1 << s, h = m >> 1;
        gl_t wm = gl_pow(root, n / m);
        gl_t *tw = malloc(h * sizeof(gl_t));
        tw[0] = 1;
        for (size_t j = 1; j < h; j++) tw[j] = gl_mul(tw[j - 1], wm);
        for (size_t k = 0; k < n; k += m)
            for (size_t j = 0; j < h; j++) {
                gl_t u = a[k + j], v = gl_mul(a[k + j + h], tw[j]);
                a[k + j] = gl_add(u, v);
                a[k + j + h] = gl_sub(u, v);
            }
        free(tw);
    }
}

void or_fft(gl_t *a, unsigned log_n) {
    if (log_n == 0) return;
    ntt_core(a, log_n, gl_root_of_unity(log_n));
}

void or_ifft(gl_t *a, unsigned log_n) {
    size_t n = (size_t)1 << log_n;
    if (log_n) ntt_core(a, log_n, gl_inv(gl_root_of_unity(log_n)));
    gl_t ninv = gl_inv(gl_from_u64(n));
    for (size_t i = 0; i < n; i++) a[i] = gl_mul(a[i], ninv);
}

void or_coset_fft(gl_t *a, unsigned log_n, gl_t shift) {
    size_t n = (size_t)1 << log_n;
    gl_t p = 1;
    for (size_t i = 0; i < n; i++) { a[i] = gl_mul(a[i], p); p = gl_mul(p, shift); }
    or_fft(a, log_n);
}

void or_coset_ifft(gl_t *a, unsigned log_n, gl_t shift) {
    size_t n = (size_t)1 << log_n;
    or_ifft(a, log_n);
    gl_t si = gl_inv(shift), p = 1;
    for (size_t i = 0; i < n; i++) { a[i] = gl_mul(a[i], p); p = gl_mul(p, si); }
}

void or_lde(const gl_t *coeffs, unsigned log_n, unsigned rate_bits, gl_t shift, gl_t *out) {
    size_t n = (size_t)1 << log_n, N = n << rate_bits;
    memcpy(out, coeffs, n * sizeof(gl_t));
    memset(out + n, 0, (N - n) * sizeof(gl_t));
    or_coset_fft(out, log_n + rate_bits, shift);
}

void or_fft_ext(glx_t *a, unsigned log_n) {
    size_t n = (size_t)1 << log_n;
    gl_t *c0 = malloc(n * sizeof(gl_t)), *c1 = malloc(n * sizeof(gl_t));
    for (size_t i = 0; i < n; i++) { c0[i] = a[i].c0; c1[i] = a[i].c1; }
    or_fft(c0, log_n);
    or_fft(c1, log_n);
    for (size_t i = 0; i < n; i++) a[i] = glx(c0[i], c1[i]);
    free(c0); free(c1);
}

void or_coset_fft_ext(glx_t *a, unsigned log_n, gl_t shift) {
    size_t n = (size_t)1 << log_n;
    gl_t p = 1;
    for (size_t i = 0; i < n; i++) { a[i] = glx_scale(a[i], p); p = gl_mul(p, shift); }
    or_fft_ext(a, log_n);
}
