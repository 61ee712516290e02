/*
 * oracle/fft.h — radix-2 NTT family over Goldilocks.  TEST INFRASTRUCTURE ONLY.
 * Restates qp-plonky2-field 1.1.1 field/src/fft.rs + polynomial/mod.rs
 * (fft, ifft, coset_fft, coset_ifft, lde) — natural-order in and out.
 * Domain: w_n = primitive_root_of_unity(log n); coset shift g = GL_GEN.
 * Reference call site: PolynomialBatch::from_values/from_coeffs
 * (wormhole/prover/src/lib.rs:233-237 -> plonky2 fri/oracle.rs).
 */
#ifndef QP_ORACLE_FFT_H
#define QP_ORACLE_FFT_H
#include "gl.h"
void or_fft(gl_t *a, unsigned log_n);                 /* coeffs -> values (in place) */
void or_ifft(gl_t *a, unsigned log_n);                /* values -> coeffs (in place) */
void or_coset_fft(gl_t *a, unsigned log_n, gl_t shift);
void or_coset_ifft(gl_t *a, unsigned log_n, gl_t shift);
/* out[N] = coset_fft(zero-pad(coeffs[n], N), shift), N = n << rate_bits */
void or_lde(const gl_t *coeffs, unsigned log_n, unsigned rate_bits, gl_t shift, gl_t *out);
void or_reverse_index_bits(gl_t *a, unsigned log_n);
/* extension-field variants (componentwise, twiddles are base-field) */
void or_fft_ext(glx_t *a, unsigned log_n);
void or_coset_fft_ext(glx_t *a, unsigned log_n, gl_t shift);
#endif
