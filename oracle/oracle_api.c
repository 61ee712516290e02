/*
 * oracle/oracle_api.c — flat C entry points for tests (ctypes).
 * TEST INFRASTRUCTURE ONLY: tests/, bench.py cpu_baseline and
 * __graft_entry__.smoke() are the only callers.
 */
#include "plonk.h"
#include "poseidon.h"
#include "fft.h"
#include "merkle.h"
#include "challenger.h"
#include <omp.h>
#include <stdlib.h>
#include <string.h>

void ora_permute(uint64_t *s) { ps_permute(s); }
void ora_hash_no_pad(const uint64_t *in, size_t n, uint64_t *out) { ps_hash_no_pad(in, n, out); }
void ora_hash_or_noop(const uint64_t *in, size_t n, uint64_t *out) { ps_hash_or_noop(in, n, out); }
void ora_two_to_one(const uint64_t *a, const uint64_t *b, uint64_t *out) { ps_two_to_one(a, b, out); }
void ora_hash_pad(const uint64_t *in, size_t n, uint64_t *out) { ps_hash_pad(in, n, out); }
void ora_mul_many(const uint64_t *a, const uint64_t *b, uint64_t *o, size_t n) {
    for (size_t i = 0; i < n; i++) o[i] = gl_mul(a[i], b[i]);
}
void ora_fft(uint64_t *a, unsigned log_n) { or_fft(a, log_n); }
void ora_ifft(uint64_t *a, unsigned log_n) { or_ifft(a, log_n); }
void ora_coset_fft(uint64_t *a, unsigned log_n, uint64_t shift) { or_coset_fft(a, log_n, shift); }
void ora_coset_ifft(uint64_t *a, unsigned log_n, uint64_t shift) { or_coset_ifft(a, log_n, shift); }
void ora_lde(const uint64_t *c, unsigned log_n, unsigned rate_bits, uint64_t shift, uint64_t *out) {
    or_lde(c, log_n, rate_bits, shift, out);
}
uint64_t ora_root_of_unity(unsigned k) { return gl_root_of_unity(k); }

/* PolynomialBatch::from_values restated: values col-major [npolys][n] ->
 * coeffs (optional), LDE leaves row-major bit-reversed [N][npolys(+salt)],
 * Merkle cap.  Salt (row-major [N][salt]) appended to each leaf. */
int ora_commit_values(const uint64_t *vals, unsigned npolys, unsigned log_n, unsigned rate_bits, unsigned cap_h,
                      const uint64_t *salt, unsigned nsalt, int from_coeffs, uint64_t *coeffs_out,
                      uint64_t *leaves_out, uint64_t *cap_out) {
    size_t n = (size_t)1 << log_n, N = n << rate_bits;
    unsigned W = npolys + nsalt;
    uint64_t *co = malloc(n * 8), *lde = malloc(N * 8);
    uint64_t *leaves = leaves_out ? leaves_out : malloc(N * W * 8);
    for (unsigned p = 0; p < npolys; p++) {
        memcpy(co, vals + (size_t)p * n, n * 8);
        if (!from_coeffs) or_ifft(co, log_n);
        if (coeffs_out) memcpy(coeffs_out + (size_t)p * n, co, n * 8);
        or_lde(co, log_n, rate_bits, GL_GEN, lde);
        for (size_t j = 0; j < N; j++) leaves[rev_bits(j, log_n + rate_bits) * W + p] = lde[j];
    }
    for (size_t j = 0; j < N; j++)
        for (unsigned s = 0; s < nsalt; s++) leaves[j * W + npolys + s] = salt[j * nsalt + s];
    or_merkle_t *t = or_merkle_build(leaves, log_n + rate_bits, W, cap_h);
    if (!t) return -1;
    or_merkle_cap(t, cap_out);
    or_merkle_free(t);
    if (!leaves_out) free(leaves);
    free(co); free(lde);
    return 0;
}

int ora_merkle(const uint64_t *leaves, unsigned log_n, size_t width, unsigned cap_h, uint64_t *cap_out,
               const uint64_t *indices, size_t nidx, uint64_t *sibs_out) {
    or_merkle_t *t = or_merkle_build(leaves, log_n, width, cap_h);
    if (!t) return -1;
    or_merkle_cap(t, cap_out);
    for (size_t i = 0; i < nidx; i++) or_merkle_prove(t, indices[i], sibs_out + i * 4 * (log_n - cap_h));
    or_merkle_free(t);
    return 0;
}

/* full verification of a proof against verifier-only + common data bytes */
/* OpenMP threads of the prover/verifier loops (bench.py's cpu_baseline sizes
 * them to the host cores the job may use) */
void ora_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

int ora_verify(const uint8_t *vd, size_t vlen, const uint8_t *pb, size_t plen) {
    or_common_t c;
    or_verifier_only_t v;
    int e = or_parse_verifier(vd, vlen, &v, &c);
    if (e) return 100 - e;
    or_proof_t *p = NULL;
    e = or_parse_proof(pb, plen, &c, &p);
    if (e) { free(v.constants_sigmas_cap); return 200 - e; }
    int rc = or_verify(&c, &v, p);
    or_proof_free(p);
    free(v.constants_sigmas_cap);
    return rc;
}

/* parse + re-serialise (byte-identity test); returns written length or <0 */
long ora_proof_roundtrip(const uint8_t *cb, size_t clen, const uint8_t *pb, size_t plen, uint8_t *out) {
    or_common_t c;
    size_t used;
    int e = or_parse_common(cb, clen, &used, &c);
    if (e) return e;
    or_proof_t *p = NULL;
    e = or_parse_proof(pb, plen, &c, &p);
    if (e) return e - 100;
    size_t n = or_write_proof(p, out);
    or_proof_free(p);
    return (long)n;
}

long ora_common_roundtrip(const uint8_t *cb, size_t clen, uint8_t *out) {
    or_common_t c;
    size_t used;
    int e = or_parse_common(cb, clen, &used, &c);
    if (e) return e;
    if (used != clen) return -99;
    return (long)or_write_common(&c, out);
}

/* challenges of a proof (for golden vectors): out = betas,gammas,alphas (nc each),
 * zeta(2), fri_alpha(2), fri_betas(2 x layers), pow_response, query indices */
int ora_challenges(const uint8_t *vd, size_t vlen, const uint8_t *pb, size_t plen, uint64_t *out) {
    or_common_t c;
    or_verifier_only_t v;
    if (or_parse_verifier(vd, vlen, &v, &c)) return -1;
    or_proof_t *p = NULL;
    if (or_parse_proof(pb, plen, &c, &p)) return -2;
    or_challenges_t ch;
    or_get_challenges(&c, v.circuit_digest, p, &ch);
    size_t k = 0;
    unsigned nc = (unsigned)c.num_challenges;
    for (unsigned i = 0; i < nc; i++) out[k++] = ch.betas[i];
    for (unsigned i = 0; i < nc; i++) out[k++] = ch.gammas[i];
    for (unsigned i = 0; i < nc; i++) out[k++] = ch.alphas[i];
    out[k++] = ch.zeta.c0; out[k++] = ch.zeta.c1;
    out[k++] = ch.fri_alpha.c0; out[k++] = ch.fri_alpha.c1;
    for (unsigned l = 0; l < p->d.num_layers; l++) { out[k++] = ch.fri_betas[l].c0; out[k++] = ch.fri_betas[l].c1; }
    out[k++] = ch.pow_response;
    for (unsigned q = 0; q < p->d.nq; q++) out[k++] = ch.query_indices[q];
    or_proof_free(p);
    free(v.constants_sigmas_cap);
    return (int)k;
}

/* circuit digest = hash_no_pad(constants_sigmas_cap || hash_pad(domain_sep=[]) || degree_bits)
 * (upstream plonk/circuit_builder.rs build) — checked against verifier.bin */
void ora_circuit_digest(const uint64_t *cap, size_t cap_len, uint64_t degree_bits, uint64_t *out) {
    size_t m = cap_len * 4 + 4 + 1;
    uint64_t *buf = malloc(m * 8);
    memcpy(buf, cap, cap_len * 32);
    ps_hash_pad(NULL, 0, buf + cap_len * 4);
    buf[cap_len * 4 + 4] = degree_bits;
    ps_hash_no_pad(buf, m, out);
    free(buf);
}

/* Merkle self-consistency for proofs without verifier data: find the leaf
 * index (low nsib bits) whose path from `leaf` lands on some cap entry.
 * Returns the full index (cap entry << nsib | low bits) or -1. */
long ora_merkle_find_index(const uint64_t *leaf, size_t width, const uint64_t *sibs, unsigned nsib,
                           const uint64_t *cap, unsigned cap_h) {
    for (uint64_t low = 0; low < ((uint64_t)1 << nsib); low++) {
        gl_t cur[4];
        ps_hash_or_noop(leaf, width, cur);
        for (unsigned k = 0; k < nsib; k++) {
            gl_t o[4];
            if ((low >> k) & 1) ps_two_to_one(sibs + 4 * k, cur, o);
            else ps_two_to_one(cur, sibs + 4 * k, o);
            memcpy(cur, o, 32);
        }
        for (uint64_t ci = 0; ci < ((uint64_t)1 << cap_h); ci++)
            if (!memcmp(cur, cap + 4 * ci, 32)) return (long)((ci << nsib) | low);
    }
    return -1;
}

int or_prove(const uint8_t *common_bytes, size_t clen, const gl_t *consts_sigmas, const gl_t *wires,
             const gl_t *pis, size_t npis, uint8_t *proof_out, size_t out_cap, size_t *out_len,
             gl_t *cs_cap_out, gl_t *digest_out);
/* full CPU prove; also returns the verifier-only data (cap, digest) */
int ora_prove(const uint8_t *cb, size_t clen, const uint64_t *cs, const uint64_t *wires, const uint64_t *pis,
              size_t npis, uint8_t *out, size_t cap, size_t *len, uint64_t *cs_cap, uint64_t *digest) {
    return or_prove(cb, clen, cs, wires, pis, npis, out, cap, len, cs_cap, digest);
}

/* Witness check on H: every filtered gate constraint vanishes at every row,
 * and the copy constraints hold (permutation grand product == 1 for fixed
 * pseudo-random beta, gamma).  Returns -1 if satisfied, the first failing
 * row, or -2 for a failed permutation check, -3 for bad input. */
long ora_check_witness(const uint8_t *cb, size_t clen, const uint64_t *cs, const uint64_t *wires,
                       const uint64_t *pis, size_t npis) {
    or_common_t c;
    size_t used;
    if (or_parse_common(cb, clen, &used, &c) || used != clen) return -3;
    size_t n = (size_t)1 << c.degree_bits;
    unsigned W = (unsigned)c.num_wires, R = (unsigned)c.num_routed_wires, NC = (unsigned)c.num_constants;
    gl_t pih[4];
    ps_hash_no_pad(pis, npis, pih);
    gl_t lc[64], lw[256], out[512];
    for (size_t i = 0; i < n; i++) {
        for (unsigned k = 0; k < NC + R; k++) lc[k] = cs[(size_t)k * n + i];
        for (unsigned k = 0; k < W; k++) lw[k] = wires[(size_t)k * n + i];
        or_eval_gate_constraints_base(&c, lc, lw, pih, out);
        for (unsigned k = 0; k < c.num_gate_constraints; k++)
            if (out[k]) return (long)i;
    }
    gl_t beta = 0x1234567890abcdefULL % GL_P, gamma = 0x0fedcba987654321ULL % GL_P;
    gl_t w = gl_root_of_unity((unsigned)c.degree_bits), x = 1, num = 1, den = 1;
    for (size_t i = 0; i < n; i++) {
        for (unsigned j = 0; j < R; j++) {
            gl_t wv = wires[(size_t)j * n + i];
            num = gl_mul(num, gl_add(gl_add(wv, gl_mul(beta, gl_mul(c.k_is[j], x))), gamma));
            den = gl_mul(den, gl_add(gl_add(wv, gl_mul(beta, cs[(size_t)(NC + j) * n + i])), gamma));
        }
        x = gl_mul(x, w);
    }
    return num == den ? -1 : -2;
}

/* Values-form polynomial evaluation at extension points (layout-parity tests):
 * f(x) = (x^n - 1)/n * sum_r v_r w^r / (x - w^r) for v over H = <w>, |H| = n.
 * vals col-major [ncols][n]; xs [nx][2] (c0, c1); out [ncols][nx][2].  The
 * reference opens every preprocessed / wire column at the query points
 * g * w_N^rev(i) (base field) and at zeta (extension), so this is what the
 * fixture comparisons need. */
void ora_eval_values(const uint64_t *vals, size_t ncols, unsigned log_n, const uint64_t *xs, size_t nx,
                     uint64_t *out) {
    size_t n = (size_t)1 << log_n;
    gl_t w = gl_root_of_unity(log_n), ninv = gl_inv((gl_t)n);
    glx_t *wt = malloc(n * sizeof(glx_t));
    for (size_t k = 0; k < nx; k++) {
        glx_t x = glx(xs[2 * k], xs[2 * k + 1]);
        glx_t c = glx_scale(glx_sub(glx_exp_power_of_2(x, log_n), glx_from(1)), ninv);
        gl_t wr = 1;
        for (size_t r = 0; r < n; r++) {
            wt[r] = glx_scale(glx_mul(c, glx_inv(glx_sub(x, glx_from(wr)))), wr);
            wr = gl_mul(wr, w);
        }
        for (size_t col = 0; col < ncols; col++) {
            glx_t acc = glx_from(0);
            const uint64_t *v = vals + col * n;
            for (size_t r = 0; r < n; r++)
                if (v[r]) acc = glx_add(acc, glx_scale(wt[r], v[r]));
            out[(col * nx + k) * 2] = acc.c0;
            out[(col * nx + k) * 2 + 1] = acc.c1;
        }
    }
    free(wt);
}
