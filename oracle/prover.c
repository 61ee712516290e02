/*
 * oracle/prover.c — plonky2 prove() restated on the CPU.  TEST INFRASTRUCTURE
 * ONLY: the byte-level checker for the HIP prover and bench.py's
 * cpu_baseline ("port"), never part of the product path.
 *
 * Follows qp-plonky2 1.1.1 (not vendored):
 *   plonk/prover.rs   prove, wires_permutation_partial_products_and_zs,
 *                     compute_quotient_polys, OpeningSet::new
 *   fri/oracle.rs     PolynomialBatch::{from_values, from_coeffs, prove_openings}
 *   fri/prover.rs     fri_proof, fri_committed_trees, fri_proof_of_work,
 *                     fri_prover_query_rounds
 * with the transcript of SURVEY.md A.4.  The PoW witness is the minimal one
 * (the reference's rayon find_any is nondeterministic; any valid witness
 * verifies — SURVEY.md 0.5(a)).  Non-zk (no salts).
 * Reference call site: WormholeProver::prove (wormhole/prover/src/lib.rs:233-237).
 */
#include "plonk.h"

/* Test-only: force the PoW witness instead of grinding for the minimal one.
 * The reference's find_any witness is nondeterministic, so
 * reproducing one of its proofs byte for byte needs its witness; the
 * transcript checks it like any other (ora_verify). */
static int or_pow_forced_on = 0;
static gl_t or_pow_forced = 0;
void ora_force_pow_witness(uint64_t w, int on) {
    or_pow_forced = w;
    or_pow_forced_on = on;
}

#include "poseidon.h"
#include "fft.h"
#include "merkle.h"
#include "challenger.h"
#include <stdlib.h>
#include <string.h>

typedef struct {
    unsigned npolys, log_n, rate_bits;
    gl_t *coeffs;   /* [npolys][n] */
    gl_t *leaves;   /* [N][npolys] row-major, leaf order */
    or_merkle_t *tree;
} batch_t;

static void batch_from_coeffs(batch_t *b, gl_t *coeffs, unsigned npolys, unsigned log_n, unsigned rate_bits,
                              unsigned cap_h) {
    size_t n = (size_t)1 << log_n, N = n << rate_bits;
    unsigned logN = log_n + rate_bits;
    b->npolys = npolys; b->log_n = log_n; b->rate_bits = rate_bits;
    b->coeffs = coeffs;
    b->leaves = malloc(N * npolys * sizeof(gl_t));
#pragma omp parallel for schedule(dynamic)
    for (unsigned p = 0; p < npolys; p++) {
        gl_t *lde = malloc(N * sizeof(gl_t));
        or_lde(coeffs + p * n, log_n, rate_bits, GL_GEN, lde);
        for (size_t j = 0; j < N; j++) b->leaves[rev_bits(j, logN) * npolys + p] = lde[j];
        free(lde);
    }
    b->tree = or_merkle_build(b->leaves, logN, npolys, cap_h);
}

static void batch_from_values(batch_t *b, const gl_t *values, unsigned npolys, unsigned log_n, unsigned rate_bits,
                              unsigned cap_h) {
    size_t n = (size_t)1 << log_n;
    gl_t *coeffs = malloc(n * npolys * sizeof(gl_t));
    memcpy(coeffs, values, n * npolys * sizeof(gl_t));
#pragma omp parallel for
    for (unsigned p = 0; p < npolys; p++) or_ifft(coeffs + p * n, log_n);
    batch_from_coeffs(b, coeffs, npolys, log_n, rate_bits, cap_h);
}

static void batch_free(batch_t *b) {
    free(b->coeffs); free(b->leaves); or_merkle_free(b->tree);
}

static glx_t eval_coeffs_ext(const gl_t *c, size_t n, glx_t x) {
    glx_t acc = glx(0, 0);
    for (size_t i = n; i-- > 0;) acc = glx_add(glx_mul(acc, x), glx_from(c[i]));
    return acc;
}

/* batch inverse (Montgomery) */
static void batch_inv(gl_t *v, size_t n) {
    gl_t *pre = malloc(n * sizeof(gl_t));
    gl_t acc = 1;
    for (size_t i = 0; i < n; i++) { pre[i] = acc; acc = gl_mul(acc, v[i]); }
    gl_t inv = gl_inv(acc);
    for (size_t i = n; i-- > 0;) { gl_t t = gl_mul(inv, pre[i]); inv = gl_mul(inv, v[i]); v[i] = t; }
    free(pre);
}

/* wires_permutation_partial_products_and_zs (plonk/prover.rs): values of
 * [Z_0..Z_nc-1, partial products of challenge 0, of challenge 1, ...] over H */
static void zs_values(const or_common_t *cp, unsigned log_n, const gl_t *consts_sigmas, const gl_t *wires,
                      const gl_t *betas, const gl_t *gammas, gl_t *zs_vals) {
    const or_common_t c = *cp;
    const size_t n = (size_t)1 << log_n;
    const unsigned nc = (unsigned)c.num_challenges, R = (unsigned)c.num_routed_wires;
    const unsigned NCONST = (unsigned)c.num_constants, npp = (unsigned)c.num_partial_products;
    const unsigned qdf = (unsigned)c.quotient_degree_factor;
    const gl_t w = gl_root_of_unity(log_n);
    const gl_t *sig = consts_sigmas + (size_t)NCONST * n;
    unsigned nchunks = (R + qdf - 1) / qdf;
    gl_t *chunkprod = malloc((size_t)n * nchunks * sizeof(gl_t));
    for (unsigned ch = 0; ch < nc; ch++) {
        gl_t x = 1;
        for (size_t i = 0; i < n; i++) {
            gl_t den[256], num[256];
            for (unsigned j = 0; j < R; j++) {
                gl_t wv = wires[(size_t)j * n + i];
                num[j] = gl_add(gl_add(wv, gl_mul(betas[ch], gl_mul(c.k_is[j], x))), gammas[ch]);
                den[j] = gl_add(gl_add(wv, gl_mul(betas[ch], sig[(size_t)j * n + i])), gammas[ch]);
            }
            batch_inv(den, R);
            for (unsigned k = 0; k < nchunks; k++) {
                gl_t pr = 1;
                for (unsigned j = k * qdf; j < (k + 1) * qdf && j < R; j++) pr = gl_mul(pr, gl_mul(num[j], den[j]));
                chunkprod[i * nchunks + k] = pr;
            }
            x = gl_mul(x, w);
        }
        gl_t z = 1;
        for (size_t i = 0; i < n; i++) {
            zs_vals[(size_t)ch * n + i] = z;
            gl_t acc = z;
            for (unsigned k = 0; k < nchunks; k++) {
                acc = gl_mul(acc, chunkprod[i * nchunks + k]);
                if (k < npp) zs_vals[((size_t)nc + ch * npp + k) * n + i] = acc;
            }
            z = acc;
        }
    }
    free(chunkprod);
}

/* compute_quotient_polys (plonk/prover.rs): the vanishing polynomial at every
 * point of the LDE coset from the leaf-order rows of the three committed
 * batches (constants||sigmas, wires, zs||partial products), alpha-reduced per
 * challenge, divided by Z_H, coset-iFFT'd and split: qcoeffs [nc*qdf][n]. */
static void quotient_coeffs(const or_common_t *cp, unsigned log_n, const gl_t *cs_leaves, const gl_t *w_leaves,
                            const gl_t *z_leaves, const gl_t *betas, const gl_t *gammas, const gl_t *alphas,
                            const gl_t *pih, gl_t *qcoeffs) {
    const or_common_t c = *cp;
    const unsigned rb = (unsigned)c.fri_params_config.rate_bits;
    const size_t n = (size_t)1 << log_n, N = n << rb;
    const unsigned logN = log_n + rb;
    const unsigned nc = (unsigned)c.num_challenges, R = (unsigned)c.num_routed_wires, W = (unsigned)c.num_wires;
    const unsigned NCONST = (unsigned)c.num_constants, npp = (unsigned)c.num_partial_products;
    const unsigned qdf = (unsigned)c.quotient_degree_factor;
    const unsigned ncs = NCONST + R, nzs = nc * (1 + npp);
    gl_t *qvals = malloc((size_t)nc * N * sizeof(gl_t)); /* natural point order */
    {
        const gl_t wN = gl_root_of_unity(logN);
        const unsigned nterms = nc + nc * (npp + 1) + (unsigned)c.num_gate_constraints;
        const unsigned nchunks = (R + qdf - 1) / qdf;
        /* 1/(x^n - 1) is 2^rb-periodic: x^n = g^n w_N^{i n} */
        gl_t zh_inv[64];
        for (size_t i = 0; i < ((size_t)1 << rb); i++)
            zh_inv[i] = gl_inv(gl_sub(gl_pow(gl_mul(GL_GEN, gl_pow(wN, i)), n), 1));
        const gl_t ninv = gl_inv(gl_from_u64(n));
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < N; i++) {
            gl_t terms[512];
            gl_t x = gl_mul(GL_GEN, gl_pow(wN, i));
            size_t li = rev_bits(i, logN), lin = rev_bits((i + ((size_t)1 << rb)) % N, logN);
            const gl_t *lc = cs_leaves + li * ncs;
            const gl_t *lw = w_leaves + li * W;
            const gl_t *lz = z_leaves + li * nzs;
            const gl_t *lzn = z_leaves + lin * nzs;
            unsigned k = 0;
            gl_t zh = gl_sub(gl_pow(x, n), 1);
            gl_t l0 = gl_mul(zh, gl_inv(gl_mul(gl_sub(x, 1), gl_from_u64(n))));
            (void)ninv;
            for (unsigned ch = 0; ch < nc; ch++) terms[k++] = gl_mul(l0, gl_sub(lz[ch], 1));
            for (unsigned ch = 0; ch < nc; ch++) {
                const gl_t *pp = lz + nc + ch * npp;
                for (unsigned ck = 0; ck < nchunks; ck++) {
                    gl_t num = 1, den = 1;
                    for (unsigned j = ck * qdf; j < (ck + 1) * qdf && j < R; j++) {
                        num = gl_mul(num, gl_add(gl_add(lw[j], gl_mul(betas[ch], gl_mul(c.k_is[j], x))), gammas[ch]));
                        den = gl_mul(den, gl_add(gl_add(lw[j], gl_mul(betas[ch], lc[NCONST + j])), gammas[ch]));
                    }
                    gl_t prev = ck == 0 ? lz[ch] : pp[ck - 1];
                    gl_t next = ck == nchunks - 1 ? lzn[ch] : pp[ck];
                    terms[k++] = gl_sub(gl_mul(prev, num), gl_mul(next, den));
                }
            }
            or_eval_gate_constraints_base(&c, lc, lw, pih, terms + k);
            k += (unsigned)c.num_gate_constraints;
            (void)nterms;
            gl_t zi = zh_inv[i & (((size_t)1 << rb) - 1)];
            for (unsigned ch = 0; ch < nc; ch++) {
                gl_t acc = 0;
                for (unsigned j = k; j-- > 0;) acc = gl_add(gl_mul(acc, alphas[ch]), terms[j]);
                qvals[(size_t)ch * N + i] = gl_mul(acc, zi);
            }
        }
    }
    for (unsigned ch = 0; ch < nc; ch++) {
        or_coset_ifft(qvals + (size_t)ch * N, logN, GL_GEN);
        for (unsigned j = 0; j < qdf; j++)
            memcpy(qcoeffs + ((size_t)ch * qdf + j) * n, qvals + (size_t)ch * N + (size_t)j * n, n * sizeof(gl_t));
    }
    free(qvals);
}

/* PolynomialBatch::prove_openings (fri/oracle.rs): the initial FRI polynomial
 * alpha^nc * (P_zeta(X) - P_zeta(zeta)) / (X - zeta) + (P_next(X) - P_next(g zeta)) / (X - g zeta),
 * P_zeta = the alpha-reduced polys of the 4 oracles in order, P_next = the
 * first nc polys of oracle 2 (the Z polys); fin gets n coefficients */
static void fri_initial(const gl_t *const coeffs[4], const unsigned npolys[4], unsigned nc, size_t n, glx_t alpha,
                        glx_t zeta, glx_t zeta_next, glx_t *fin) {
    /* zeta batch: all polys of the 4 oracles in order; Horner over the reversed list */
    glx_t *comp = calloc(n, sizeof(glx_t));
    for (int o = 3; o >= 0; o--)
        for (unsigned pi = npolys[o]; pi-- > 0;) {
            const gl_t *cf = coeffs[o] + (size_t)pi * n;
            for (size_t k = 0; k < n; k++) comp[k] = glx_add(glx_mul(comp[k], alpha), glx_from(cf[k]));
        }
    /* divide_by_linear(zeta) */
    glx_t *q1 = calloc(n, sizeof(glx_t));
    glx_t acc = glx(0, 0);
    for (size_t k = n; k-- > 1;) { acc = glx_add(glx_mul(acc, zeta), comp[k]); q1[k - 1] = acc; }
    /* next batch: Z polys */
    glx_t *comp2 = calloc(n, sizeof(glx_t));
    for (unsigned pi = nc; pi-- > 0;) {
        const gl_t *cf = coeffs[2] + (size_t)pi * n;
        for (size_t k = 0; k < n; k++) comp2[k] = glx_add(glx_mul(comp2[k], alpha), glx_from(cf[k]));
    }
    glx_t *q2 = calloc(n, sizeof(glx_t));
    acc = glx(0, 0);
    for (size_t k = n; k-- > 1;) { acc = glx_add(glx_mul(acc, zeta_next), comp2[k]); q2[k - 1] = acc; }
    glx_t ap = glx_pow(alpha, nc);
    for (size_t k = 0; k < n; k++) fin[k] = glx_add(glx_mul(q1[k], ap), q2[k]);
    free(comp); free(comp2); free(q1); free(q2);
}

int or_prove(const uint8_t *common_bytes, size_t clen, const gl_t *consts_sigmas, const gl_t *wires,
             const gl_t *pis, size_t npis, uint8_t *proof_out, size_t out_cap, size_t *out_len,
             gl_t *cs_cap_out, gl_t *digest_out) {
    or_common_t c;
    size_t used;
    if (or_parse_common(common_bytes, clen, &used, &c) || used != clen) return -1;
    if (c.hiding) return -2; /* zk salts not restated */
    or_dims_t d;
    or_dims(&c, &d);
    const unsigned log_n = d.log_n, rb = (unsigned)c.fri_params_config.rate_bits;
    const unsigned cap_h = (unsigned)c.fri_params_config.cap_height;
    const size_t n = (size_t)1 << log_n, N = n << rb;
    const unsigned logN = log_n + rb;
    const unsigned nc = (unsigned)c.num_challenges, R = (unsigned)c.num_routed_wires, W = (unsigned)c.num_wires;
    const unsigned NCONST = (unsigned)c.num_constants, npp = (unsigned)c.num_partial_products;
    const unsigned qdf = (unsigned)c.quotient_degree_factor;
    const unsigned ncs = NCONST + R, nzs = nc * (1 + npp), nq = nc * qdf;
    const size_t cap_len = (size_t)1 << cap_h;
    if (npis != c.num_public_inputs) return -3;

    /* preprocessing: constants || sigmas commitment + circuit digest */
    batch_t bcs, bw, bz, bq;
    batch_from_values(&bcs, consts_sigmas, ncs, log_n, rb, cap_h);
    gl_t cs_cap[64 * 4], digest[4];
    or_merkle_cap(bcs.tree, cs_cap);
    {
        gl_t buf[64 * 4 + 8];
        memcpy(buf, cs_cap, cap_len * 32);
        ps_hash_pad(NULL, 0, buf + cap_len * 4);
        buf[cap_len * 4 + 4] = log_n;
        ps_hash_no_pad(buf, cap_len * 4 + 5, digest);
    }
    if (cs_cap_out) memcpy(cs_cap_out, cs_cap, cap_len * 32);
    if (digest_out) memcpy(digest_out, digest, 32);

    or_proof_t *p = or_proof_alloc(&d, npis);
    memcpy(p->pis, pis, npis * sizeof(gl_t));
    gl_t pih[4];
    ps_hash_no_pad(pis, npis, pih);

    /* 1. wires */
    batch_from_values(&bw, wires, W, log_n, rb, cap_h);
    or_merkle_cap(bw.tree, p->wires_cap);
    or_chal_t t;
    or_chal_init(&t);
    or_chal_observe_n(&t, digest, 4);
    or_chal_observe_n(&t, pih, 4);
    or_chal_observe_n(&t, p->wires_cap, cap_len * 4);
    gl_t betas[4], gammas[4], alphas[4];
    for (unsigned i = 0; i < nc; i++) betas[i] = or_chal_get(&t);
    for (unsigned i = 0; i < nc; i++) gammas[i] = or_chal_get(&t);

    /* 2. partial products and Z (plonk/prover.rs wires_permutation_partial_products_and_zs) */
    gl_t *zs_vals = calloc((size_t)nzs * n, sizeof(gl_t)); /* [Z_0..Z_nc-1, pp_0[0..npp], pp_1..] */
    zs_values(&c, log_n, consts_sigmas, wires, betas, gammas, zs_vals);
    batch_from_values(&bz, zs_vals, nzs, log_n, rb, cap_h);
    free(zs_vals);
    or_merkle_cap(bz.tree, p->zs_cap);
    or_chal_observe_n(&t, p->zs_cap, cap_len * 4);
    for (unsigned i = 0; i < nc; i++) alphas[i] = or_chal_get(&t);

    /* 3. quotient polys (plonk/prover.rs compute_quotient_polys) */
    gl_t *qcoeffs = malloc((size_t)nq * n * sizeof(gl_t));
    quotient_coeffs(&c, log_n, bcs.leaves, bw.leaves, bz.leaves, betas, gammas, alphas, pih, qcoeffs);
    batch_from_coeffs(&bq, qcoeffs, nq, log_n, rb, cap_h);
    or_merkle_cap(bq.tree, p->quot_cap);
    or_chal_observe_n(&t, p->quot_cap, cap_len * 4);
    glx_t zeta = or_chal_get_ext(&t);

    /* 4. openings (OpeningSet::new) */
    const gl_t g_n = gl_root_of_unity(log_n);
    const glx_t zeta_next = glx_scale(zeta, g_n);
    for (unsigned i = 0; i < ncs; i++) p->constants[i] = eval_coeffs_ext(bcs.coeffs + (size_t)i * n, n, zeta);
    for (unsigned i = 0; i < W; i++) p->wires[i] = eval_coeffs_ext(bw.coeffs + (size_t)i * n, n, zeta);
    for (unsigned i = 0; i < nc; i++) {
        p->zs[i] = eval_coeffs_ext(bz.coeffs + (size_t)i * n, n, zeta);
        p->zs_next[i] = eval_coeffs_ext(bz.coeffs + (size_t)i * n, n, zeta_next);
    }
    for (unsigned i = 0; i < nc * npp; i++) p->pp[i] = eval_coeffs_ext(bz.coeffs + (size_t)(nc + i) * n, n, zeta);
    for (unsigned i = 0; i < nq; i++) p->quotient[i] = eval_coeffs_ext(bq.coeffs + (size_t)i * n, n, zeta);
    for (unsigned i = 0; i < ncs; i++) or_chal_observe_ext(&t, p->constants[i]);
    for (unsigned i = 0; i < W; i++) or_chal_observe_ext(&t, p->wires[i]);
    for (unsigned i = 0; i < nc; i++) or_chal_observe_ext(&t, p->zs[i]);
    for (unsigned i = 0; i < nc * npp; i++) or_chal_observe_ext(&t, p->pp[i]);
    for (unsigned i = 0; i < nq; i++) or_chal_observe_ext(&t, p->quotient[i]);
    for (unsigned i = 0; i < nc; i++) or_chal_observe_ext(&t, p->zs_next[i]);

    /* 5. FRI (PolynomialBatch::prove_openings + fri_proof) */
    glx_t alpha = or_chal_get_ext(&t);
    glx_t *fin = calloc(N, sizeof(glx_t)); /* final poly coefficients, zero-padded to N */
    {
        const gl_t *coeffs[4] = {bcs.coeffs, bw.coeffs, bz.coeffs, bq.coeffs};
        const unsigned npolys[4] = {bcs.npolys, bw.npolys, bz.npolys, bq.npolys};
        fri_initial(coeffs, npolys, nc, n, alpha, zeta, zeta_next, fin);
    }
    glx_t *vals = malloc(N * sizeof(glx_t));
    memcpy(vals, fin, N * sizeof(glx_t));
    or_coset_fft_ext(vals, logN, GL_GEN);
    or_merkle_t *ltrees[OR_MAX_LAYERS];
    glx_t betas_fri[OR_MAX_LAYERS];
    size_t cur = N;
    unsigned curlog = logN;
    gl_t shift = GL_GEN;
    glx_t *cf = fin;
    for (unsigned l = 0; l < d.num_layers; l++) {
        unsigned ab = d.arity_bits[l], ar = 1u << ab;
        /* reverse_index_bits + chunk(arity) -> leaves of 2*arity felts */
        size_t nleaves = cur >> ab;
        gl_t *leaves = malloc(cur * 2 * sizeof(gl_t));
        for (size_t j = 0; j < cur; j++) {
            glx_t v = vals[rev_bits(j, curlog)];
            leaves[2 * j] = v.c0; leaves[2 * j + 1] = v.c1;
        }
        ltrees[l] = or_merkle_build(leaves, curlog - ab, 2 * ar, cap_h);
        free(leaves);
        or_merkle_cap(ltrees[l], p->commit_caps + (size_t)l * cap_len * 4);
        or_chal_observe_n(&t, p->commit_caps + (size_t)l * cap_len * 4, cap_len * 4);
        betas_fri[l] = or_chal_get_ext(&t);
        /* fold coefficients: chunks of arity reduced with powers of beta */
        glx_t *nc2 = calloc(nleaves, sizeof(glx_t));
        for (size_t j = 0; j < nleaves; j++) {
            glx_t a = glx(0, 0);
            for (unsigned k = ar; k-- > 0;) a = glx_add(glx_mul(a, betas_fri[l]), cf[j * ar + k]);
            nc2[j] = a;
        }
        if (cf != fin) free(cf);
        cf = nc2;
        shift = gl_pow(shift, ar);
        cur = nleaves;
        curlog -= ab;
        free(vals);
        vals = malloc(cur * sizeof(glx_t));
        memcpy(vals, cf, cur * sizeof(glx_t));
        or_coset_fft_ext(vals, curlog, shift);
    }
    free(vals);
    for (unsigned i = 0; i < d.final_poly_len; i++) p->final_poly[i] = cf[i];
    if (cf != fin) free(cf);
    free(fin);
    for (unsigned i = 0; i < d.final_poly_len; i++) or_chal_observe_ext(&t, p->final_poly[i]);

    /* 6. proof of work: minimal witness (or the forced one, test-only) */
    if (or_pow_forced_on) {
        p->pow_witness = or_pow_forced;
        or_chal_observe(&t, or_pow_forced);
        (void)or_chal_get(&t);
    } else {
        gl_t st[12];
        memcpy(st, t.state, sizeof(st));
        for (unsigned i = 0; i < t.nin; i++) st[i] = t.in[i];
        unsigned pos = t.nin;
        const unsigned bits = c.fri_params_config.pow_bits;
        gl_t found = 0;
        int ok = 0;
        for (gl_t cand = 0; !ok; cand++) {
            gl_t s[12];
            memcpy(s, st, sizeof(s));
            s[pos] = cand;
            ps_permute(s);
            gl_t r = s[7];
            if ((r >> (64 - bits)) == 0) { found = cand; ok = 1; }
        }
        p->pow_witness = found;
        or_chal_observe(&t, found);
        (void)or_chal_get(&t);
    }

    /* 7. query rounds */
    for (unsigned q = 0; q < d.nq; q++) {
        size_t xi = or_chal_get(&t) % N;
        const batch_t *bs[4] = {&bcs, &bw, &bz, &bq};
        for (int o = 0; o < 4; o++) {
            memcpy(p->q_leaf[o][q], bs[o]->leaves + xi * bs[o]->npolys, bs[o]->npolys * sizeof(gl_t));
            or_merkle_prove(bs[o]->tree, xi, p->q_sib[o][q]);
        }
        for (unsigned l = 0; l < d.num_layers; l++) {
            unsigned ab = d.arity_bits[l], ar = 1u << ab;
            size_t li = xi >> ab;
            const gl_t *leaf = ltrees[l]->leaves + li * 2 * ar;
            for (unsigned k = 0; k < ar; k++) p->q_evals[l][q][k] = glx(leaf[2 * k], leaf[2 * k + 1]);
            or_merkle_prove(ltrees[l], li, p->q_lsib[l][q]);
            xi = li;
        }
    }
    for (unsigned l = 0; l < d.num_layers; l++) or_merkle_free(ltrees[l]);
    batch_free(&bcs); batch_free(&bw); batch_free(&bz); batch_free(&bq);

    size_t len = or_write_proof(p, NULL);
    if (out_len) *out_len = len;
    int rc = 0;
    if (proof_out) {
        if (len > out_cap) rc = -4;
        else or_write_proof(p, proof_out);
    }
    or_proof_free(p);
    return rc;
}

/* qp_quotient checker: commits the three value batches like or_prove and
 * returns quotient coefficients [nc*qdf][n] (plonk/prover.rs compute_quotient_polys) */
int ora_quotient(const uint8_t *common_bytes, size_t clen, const gl_t *consts_sigmas, const gl_t *wires,
                 const gl_t *zs_vals, const gl_t *betas, const gl_t *gammas, const gl_t *alphas, const gl_t *pih,
                 gl_t *qcoeffs_out) {
    or_common_t c;
    size_t used;
    if (or_parse_common(common_bytes, clen, &used, &c) || used != clen) return -1;
    or_dims_t d;
    or_dims(&c, &d);
    const unsigned log_n = d.log_n, rb = (unsigned)c.fri_params_config.rate_bits;
    const unsigned nc = (unsigned)c.num_challenges, R = (unsigned)c.num_routed_wires;
    const unsigned ncs = (unsigned)c.num_constants + R, nzs = nc * (1 + (unsigned)c.num_partial_products);
    batch_t bcs, bw, bz;
    batch_from_values(&bcs, consts_sigmas, ncs, log_n, rb, 0);
    batch_from_values(&bw, wires, (unsigned)c.num_wires, log_n, rb, 0);
    batch_from_values(&bz, zs_vals, nzs, log_n, rb, 0);
    quotient_coeffs(&c, log_n, bcs.leaves, bw.leaves, bz.leaves, betas, gammas, alphas, pih, qcoeffs_out);
    batch_free(&bcs); batch_free(&bw); batch_free(&bz);
    return 0;
}

/* one fri_committed_trees layer (fri/prover.rs): values = coset_fft(coeffs
 * zero-padded to 2^log_values, shift), reverse_index_bits, leaves of 2^ab ext
 * values; cap, and for leaf indices idx[] the leaf evals [2^ab][2] and siblings.
 * coeffs is [2][2^log_coeffs] (c0 row, c1 row) like the C ABI. */
int ora_fri_layer(const gl_t *coeffs, unsigned log_coeffs, unsigned log_values, gl_t shift, unsigned ab,
                  unsigned cap_h, gl_t *cap_out, const uint32_t *idx, unsigned nidx, gl_t *evals_out,
                  gl_t *sibs_out) {
    if (log_coeffs > log_values || ab + cap_h > log_values) return -1;
    const size_t Lc = (size_t)1 << log_coeffs, Lv = (size_t)1 << log_values;
    glx_t *vals = calloc(Lv, sizeof(glx_t));
    for (size_t i = 0; i < Lc; i++) vals[i] = glx(coeffs[i], coeffs[Lc + i]);
    or_coset_fft_ext(vals, log_values, shift);
    gl_t *leaves = malloc(Lv * 2 * sizeof(gl_t));
    for (size_t j = 0; j < Lv; j++) {
        glx_t v = vals[rev_bits(j, log_values)];
        leaves[2 * j] = v.c0; leaves[2 * j + 1] = v.c1;
    }
    free(vals);
    const size_t W = (size_t)2 << ab;
    const unsigned depth = log_values - ab - cap_h;
    or_merkle_t *t = or_merkle_build(leaves, log_values - ab, W, cap_h);
    free(leaves);
    or_merkle_cap(t, cap_out);
    for (unsigned q = 0; q < nidx; q++) {
        memcpy(evals_out + q * W, t->leaves + (size_t)idx[q] * W, W * sizeof(gl_t));
        or_merkle_prove(t, idx[q], sibs_out + (size_t)q * depth * 4);
    }
    or_merkle_free(t);
    return 0;
}

/* the coefficient fold of fri_committed_trees: chunks of 2^ab reduced with powers of beta */
void ora_fri_fold(const gl_t *coeffs, unsigned log_coeffs, unsigned ab, const gl_t *beta, gl_t *out) {
    const size_t L = (size_t)1 << log_coeffs, Lo = L >> ab, ar = (size_t)1 << ab;
    const glx_t b = glx(beta[0], beta[1]);
    for (size_t j = 0; j < Lo; j++) {
        glx_t a = glx(0, 0);
        for (size_t k = ar; k-- > 0;) a = glx_add(glx_mul(a, b), glx(coeffs[j * ar + k], coeffs[L + j * ar + k]));
        out[j] = a.c0; out[Lo + j] = a.c1;
    }
}

/* fri_proof_of_work: minimal witness for one duplex state (lanes 0..pos-1 hold
 * the pending inputs) */
gl_t ora_pow_grind(const gl_t *state, unsigned pos, unsigned bits) {
    for (gl_t cand = 0;; cand++) {
        gl_t s[12];
        memcpy(s, state, sizeof(s));
        s[pos] = cand;
        ps_permute(s);
        if ((s[7] >> (64 - bits)) == 0) return cand;
    }
}

/* qp_quotient checker for an arbitrary gate description (the layout of
 * include/qpgpu.h qp_gate_desc, mirrored here so the oracle includes nothing
 * of the product): builds the CommonCircuitData fields the vanishing
 * polynomial reads (k_is = g^j, plonky2's get_unique_coset_shifts) and runs
 * quotient_coeffs.  Values: consts_sigmas [num_constants + R][n], wires
 * [num_wires][n], zs_pp [2 * nchunks][n]. */
typedef struct {
    uint32_t num_gates, kind[16], param[16], param2[16], param3[16], selector_index[16];
    uint32_t num_selectors, group_lo[16], group_hi[16];
    uint32_t num_constants, num_routed_wires, num_wires, quotient_degree_factor, num_challenges,
        num_gate_constraints;
} ora_gate_desc_t;

static const uint32_t ORA_ID_OF_KIND[14] = {G_NOOP, G_CONSTANT, G_PUBLIC_INPUT, G_BASE_SUM, G_ARITHMETIC, G_POSEIDON,
                                            G_ARITH_EXT, G_MUL_EXT, G_RANDOM_ACCESS, G_EXPONENTIATION, G_REDUCING,
                                            G_REDUCING_EXT, G_POSEIDON_MDS, G_COSET_INTERP};

/* unfiltered constraints of gate gi of a description at one row: returns the
 * count (constants = the gate constants after the selector columns) */
long ora_gate_eval(const ora_gate_desc_t *g, unsigned gi, const gl_t *constants, const gl_t *wires,
                   const gl_t *pih, gl_t *out) {
    if (gi >= g->num_gates || g->kind[gi] >= 14) return -1;
    or_gate_t gt = {ORA_ID_OF_KIND[g->kind[gi]], g->param[gi], g->param2[gi], g->param3[gi]};
    return (long)or_gate_eval_base(&gt, constants, wires, pih, out);
}

int ora_quotient_desc(const ora_gate_desc_t *g, unsigned log_n, unsigned rate_bits, const gl_t *consts_sigmas,
                      const gl_t *wires, const gl_t *zs_vals, const gl_t *betas, const gl_t *gammas,
                      const gl_t *alphas, const gl_t *pih, gl_t *qcoeffs_out) {
    if (g->num_gates == 0 || g->num_gates > 16 || g->num_challenges != 2 || g->num_routed_wires > 256) return -1;
    or_common_t *c = calloc(1, sizeof(or_common_t));
    c->fri_params_config.rate_bits = rate_bits;
    c->degree_bits = log_n;
    c->num_challenges = 2;
    c->num_wires = g->num_wires;
    c->num_routed_wires = g->num_routed_wires;
    c->num_constants = g->num_constants;
    c->quotient_degree_factor = g->quotient_degree_factor;
    const unsigned nchunks = (g->num_routed_wires + g->quotient_degree_factor - 1) / g->quotient_degree_factor;
    c->num_partial_products = nchunks - 1;
    c->num_gate_constraints = g->num_gate_constraints;
    c->num_k_is = g->num_routed_wires;
    for (unsigned j = 0; j < g->num_routed_wires; j++) c->k_is[j] = gl_pow(GL_GEN, j);
    c->num_gates = g->num_gates;
    c->num_selector_indices = g->num_gates;
    for (unsigned i = 0; i < g->num_gates; i++) {
        if (g->kind[i] >= 14) { free(c); return -1; }
        c->gates[i].id = ORA_ID_OF_KIND[g->kind[i]];
        c->gates[i].p0 = g->param[i];
        c->gates[i].p1 = g->param2[i];
        c->gates[i].p2 = g->param3[i];
        c->selector_indices[i] = g->selector_index[i];
    }
    c->num_groups = g->num_selectors;
    for (unsigned i = 0; i < g->num_selectors; i++) { c->groups[i][0] = g->group_lo[i]; c->groups[i][1] = g->group_hi[i]; }
    const unsigned ncs = g->num_constants + g->num_routed_wires, nzs = 2 * nchunks;
    batch_t bcs, bw, bz;
    batch_from_values(&bcs, consts_sigmas, ncs, log_n, rate_bits, 0);
    batch_from_values(&bw, wires, g->num_wires, log_n, rate_bits, 0);
    batch_from_values(&bz, zs_vals, nzs, log_n, rate_bits, 0);
    quotient_coeffs(c, log_n, bcs.leaves, bw.leaves, bz.leaves, betas, gammas, alphas, pih, qcoeffs_out);
    batch_free(&bcs); batch_free(&bw); batch_free(&bz);
    free(c);
    return 0;
}

/* checker hooks for a seam-composed prove (tests/seam_prover.py): the host
 * steps plonky2 keeps when the GPU seams take the rest */
int ora_zs_values(const uint8_t *common_bytes, size_t clen, const gl_t *consts_sigmas, const gl_t *wires,
                  const gl_t *betas, const gl_t *gammas, gl_t *zs_out) {
    or_common_t c;
    size_t used;
    if (or_parse_common(common_bytes, clen, &used, &c) || used != clen) return -1;
    zs_values(&c, (unsigned)c.degree_bits, consts_sigmas, wires, betas, gammas, zs_out);
    return 0;
}

/* out[p] = coeffs[p](x) in the extension (ext x as [2]) */
void ora_eval_ext(const gl_t *coeffs, unsigned npolys, unsigned log_n, const gl_t *x, gl_t *out) {
    const size_t n = (size_t)1 << log_n;
    for (unsigned p = 0; p < npolys; p++) {
        glx_t v = eval_coeffs_ext(coeffs + (size_t)p * n, n, glx(x[0], x[1]));
        out[2 * p] = v.c0; out[2 * p + 1] = v.c1;
    }
}

/* initial FRI polynomial from the 4 oracles' coefficient matrices: fin_out [n][2] */
void ora_fri_initial(const gl_t *cs, unsigned ncs, const gl_t *w, unsigned nw, const gl_t *z, unsigned nz,
                     const gl_t *q, unsigned nq, unsigned nc, unsigned log_n, const gl_t *alpha, const gl_t *zeta,
                     const gl_t *zeta_next, gl_t *fin_out) {
    const size_t n = (size_t)1 << log_n;
    const gl_t *coeffs[4] = {cs, w, z, q};
    const unsigned np[4] = {ncs, nw, nz, nq};
    glx_t *fin = calloc(n, sizeof(glx_t));
    fri_initial(coeffs, np, nc, n, glx(alpha[0], alpha[1]), glx(zeta[0], zeta[1]), glx(zeta_next[0], zeta_next[1]),
                fin);
    for (size_t k = 0; k < n; k++) { fin_out[2 * k] = fin[k].c0; fin_out[2 * k + 1] = fin[k].c1; }
    free(fin);
}
