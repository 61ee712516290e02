/*
 * oracle/verifier.c — plonky2 verifier restated (upstream plonk/verifier.rs,
 * plonk/get_challenges.rs, plonk/vanishing_poly.rs eval_vanishing_poly,
 * fri/verifier.rs, fri/challenges.rs).  TEST INFRASTRUCTURE ONLY.
 * Transcript: SURVEY.md A.4; vanishing poly: A.5; FRI: A.7.
 * First golden check: accepts wormhole/bench-data/proof.bin under
 * wormhole/bench-data/verifier.bin (the reference's verifier bench,
 * wormhole/verifier/benches/verifier.rs:11-20).
 */
#include "plonk.h"
#include "poseidon.h"
#include "challenger.h"
#include "merkle.h"
#include <stdlib.h>
#include <string.h>

static const char *ERRS[] = {
    "ok", "public-input count mismatch", "zeta in subgroup", "vanishing/quotient identity",
    "pow response", "initial merkle path", "fri layer consistency", "fri layer merkle path",
    "final polynomial", "malformed"};
const char *or_verify_error(int code) { return (code >= 0 && code <= 9) ? ERRS[code] : "?"; }

void or_get_challenges(const or_common_t *c, const gl_t digest[4], const or_proof_t *p, or_challenges_t *ch) {
    const or_dims_t *d = &p->d;
    or_chal_t t;
    or_chal_init(&t);
    gl_t pih[4];
    ps_hash_no_pad(p->pis, p->num_pis, pih);
    or_chal_observe_n(&t, digest, 4);
    or_chal_observe_n(&t, pih, 4);
    or_chal_observe_n(&t, p->wires_cap, (size_t)d->cap_len * 4);
    unsigned nc = (unsigned)c->num_challenges;
    for (unsigned i = 0; i < nc; i++) ch->betas[i] = or_chal_get(&t);
    for (unsigned i = 0; i < nc; i++) ch->gammas[i] = or_chal_get(&t);
    or_chal_observe_n(&t, p->zs_cap, (size_t)d->cap_len * 4);
    for (unsigned i = 0; i < nc; i++) ch->alphas[i] = or_chal_get(&t);
    or_chal_observe_n(&t, p->quot_cap, (size_t)d->cap_len * 4);
    ch->zeta = or_chal_get_ext(&t);
    /* observe openings: batch zeta = constants, sigmas, wires, zs, pp, quotient; batch g*zeta = zs_next */
    for (unsigned i = 0; i < d->oracle_unsalted[0]; i++) or_chal_observe_ext(&t, p->constants[i]);
    for (unsigned i = 0; i < d->oracle_unsalted[1]; i++) or_chal_observe_ext(&t, p->wires[i]);
    for (unsigned i = 0; i < nc; i++) or_chal_observe_ext(&t, p->zs[i]);
    unsigned npp = d->oracle_unsalted[2] - nc;
    for (unsigned i = 0; i < npp; i++) or_chal_observe_ext(&t, p->pp[i]);
    for (unsigned i = 0; i < d->oracle_unsalted[3]; i++) or_chal_observe_ext(&t, p->quotient[i]);
    for (unsigned i = 0; i < nc; i++) or_chal_observe_ext(&t, p->zs_next[i]);
    ch->fri_alpha = or_chal_get_ext(&t);
    for (unsigned l = 0; l < d->num_layers; l++) {
        or_chal_observe_n(&t, p->commit_caps + (size_t)l * d->cap_len * 4, (size_t)d->cap_len * 4);
        ch->fri_betas[l] = or_chal_get_ext(&t);
    }
    for (unsigned i = 0; i < d->final_poly_len; i++) or_chal_observe_ext(&t, p->final_poly[i]);
    or_chal_observe(&t, p->pow_witness);
    ch->pow_response = or_chal_get(&t);
    uint64_t N = (uint64_t)1 << d->log_N;
    for (unsigned q = 0; q < d->nq && q < 64; q++) ch->query_indices[q] = or_chal_get(&t) % N;
}

/* sum_i t_i a^i (Horner over the reversed list) */
static glx_t reduce_with_powers_x(const glx_t *t, size_t n, glx_t a) {
    glx_t acc = glx(0, 0);
    for (size_t i = n; i-- > 0;) acc = glx_add(glx_mul(acc, a), t[i]);
    return acc;
}

/* eval_vanishing_poly at an extension point, openings given */
static void vanishing_at(const or_common_t *c, const or_proof_t *p, const or_challenges_t *ch,
                         const gl_t pih[4], glx_t x, glx_t *out /* [num_challenges] */) {
    const or_dims_t *d = &p->d;
    unsigned nc = (unsigned)c->num_challenges, R = (unsigned)c->num_routed_wires;
    unsigned nconst = (unsigned)c->num_constants, npp = (unsigned)c->num_partial_products;
    unsigned qdf = (unsigned)c->quotient_degree_factor;
    size_t nterms = nc + nc * (npp + 1) + c->num_gate_constraints;
    glx_t *terms = calloc(nterms, sizeof(glx_t));
    size_t k = 0;
    /* L_0(x) = (x^n - 1) / (n (x - 1)) */
    glx_t xn = glx_exp_power_of_2(x, d->log_n);
    glx_t zh = glx_sub(xn, glx(1, 0));
    glx_t l0 = glx_mul(zh, glx_inv(glx_scale(glx_sub(x, glx(1, 0)), gl_from_u64((uint64_t)1 << d->log_n))));
    for (unsigned i = 0; i < nc; i++) terms[k++] = glx_mul(l0, glx_sub(p->zs[i], glx(1, 0)));
    const glx_t *sig = p->constants + nconst;
    for (unsigned i = 0; i < nc; i++) {
        const glx_t *partials = p->pp + (size_t)i * npp;
        unsigned nchunks = (R + qdf - 1) / qdf;
        for (unsigned ch_i = 0; ch_i < nchunks; ch_i++) {
            glx_t num = glx(1, 0), den = glx(1, 0);
            for (unsigned j = ch_i * qdf; j < (ch_i + 1) * qdf && j < R; j++) {
                glx_t wv = p->wires[j];
                glx_t nn = glx_add(glx_add(wv, glx_scale(x, gl_mul(ch->betas[i], c->k_is[j]))), glx_from(ch->gammas[i]));
                glx_t dd = glx_add(glx_add(wv, glx_scale(sig[j], ch->betas[i])), glx_from(ch->gammas[i]));
                num = glx_mul(num, nn);
                den = glx_mul(den, dd);
            }
            glx_t prev = ch_i == 0 ? p->zs[i] : partials[ch_i - 1];
            glx_t next = ch_i == nchunks - 1 ? p->zs_next[i] : partials[ch_i];
            terms[k++] = glx_sub(glx_mul(prev, num), glx_mul(next, den));
        }
    }
    or_eval_gate_constraints_ext(c, p->constants, p->wires, pih, terms + k);
    k += c->num_gate_constraints;
    for (unsigned i = 0; i < nc; i++) out[i] = reduce_with_powers_x(terms, k, glx_from(ch->alphas[i]));
    free(terms);
}

/* barycentric interpolation of (x_i, y_i) evaluated at z (upstream interpolation.rs) */
static glx_t interpolate_x(const glx_t *xs, const glx_t *ys, size_t n, glx_t z) {
    glx_t res = glx(0, 0);
    for (size_t i = 0; i < n; i++) {
        glx_t w = glx(1, 0);
        for (size_t j = 0; j < n; j++) if (j != i) w = glx_mul(w, glx_sub(xs[i], xs[j]));
        glx_t term = glx_mul(ys[i], glx_inv(w));
        for (size_t j = 0; j < n; j++) if (j != i) term = glx_mul(term, glx_sub(z, xs[j]));
        res = glx_add(res, term);
    }
    return res;
}

int or_verify(const or_common_t *c, const or_verifier_only_t *v, const or_proof_t *p) {
    const or_dims_t *d = &p->d;
    if (p->num_pis != c->num_public_inputs) return 1;
    or_challenges_t ch;
    or_get_challenges(c, v->circuit_digest, p, &ch);
    gl_t pih[4];
    ps_hash_no_pad(p->pis, p->num_pis, pih);
    unsigned nc = (unsigned)c->num_challenges, qdf = (unsigned)c->quotient_degree_factor;
    /* zeta^n != 1 */
    glx_t zn = glx_exp_power_of_2(ch.zeta, d->log_n);
    if (glx_eq(zn, glx(1, 0))) return 2;
    glx_t van[8];
    vanishing_at(c, p, &ch, pih, ch.zeta, van);
    glx_t zh = glx_sub(zn, glx(1, 0));
    for (unsigned i = 0; i < nc; i++) {
        glx_t t = reduce_with_powers_x(p->quotient + (size_t)i * qdf, qdf, zn);
        if (!glx_eq(van[i], glx_mul(zh, t))) return 3;
    }
    /* PoW */
    uint64_t resp = ch.pow_response;
    int lz = resp ? __builtin_clzll(resp) : 64;
    if (lz < (int)c->fri_params_config.pow_bits) return 4;
    /* FRI */
    glx_t g_n = glx_from(gl_root_of_unity(d->log_n));
    glx_t zeta_next = glx_mul(g_n, ch.zeta);
    glx_t a = ch.fri_alpha;
    /* reduced openings per batch */
    glx_t *zb = malloc(sizeof(glx_t) * d->num_openings_zeta);
    unsigned m = 0;
    for (unsigned i = 0; i < d->oracle_unsalted[0]; i++) zb[m++] = p->constants[i];
    for (unsigned i = 0; i < d->oracle_unsalted[1]; i++) zb[m++] = p->wires[i];
    for (unsigned i = 0; i < nc; i++) zb[m++] = p->zs[i];
    for (unsigned i = 0; i < d->oracle_unsalted[2] - nc; i++) zb[m++] = p->pp[i];
    for (unsigned i = 0; i < d->oracle_unsalted[3]; i++) zb[m++] = p->quotient[i];
    glx_t red0 = reduce_with_powers_x(zb, m, a);
    glx_t red1 = reduce_with_powers_x(p->zs_next, nc, a);
    glx_t a_pow_nc = glx_pow(a, nc); /* shift applied to the zeta batch before adding the next batch */
    gl_t g = GL_GEN;
    gl_t w_N = gl_root_of_unity(d->log_N);
    int rc = 0;
    glx_t *ev = malloc(sizeof(glx_t) * d->num_openings_zeta);
    for (unsigned q = 0; q < d->nq && !rc; q++) {
        uint64_t xi = ch.query_indices[q];
        const gl_t *caps[4] = {v->constants_sigmas_cap, p->wires_cap, p->zs_cap, p->quot_cap};
        for (int o = 0; o < 4; o++)
            if (!or_merkle_verify(p->q_leaf[o][q], d->oracle_width[o], xi, caps[o],
                                  (unsigned)c->fri_params_config.cap_height, p->q_sib[o][q], d->init_sibs)) {
                rc = 5;
                break;
            }
        if (rc) break;
        gl_t sx = gl_mul(g, gl_pow(w_N, rev_bits(xi, d->log_N)));
        /* fri_combine_initial */
        m = 0;
        for (int o = 0; o < 4; o++)
            for (unsigned i = 0; i < d->oracle_unsalted[o]; i++) ev[m++] = glx_from(p->q_leaf[o][q][i]);
        glx_t r0 = reduce_with_powers_x(ev, m, a);
        glx_t en[8];
        for (unsigned i = 0; i < nc; i++) en[i] = glx_from(p->q_leaf[2][q][i]);
        glx_t r1 = reduce_with_powers_x(en, nc, a);
        glx_t sxx = glx_from(sx);
        glx_t s0 = glx_mul(glx_sub(r0, red0), glx_inv(glx_sub(sxx, ch.zeta)));
        glx_t s1 = glx_mul(glx_sub(r1, red1), glx_inv(glx_sub(sxx, zeta_next)));
        glx_t old = glx_add(glx_mul(s0, a_pow_nc), s1);
        for (unsigned l = 0; l < d->num_layers; l++) {
            unsigned ab = d->arity_bits[l], ar = 1u << ab;
            const glx_t *evals = p->q_evals[l][q];
            uint64_t coset = xi >> ab, within = xi & (ar - 1);
            if (!glx_eq(evals[within], old)) { rc = 6; break; }
            /* compute_evaluation: interpolate over the coset at beta */
            glx_t rev_e[64], pts[64];
            for (unsigned i = 0; i < ar; i++) rev_e[rev_bits(i, ab)] = evals[i];
            gl_t ga = gl_root_of_unity(ab);
            uint64_t rw = rev_bits(within, ab);
            gl_t start = gl_mul(sx, gl_pow(ga, (ar - rw) % ar));
            gl_t y = start;
            for (unsigned i = 0; i < ar; i++) { pts[i] = glx_from(y); y = gl_mul(y, ga); }
            old = interpolate_x(pts, rev_e, ar, ch.fri_betas[l]);
            gl_t flat[128];
            for (unsigned i = 0; i < ar; i++) { flat[2 * i] = evals[i].c0; flat[2 * i + 1] = evals[i].c1; }
            if (!or_merkle_verify(flat, 2 * ar, coset, p->commit_caps + (size_t)l * d->cap_len * 4,
                                  (unsigned)c->fri_params_config.cap_height, p->q_lsib[l][q], d->layer_sibs[l])) {
                rc = 7;
                break;
            }
            sx = gl_pow(sx, ar);
            xi = coset;
        }
        if (rc) break;
        /* final poly at sx */
        glx_t fx = glx(0, 0), sxe = glx_from(sx);
        for (unsigned i = d->final_poly_len; i-- > 0;) fx = glx_add(glx_mul(fx, sxe), p->final_poly[i]);
        if (!glx_eq(fx, old)) rc = 8;
    }
    free(zb); free(ev);
    return rc;
}
