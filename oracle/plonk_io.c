/*
 * oracle/plonk_io.c — byte layouts of plonky2 CommonCircuitData,
 * VerifierOnlyCircuitData and ProofWithPublicInputs (upstream
 * util/serialization.rs).  TEST INFRASTRUCTURE ONLY.
 * Pinned: parses wormhole/bench-data/{common,verifier,proof}.bin and
 * wormhole/aggregator/data/dummy_proof{,_zk}.bin to their exact lengths and
 * re-serialises them byte-identically (tests/test_oracle_golden.py).
 */
#include "plonk.h"
#include <stdlib.h>
#include <string.h>

typedef struct { const uint8_t *b; size_t len, pos; int err; } rd_t;

static uint64_t rd_u64(rd_t *r) {
    if (r->pos + 8 > r->len) { r->err = 1; return 0; }
    uint64_t v; memcpy(&v, r->b + r->pos, 8); r->pos += 8; return v;
}
static uint32_t rd_u32(rd_t *r) {
    if (r->pos + 4 > r->len) { r->err = 1; return 0; }
    uint32_t v; memcpy(&v, r->b + r->pos, 4); r->pos += 4; return v;
}
static uint8_t rd_u8(rd_t *r) {
    if (r->pos + 1 > r->len) { r->err = 1; return 0; }
    return r->b[r->pos++];
}
static gl_t rd_fe(rd_t *r) {
    uint64_t v = rd_u64(r);
    if (v >= GL_P) r->err = 2;
    return v;
}
static glx_t rd_fx(rd_t *r) { gl_t a = rd_fe(r); gl_t b = rd_fe(r); return glx(a, b); }

typedef struct { uint8_t *b; size_t pos; } wr_t;
static void wr_bytes(wr_t *w, const void *p, size_t n) { if (w->b) memcpy(w->b + w->pos, p, n); w->pos += n; }
static void wr_u64(wr_t *w, uint64_t v) { wr_bytes(w, &v, 8); }
static void wr_u32(wr_t *w, uint32_t v) { wr_bytes(w, &v, 4); }
static void wr_u8(wr_t *w, uint8_t v) { wr_bytes(w, &v, 1); }
static void wr_fx(wr_t *w, glx_t x) { wr_u64(w, x.c0); wr_u64(w, x.c1); }

static void rd_fri_config(rd_t *r, or_fri_config_t *f) {
    f->rate_bits = rd_u64(r);
    f->cap_height = rd_u64(r);
    f->num_query_rounds = rd_u64(r);
    f->pow_bits = rd_u32(r);
    f->strategy = rd_u8(r);
    if (f->strategy == 1) { f->strat_a = rd_u64(r); f->strat_b = rd_u64(r); }
    else if (f->strategy == 2) { uint8_t some = rd_u8(r); f->strat_a = some; if (some) f->strat_b = rd_u64(r); }
    else r->err = 3; /* Fixed(seq) not used by the reference configs */
}
static void wr_fri_config(wr_t *w, const or_fri_config_t *f) {
    wr_u64(w, f->rate_bits); wr_u64(w, f->cap_height); wr_u64(w, f->num_query_rounds);
    wr_u32(w, f->pow_bits); wr_u8(w, f->strategy);
    if (f->strategy == 1) { wr_u64(w, f->strat_a); wr_u64(w, f->strat_b); }
    else if (f->strategy == 2) { wr_u8(w, (uint8_t)f->strat_a); if (f->strat_a) wr_u64(w, f->strat_b); }
}

/* gate parameter layout per upstream Gate::serialize */
static void rd_gate(rd_t *r, or_gate_t *g) {
    g->id = rd_u32(r);
    g->p0 = g->p1 = g->p2 = 0;
    switch (g->id) {
    case G_ARITHMETIC: case G_ARITH_EXT: case G_BASE_SUM: case G_CONSTANT: case G_MUL_EXT:
    case G_REDUCING: case G_REDUCING_EXT: case G_EXPONENTIATION:
        g->p0 = rd_u64(r); break;
    case G_NOOP: case G_POSEIDON: case G_PUBLIC_INPUT: case G_POSEIDON_MDS: break;
    case G_RANDOM_ACCESS: g->p0 = rd_u64(r); g->p1 = rd_u64(r); g->p2 = rd_u64(r); break;
    case G_COSET_INTERP: { /* subgroup_bits, degree, barycentric_weights (field vec; recomputed) */
        g->p0 = rd_u64(r); g->p1 = rd_u64(r);
        uint64_t nw = rd_u64(r);
        if (g->p0 > 6 || nw != ((uint64_t)1 << g->p0) || g->p1 < 2) { r->err = 4; break; }
        for (uint64_t i = 0; i < nw; i++) rd_u64(r);
        break;
    }
    default: r->err = 4; break; /* Lookup gates: not supported */
    }
}
static void wr_gate(wr_t *w, const or_gate_t *g) {
    wr_u32(w, g->id);
    switch (g->id) {
    case G_ARITHMETIC: case G_ARITH_EXT: case G_BASE_SUM: case G_CONSTANT: case G_MUL_EXT:
    case G_REDUCING: case G_REDUCING_EXT: case G_EXPONENTIATION: wr_u64(w, g->p0); break;
    case G_RANDOM_ACCESS: wr_u64(w, g->p0); wr_u64(w, g->p1); wr_u64(w, g->p2); break;
    case G_COSET_INTERP: { /* weights of the subgroup: w^i / n */
        const uint64_t np = (uint64_t)1 << g->p0;
        const gl_t om = gl_root_of_unity((unsigned)g->p0), ninv = gl_inv(np);
        gl_t x = 1;
        wr_u64(w, g->p0); wr_u64(w, g->p1); wr_u64(w, np);
        for (uint64_t i = 0; i < np; i++) { wr_u64(w, gl_mul(x, ninv)); x = gl_mul(x, om); }
        break;
    }
    default: break;
    }
}

int or_parse_common(const uint8_t *buf, size_t len, size_t *consumed, or_common_t *c) {
    rd_t r = {buf, len, 0, 0};
    memset(c, 0, sizeof(*c));
    c->num_wires = rd_u64(&r); c->num_routed_wires = rd_u64(&r); c->config_num_constants = rd_u64(&r);
    c->security_bits = rd_u64(&r); c->num_challenges = rd_u64(&r);
    c->max_quotient_degree_factor = rd_u64(&r);
    c->use_base_arithmetic_gate = rd_u8(&r); c->zero_knowledge = rd_u8(&r);
    rd_fri_config(&r, &c->fri_config);
    rd_fri_config(&r, &c->fri_params_config);
    c->num_layers = rd_u64(&r);
    if (c->num_layers > OR_MAX_LAYERS) return -10;
    for (uint64_t i = 0; i < c->num_layers; i++) c->arity_bits[i] = rd_u64(&r);
    c->degree_bits = rd_u64(&r);
    c->hiding = rd_u8(&r);
    c->num_selector_indices = rd_u64(&r);
    if (c->num_selector_indices > OR_MAX_GATES) return -11;
    for (uint64_t i = 0; i < c->num_selector_indices; i++) c->selector_indices[i] = rd_u64(&r);
    c->num_groups = rd_u64(&r);
    if (c->num_groups > OR_MAX_GATES) return -12;
    for (uint64_t i = 0; i < c->num_groups; i++) { c->groups[i][0] = rd_u64(&r); c->groups[i][1] = rd_u64(&r); }
    c->quotient_degree_factor = rd_u64(&r); c->num_gate_constraints = rd_u64(&r);
    c->num_constants = rd_u64(&r); c->num_public_inputs = rd_u64(&r);
    c->num_k_is = rd_u64(&r);
    if (c->num_k_is > 256) return -13;
    for (uint64_t i = 0; i < c->num_k_is; i++) c->k_is[i] = rd_fe(&r);
    c->num_partial_products = rd_u64(&r); c->num_lookup_polys = rd_u64(&r);
    c->num_lookup_selectors = rd_u64(&r); c->num_luts = rd_u64(&r);
    if (c->num_luts) return -14;
    c->num_gates = rd_u64(&r);
    if (c->num_gates > OR_MAX_GATES) return -15;
    for (uint64_t i = 0; i < c->num_gates; i++) rd_gate(&r, &c->gates[i]);
    if (r.err) return -r.err;
    if (consumed) *consumed = r.pos;
    return 0;
}

size_t or_write_common(const or_common_t *c, uint8_t *out) {
    wr_t w = {out, 0};
    wr_u64(&w, c->num_wires); wr_u64(&w, c->num_routed_wires); wr_u64(&w, c->config_num_constants);
    wr_u64(&w, c->security_bits); wr_u64(&w, c->num_challenges); wr_u64(&w, c->max_quotient_degree_factor);
    wr_u8(&w, c->use_base_arithmetic_gate); wr_u8(&w, c->zero_knowledge);
    wr_fri_config(&w, &c->fri_config);
    wr_fri_config(&w, &c->fri_params_config);
    wr_u64(&w, c->num_layers);
    for (uint64_t i = 0; i < c->num_layers; i++) wr_u64(&w, c->arity_bits[i]);
    wr_u64(&w, c->degree_bits); wr_u8(&w, c->hiding);
    wr_u64(&w, c->num_selector_indices);
    for (uint64_t i = 0; i < c->num_selector_indices; i++) wr_u64(&w, c->selector_indices[i]);
    wr_u64(&w, c->num_groups);
    for (uint64_t i = 0; i < c->num_groups; i++) { wr_u64(&w, c->groups[i][0]); wr_u64(&w, c->groups[i][1]); }
    wr_u64(&w, c->quotient_degree_factor); wr_u64(&w, c->num_gate_constraints);
    wr_u64(&w, c->num_constants); wr_u64(&w, c->num_public_inputs);
    wr_u64(&w, c->num_k_is);
    for (uint64_t i = 0; i < c->num_k_is; i++) wr_u64(&w, c->k_is[i]);
    wr_u64(&w, c->num_partial_products); wr_u64(&w, c->num_lookup_polys);
    wr_u64(&w, c->num_lookup_selectors); wr_u64(&w, c->num_luts);
    wr_u64(&w, c->num_gates);
    for (uint64_t i = 0; i < c->num_gates; i++) wr_gate(&w, &c->gates[i]);
    return w.pos;
}

int or_parse_verifier(const uint8_t *buf, size_t len, or_verifier_only_t *v, or_common_t *c) {
    rd_t r = {buf, len, 0, 0};
    v->cap_height = rd_u64(&r);
    if (v->cap_height > 20) return -20;
    size_t cl = (size_t)1 << v->cap_height;
    v->constants_sigmas_cap = malloc(cl * 32);
    for (size_t i = 0; i < cl * 4; i++) v->constants_sigmas_cap[i] = rd_fe(&r);
    for (int i = 0; i < 4; i++) v->circuit_digest[i] = rd_fe(&r);
    if (r.err) return -r.err;
    size_t used = 0;
    int e = or_parse_common(buf + r.pos, len - r.pos, &used, c);
    if (e) return e;
    if (r.pos + used != len) return -21;
    return 0;
}

void or_dims(const or_common_t *c, or_dims_t *d) {
    memset(d, 0, sizeof(*d));
    d->log_n = (unsigned)c->degree_bits;
    d->log_N = d->log_n + (unsigned)c->fri_params_config.rate_bits;
    d->cap_len = 1u << c->fri_params_config.cap_height;
    d->salt = c->hiding ? 4 : 0;
    unsigned nc = (unsigned)c->num_challenges;
    d->oracle_unsalted[0] = (unsigned)(c->num_constants + c->num_routed_wires);
    d->oracle_unsalted[1] = (unsigned)c->num_wires;
    d->oracle_unsalted[2] = nc * (1 + (unsigned)c->num_partial_products);
    d->oracle_unsalted[3] = nc * (unsigned)c->quotient_degree_factor;
    d->oracle_width[0] = d->oracle_unsalted[0];
    for (int o = 1; o < 4; o++) d->oracle_width[o] = d->oracle_unsalted[o] + d->salt;
    d->init_sibs = d->log_N - (unsigned)c->fri_params_config.cap_height;
    d->num_layers = (unsigned)c->num_layers;
    unsigned lg = d->log_N, tot = 0;
    for (unsigned l = 0; l < d->num_layers; l++) {
        d->arity_bits[l] = (unsigned)c->arity_bits[l];
        lg -= d->arity_bits[l];
        d->layer_sibs[l] = lg - (unsigned)c->fri_params_config.cap_height;
        tot += d->arity_bits[l];
    }
    d->final_poly_len = 1u << (d->log_n - tot);
    d->num_openings_zeta = d->oracle_unsalted[0] + d->oracle_unsalted[1] + d->oracle_unsalted[2] +
                           d->oracle_unsalted[3];
    d->num_openings_next = nc;
    d->nq = (unsigned)c->fri_params_config.num_query_rounds;
}

static void *xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

or_proof_t *or_proof_alloc(const or_dims_t *d, uint64_t num_pis) {
    or_proof_t *p = calloc(1, sizeof(*p));
    p->d = *d;
    size_t cl = d->cap_len;
    p->wires_cap = xcalloc(cl * 4, 8); p->zs_cap = xcalloc(cl * 4, 8); p->quot_cap = xcalloc(cl * 4, 8);
    unsigned nsig = d->oracle_unsalted[0];
    (void)nsig;
    p->constants = xcalloc(d->oracle_unsalted[0], sizeof(glx_t));
    p->sigmas = p->constants; /* split view set by caller via counts; see or_proof_views */
    p->wires = xcalloc(d->oracle_unsalted[1], sizeof(glx_t));
    p->zs = xcalloc(d->num_openings_next, sizeof(glx_t));
    p->zs_next = xcalloc(d->num_openings_next, sizeof(glx_t));
    p->pp = xcalloc(d->oracle_unsalted[2], sizeof(glx_t));
    p->quotient = xcalloc(d->oracle_unsalted[3], sizeof(glx_t));
    p->commit_caps = xcalloc((size_t)d->num_layers * cl * 4, 8);
    for (int o = 0; o < 4; o++) {
        p->q_leaf[o] = xcalloc(d->nq, sizeof(gl_t *));
        p->q_sib[o] = xcalloc(d->nq, sizeof(gl_t *));
        for (unsigned q = 0; q < d->nq; q++) {
            p->q_leaf[o][q] = xcalloc(d->oracle_width[o], 8);
            p->q_sib[o][q] = xcalloc((size_t)d->init_sibs * 4, 8);
        }
    }
    for (unsigned l = 0; l < d->num_layers; l++) {
        p->q_evals[l] = xcalloc(d->nq, sizeof(glx_t *));
        p->q_lsib[l] = xcalloc(d->nq, sizeof(gl_t *));
        for (unsigned q = 0; q < d->nq; q++) {
            p->q_evals[l][q] = xcalloc((size_t)1 << d->arity_bits[l], sizeof(glx_t));
            p->q_lsib[l][q] = xcalloc((size_t)d->layer_sibs[l] * 4, 8);
        }
    }
    p->final_poly = xcalloc(d->final_poly_len, sizeof(glx_t));
    p->num_pis = num_pis;
    p->pis = xcalloc(num_pis, 8);
    return p;
}

void or_proof_free(or_proof_t *p) {
    if (!p) return;
    const or_dims_t *d = &p->d;
    free(p->wires_cap); free(p->zs_cap); free(p->quot_cap);
    free(p->constants); free(p->wires); free(p->zs); free(p->zs_next); free(p->pp); free(p->quotient);
    free(p->commit_caps);
    for (int o = 0; o < 4; o++) {
        for (unsigned q = 0; q < d->nq; q++) { free(p->q_leaf[o][q]); free(p->q_sib[o][q]); }
        free(p->q_leaf[o]); free(p->q_sib[o]);
    }
    for (unsigned l = 0; l < d->num_layers; l++) {
        for (unsigned q = 0; q < d->nq; q++) { free(p->q_evals[l][q]); free(p->q_lsib[l][q]); }
        free(p->q_evals[l]); free(p->q_lsib[l]);
    }
    free(p->final_poly); free(p->pis); free(p);
}

/* Openings: constants(num_constants) sigmas(num_routed) live in p->constants
 * (one array of oracle_unsalted[0]); wires; zs; zs_next; partial products;
 * quotient.  Serialised order: constants, sigmas, wires, zs, zs_next,
 * partial_products, quotient (lookup vectors empty). */
int or_parse_proof(const uint8_t *buf, size_t len, const or_common_t *c, or_proof_t **out) {
    or_dims_t d;
    or_dims(c, &d);
    rd_t r = {buf, len, 0, 0};
    or_proof_t *p = or_proof_alloc(&d, 0);
    size_t cl = d.cap_len;
    for (size_t i = 0; i < cl * 4; i++) p->wires_cap[i] = rd_fe(&r);
    for (size_t i = 0; i < cl * 4; i++) p->zs_cap[i] = rd_fe(&r);
    for (size_t i = 0; i < cl * 4; i++) p->quot_cap[i] = rd_fe(&r);
    for (unsigned i = 0; i < d.oracle_unsalted[0]; i++) p->constants[i] = rd_fx(&r);
    for (unsigned i = 0; i < d.oracle_unsalted[1]; i++) p->wires[i] = rd_fx(&r);
    for (unsigned i = 0; i < d.num_openings_next; i++) p->zs[i] = rd_fx(&r);
    for (unsigned i = 0; i < d.num_openings_next; i++) p->zs_next[i] = rd_fx(&r);
    unsigned npp = d.oracle_unsalted[2] - d.num_openings_next;
    for (unsigned i = 0; i < npp; i++) p->pp[i] = rd_fx(&r);
    for (unsigned i = 0; i < d.oracle_unsalted[3]; i++) p->quotient[i] = rd_fx(&r);
    for (size_t i = 0; i < (size_t)d.num_layers * cl * 4; i++) p->commit_caps[i] = rd_fe(&r);
    for (unsigned q = 0; q < d.nq; q++) {
        for (int o = 0; o < 4; o++) {
            for (unsigned i = 0; i < d.oracle_width[o]; i++) p->q_leaf[o][q][i] = rd_fe(&r);
            unsigned ns = rd_u8(&r);
            if (ns != d.init_sibs) { r.err = 5; break; }
            for (unsigned i = 0; i < ns * 4; i++) p->q_sib[o][q][i] = rd_fe(&r);
        }
        for (unsigned l = 0; l < d.num_layers; l++) {
            unsigned ar = 1u << d.arity_bits[l];
            for (unsigned i = 0; i < ar; i++) p->q_evals[l][q][i] = rd_fx(&r);
            unsigned ns = rd_u8(&r);
            if (ns != d.layer_sibs[l]) { r.err = 6; break; }
            for (unsigned i = 0; i < ns * 4; i++) p->q_lsib[l][q][i] = rd_fe(&r);
        }
        if (r.err) break;
    }
    for (unsigned i = 0; i < d.final_poly_len; i++) p->final_poly[i] = rd_fx(&r);
    p->pow_witness = rd_fe(&r);
    p->num_pis = rd_u64(&r);
    if (p->num_pis > (1u << 20)) r.err = 7;  /* sanity bound (a 2048-leaf root carries 32,768) */
    if (!r.err) {
        free(p->pis);
        p->pis = xcalloc(p->num_pis, 8);
        for (uint64_t i = 0; i < p->num_pis; i++) p->pis[i] = rd_fe(&r);
    }
    if (r.err || r.pos != len) {
        int e = r.err ? -r.err : -30;
        or_proof_free(p);
        return e;
    }
    *out = p;
    return 0;
}

size_t or_write_proof(const or_proof_t *p, uint8_t *out) {
    const or_dims_t *d = &p->d;
    wr_t w = {out, 0};
    size_t cl = d->cap_len;
    for (size_t i = 0; i < cl * 4; i++) wr_u64(&w, p->wires_cap[i]);
    for (size_t i = 0; i < cl * 4; i++) wr_u64(&w, p->zs_cap[i]);
    for (size_t i = 0; i < cl * 4; i++) wr_u64(&w, p->quot_cap[i]);
    for (unsigned i = 0; i < d->oracle_unsalted[0]; i++) wr_fx(&w, p->constants[i]);
    for (unsigned i = 0; i < d->oracle_unsalted[1]; i++) wr_fx(&w, p->wires[i]);
    for (unsigned i = 0; i < d->num_openings_next; i++) wr_fx(&w, p->zs[i]);
    for (unsigned i = 0; i < d->num_openings_next; i++) wr_fx(&w, p->zs_next[i]);
    unsigned npp = d->oracle_unsalted[2] - d->num_openings_next;
    for (unsigned i = 0; i < npp; i++) wr_fx(&w, p->pp[i]);
    for (unsigned i = 0; i < d->oracle_unsalted[3]; i++) wr_fx(&w, p->quotient[i]);
    for (size_t i = 0; i < (size_t)d->num_layers * cl * 4; i++) wr_u64(&w, p->commit_caps[i]);
    for (unsigned q = 0; q < d->nq; q++) {
        for (int o = 0; o < 4; o++) {
            for (unsigned i = 0; i < d->oracle_width[o]; i++) wr_u64(&w, p->q_leaf[o][q][i]);
            wr_u8(&w, (uint8_t)d->init_sibs);
            for (unsigned i = 0; i < d->init_sibs * 4; i++) wr_u64(&w, p->q_sib[o][q][i]);
        }
        for (unsigned l = 0; l < d->num_layers; l++) {
            unsigned ar = 1u << d->arity_bits[l];
            for (unsigned i = 0; i < ar; i++) wr_fx(&w, p->q_evals[l][q][i]);
            wr_u8(&w, (uint8_t)d->layer_sibs[l]);
            for (unsigned i = 0; i < d->layer_sibs[l] * 4; i++) wr_u64(&w, p->q_lsib[l][q][i]);
        }
    }
    for (unsigned i = 0; i < d->final_poly_len; i++) wr_fx(&w, p->final_poly[i]);
    wr_u64(&w, p->pow_witness);
    wr_u64(&w, p->num_pis);
    for (uint64_t i = 0; i < p->num_pis; i++) wr_u64(&w, p->pis[i]);
    return w.pos;
}
