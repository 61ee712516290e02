/*
 * oracle/plonk.h — plonky2 circuit/proof data model, byte IO, gate constraints,
 * verifier and CPU prover, restated in C.  TEST INFRASTRUCTURE ONLY: the
 * checker for the HIP product path, never linked into it.
 *
 * Restates qp-plonky2 1.1.1 (Cargo.lock:489-512, not vendored):
 *   util/serialization.rs   (byte layouts: SURVEY.md A.6, [FIX] from
 *                            wormhole/bench-data/{common,verifier,proof}.bin and
 *                            wormhole/aggregator/data/dummy_proof*.bin)
 *   plonk/vanishing_poly.rs, gates/ modules (A.5 per-gate formulas)
 *   plonk/verifier.rs, fri/verifier.rs (A.4 transcript, A.7 FRI)
 *   plonk/prover.rs, fri/oracle.rs, fri/prover.rs (prover side of the same)
 * Reference call sites: wormhole/verifier/src/lib.rs:155-159 (verify),
 * wormhole/prover/src/lib.rs:233-237 (prove).
 */
#ifndef QP_ORACLE_PLONK_H
#define QP_ORACLE_PLONK_H
#include "gl.h"

#define OR_MAX_GATES 32
#define OR_MAX_LAYERS 8

/* gate ids = plonky2 DefaultGateSerializer order */
enum {
    G_ARITHMETIC = 0, G_ARITH_EXT = 1, G_BASE_SUM = 2, G_CONSTANT = 3, G_COSET_INTERP = 4,
    G_EXPONENTIATION = 5, G_LOOKUP = 6, G_LOOKUP_TABLE = 7, G_MUL_EXT = 8, G_NOOP = 9,
    G_POSEIDON_MDS = 10, G_POSEIDON = 11, G_PUBLIC_INPUT = 12, G_RANDOM_ACCESS = 13,
    G_REDUCING_EXT = 14, G_REDUCING = 15
};

typedef struct {
    uint32_t id;
    uint64_t p0, p1, p2; /* gate parameters (num_ops / num_limbs / num_consts ...) */
} or_gate_t;

typedef struct {
    uint64_t rate_bits, cap_height, num_query_rounds;
    uint32_t pow_bits;
    uint8_t strategy; uint64_t strat_a, strat_b;
} or_fri_config_t;

typedef struct {
    /* CircuitConfig */
    uint64_t num_wires, num_routed_wires, config_num_constants, security_bits, num_challenges,
        max_quotient_degree_factor;
    uint8_t use_base_arithmetic_gate, zero_knowledge;
    or_fri_config_t fri_config;
    /* FriParams */
    or_fri_config_t fri_params_config;
    uint64_t num_layers, arity_bits[OR_MAX_LAYERS];
    uint64_t degree_bits;
    uint8_t hiding;
    /* SelectorsInfo */
    uint64_t num_selector_indices, selector_indices[OR_MAX_GATES];
    uint64_t num_groups, groups[OR_MAX_GATES][2];
    uint64_t quotient_degree_factor, num_gate_constraints, num_constants, num_public_inputs;
    uint64_t num_k_is; gl_t k_is[256];
    uint64_t num_partial_products, num_lookup_polys, num_lookup_selectors, num_luts;
    uint64_t num_gates; or_gate_t gates[OR_MAX_GATES];
} or_common_t;

typedef struct {
    uint64_t cap_height;
    gl_t *constants_sigmas_cap; /* 2^h x 4 */
    gl_t circuit_digest[4];
} or_verifier_only_t;

/* derived sizes */
typedef struct {
    unsigned log_n, log_N, cap_len, salt;
    unsigned oracle_width[4];      /* leaf widths incl. salt */
    unsigned oracle_unsalted[4];   /* poly counts (what FRI opens) */
    unsigned init_sibs;            /* log_N - cap_height */
    unsigned num_layers, arity_bits[OR_MAX_LAYERS], layer_sibs[OR_MAX_LAYERS];
    unsigned final_poly_len;
    unsigned num_openings_zeta, num_openings_next;
    unsigned nq; /* query rounds */
} or_dims_t;

typedef struct {
    or_dims_t d;
    gl_t *wires_cap, *zs_cap, *quot_cap;   /* cap_len x 4 each */
    glx_t *constants, *sigmas, *wires, *zs, *zs_next, *pp, *quotient;
    gl_t *commit_caps;                     /* num_layers x cap_len x 4 */
    /* queries: for q: oracle o: leaf[oracle_width[o]] + sibs[init_sibs x 4]
     *          layer l: evals[arity] (ext) + sibs[layer_sibs[l] x 4] */
    gl_t **q_leaf[4], **q_sib[4];
    glx_t **q_evals[OR_MAX_LAYERS]; gl_t **q_lsib[OR_MAX_LAYERS];
    glx_t *final_poly;
    gl_t pow_witness;
    uint64_t num_pis; gl_t *pis;
} or_proof_t;

int or_parse_common(const uint8_t *buf, size_t len, size_t *consumed, or_common_t *c);
size_t or_write_common(const or_common_t *c, uint8_t *out /* NULL = size only */);
int or_parse_verifier(const uint8_t *buf, size_t len, or_verifier_only_t *v, or_common_t *c);
void or_dims(const or_common_t *c, or_dims_t *d);
or_proof_t *or_proof_alloc(const or_dims_t *d, uint64_t num_pis);
void or_proof_free(or_proof_t *p);
int or_parse_proof(const uint8_t *buf, size_t len, const or_common_t *c, or_proof_t **out);
size_t or_write_proof(const or_proof_t *p, uint8_t *out /* NULL = size only */);

/* gate constraints, accumulated with selector filters: out[num_gate_constraints] */
void or_eval_gate_constraints_ext(const or_common_t *c, const glx_t *local_constants,
                                  const glx_t *local_wires, const gl_t pi_hash[4], glx_t *out);
void or_eval_gate_constraints_base(const or_common_t *c, const gl_t *local_constants,
                                   const gl_t *local_wires, const gl_t pi_hash[4], gl_t *out);
unsigned or_gate_num_constraints(const or_gate_t *g);
unsigned or_gate_eval_base(const or_gate_t *g, const gl_t *c, const gl_t *w, const gl_t pi[4], gl_t *out);

/* verifier: 0 = ok, else a failing-check code (see or_verify_error) */
int or_verify(const or_common_t *c, const or_verifier_only_t *v, const or_proof_t *p);
const char *or_verify_error(int code);

typedef struct {
    gl_t betas[4], gammas[4], alphas[4];
    glx_t zeta, fri_alpha, fri_betas[OR_MAX_LAYERS];
    gl_t pow_response;
    uint64_t query_indices[64];
} or_challenges_t;
void or_get_challenges(const or_common_t *c, const gl_t circuit_digest[4], const or_proof_t *p,
                       or_challenges_t *ch);

#endif
