/*
 * qpgpu.h — C ABI of the MI355X (gfx950) Plonky2 prover backend.
 *
 * The reference (aletheia-labs/qp-zk-circuits-rm) has no FFI: its hot path is
 * the Rust crate qp-plonky2 1.1.1 called from qp-wormhole-prover.  Each entry
 * point below names the plonky2 routine it replaces and the reference call
 * site that reaches it.  A Rust binding is a
 * `[patch.crates-io]` qp-plonky2 whose routines call these functions
 * (INTEGRATION.md).
 *
 * Conventions
 *   - Field elements are canonical Goldilocks u64 (p = 2^64 - 2^32 + 1);
 *     extension elements are (c0, c1) pairs, X^2 = 7.
 *   - Host buffers are caller-owned and only borrowed for the call.  Device
 *     objects (qp_ctx, qp_batch, qp_prover) are opaque handles released by
 *     their _free / _destroy function.
 *   - `_dev` variants take device pointers and run on the context's stream
 *     without synchronising (inputs already resident in HBM).
 *   - Every function returns a qp_status; it never aborts or throws across
 *     the ABI.  qp_ctx_last_error() gives the message of the last failure.
 *   - A qp_ctx is single-thread-affine (one HIP stream); concurrent callers
 *     use distinct contexts, which are independent.
 */
#ifndef QPGPU_H
#define QPGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    QP_OK = 0,
    QP_ERR_ARG = 1,      /* bad shape / null pointer / out-of-range index */
    QP_ERR_HIP = 2,      /* HIP runtime error (no device, launch failure) */
    QP_ERR_OOM = 3,      /* device allocation failed */
    QP_ERR_STATE = 4,    /* call order violated (e.g. prove before commit) */
    QP_ERR_WITNESS = 5,  /* witness conflict ("set twice with different values") or unsatisfied */
    QP_ERR_FORMAT = 6    /* malformed serialized input */
} qp_status;

typedef struct qp_ctx qp_ctx;
typedef struct qp_batch qp_batch;

/* ---- context ---------------------------------------------------------- */
int qp_ctx_create(int device, qp_ctx **out);
void qp_ctx_destroy(qp_ctx *ctx);
const char *qp_ctx_last_error(const qp_ctx *ctx);
/* run subsequent work on an external HIP stream (e.g. torch's); NULL = own stream */
int qp_ctx_set_stream(qp_ctx *ctx, void *hip_stream);
int qp_ctx_synchronize(qp_ctx *ctx);
/* re-create the context's own stream at the device's greatest stream priority
 * (high != 0) or the default one; call before any work is queued on it */
int qp_ctx_set_priority(qp_ctx *ctx, int high);
/* library build/version string */
const char *qp_version(void);

/* ---- PolynomialBatch (plonky2 fri/oracle.rs) ----------------------------
 * Replaces PolynomialBatch::from_values (ifft -> coset LDE -> transpose ->
 * reverse_index_bits -> MerkleTree::new).  Reached from
 * WormholeProver::prove (wormhole/prover/src/lib.rs:233-237) for the wires,
 * zs/partial-products and quotient commitments, and from
 * WormholeProver::new -> CircuitBuilder::build (lib.rs:190-202) for the
 * constants/sigmas commitment.
 *   values: column-major [npolys][2^log_n]; salt: row-major [N][nsalt] (may be
 *   NULL when nsalt == 0), N = 2^(log_n+rate_bits).
 *   coeffs_out (optional): [npolys][2^log_n]; cap_out: [2^cap_height][4].
 *   out (optional): keeps the LDE matrix + tree resident for openings.     */
int qp_commit_values(qp_ctx *ctx, const uint64_t *values, uint32_t npolys, uint32_t log_n, uint32_t rate_bits,
                     uint32_t cap_height, const uint64_t *salt, uint32_t nsalt, uint64_t *coeffs_out,
                     uint64_t *cap_out, qp_batch **out);
/* PolynomialBatch::from_coeffs (quotient chunks) — same, from coefficients */
int qp_commit_coeffs(qp_ctx *ctx, const uint64_t *coeffs, uint32_t npolys, uint32_t log_n, uint32_t rate_bits,
                     uint32_t cap_height, const uint64_t *salt, uint32_t nsalt, uint64_t *cap_out, qp_batch **out);
/* device-resident variant: d_values [nbat][npolys][n] on the device; d_cap_out
 * [nbat][2^cap_h][4] on the device; no host sync.  Batches are independent
 * polynomial batches of identical shape (one per proof).                   */
int qp_commit_values_dev(qp_ctx *ctx, const uint64_t *d_values, uint32_t nbat, uint32_t npolys, uint32_t log_n,
                         uint32_t rate_bits, uint32_t cap_height, uint64_t *d_cap_out, qp_batch **out);

/* MerkleTree::get + MerkleTree::prove for a list of leaf indices:
 * leaves_out [nidx][npolys+nsalt], siblings_out [nidx][log_N - cap_h][4]    */
int qp_batch_open(qp_batch *b, const uint32_t *leaf_idx, uint32_t nidx, uint64_t *leaves_out,
                  uint64_t *siblings_out);
/* copies the LDE matrix, leaf order, column-major [npolys][N] (tests) */
int qp_batch_lde(qp_batch *b, uint64_t *out);
/* copies the coefficients [npolys][n] */
int qp_batch_coeffs(qp_batch *b, uint64_t *out);
void qp_batch_free(qp_batch *b);

/* ---- primitives (plonky2 field/fft.rs, hash/poseidon.rs) ----------------- */
/* PolynomialValues::ifft for ncols columns, in place, column-major          */
int qp_ifft(qp_ctx *ctx, uint64_t *data, uint32_t ncols, uint32_t log_n);
/* PolynomialCoeffs::lde(rate_bits).coset_fft(shift), output in Merkle-leaf
 * (bit-reversed) row order, column-major [ncols][N]                         */
int qp_lde(qp_ctx *ctx, const uint64_t *coeffs, uint32_t ncols, uint32_t log_n, uint32_t rate_bits, uint64_t shift,
           uint64_t *out);
/* Poseidon permutation of n 12-element states, in place                   */
int qp_poseidon_permute(qp_ctx *ctx, uint64_t *states, uint64_t n);
/* PoseidonHash::hash_no_pad on the host (no device): used to build circuit
 * inputs (nullifier, unspendable account, storage-proof roots)            */
int qp_hash_no_pad(const uint64_t *in, size_t n, uint64_t *out4);


/* ---- circuits and witnesses (host; no device needed) ---------------------
 * Native equivalent of plonky2's CircuitBuilder::build / build_prover and
 * generate_partial_witness for the reference circuits.                     */
typedef struct qp_circuit qp_circuit;
typedef struct qp_witness qp_witness;

/* CircuitInputs (wormhole/circuit/src/inputs.rs:25-52) in byte form */
typedef struct {
    uint8_t funding_amount[16];        /* u128, little-endian */
    uint8_t nullifier[32];
    uint8_t root_hash[32];
    uint8_t exit_account[32];
    uint8_t secret[32];
    uint64_t transfer_count;
    uint8_t funding_account[32];
    uint8_t unspendable_account[32];
    uint32_t num_nodes;                /* storage proof length (<= 20) */
    const uint8_t *const *nodes;       /* node byte strings */
    const uint32_t *node_lens;
    const uint64_t *indices;           /* hex-character child-hash indices */
    /* values of the PublicInputGate row's unused wires 4..num_wires-1
     * (num_wires - 4 canonical felts), which the reference fills from
     * RandomValueGenerator (plonky2 CircuitBuilder::build,
     * randomize_unused_pi_wires; qp-plonky2 under both configs).  Passing the
     * values a reference proof holds reproduces that proof's wires.  NULL =
     * zeros under standard_recursion_config; under the zk config derived
     * deterministically from the private inputs (a Poseidon nonce; DESIGN.md
     * "zk").                                                                 */
    const uint64_t *zk_randomness;
} qp_wormhole_inputs;

/* WormholeCircuit::new(config) + build_prover (wormhole/circuit/src/circuit.rs:76-108,
 * wormhole/prover/src/lib.rs:190-202) — host part.  zero_knowledge selects
 * standard_recursion_zk_config vs standard_recursion_config.  Under the
 * workspace's `no_random` feature the two share the preprocessing and proof
 * shape (no salt columns; tests/test_current_circuit_fixture.py) and both
 * fill the PublicInputGate row's spare cells (qp_wormhole_inputs.zk_randomness);
 * the constants||sigmas columns equal the reference's
 * (tests/test_reference_layout.py).                                        */
int qp_wormhole_circuit_new(int zero_knowledge, qp_circuit **out);
void qp_circuit_free(qp_circuit *c);
/* info[0..6] = degree_bits, num_wires, num_routed_wires, num_constants,
 *              num_public_inputs, gates used (before padding), num_gate_constraints
 * info[7..8] = witness generators, dependency levels of the device schedule
 * (info must hold 9 words)                                                  */
int qp_circuit_info(const qp_circuit *c, uint32_t *info);
/* generator and gate-row census: gens[k] = generators of GenKind k (constant,
 * arithmetic, Poseidon, BaseSum split, equality, wire split, extension
 * division, RandomAccess, ArithmeticExtension, MulExtension, Reducing,
 * ReducingExtension, PoseidonMds, CosetInterpolation: 14 words); rows[k] =
 * gate rows of kind k (noop, constant, public input, BaseSum, arithmetic,
 * Poseidon, RandomAccess, ArithmeticExtension, MulExtension, Reducing,
 * ReducingExtension, PoseidonMds, CosetInterpolation: 13 words; the n rows
 * of the trace, padding counted as noop); level_gens (may be null; 14 words
 * per device-witness level, info word 8 levels) = the generators of each
 * dependency level by kind.  Test/diagnostic entry point.                   */
int qp_circuit_census(const qp_circuit *c, uint32_t *gens, uint32_t *rows, uint32_t *level_gens);
/* the device witness's host part: gens[k] (14 words, GenKind order as above)
 * = generators the host runs before the device schedule (Poseidon chains over
 * inputs alone at least 64 permutations deep -- the public-input hashes and
 * the transcript sponges behind them -- with the constants they read);
 * *slots = value slots set on the host (commit()'s inputs and those chains'
 * outputs); *chains (may be null) = independent chains among them (a batch
 * smaller than the host pool runs them in parallel).  Test/diagnostic entry
 * point.                                                                      */
int qp_circuit_host_chains(const qp_circuit *c, uint32_t *gens, uint32_t *slots, uint32_t *chains);
/* CommonCircuitData::to_bytes (plonky2 util/serialization.rs) */
int qp_circuit_common_data(const qp_circuit *c, uint8_t *out, size_t cap, size_t *len);
/* preprocessed constants||sigmas values over H, [num_constants+num_routed][n] */
int qp_circuit_constants_sigmas(const qp_circuit *c, uint64_t *out);
/* their coefficients (PolynomialValues::ifft per column, host), the polynomials
 * of ProverOnlyCircuitData.constants_sigmas_commitment                     */
int qp_circuit_constants_sigmas_coeffs(const qp_circuit *c, uint64_t *out);
/* ProverOnlyCircuitData::to_bytes through DefaultGeneratorSerializer (the
 * prover.bin of wormhole/circuit-builder/src/lib.rs:53-59, read by
 * WormholeProver::new_from_bytes, prover/src/lib.rs:104-137) of a leaf circuit
 * (Wormhole, voting; QP_ERR_ARG for an aggregation circuit), computed on the
 * host: generators, watch index, the constants||sigmas PolynomialBatch with its
 * Merkle tree, sigmas, subgroup, public inputs, representative map, fft root
 * table, circuit digest.  out == NULL: *len = the size (the bytes are kept until
 * the copying call).  Restated from upstream plonky2; parity unpinned.        */
int qp_circuit_prover_only_bytes(const qp_circuit *c, uint8_t *out, size_t cap, size_t *len);
/* WormholeProver::commit (lib.rs:209-225) + witness generation.  On a witness
 * conflict returns QP_ERR_WITNESS with the reference's message in err.     */
int qp_wormhole_commit(const qp_circuit *c, const qp_wormhole_inputs *in, qp_witness **out, char *err,
                       size_t errcap);
/* VotePublicInputs + VotePrivateInputs (voting/src/lib.rs:26-52), felt form */
typedef struct {
    uint64_t proposal_id[4];
    uint64_t merkle_root[4];
    uint64_t nullifier[4];
    uint8_t vote;                      /* 0 = no, 1 = yes */
    uint64_t private_key[4];
    uint32_t num_siblings;             /* merkle_siblings.len() */
    const uint64_t *siblings;          /* [num_siblings][4] */
    uint32_t num_path_indices;         /* path_indices.len() */
    const uint8_t *path_indices;       /* [num_path_indices], 0 = left, 1 = right */
    uint64_t actual_merkle_depth;
    const uint64_t *zk_randomness;     /* as in qp_wormhole_inputs */
} qp_voting_inputs;

/* VoteTargets::new + VoteCircuitData::circuit + builder.build()
 * (voting/src/lib.rs:71-197, :346-357) — host part.                         */
int qp_voting_circuit_new(int zero_knowledge, qp_circuit **out);
/* VoteCircuitData::fill_targets (voting/src/lib.rs:199-261) + witness
 * generation.  Input validation errors return QP_ERR_ARG and witness
 * conflicts (an invalid Merkle proof or nullifier: plonky2's prove() fails)
 * QP_ERR_WITNESS, both with the reference's message in err.               */
int qp_voting_commit(const qp_circuit *c, const qp_voting_inputs *in, qp_witness **out, char *err, size_t errcap);
/* ---- recursive aggregation (wormhole/aggregator/src/circuits/tree.rs) -----
 * aggregate_chunk's circuit (tree.rs:106-127): a native recursive verifier
 * (plonky2 verify_proof: in-circuit challenger, vanishing polynomial at zeta,
 * FRI with Merkle paths to the caps, coset interpolation, PoW) of nproofs
 * proofs of the circuit whose CommonCircuitData bytes are inner_common (this
 * library's leaf or aggregation circuits), their public inputs registered in
 * order.  Prove it from chunks with qp_prover_prove_aggregation (witness
 * generation on the device) or from host witnesses (qp_aggregation_commit +
 * qp_prover_prove).                                                        */
int qp_aggregation_circuit_new(const uint8_t *inner_common, size_t len, uint32_t nproofs, qp_circuit **out);
/* one aggregate_chunk call's inputs (tree.rs:129-134): verifier_only =
 * VerifierOnlyCircuitData bytes of the inner circuit (cap height u64, cap,
 * circuit digest), proofs = nproofs serialized ProofWithPublicInputs,
 * zk_randomness = the PublicInputGate row's num_wires - 4 random cells (NULL:
 * OS randomness under the zk config, zeros otherwise).                      */
typedef struct {
    const uint8_t *verifier_only;
    size_t vlen;
    const uint8_t *const *proofs;
    const size_t *lens;
    uint32_t nproofs;
    const uint64_t *zk_randomness;
} qp_aggregation_chunk;
/* aggregate_chunk's witness on the host (set_verifier_data_target +
 * set_proof_with_pis_target + generate_partial_witness).  An invalid inner
 * proof fails witness generation (QP_ERR_WITNESS), as plonky2's prove() of the
 * aggregation circuit fails.  zk_randomness: as in qp_aggregation_chunk.    */
int qp_aggregation_commit(const qp_circuit *c, const uint8_t *verifier_only, size_t vlen,
                          const uint8_t *const *proofs, const size_t *lens, uint32_t nproofs,
                          const uint64_t *zk_randomness, qp_witness **out, char *err, size_t errcap);
/* full wire matrix, column-major [num_wires][n] */
int qp_witness_wires(const qp_witness *w, uint64_t *out);
int qp_witness_public_inputs(const qp_witness *w, uint64_t *out, uint32_t cap, uint32_t *n);
void qp_witness_free(qp_witness *w);

/* ---- prover (device) -------------------------------------------------------
 * plonky2 prove() (plonk/prover.rs) for B proofs of one circuit at a time,
 * replacing ProverCircuitData::prove as called by WormholeProver::prove
 * (wormhole/prover/src/lib.rs:233-237) and by the aggregator
 * (wormhole/aggregator/src/circuits/tree.rs:136).  qp_prover_new runs the
 * circuit's device preprocessing (constants/sigmas LDE + Merkle cap, circuit
 * digest: CircuitBuilder::build) and sizes the workspace for max_batch proofs.
 * Proof bytes follow ProofWithPublicInputs::to_bytes; the PoW witness is the
 * minimal one, so proofs are a deterministic function of the witness.      */
typedef struct qp_prover qp_prover;
int qp_prover_new(qp_ctx *ctx, const qp_circuit *c, uint32_t max_batch, qp_prover **out);
void qp_prover_free(qp_prover *p);
int qp_prover_proof_size(const qp_prover *p, size_t *len);
/* VerifierOnlyCircuitData || CommonCircuitData bytes (cap height, constants/sigmas
 * cap, circuit digest, common data) — the wormhole/bench-data/verifier.bin layout */
int qp_prover_verifier_data(const qp_prover *p, uint8_t *out, size_t cap, size_t *len);
/* prove from witnesses made by qp_wormhole_commit; proof b at out + b*stride */
int qp_prover_prove(qp_prover *p, const qp_witness *const *w, uint32_t nproofs, uint8_t *out, size_t stride,
                    size_t *lens);
/* prove from raw wire matrices [nproofs][num_wires][n] + public inputs [nproofs][npis] */
int qp_prover_prove_wires(qp_prover *p, const uint64_t *wires, const uint64_t *pis, uint32_t nproofs, uint8_t *out,
                          size_t stride, size_t *lens);
/* End to end: WormholeProver::commit(inputs) + prove() (wormhole/prover/src/lib.rs:
 * 209-237) for a batch of CircuitInputs.  commit() (the fragments' fill_targets)
 * runs on the host thread pool; generate_partial_witness (plonky2
 * iop/generator.rs: Poseidon, BaseSum, arithmetic, equality and constant
 * generators) runs on the device, one workgroup per proof, level by level;
 * then the proof.  A witness conflict returns QP_ERR_WITNESS with the
 * reference's "set twice with different values" message naming the proof. */
int qp_prover_prove_wormhole_inputs(qp_prover *p, const qp_wormhole_inputs *in, uint32_t nproofs, uint8_t *out,
                                    size_t stride, size_t *lens);
/* the same for the voting circuit: VoteCircuitData::fill_targets + prove
 * (voting/src/lib.rs:199-261, :346-357)                                     */
int qp_prover_prove_voting_inputs(qp_prover *p, const qp_voting_inputs *in, uint32_t nproofs, uint8_t *out,
                                  size_t stride, size_t *lens);
/* the same for aggregation circuits: nchunks aggregate_chunk calls
 * (tree.rs:106-143) proven as one batch — the chunks' proof bytes are
 * deserialized into the circuit's input targets on the host pool, the
 * recursive verifier's generators (Poseidon, arithmetic, BaseSum, wire split,
 * extension division, RandomAccess, ...) run on the device; an invalid inner
 * proof returns QP_ERR_WITNESS naming the chunk.                            */
int qp_prover_prove_aggregation(qp_prover *p, const qp_aggregation_chunk *chunks, uint32_t nchunks, uint8_t *out,
                                size_t stride, size_t *lens);
/* same, with the wire matrices already resident on the device:
 * d_wires = device pointer [nproofs][num_wires][n]; pis on the host          */
int qp_prover_prove_wires_dev(qp_prover *p, const uint64_t *d_wires, const uint64_t *pis, uint32_t nproofs,
                              uint8_t *out, size_t stride, size_t *lens);
/* HIP-event timing of the hot kernels on the prover's stream (off by default):
 * slot 0 = wires LDE (NTT; units = algorithmic bytes 8*(n+N) per column),
 * 1 = wires leaf hashing (units = permutations), 2 = wires Merkle levels
 * (units = permutations), 3 = quotient evaluation (units = LDE points)     */
int qp_prover_set_timing(qp_prover *p, int enable);
/* TEST-ONLY: use `witness` as every proof's FRI proof-of-work witness instead
 * of grinding the minimal one (enable = 0 restores grinding).  The reference's
 * rayon find_any witness is nondeterministic, so reproducing one of its proofs
 * byte for byte needs its witness (tests/test_gpu_reference_proof.py); a
 * witness without the required leading zeros gives a proof that fails
 * verification.                                                            */
int qp_prover_debug_force_pow(qp_prover *p, uint64_t witness, int enable);
/* TEST-ONLY: release one of the prover's device tables ("wg_wslot_cm",
 * "wg_gens" or "qtab") to check that a launch whose table is missing returns
 * QP_ERR_STATE naming it instead of faulting (every prove entry point checks
 * the tables its kernels read before launching them).                      */
int qp_prover_debug_drop_table(qp_prover *p, const char *name);
/* host threads (the caller included) of the prover's pool for commit() and the
 * per-proof host stages; default min(hardware threads, 16).  Several provers in
 * one process should split the host cores (cores / provers each).           */
int qp_prover_set_host_threads(qp_prover *p, uint32_t nthreads);
int qp_prover_kernel_stats(qp_prover *p, double *ms, double *units, uint64_t *launches, uint32_t n, int reset);
/* accumulated host wall time per stage (ms): [0] commit wires, [1] zs, [2] quotient,
 * [3] openings, [4] FRI, [5] PoW, [6] queries, [7] serialize, [8] commit() of the
 * inputs (host), [9] device witness generation; reset != 0 clears */
int qp_prover_stage_times(qp_prover *p, double *ms, uint32_t n, int reset);

/* ---- routine-level seams ---------------------------------
 * The pieces of plonky2's prove() (qp-plonky2 1.1.1 plonk/prover.rs,
 * fri/prover.rs) a patched crate routes to the GPU for any circuit over the
 * supported gate set within the shape limits below — e.g. the aggregator's
 * per-chunk circuits (wormhole/aggregator/src/circuits/tree.rs:127-136).  The
 * Fiat-Shamir transcript stays with the caller (INTEGRATION.md shows the call
 * sequence).
 *
 * Shape limits (a call outside them returns QP_ERR_ARG with the reason in the
 * context's last error, never a wrong result): commitments of up to 2^16
 * values per polynomial with LDE domains up to 2^18 points (log_n + rate_bits
 * <= 18, i.e. circuits up to degree 2^15 at rate 3, the top of a 2048-leaf
 * aggregation tree, and the level-1 circuits of 5- to 7-ary trees);
 * qp_quotient: 2^6 <= degree <= 2^15 (the same kernels as the whole-circuit
 * prover; above 2^14 the coset iNTT runs its first levels in HBM), 2
 * challenges, quotient_degree_factor == 2^rate_bits <= 16, at most 16 gates,
 * unsalted batches of one; qp_fri_layer_commit: at most 2^16 nonzero
 * coefficients.                                                             */

/* gate kinds of CommonCircuitData.gates (DefaultGateSerializer ids in brackets).
 * 0-5: the leaf circuits' gates (fast single-read quotient kernel); 6-13: the
 * recursive-verifier gates of the aggregator circuits (tree.rs:106-143; generic
 * quotient kernel; parity unpinned: no reference fixture holds such a circuit). */
enum { QP_GATE_NOOP = 0 /* 9 */, QP_GATE_CONSTANT = 1 /* 3 */, QP_GATE_PUBLIC_INPUT = 2 /* 12 */,
       QP_GATE_BASE_SUM = 3 /* 2, BaseSumGate<2> */, QP_GATE_ARITHMETIC = 4 /* 0 */, QP_GATE_POSEIDON = 5 /* 11 */,
       QP_GATE_ARITHMETIC_EXTENSION = 6 /* 1 */, QP_GATE_MUL_EXTENSION = 7 /* 8 */,
       QP_GATE_RANDOM_ACCESS = 8 /* 13 */, QP_GATE_EXPONENTIATION = 9 /* 5 */, QP_GATE_REDUCING = 10 /* 15 */,
       QP_GATE_REDUCING_EXTENSION = 11 /* 14 */, QP_GATE_POSEIDON_MDS = 12 /* 10 */,
       QP_GATE_COSET_INTERPOLATION = 13 /* 4 */ };
#define QP_MAX_GATES 16

/* the parts of CommonCircuitData the vanishing polynomial reads */
typedef struct {
    uint32_t num_gates;                    /* <= QP_MAX_GATES, in CommonCircuitData.gates order */
    uint32_t kind[QP_MAX_GATES];           /* QP_GATE_* */
    uint32_t param[QP_MAX_GATES];          /* Constant num_consts, BaseSum num_limbs, Arithmetic(Extension) /
                                              MulExtension num_ops, RandomAccess bits, Exponentiation
                                              num_power_bits, Reducing(Extension) num_coeffs,
                                              CosetInterpolation subgroup_bits */
    uint32_t param2[QP_MAX_GATES];         /* RandomAccess num_copies, CosetInterpolation degree */
    uint32_t param3[QP_MAX_GATES];         /* RandomAccess num_extra_constants */
    uint32_t selector_index[QP_MAX_GATES]; /* selectors_info.selector_indices */
    uint32_t num_selectors;                /* selectors_info.groups.len() */
    uint32_t group_lo[QP_MAX_GATES], group_hi[QP_MAX_GATES];
    uint32_t num_constants;                /* selectors + gate constants */
    uint32_t num_routed_wires, num_wires, quotient_degree_factor, num_challenges, num_gate_constraints;
} qp_gate_desc;

/* fill a qp_gate_desc from a built circuit of this library */
int qp_circuit_gate_desc(const qp_circuit *c, qp_gate_desc *g);

/* compute_quotient_polys (plonk/prover.rs): vanishing polynomial at every
 * point of the LDE coset from the committed batches (constants||sigmas, wires,
 * zs||partial products; qp_commit_values batches of one, kept), alpha-reduced
 * per challenge, divided by Z_H, coset-iFFT'd and split:
 * quotient_coeffs_out [num_challenges * quotient_degree_factor][n].
 * betas/gammas/alphas [num_challenges] (num_challenges == 2), pi_hash =
 * hash_no_pad(public inputs).  Replaces prover.rs:compute_quotient_polys as
 * reached from CircuitData::prove (tree.rs:136, lib.rs:233-237).            */
int qp_quotient(qp_ctx *ctx, const qp_batch *cs, const qp_batch *wires, const qp_batch *zs_pp, const qp_gate_desc *g,
                const uint64_t *betas, const uint64_t *gammas, const uint64_t *alphas, const uint64_t pi_hash[4],
                uint64_t *quotient_coeffs_out);

/* one reduction layer of fri_committed_trees (fri/prover.rs): values =
 * coeffs.coset_fft(shift) of size 2^log_values, reverse_index_bits, leaves of
 * 2^arity_bits ext values, MerkleTree -> cap_out [2^cap_height][4].  coeffs are
 * ext coefficients as two rows [2][2^log_coeffs] (c0, c1); the reference keeps
 * them full length with a zero tail, so log_coeffs may equal log_values: only
 * the nonzero prefix (at most 2^16 coefficients) is transformed.  The caller
 * observes the cap, draws beta and calls qp_fri_fold; out (optional) keeps the
 * layer for qp_fri_layer_open in the query rounds.  A layer uses its context's
 * stream: free it (qp_fri_layer_free) before qp_ctx_destroy.                */
typedef struct qp_fri_layer qp_fri_layer;
int qp_fri_layer_commit(qp_ctx *ctx, const uint64_t *coeffs, uint32_t log_coeffs, uint32_t log_values, uint64_t shift,
                        uint32_t arity_bits, uint32_t cap_height, uint64_t *cap_out, qp_fri_layer **out);
/* leaf evals_out [nidx][2^arity_bits][2] (ext, c0 c1) and Merkle siblings
 * [nidx][log_leaves - cap_height][4] of layer leaves idx[]                 */
int qp_fri_layer_open(qp_fri_layer *layer, const uint32_t *idx, uint32_t nidx, uint64_t *evals_out,
                      uint64_t *siblings_out);
void qp_fri_layer_free(qp_fri_layer *layer);
/* coeffs_out[k] = sum_{i < 2^arity_bits} beta^i coeffs[2^arity_bits k + i]
 * (reduce_with_powers over chunks), ext rows [2][2^(log_coeffs - arity_bits)] */
int qp_fri_fold(qp_ctx *ctx, const uint64_t *coeffs, uint32_t log_coeffs, uint32_t arity_bits, const uint64_t beta[2],
                uint64_t *coeffs_out);

/* fri_proof_of_work (fri/prover.rs) for n transcripts: states [n][12] are the
 * duplex intermediate states (sponge_state with the pending input_buffer
 * written into lanes 0..pos-1), pos[b] = input_buffer.len() < 8.  Returns the
 * MINIMAL witness w with leading_zeros(permute(state with lane pos = w)[7])
 * >= pow_bits, 1 <= pow_bits <= 32 (the reference's rayon find_any returns any
 * such w).                                                                 */
int qp_pow_grind(qp_ctx *ctx, const uint64_t *states, const uint32_t *pos, uint32_t n, uint32_t pow_bits,
                 uint64_t *witness_out);

#ifdef __cplusplus
}
#endif
#endif
