// recursion.h — the recursive verifier on the native builder: plonky2's
// verify_proof gadget (plonk/recursive_verifier.rs, fri/recursive_verifier.rs,
// iop/challenger.rs RecursiveChallenger, gadgets/*) as the Wormhole aggregator
// calls it from aggregate_chunk (wormhole/aggregator/src/circuits/tree.rs:106-143):
//   add_virtual_verifier_data + per proof add_virtual_proof_with_pis,
//   verify_proof, register_public_inputs(proof.public_inputs).
//
// The inner circuits are this library's: the Wormhole / voting leaf circuits
// (Noop, Constant, PublicInput, BaseSum, Arithmetic, Poseidon) and the
// aggregation circuits themselves.  The gadgets are upstream's recursive
// verifier's, on upstream's gates: extension arithmetic on
// ArithmeticExtension / MulExtension ops (special cases and operation dedup as
// gadgets/arithmetic_extension.rs), divisions through an inverse generator,
// the in-circuit Poseidon gate evaluation on PoseidonMds layers, the alpha
// reductions on Reducing / ReducingExtension rows, the FRI coset checks on
// CosetInterpolation rows, Merkle caps and coset evaluations selected with
// RandomAccess copies.  Two degree-13 Wormhole proofs then fit 2^13 rows
// (7,596 gates), and so do two aggregation proofs (7,917).  Values are pinned
// (every challenge, vanishing term and FRI check equals plonky2's, SURVEY.md
// A.4-A.7: the reference's own proofs verify inside); the gate layout restates
// upstream without a fixture (parity unpinned).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>
#include "circuit.h"

namespace qr {

using qc::F;
using qc::Target;

using qc::ExtT;

// CommonCircuitData of the circuit whose proofs are verified (parsed bytes)
struct InnerCommon {
  std::vector<uint8_t> bytes;
  uint32_t num_wires = 0, num_routed_wires = 0, config_num_constants = 0, num_challenges = 0;
  uint32_t rate_bits = 0, cap_height = 0, num_query_rounds = 0, pow_bits = 0;
  std::vector<uint32_t> arity_bits;
  uint32_t degree_bits = 0;
  bool hiding = false, zero_knowledge = false;
  std::vector<uint32_t> selector_indices;
  std::vector<std::pair<uint32_t, uint32_t>> groups;
  uint32_t quotient_degree_factor = 0, num_gate_constraints = 0, num_constants = 0, num_public_inputs = 0;
  std::vector<F> k_is;
  uint32_t num_partial_products = 0;
  struct Gate {
    uint32_t id;    // DefaultGateSerializer tag
    uint64_t p[3];  // parameters in serialization order
  };
  std::vector<Gate> gates;
  uint32_t final_poly_len() const;
  uint32_t width(int oracle) const;  // unsalted leaf widths of the 4 initial trees
};
// CommonCircuitData::from_bytes for the supported gate set; "" or an error
std::string parse_common(const uint8_t *b, size_t n, InnerCommon &out);

struct QueryTargets {
  std::vector<Target> leaf[4], sib[4];           // initial trees
  std::vector<std::vector<ExtT>> evals;          // per FRI layer: 2^arity ext values
  std::vector<std::vector<Target>> lsib;         // per FRI layer: siblings (4 felts each)
};
struct ProofTargets {  // ProofWithPublicInputsTarget
  std::vector<Target> wires_cap, zs_cap, quot_cap;
  std::vector<ExtT> constants_sigmas, wires, zs, zs_next, pp, quotient;  // openings
  std::vector<std::vector<Target>> commit_caps;
  std::vector<QueryTargets> queries;
  std::vector<ExtT> final_poly;
  Target pow_witness;
  std::vector<Target> pis;
};
struct AggregationTargets {
  InnerCommon inner;
  std::vector<Target> vd_cap, vd_digest;  // VerifierCircuitTarget (add_virtual_verifier_data)
  std::vector<ProofTargets> proofs;
};

// aggregate_chunk's circuit: nproofs inner proofs verified against one virtual
// verifier data, their public inputs registered in order
AggregationTargets build_aggregation(qc::CircuitBuilder &b, const InnerCommon &inner, uint32_t nproofs);

// aggregate_chunk's witness: set_verifier_data_target + set_proof_with_pis_target.
// vo = VerifierOnlyCircuitData bytes (cap height u64, cap, circuit digest).
std::string fill_aggregation(const AggregationTargets &t, const uint8_t *vo, size_t volen,
                             const uint8_t *const *proofs, const size_t *lens, uint32_t nproofs, qc::Witness &w);

// proof size (bytes) of a proof of `inner` with `npis` public inputs
size_t proof_bytes(const InnerCommon &inner, uint32_t npis);

}  // namespace qr
