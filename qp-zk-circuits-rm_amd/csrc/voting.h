// voting.h — the voting circuit (voting/src/lib.rs) on the native builder:
// 32-level Poseidon Merkle membership of hash(private key) + nullifier
// hash(leaf ‖ proposal id) + a boolean vote, all reusing the common/ gadgets
// (is_const_less_than, select, hash_n_to_hash_no_pad) the Wormhole circuit uses.
#pragma once
#include <stdint.h>
#include <array>
#include <string>
#include <vector>
#include "circuit.h"

namespace qv {

using qc::F;
using qc::Target;

constexpr uint32_t MAX_MERKLE_DEPTH = 32;  // voting/src/lib.rs:21

struct VoteTargets {  // voting/src/lib.rs:56-69
  std::vector<Target> proposal_id, expected_merkle_root, expected_nullifier, private_key;
  Target vote;
  std::vector<std::vector<Target>> merkle_siblings;
  std::vector<Target> path_indices;
  Target actual_merkle_depth;
};

// VotePublicInputs / VotePrivateInputs (voting/src/lib.rs:26-52), felt form
struct VoteInputs {
  F proposal_id[4] = {0}, merkle_root[4] = {0}, nullifier[4] = {0};
  bool vote = false;
  F private_key[4] = {0};
  std::vector<std::array<F, 4>> merkle_siblings;
  std::vector<bool> path_indices;
  uint64_t actual_merkle_depth = 0;
};

// VoteTargets::new + VoteCircuitData::circuit (voting/src/lib.rs:71-100, :123-197)
VoteTargets build_voting(qc::CircuitBuilder &b);

// VoteCircuitData::fill_targets (voting/src/lib.rs:199-261): "" on success or
// the reference's error message.
std::string fill_targets(const VoteTargets &t, const VoteInputs &in, qc::Witness &w);

}  // namespace qv
