// voting.cpp — the voting circuit on the native builder (voting/src/lib.rs).
//   VoteTargets::new           voting/src/lib.rs:71-100
//   VoteCircuitData::circuit   voting/src/lib.rs:123-197
//   fill_targets               voting/src/lib.rs:199-261
//   is_const_less_than / xor   common/src/gadgets.rs:14-65
#include "voting.h"
#include "field.h"

namespace qv {

using qc::CircuitBuilder;

VoteTargets build_voting(CircuitBuilder &b) {
  VoteTargets t;
  // public inputs in the reference's registration order
  t.proposal_id = b.add_virtual_hash_public_input();
  t.expected_merkle_root = b.add_virtual_hash_public_input();
  t.vote = b.add_virtual_bool_target_safe();
  b.register_public_input(t.vote);
  t.expected_nullifier = b.add_virtual_hash_public_input();
  // private inputs
  t.private_key = b.add_virtual_hash();
  for (uint32_t i = 0; i < MAX_MERKLE_DEPTH; i++) t.merkle_siblings.push_back(b.add_virtual_hash());
  for (uint32_t i = 0; i < MAX_MERKLE_DEPTH; i++) t.path_indices.push_back(b.add_virtual_bool_target_safe());
  t.actual_merkle_depth = b.add_virtual_target();

  b.mark_inputs(t.proposal_id);
  b.mark_inputs(t.expected_merkle_root);
  b.mark_input(t.vote);
  b.mark_inputs(t.expected_nullifier);
  b.mark_inputs(t.private_key);
  for (auto &s : t.merkle_siblings) b.mark_inputs(s);
  b.mark_inputs(t.path_indices);
  b.mark_input(t.actual_merkle_depth);

  // 1. Merkle proof verification
  const auto leaf_hash = b.hash_n_to_hash_no_pad(t.private_key);
  auto current = leaf_hash;
  // usize::BITS - (MAX_MERKLE_DEPTH - 1).leading_zeros()
  const uint32_t n_log = 32 - __builtin_clz(MAX_MERKLE_DEPTH - 1);
  for (uint32_t i = 0; i < MAX_MERKLE_DEPTH; i++) {
    Target is_active = qc::is_const_less_than(b, i, t.actual_merkle_depth, n_log);
    const auto &sib = t.merkle_siblings[i];
    Target path = t.path_indices[i];
    std::vector<Target> combined, right;
    for (int k = 0; k < 4; k++) {
      combined.push_back(b.select(path, sib[k], current[k]));
      right.push_back(b.select(path, current[k], sib[k]));
    }
    combined.insert(combined.end(), right.begin(), right.end());
    auto parent = b.hash_n_to_hash_no_pad(combined);
    std::vector<Target> next;
    for (int k = 0; k < 4; k++) next.push_back(b.select(is_active, parent[k], current[k]));
    current = next;
  }
  b.connect_hashes(current, t.expected_merkle_root);
  // 2. nullifier = H(leaf_hash ‖ proposal_id)
  std::vector<Target> nin = leaf_hash;
  nin.insert(nin.end(), t.proposal_id.begin(), t.proposal_id.end());
  auto nullifier = b.hash_n_to_hash_no_pad(nin);
  b.connect_hashes(nullifier, t.expected_nullifier);
  // 3. the vote is boolean by add_virtual_bool_target_safe
  return t;
}

static bool set4(qc::Witness &w, const std::vector<Target> &ts, const F *v) {
  for (size_t i = 0; i < ts.size(); i++)
    if (!w.set(ts[i], gl::canon(v[i]))) return false;
  return true;
}

std::string fill_targets(const VoteTargets &t, const VoteInputs &in, qc::Witness &w) {
  const char *conflict = "Partition containing a target was set twice with different values";
  if (in.actual_merkle_depth > MAX_MERKLE_DEPTH)
    return "Merkle tree depth " + std::to_string(in.actual_merkle_depth) + " exceeds maximum allowed depth " +
           std::to_string(MAX_MERKLE_DEPTH);
  if (in.merkle_siblings.size() != in.path_indices.size())
    return "Merkle proof length mismatch: " + std::to_string(in.merkle_siblings.size()) + " siblings vs " +
           std::to_string(in.path_indices.size()) + " path indices";
  if (!set4(w, t.proposal_id, in.proposal_id)) return conflict;
  if (!set4(w, t.expected_merkle_root, in.merkle_root)) return conflict;
  if (!w.set(t.vote, in.vote ? 1 : 0)) return conflict;
  if (!set4(w, t.expected_nullifier, in.nullifier)) return conflict;
  if (!set4(w, t.private_key, in.private_key)) return conflict;
  if (!w.set(t.actual_merkle_depth, in.actual_merkle_depth)) return conflict;
  const F zero[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < MAX_MERKLE_DEPTH; i++) {
    if (i < in.actual_merkle_depth) {
      // the reference indexes merkle_siblings[i] here (a Rust bounds panic when shorter)
      if (i >= in.merkle_siblings.size())
        return "index out of bounds: the len is " + std::to_string(in.merkle_siblings.size()) + " but the index is " +
               std::to_string(i);
      if (!set4(w, t.merkle_siblings[i], in.merkle_siblings[i].data())) return conflict;
      if (!w.set(t.path_indices[i], in.path_indices[i] ? 1 : 0)) return conflict;
    } else {
      if (!set4(w, t.merkle_siblings[i], zero)) return conflict;
      if (!w.set(t.path_indices[i], 0)) return conflict;
    }
  }
  return "";
}

}  // namespace qv
