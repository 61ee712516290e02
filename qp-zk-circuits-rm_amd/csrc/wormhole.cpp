// wormhole.cpp — the Wormhole circuit on the native builder.  Each fragment
// follows its reference file:
//   Nullifier::circuit          wormhole/circuit/src/nullifier.rs:215-242
//   UnspendableAccount::circuit wormhole/circuit/src/unspendable_account.rs:182-208
//   StorageProof::circuit       wormhole/circuit/src/storage_proof/mod.rs:140-244
//   SubstrateAccount::circuit   wormhole/circuit/src/substrate_account.rs:84-97
//   connect_shared_targets      wormhole/circuit/src/circuit.rs:111-137
//   is_const_less_than / xor    common/src/gadgets.rs:14-65
#include "wormhole.h"
#include <string.h>
#include "field.h"

namespace qw {

using qc::CircuitBuilder;

std::vector<F> injective_bytes_to_felts(const uint8_t *b, size_t n) {
  std::vector<F> out;
  for (size_t i = 0; i < n; i += 4) {
    uint32_t v = 0;
    for (size_t k = 0; k < 4 && i + k < n; k++) v |= (uint32_t)b[i + k] << (8 * k);
    out.push_back(v);
  }
  return out;
}

static void injective_string_to_felt(const char *s, F out[2]) {
  auto v = injective_bytes_to_felts((const uint8_t *)s, 8);
  out[0] = v[0];
  out[1] = v[1];
}

bool digest_bytes_to_felts(const uint8_t b[32], F out[4]) {
  bool ok = true;
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b[8 * i + k] << (8 * k);
    if (v >= gl::P) ok = false;
    out[i] = gl::canon(v);
  }
  return ok;
}

void u64_to_felts(uint64_t x, F out[2]) {
  out[0] = (x >> 32) & 0xFFFFFFFFull;
  out[1] = x & 0xFFFFFFFFull;
}

void u128_to_felts(uint64_t lo, uint64_t hi, F out[4]) {
  out[0] = (hi >> 32) & 0xFFFFFFFFull;
  out[1] = hi & 0xFFFFFFFFull;
  out[2] = (lo >> 32) & 0xFFFFFFFFull;
  out[3] = lo & 0xFFFFFFFFull;
}

WormholeTargets build_wormhole(CircuitBuilder &b) {
  WormholeTargets t;
  // CircuitTargets::new (targets + public inputs in the reference's order)
  t.nullifier.hash = b.add_virtual_hash_public_input();
  t.nullifier.secret = b.add_virtual_targets(SECRET_NUM_TARGETS);
  t.nullifier.transfer_count = b.add_virtual_targets(2);
  t.unspendable.account_id = b.add_virtual_hash();
  t.unspendable.secret = b.add_virtual_targets(SECRET_NUM_TARGETS);
  for (uint32_t i = 0; i < MAX_PROOF_LEN; i++) t.storage.proof_data.push_back(b.add_virtual_targets(PROOF_NODE_MAX_SIZE_F));
  t.storage.indices = b.add_virtual_targets(MAX_PROOF_LEN);
  t.storage.root_hash = b.add_virtual_hash_public_input();
  t.storage.proof_len = b.add_virtual_target();
  t.storage.leaf.transfer_count = b.add_virtual_targets(2);
  t.storage.leaf.funding_account = b.add_virtual_hash();
  t.storage.leaf.to_account = b.add_virtual_hash();
  for (int i = 0; i < 4; i++) t.storage.leaf.funding_amount.push_back(b.add_virtual_public_input());
  t.exit_address = b.add_virtual_hash_public_input();

  // the targets commit() sets
  b.mark_inputs(t.nullifier.hash);
  b.mark_inputs(t.nullifier.secret);
  b.mark_inputs(t.nullifier.transfer_count);
  b.mark_inputs(t.unspendable.account_id);
  b.mark_inputs(t.unspendable.secret);
  for (auto &nd : t.storage.proof_data) b.mark_inputs(nd);
  b.mark_inputs(t.storage.indices);
  b.mark_inputs(t.storage.root_hash);
  b.mark_input(t.storage.proof_len);
  b.mark_inputs(t.storage.leaf.transfer_count);
  b.mark_inputs(t.storage.leaf.funding_account);
  b.mark_inputs(t.storage.leaf.to_account);
  b.mark_inputs(t.storage.leaf.funding_amount);
  b.mark_inputs(t.exit_address);

  // Nullifier::circuit
  {
    F salt[2];
    injective_string_to_felt("~nullif~", salt);
    std::vector<Target> pre = {b.constant(salt[0]), b.constant(salt[1])};
    pre.insert(pre.end(), t.nullifier.secret.begin(), t.nullifier.secret.end());
    pre.insert(pre.end(), t.nullifier.transfer_count.begin(), t.nullifier.transfer_count.end());
    for (Target x : pre) b.range_check(x, 32);
    auto inner = b.hash_n_to_hash_no_pad(pre);
    auto computed = b.hash_n_to_hash_no_pad(inner);
    b.connect_hashes(computed, t.nullifier.hash);
  }
  // UnspendableAccount::circuit
  {
    F salt[2];
    injective_string_to_felt("wormhole", salt);
    std::vector<Target> pre = {b.constant(salt[0]), b.constant(salt[1])};
    for (Target x : pre) b.range_check(x, 32);
    pre.insert(pre.end(), t.unspendable.secret.begin(), t.unspendable.secret.end());
    auto inner = b.hash_n_to_hash_no_pad(pre);
    auto gen = b.hash_n_to_hash_no_pad(inner);
    b.connect_hashes(gen, t.unspendable.account_id);
  }
  // StorageProof::circuit
  {
    const LeafTargets &lf = t.storage.leaf;
    std::vector<Target> l32 = lf.transfer_count;
    l32.insert(l32.end(), lf.funding_amount.begin(), lf.funding_amount.end());
    for (Target x : l32) b.range_check(x, 32);
    std::vector<Target> leaf_vec = lf.transfer_count;
    leaf_vec.insert(leaf_vec.end(), lf.funding_account.begin(), lf.funding_account.end());
    leaf_vec.insert(leaf_vec.end(), lf.to_account.begin(), lf.to_account.end());
    leaf_vec.insert(leaf_vec.end(), lf.funding_amount.begin(), lf.funding_amount.end());
    auto leaf_hash = b.hash_n_to_hash_no_pad(leaf_vec);
    Target two_pow_32 = b.constant(1ull << 32);
    std::vector<Target> prev = t.storage.root_hash;
    const uint32_t n_log = 32 - __builtin_clz(MAX_PROOF_LEN - 1);
    for (uint32_t i = 0; i < MAX_PROOF_LEN; i++) {
      const auto &node = t.storage.proof_data[i];
      Target is_proof_node = is_const_less_than(b, i, t.storage.proof_len, n_log);
      Target i_t = b.constant(i);
      Target is_leaf_node = b.is_equal(i_t, t.storage.proof_len);
      auto computed = b.hash_n_to_hash_no_pad(node);
      for (int y = 0; y < 4; y++) {
        Target diff = b.sub(computed[y], prev[y]);
        Target res = b.mul(diff, is_proof_node);
        b.connect(res, b.zero());
      }
      Target z = b.zero();
      std::vector<Target> found = {z, z, z, z};
      Target expected = t.storage.indices[i];
      for (uint32_t j = 0; j < PROOF_NODE_MAX_SIZE_F - 8; j++) {
        b.range_check(node[j], 32);
        Target felt_index = b.constant(j);
        Target is_start = b.is_equal(felt_index, expected);
        auto combine = [&](Target lo, Target hi) {
          Target hs = b.mul(hi, two_pow_32);
          return b.add(lo, hs);
        };
        Target h0 = combine(node[j], node[j + 1]);
        Target h1 = combine(node[j + 2], node[j + 3]);
        Target h2 = combine(node[j + 4], node[j + 5]);
        Target h3 = combine(node[j + 6], node[j + 7]);
        found[0] = b.select(is_start, h0, found[0]);
        found[1] = b.select(is_start, h1, found[1]);
        found[2] = b.select(is_start, h2, found[2]);
        found[3] = b.select(is_start, h3, found[3]);
      }
      for (uint32_t j = PROOF_NODE_MAX_SIZE_F - 8; j < PROOF_NODE_MAX_SIZE_F; j++) b.range_check(node[j], 32);
      for (int y = 1; y < 4; y++) {
        Target diff = b.sub(leaf_hash[y], prev[y]);
        Target res = b.mul(diff, is_leaf_node);
        b.connect(res, b.zero());
      }
      prev = found;
    }
  }
  // SubstrateAccount::circuit: exit address is a public input only.
  // connect_shared_targets
  for (uint32_t i = 0; i < SECRET_NUM_TARGETS; i++) b.connect(t.nullifier.secret[i], t.unspendable.secret[i]);
  for (uint32_t i = 0; i < 2; i++) b.connect(t.nullifier.transfer_count[i], t.storage.leaf.transfer_count[i]);
  b.connect_hashes(t.unspendable.account_id, t.storage.leaf.to_account);
  return t;
}

static bool set_all(qc::Witness &w, const std::vector<Target> &ts, const F *v) {
  for (size_t i = 0; i < ts.size(); i++)
    if (!w.set(ts[i], v[i])) return false;
  return true;
}

std::string commit(const WormholeTargets &t, const CircuitInputs &in, qc::Witness &w) {
  const char *conflict = "Partition containing a target was set twice with different values";
  F d[4], tc[2], amt[4];
  // Nullifier::fill_targets (nullifier.rs:244-254)
  if (!digest_bytes_to_felts(in.nullifier, d)) return "nullifier digest chunk out of field range";
  if (!set_all(w, t.nullifier.hash, d)) return conflict;
  auto secret = injective_bytes_to_felts(in.secret, 32);
  if (!set_all(w, t.nullifier.secret, secret.data())) return conflict;
  u64_to_felts(in.transfer_count, tc);
  if (!set_all(w, t.nullifier.transfer_count, tc)) return conflict;
  // UnspendableAccount::fill_targets
  if (!digest_bytes_to_felts(in.unspendable_account, d)) return "unspendable account chunk out of field range";
  if (!set_all(w, t.unspendable.account_id, d)) return conflict;
  if (!set_all(w, t.unspendable.secret, secret.data())) return conflict;
  // StorageProof::fill_targets (storage_proof/mod.rs:246-301)
  if (in.storage_proof.size() != in.storage_indices.size())
    return "indices length must be equal to proof length";
  if (!digest_bytes_to_felts(in.root_hash, d)) return "root hash chunk out of field range";
  if (!set_all(w, t.storage.root_hash, d)) return conflict;
  if (in.storage_proof.size() > MAX_PROOF_LEN)
    return "proof length exceeds maximum allowed length: " + std::to_string(in.storage_proof.size()) + " > 20";
  if (!w.set(t.storage.proof_len, in.storage_proof.size())) return conflict;
  for (uint32_t i = 0; i < MAX_PROOF_LEN; i++) {
    std::vector<F> node(PROOF_NODE_MAX_SIZE_F, 0);
    if (i < in.storage_proof.size()) {
      auto f = injective_bytes_to_felts(in.storage_proof[i].data(), in.storage_proof[i].size());
      if (f.size() > PROOF_NODE_MAX_SIZE_F)
        return "proof node at index " + std::to_string(i) + " is too large: " + std::to_string(f.size());
      for (size_t k = 0; k < f.size(); k++) node[k] = f[k];
    }
    if (!set_all(w, t.storage.proof_data[i], node.data())) return conflict;
  }
  for (uint32_t i = 0; i < MAX_PROOF_LEN; i++) {
    F idx = i < in.storage_indices.size() ? in.storage_indices[i] / 8 : 0;
    if (!w.set(t.storage.indices[i], idx)) return conflict;
  }
  if (!set_all(w, t.storage.leaf.transfer_count, tc)) return conflict;
  if (!digest_bytes_to_felts(in.funding_account, d)) return "funding account chunk out of field range";
  if (!set_all(w, t.storage.leaf.funding_account, d)) return conflict;
  if (!digest_bytes_to_felts(in.unspendable_account, d)) return "unspendable account chunk out of field range";
  if (!set_all(w, t.storage.leaf.to_account, d)) return conflict;
  u128_to_felts(in.funding_amount_lo, in.funding_amount_hi, amt);
  if (!set_all(w, t.storage.leaf.funding_amount, amt)) return conflict;
  // SubstrateAccount (exit) fill_targets
  if (!digest_bytes_to_felts(in.exit_account, d)) return "exit account chunk out of field range";
  if (!set_all(w, t.exit_address, d)) return conflict;
  return "";
}

}  // namespace qw
