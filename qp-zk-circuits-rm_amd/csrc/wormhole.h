// wormhole.h — the Wormhole circuit (nullifier, unspendable account,
// storage proof, exit account) on the native builder, plus commit()
// (the fragments' fill_targets) — wormhole/circuit/src/circuit.rs:63-137.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>
#include "circuit.h"

namespace qw {

using qc::F;
using qc::Target;

constexpr uint32_t MAX_PROOF_LEN = 20;          // storage_proof/mod.rs:21
constexpr uint32_t PROOF_NODE_MAX_SIZE_F = 188;  // storage_proof/mod.rs:22
constexpr uint32_t SECRET_NUM_TARGETS = 8;

struct NullifierTargets {  // nullifier.rs:195-210
  std::vector<Target> hash, secret, transfer_count;
};
struct UnspendableTargets {  // unspendable_account.rs:165-180
  std::vector<Target> account_id, secret;
};
struct LeafTargets {  // storage_proof/leaf.rs:17-55
  std::vector<Target> transfer_count, funding_account, to_account, funding_amount;
};
struct StorageProofTargets {  // storage_proof/mod.rs:26-56
  std::vector<Target> root_hash;
  Target proof_len;
  std::vector<std::vector<Target>> proof_data;
  std::vector<Target> indices;
  LeafTargets leaf;
};
struct WormholeTargets {  // circuit.rs:44-62
  NullifierTargets nullifier;
  UnspendableTargets unspendable;
  StorageProofTargets storage;
  std::vector<Target> exit_address;
};

// CircuitInputs (wormhole/circuit/src/inputs.rs:25-52), byte form
struct CircuitInputs {
  // public
  uint64_t funding_amount_lo = 0, funding_amount_hi = 0;  // u128
  uint8_t nullifier[32] = {0}, root_hash[32] = {0}, exit_account[32] = {0};
  // private
  uint8_t secret[32] = {0};
  uint64_t transfer_count = 0;
  uint8_t funding_account[32] = {0}, unspendable_account[32] = {0};
  std::vector<std::vector<uint8_t>> storage_proof;
  std::vector<uint64_t> storage_indices;  // hex-character indices (ProcessedStorageProof)
};

// WormholeCircuit::new: all four fragments + connect_shared_targets
WormholeTargets build_wormhole(qc::CircuitBuilder &b);

// WormholeProver::commit: fill every fragment's targets.  Returns "" on
// success or the reference's error message.
std::string commit(const WormholeTargets &t, const CircuitInputs &in, qc::Witness &w);

// codecs (common/src/utils.rs)
std::vector<F> injective_bytes_to_felts(const uint8_t *b, size_t n);
bool digest_bytes_to_felts(const uint8_t b[32], F out[4]);  // false if a limb >= p
void u64_to_felts(uint64_t x, F out[2]);
void u128_to_felts(uint64_t lo, uint64_t hi, F out[4]);

}  // namespace qw
