// circuit_obj.h — definitions behind qp_circuit / qp_witness handles.
#pragma once
#include <stdint.h>
#include <mutex>
#include <vector>
#include "circuit.h"
#include "recursion.h"
#include "voting.h"
#include "wormhole.h"

struct qp_circuit {
  enum Kind { WORMHOLE = 1, VOTING = 2, AGGREGATION = 3 } kind = WORMHOLE;
  qc::CircuitData cd;
  qw::WormholeTargets wormhole;
  qv::VoteTargets voting;
  qr::AggregationTargets aggregation;
  uint32_t gates_used = 0;
  // upstream-format prover.bin between qp_circuit_prover_only_bytes' size and copy calls
  mutable std::vector<uint8_t> prover_bin;  // guarded by prover_bin_mu
  mutable std::mutex prover_bin_mu;
};

// commit(): the fragments' fill_targets into w (no generation); "" on success,
// else the reference's message; *code receives the qp_status to return
std::string wormhole_fill(const qp_circuit *c, const void *in /* qp_wormhole_inputs */, qc::Witness &w, int *code);
std::string voting_fill(const qp_circuit *c, const void *in /* qp_voting_inputs */, qc::Witness &w, int *code);
std::string aggregation_fill(const qp_circuit *c, const void *in /* qp_aggregation_chunk */, qc::Witness &w,
                             int *code);

struct qp_witness {
  explicit qp_witness(const qp_circuit *c) : circuit(c), w(c->cd) {}
  const qp_circuit *circuit;
  qc::Witness w;
};
