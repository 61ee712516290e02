// witness_kernels.h — launch interface of witness.hip (device witness generation).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qpk {

struct WitnessGenArgs {
  uint64_t *vals;             // [B][v_bstride] slot values
  uint64_t v_bstride;
  const uint64_t *gens;       // qc::DevGen records (40 B each), level order
  const uint32_t *level_off;  // [nlevels + 1]
  const uint32_t *level_pos;  // [nlevels][2]: first Poseidon generator, count
  uint32_t nlevels;
  uint32_t coop_max;          // levels with at most this many Poseidons run them cooperatively
  uint32_t row;               // cooperative Poseidons one per 16-lane row (else one per wave)
  const uint32_t *wslot;      // row-major wire -> slot map [n][W]
  uint32_t W, limbs, zero_slot, num_consts;
  uint32_t *err;              // [B]: 0 = ok, else 1 + index of the first failing generator
};

__global__ void k_witness_init(uint64_t *vals, uint64_t v_bstride, uint32_t nslots, const uint32_t *in_slots,
                               const uint64_t *in_vals, uint32_t nin);
__global__ void k_witness_inputs(uint64_t *vals, uint64_t v_bstride, const uint32_t *in_slots,
                                 const uint64_t *in_vals, uint32_t nin);
__global__ void k_witness_gen(const WitnessGenArgs a);
// one dependency level of nb proofs (grid (na + Poseidon blocks, nb), 256 threads)
__global__ void k_witness_level(const WitnessGenArgs a, uint32_t l, uint32_t na);
__global__ void k_witness_expand(const uint64_t *vals, uint64_t v_bstride, const uint32_t *wslot_cm, uint64_t nwires,
                                 uint64_t *wires, uint64_t w_bstride, const uint32_t *pi_slots, uint32_t npis,
                                 uint64_t *pis);

}  // namespace qpk
