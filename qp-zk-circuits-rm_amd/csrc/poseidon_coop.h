// poseidon_coop.h — one Poseidon permutation on one wave: lane i < 12 holds
// state element i.  For work that is a chain of single permutations with too
// few of them to fill the GPU (the device witness's narrow levels, the upper
// Merkle levels of small batches): the one-lane form issues a permutation's
// ~15k instructions back to back from one wave (≈70 us at one wave per SIMD),
// this form ≈125 per round (one S-box, the MDS row of the lane from the 12
// S-box outputs broadcast by v_readlane, six products in two accumulators per
// half).  All 64 lanes must be active; lanes >= 12 compute and are ignored.
#pragma once
#include "poseidon.h"
#include "poseidon_fast.h"

namespace pc {

// MDS row of this lane (coefficients coef[j] of element j) over the 12 lanes' y
__device__ __forceinline__ uint64_t wave_mds_row(uint64_t y, const uint32_t (&coef)[12]) {
  const uint32_t lo = (uint32_t)y, hi = (uint32_t)(y >> 32);
  uint64_t al[2] = {0, 0}, ah[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const uint32_t xl = __builtin_amdgcn_readlane(lo, j), xh = __builtin_amdgcn_readlane(hi, j);
    al[j & 1] += (uint64_t)xl * coef[j];
    ah[j & 1] += (uint64_t)xh * coef[j];
  }
  return pf::reduce_row(al[0] + al[1], ah[0] + ah[1]);
}

// row i of the MDS matrix: element j's coefficient CIRC[(j - i) mod 12] (+ 8 on
// the diagonal of row 0)
__device__ __forceinline__ void mds_coef(uint32_t i, uint32_t (&coef)[12]) {
#pragma unroll
  for (int j = 0; j < 12; j++) coef[j] = ps::mds_circ((j - (int)i + 12) % 12) + (i == 0 && j == 0 ? 8u : 0u);
}

// the permutation of the state held in lanes 0..11 (x = this lane's element);
// returns this lane's element of the output (non-canonical)
__device__ __forceinline__ uint64_t permute(uint64_t x) {
  const uint32_t lane = threadIdx.x & 63, i = lane < 12 ? lane : 0;
  uint32_t coef[12];
  mds_coef(i, coef);
  x = pf::add_c(x, ps::RC_DEV[i]);
#pragma unroll 1
  for (int r = 0; r < 30; r++) {
    const bool full = r < 4 || r >= 26;
    const uint64_t y = pf::sbox(x);
    x = wave_mds_row(full || i == 0 ? y : x, coef);
    if (r < 29) x = pf::add_c(x, ps::RC_DEV[(r + 1) * 12 + i]);
  }
  return x;
}

// ---- row form: one permutation per 16-lane row (lane & 15 < 12 holds state
// element lane & 15), four per wave.  The MDS broadcasts come from DPP
// row_newbcast (a v_mov_b32_dpp per 32-bit half, full-rate VALU, no SGPR
// round trip), so the four rows' permutations share every instruction: the
// same ≈125-instruction chain per round as permute(), at a quarter of the
// waves per permutation.  A row is either wholly active or wholly inactive.

template <int J>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + J, 0xf, 0xf, false);  // row_newbcast:J
}

template <int J>
__device__ __forceinline__ void row_mds_terms(uint32_t lo, uint32_t hi, const uint32_t (&coef)[12], uint64_t (&al)[2],
                                              uint64_t (&ah)[2]) {
  al[J & 1] += (uint64_t)row_bcast<J>(lo) * coef[J];
  ah[J & 1] += (uint64_t)row_bcast<J>(hi) * coef[J];
  if constexpr (J < 11) row_mds_terms<J + 1>(lo, hi, coef, al, ah);
}

// MDS row of this lane over the 12 elements of its row
__device__ __forceinline__ uint64_t row_mds(uint64_t y, const uint32_t (&coef)[12]) {
  uint64_t al[2] = {0, 0}, ah[2] = {0, 0};
  row_mds_terms<0>((uint32_t)y, (uint32_t)(y >> 32), coef, al, ah);
  return pf::reduce_row(al[0] + al[1], ah[0] + ah[1]);
}

// the permutation of the state held in lanes 0..11 of this lane's row
__device__ __forceinline__ uint64_t permute_row(uint64_t x) {
  const uint32_t l16 = threadIdx.x & 15, i = l16 < 12 ? l16 : 0;
  uint32_t coef[12];
  mds_coef(i, coef);
  x = pf::add_c(x, ps::RC_DEV[i]);
#pragma unroll 1
  for (int r = 0; r < 30; r++) {
    const bool full = r < 4 || r >= 26;
    const uint64_t y = pf::sbox(x);
    x = row_mds(full || i == 0 ? y : x, coef);
    if (r < 29) x = pf::add_c(x, ps::RC_DEV[(r + 1) * 12 + i]);
  }
  return x;
}

}  // namespace pc
