// poseidon_dev.h — throughput form of the Poseidon permutation for gfx950
// kernels (leaf hashing, Merkle levels, PoW).  Same function as ps::permute
// (poseidon.h), different arithmetic discipline:
//   * state kept NON-canonical in [0, 2^64) between rounds (one final
//     canonicalisation of the lanes the caller reads), as plonky2's own
//     Goldilocks backend does; field values are unchanged;
//   * rounds fully unrolled in three phases so round constants are scalar
//     operands and no loop/branch executes per round;
//   * MDS: 32-bit halves times the small circulant constants accumulate in
//     u64 (< 2^41), so each output lane needs one short reduction with a
//     high word < 2^10 instead of a full 128-bit reduction.
#pragma once
#include "field.h"
#include "poseidon.h"
#include "field_nc.h"
#include "poseidon_fast.h"

namespace psd {

constexpr uint64_t EPS = 0xFFFFFFFFull;

__device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t c) { return gfn::add_c(a, c); }
__device__ __forceinline__ uint64_t reduce_nc(uint64_t lo, uint64_t hi) { return gfn::reduce(lo, hi); }
__device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) { return gfn::mul(a, b); }

__device__ __forceinline__ uint64_t sbox_nc(uint64_t x) {
  const uint64_t x2 = mul_nc(x, x);
  const uint64_t x3 = mul_nc(x2, x);
  const uint64_t x4 = mul_nc(x2, x2);
  return mul_nc(x3, x4);
}

__device__ __forceinline__ uint64_t canon(uint64_t x) { return x >= gl::P ? x - gl::P : x; }

// MDS(s)[r] = sum_i s[(i+r)%12]*CIRC[i] + 8*s[0]*(r==0), on the 32-bit halves
__device__ __forceinline__ void mds_nc(uint64_t s[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = (uint32_t)s[i];
    hi[i] = (uint32_t)(s[i] >> 32);
  }
#pragma unroll
  for (int r = 0; r < 12; r++) {
    uint64_t al = 0, ah = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      al += (uint64_t)lo[(i + r) % 12] * ps::mds_circ(i);
      ah += (uint64_t)hi[(i + r) % 12] * ps::mds_circ(i);
    }
    if (r == 0) {
      al += (uint64_t)lo[0] * 8u;
      ah += (uint64_t)hi[0] * 8u;
    }
    // value = al + ah*2^32 < 2^74 = (l1:l0) + 2^64 H with H < 2^10;
    // + H*eps = + (H << 32) - H, in 32-bit carry chains
    uint32_t c, bo, c2;
    const uint32_t l0 = (uint32_t)al;
    const uint32_t l1 = __builtin_addc((uint32_t)(al >> 32), (uint32_t)ah, 0u, &c);
    const uint32_t H = (uint32_t)(ah >> 32) + c;
    const uint32_t r0 = __builtin_subc(l0, H, 0u, &bo);
    const uint32_t r1 = __builtin_addc(l1, H - bo, 0u, &c);  // H >= bo
    const uint32_t q0 = __builtin_addc(r0, 0u - c, 0u, &c2);  // wrapped: + eps
    s[r] = gfn::pack(q0, r1 + c2);
  }
}

__device__ __forceinline__ void full_round(uint64_t s[12], int rc) {
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = sbox_nc(add_nc(s[i], ps::RC_DEV[rc * 12 + i]));
  mds_nc(s);
}

__device__ __forceinline__ void partial_round(uint64_t s[12], int rc) {
#pragma unroll
  for (int i = 1; i < 12; i++) s[i] = add_nc(s[i], ps::RC_DEV[rc * 12 + i]);
  s[0] = sbox_nc(add_nc(s[0], ps::RC_DEV[rc * 12]));
  mds_nc(s);
}

// first-generation form (carry-chain arithmetic, separate round-constant
// additions); kept for tools/poseidon_ubench.hip comparisons only
__device__ __forceinline__ void permute_nc_v1(uint64_t s[12]) {
#pragma unroll
  for (int r = 0; r < 4; r++) full_round(s, r);
#pragma unroll
  for (int r = 4; r < 26; r++) partial_round(s, r);
#pragma unroll
  for (int r = 26; r < 30; r++) full_round(s, r);
}

// permutation used by the kernels: poseidon_fast.h (2.24 vs 1.67 Gperm/s for
// permute_nc_v1 on MI355X, tools/poseidon_ubench.hip).  Mode 3 (each MDS row
// one asm block: no compiler hazard s_nops between the mads): 2.35 Gperm/s in
// isolation, leaf hash -0.8 %, Merkle levels -6 %, e2e 932 -> 942 proofs/s
// (profiles/r02_ab_poseidon_mode3.log).  Inputs in [0,2^64), outputs in
// [0,2^64) (call canon on lanes read out)
#ifndef QP_POSEIDON_MODE
#define QP_POSEIDON_MODE 3
#endif
__device__ __forceinline__ void permute_nc(uint64_t s[12]) { pf::permute_nc<QP_POSEIDON_MODE>(s); }
// two_to_one form: s[8..11] == 0 on entry, only lanes 0..3 read
__device__ __forceinline__ void permute_nc_node(uint64_t s[12]) {
  if constexpr (QP_POSEIDON_MODE == 3) pf::permute_nc_capz<0xFu>(s);
  else pf::permute_nc<QP_POSEIDON_MODE>(s);
}

__device__ __forceinline__ void permute(uint64_t s[12]) {
  permute_nc(s);
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = canon(s[i]);
}

}  // namespace psd
