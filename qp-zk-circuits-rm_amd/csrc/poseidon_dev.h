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

namespace psd {

constexpr uint64_t EPS = 0xFFFFFFFFull;

// a + b for a, b in [0, 2^64) with b < p (canonical): result in [0, 2^64).
// 32-bit carry chain (full-rate VALU) instead of 64-bit add + 64-bit compare.
__device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t b) {
  uint32_t c0, c1, c2, c3;
  uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
  // wrapped past 2^64: + eps (cannot wrap again: b < p)
  lo = __builtin_addc(lo, 0u - c1, 0u, &c2);
  hi = __builtin_addc(hi, 0u, c2, &c3);
  return ((uint64_t)hi << 32) | lo;
}

// reduce lo + 2^64 hi (any hi) to [0, 2^64) with 32-bit carry chains
__device__ __forceinline__ uint64_t reduce_nc(uint64_t lo, uint64_t hi) {
  const uint32_t hl = (uint32_t)hi, hh = (uint32_t)(hi >> 32);
  uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32), c, bo, bo2;
  // t = lo - hh ; on borrow t -= eps  (= t + 1 - 2^32)
  l0 = __builtin_subc(l0, hh, 0u, &bo);
  l1 = __builtin_subc(l1, 0u, bo, &bo2);
  l0 = __builtin_addc(l0, bo2, 0u, &c);
  l1 = l1 - bo2 + c;
  // + hl * eps = (hl << 32) - hl
  const uint32_t t0 = __builtin_subc(0u, hl, 0u, &bo);
  const uint32_t t1 = hl - bo;
  l0 = __builtin_addc(l0, t0, 0u, &c);
  l1 = __builtin_addc(l1, t1, c, &c);
  // carry out: + eps
  l0 = __builtin_addc(l0, 0u - c, 0u, &bo);
  l1 = l1 + bo;
  return ((uint64_t)l1 << 32) | l0;
}

__device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t m = (uint64_t)a1 * b0 + (p00 >> 32);
  const uint64_t m2 = (uint64_t)a0 * b1 + (uint32_t)m;
  const uint64_t h = (uint64_t)a1 * b1 + (m >> 32);
  uint32_t c;
  const uint32_t hl = __builtin_addc((uint32_t)h, (uint32_t)(m2 >> 32), 0u, &c);
  const uint32_t hh = (uint32_t)(h >> 32) + c;
  return reduce_nc(((uint64_t)(uint32_t)m2 << 32) | (uint32_t)p00, ((uint64_t)hh << 32) | hl);
}

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
    // value = al + ah*2^32 < 2^74: low word + carry, high word H < 2^10
    const uint64_t l = al + (ah << 32);
    const uint64_t H = (ah >> 32) + (l < al ? 1 : 0);
    const uint64_t t1 = (H << 32) - H;  // H * eps
    const uint64_t v = l + t1;
    s[r] = v + (v < t1 ? EPS : 0);
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

// permutation; inputs in [0,2^64), outputs in [0,2^64) (call canon on lanes read out)
__device__ __forceinline__ void permute_nc(uint64_t s[12]) {
#pragma unroll
  for (int r = 0; r < 4; r++) full_round(s, r);
#pragma unroll
  for (int r = 4; r < 26; r++) partial_round(s, r);
#pragma unroll
  for (int r = 26; r < 30; r++) full_round(s, r);
}

__device__ __forceinline__ void permute(uint64_t s[12]) {
  permute_nc(s);
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = canon(s[i]);
}

}  // namespace psd
