// field_nc.h — Goldilocks arithmetic for the throughput kernels, in the
// non-canonical representation [0, 2^64) (plonky2's own GoldilocksField
// representation; canonicalise with canon() before values leave a kernel).
//
// gfx950 runs 64-bit VALU ops (v_lshl_add_u64, v_cmp_*_u64, 64-bit shifts,
// v_mad_u64_u32) at a fraction of the 32-bit rate (PMC: SQ_INSTS_VALU_INT64),
// so everything except the four 32x32->64 partial products is written as
// 32-bit carry chains (v_add_co/v_addc/v_sub_co/v_subb).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "poseidon_fast.h"

namespace gfn {

constexpr uint64_t P = 0xFFFFFFFF00000001ull;

__device__ __forceinline__ uint64_t pack(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ uint64_t canon(uint64_t x) { return x >= P ? x - P : x; }

// a + b, any a, b in [0, 2^64)
__device__ __forceinline__ uint64_t add(uint64_t a, uint64_t b) {
  uint32_t c0, c1, c2, c3, c4;
  uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
  lo = __builtin_addc(lo, 0u - c1, 0u, &c2);  // wrapped: + eps
  hi = __builtin_addc(hi, 0u, c2, &c3);
  lo = __builtin_addc(lo, 0u - c3, 0u, &c4);  // wrapped again (both inputs > p): + eps
  hi += c4;
  return pack(lo, hi);
}

// a + b with b < p: the second wrap cannot happen
__device__ __forceinline__ uint64_t add_c(uint64_t a, uint64_t b) {
  uint32_t c0, c1, c2, c3;
  uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
  lo = __builtin_addc(lo, 0u - c1, 0u, &c2);
  hi = __builtin_addc(hi, 0u, c2, &c3);
  return pack(lo, hi);
}

// a - b, any a, b in [0, 2^64)
__device__ __forceinline__ uint64_t sub(uint64_t a, uint64_t b) {
  uint32_t b0, b1, b2, b3, b4;
  uint32_t lo = __builtin_subc((uint32_t)a, (uint32_t)b, 0u, &b0);
  uint32_t hi = __builtin_subc((uint32_t)(a >> 32), (uint32_t)(b >> 32), b0, &b1);
  lo = __builtin_subc(lo, 0u - b1, 0u, &b2);  // wrapped below 0: - eps
  hi = __builtin_subc(hi, 0u, b2, &b3);
  lo = __builtin_subc(lo, 0u - b3, 0u, &b4);  // wrapped again (b - a > p): - eps
  hi -= b4;
  return pack(lo, hi);
}

// lo + 2^64 hi -> [0, 2^64)
__device__ __forceinline__ uint64_t reduce(uint64_t lo, uint64_t hi) {
  const uint32_t hl = (uint32_t)hi, hh = (uint32_t)(hi >> 32);
  uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32), c, bo, bo2;
  l0 = __builtin_subc(l0, hh, 0u, &bo);  // lo - hh; borrow: - eps (= + 1 - 2^32)
  l1 = __builtin_subc(l1, 0u, bo, &bo2);
  l0 = __builtin_addc(l0, bo2, 0u, &c);
  l1 = l1 - bo2 + c;
  const uint32_t t0 = __builtin_subc(0u, hl, 0u, &bo);  // hl * eps = (hl << 32) - hl
  const uint32_t t1 = hl - bo;
  l0 = __builtin_addc(l0, t0, 0u, &c);
  l1 = __builtin_addc(l1, t1, c, &c);
  l0 = __builtin_addc(l0, 0u - c, 0u, &bo);  // carry out: + eps
  l1 = l1 + bo;
  return pack(l0, l1);
}

// product and sbox: the asm forms of poseidon_fast.h (5 mads + 8-op reduction)
__device__ __forceinline__ uint64_t mul(uint64_t a, uint64_t b) { return pf::mul(a, b); }

__device__ __forceinline__ uint64_t sbox(uint64_t x) { return pf::sbox(x); }

}  // namespace gfn
