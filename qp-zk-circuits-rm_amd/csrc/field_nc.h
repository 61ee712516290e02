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

// Lazily reduced sum of products (the quotient's alpha-weighted constraint
// sums): sum_i a_i b_i held as lo + 2^64 hi + 2^128 top, top counting the
// carries out of 2^128 (fewer than 2^32 terms), reduced once by value().  One
// product-accumulate is 4 mads + 1 cndmask + 3 addc, against a reduced
// product and a reduced add (13 + 6) per term.
struct Acc3 {
  uint64_t lo = 0, hi = 0;
  uint32_t top = 0;
  __device__ __forceinline__ void mac(uint64_t a, uint64_t b) {
    const uint32_t a0 = pf::lo32(a), a1 = pf::hi32(a), b0 = pf::lo32(b), b1 = pf::hi32(b);
    // L = a0 b0 + lo, carry-out cl worth 2^64; the rest of the product is then
    // the exact high part of a b + lo - cl 2^64 < 2^128, so W < 2^64
    uint64_t L, cl, U, cu, c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(L), "=s"(cl) : "v"(a0), "v"(b0), "v"(lo));
    const uint64_t T = (uint64_t)a0 * b1 + pf::hi32(L);
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(U), "=s"(cu) : "v"(a1), "v"(b0), "v"(T));
    uint32_t ce;
    asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(ce) : "s"(cu));
    const uint64_t W = (uint64_t)a1 * b1 + (((uint64_t)ce << 32) | pf::hi32(U));
    lo = ((uint64_t)pf::lo32(U) << 32) | pf::lo32(L);
    // hi += W + cl; top += the carry out
    uint32_t h0 = pf::lo32(hi), h1 = pf::hi32(hi);
    asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(h0), "=s"(c) : "v"(h0), "v"(pf::lo32(W)), "s"(cl));
    asm(QP_CWAIT "v_addc_co_u32_e64 %0, %1, %2, %3, %1" : "=v"(h1), "+s"(c) : "v"(h1), "v"(pf::hi32(W)));
    asm(QP_CWAIT "v_addc_co_u32_e64 %0, %1, %2, 0, %1" : "=v"(top), "+s"(c) : "v"(top));
    hi = ((uint64_t)h1 << 32) | h0;
  }
  // += x 2^e (0 <= e < 64) as the 128-bit integer it is: no reduction
  __device__ __forceinline__ void add_shifted(uint64_t x, uint32_t e) {
    const uint64_t xl = x << e, xh = e ? x >> (64 - e) : 0;
    uint32_t c0, c1, c2, c3, c4;
    const uint32_t l0 = __builtin_addc(pf::lo32(lo), pf::lo32(xl), 0u, &c0);
    const uint32_t l1 = __builtin_addc(pf::hi32(lo), pf::hi32(xl), c0, &c1);
    const uint32_t h0 = __builtin_addc(pf::lo32(hi), pf::lo32(xh), c1, &c2);
    const uint32_t h1 = __builtin_addc(pf::hi32(hi), pf::hi32(xh), c2, &c3);
    top = __builtin_addc(top, 0u, c3, &c4);
    lo = ((uint64_t)l1 << 32) | l0;
    hi = ((uint64_t)h1 << 32) | h0;
  }
  // 2^128 = 2^96 2^32 = -2^32 (mod p)
  __device__ __forceinline__ uint64_t value() const { return sub(reduce(lo, hi), (uint64_t)top << 32); }
};

}  // namespace gfn
