// field.h — Goldilocks field and its quadratic extension for the MI355X
// prover (host + gfx950 device).  p = 2^64 - 2^32 + 1, canonical u64.
//
// Replaces qp-plonky2-field 1.1.1 GoldilocksField / QuadraticExtension
// (Cargo.lock:514-530).  There is no 64x64->128 multiplier on
// CDNA4: products are built from four 32x32->64 partial products
// (v_mad_u64_u32 / v_mul_hi_u32) and reduced with 2^64 = 2^32 - 1, 2^96 = -1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define QP_HD __host__ __device__ __forceinline__

namespace gl {

constexpr uint64_t P = 0xFFFFFFFF00000001ull;
constexpr uint64_t EPS = 0xFFFFFFFFull;  // 2^64 mod p
constexpr uint64_t GEN = 0xc65c18b67785d900ull;          // multiplicative generator / coset shift
constexpr uint64_t TWO_ADIC_GEN = 7277203076849721926ull;  // w_{2^32}
constexpr unsigned TWO_ADICITY = 32;
constexpr uint64_t EXT_W = 7;

QP_HD uint64_t canon(uint64_t x) { return x >= P ? x - P : x; }

QP_HD uint64_t add(uint64_t a, uint64_t b) {
  // a, b canonical: a + b < 2p < 2^65
  uint64_t s = a + b;
  uint64_t c = s < a;  // wrapped past 2^64: true value s + 2^64 = s + eps (mod p)
  s += c ? EPS : 0;
  return canon(s);
}

QP_HD uint64_t sub(uint64_t a, uint64_t b) {
  uint64_t d = a - b;
  return a >= b ? d : d + P;
}

QP_HD uint64_t neg(uint64_t a) { return a ? P - a : 0; }

// reduce lo + 2^64 hi (hi < 2^64)
QP_HD uint64_t reduce128(uint64_t lo, uint64_t hi) {
  uint64_t hh = hi >> 32, hl = hi & EPS;
  uint64_t t0 = lo - hh;
  if (lo < hh) t0 -= EPS;
  uint64_t t1 = (hl << 32) - hl;  // hl * eps
  uint64_t r = t0 + t1;
  if (r < t1) r += EPS;
  return canon(r);
}

QP_HD void mul_wide(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
  uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t p00 = (uint64_t)a0 * b0;
  uint64_t p01 = (uint64_t)a0 * b1;
  uint64_t p10 = (uint64_t)a1 * b0;
  uint64_t p11 = (uint64_t)a1 * b1;
  uint64_t mid = p01 + (p00 >> 32);           // < 2^64
  uint64_t mid2 = (uint32_t)mid + p10;        // < 2^64
  lo = (mid2 << 32) | (uint32_t)p00;
  hi = p11 + (mid >> 32) + (mid2 >> 32);
#else
  unsigned __int128 r = (unsigned __int128)a * b;
  lo = (uint64_t)r;
  hi = (uint64_t)(r >> 64);
#endif
}

QP_HD uint64_t mul(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  mul_wide(a, b, lo, hi);
  return reduce128(lo, hi);
}

QP_HD uint64_t sqr(uint64_t a) { return mul(a, a); }

QP_HD uint64_t pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mul(r, a);
    a = mul(a, a);
    e >>= 1;
  }
  return r;
}

QP_HD uint64_t inv(uint64_t a) { return pow(a, P - 2); }

QP_HD uint64_t root_of_unity(unsigned log_n) {
  uint64_t r = TWO_ADIC_GEN;
  for (unsigned i = log_n; i < TWO_ADICITY; i++) r = mul(r, r);
  return r;
}

// small-constant product accumulation: s * c for c < 2^16, used by the MDS layer.
// acc_lo/acc_hi collect s_lo*c and s_hi*c separately (each < 2^48 per term).
QP_HD void mac_small(uint64_t s, uint32_t c, uint64_t &acc_lo, uint64_t &acc_hi) {
  acc_lo += (uint64_t)(uint32_t)s * c;
  acc_hi += (uint64_t)(uint32_t)(s >> 32) * c;
}
QP_HD uint64_t reduce_split(uint64_t acc_lo, uint64_t acc_hi) {
  // value = acc_lo + acc_hi * 2^32, both < 2^56
  uint64_t lo = acc_lo + (acc_hi << 32);
  uint64_t hi = (acc_hi >> 32) + (lo < acc_lo);
  return reduce128(lo, hi);
}

// ---------------- quadratic extension F[X]/(X^2 - 7) ----------------
struct ext {
  uint64_t c0, c1;
};
QP_HD ext ext_make(uint64_t a, uint64_t b) { return ext{a, b}; }
QP_HD ext ext_add(ext a, ext b) { return ext{add(a.c0, b.c0), add(a.c1, b.c1)}; }
QP_HD ext ext_sub(ext a, ext b) { return ext{sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
QP_HD ext ext_mul(ext a, ext b) {
  uint64_t t = mul(a.c1, b.c1);
  return ext{add(mul(a.c0, b.c0), mul(EXT_W, t)), add(mul(a.c0, b.c1), mul(a.c1, b.c0))};
}
QP_HD ext ext_scale(ext a, uint64_t s) { return ext{mul(a.c0, s), mul(a.c1, s)}; }
QP_HD ext ext_inv(ext a) {
  uint64_t n = sub(sqr(a.c0), mul(EXT_W, sqr(a.c1)));
  uint64_t ni = inv(n);
  return ext{mul(a.c0, ni), mul(neg(a.c1), ni)};
}
QP_HD ext ext_pow(ext a, uint64_t e) {
  ext r{1, 0};
  while (e) {
    if (e & 1) r = ext_mul(r, a);
    a = ext_mul(a, a);
    e >>= 1;
  }
  return r;
}
QP_HD bool ext_eq(ext a, ext b) { return a.c0 == b.c0 && a.c1 == b.c1; }

QP_HD uint32_t rev_bits(uint32_t x, unsigned bits) {
#ifdef __HIP_DEVICE_COMPILE__
  return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
#else
  uint32_t r = 0;
  for (unsigned i = 0; i < bits; i++) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
#endif
}

}  // namespace gl
