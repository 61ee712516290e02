// poseidon_fast.h — Poseidon (width 12, x^7, 8 full + 22 partial rounds)
// written to the measured gfx950 VALU cost model (tools/isa_rates.hip,
// profiles/r01_isa_rates.log): almost every VALU op issues at one per 4
// cycles per SIMD (add/sub/logic/mov at 2), so the permutation is bound by
// its VALU instruction count and v_mad_u64_u32 — a 32x32+64 product-sum in one
// issue — is the densest instruction there is.
//
// Hazard rule (gfx950): a VALU instruction reading a carry/mask SGPR written
// by the previous VALU instruction needs 2 wait states (hipcc puts s_nop 1
// between its own v_add_co/v_addc pairs).  Around inline asm hipcc adds only a
// fixed 1-state pad, so every asm statement below that reads a carry written
// by the preceding one opens with its own s_nop 0.
// (Dropping it measured no faster, profiles/r02_ab_carry_wait.log.)
#define QP_CWAIT "s_nop 0\n\t"
//
// Same function as ps::permute (poseidon.h); arithmetic discipline:
//   * state NON-canonical in [0, 2^64) (plonky2's GoldilocksField form);
//   * MDS row r = sum_i CIRC[i] * s[(i+r)%12] (+ DIAG) computed on 32-bit
//     halves as 24 explicit v_mad_u64_u32 with the small constants inline
//     (the compiler would otherwise strength-reduce them into longer
//     shift/add carry chains);
//   * the NEXT round's constant is folded into the first mad of each row
//     (addend = the constant's halves), so no round-constant additions are
//     executed except the first round's;
//   * each row reduces in 4 instructions: value = al + 2^32 ah with
//     al, ah < 2^41 -> t = al + eps*hi32(ah) (one mad), t.hi += lo32(ah) with
//     carry c, t += c*eps.
//   * sbox x^7 = x^3 * x^4 with a 5-mad product and an 8-instruction
//     Goldilocks reduction whose carries come straight from the mad/sub
//     carry-outs.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "poseidon.h"
#include "poseidon_mds_asm.h"
#include "poseidon_partial_consts.h"

namespace pf {

constexpr uint64_t EPS = 0xFFFFFFFFull;
constexpr uint64_t P = 0xFFFFFFFF00000001ull;

__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }

// C as a value the compiler cannot see through (an SGPR; no instruction is
// emitted for the empty asm), so x * C stays one v_mad_u64_u32
template <int C>
__device__ __forceinline__ uint32_t opaque() {
  uint32_t c;
  asm("" : "=s"(c) : "0"((uint32_t)C));
  return c;
}

// acc = x * C + add   (C an inline constant in [0, 64])
template <int C>
__device__ __forceinline__ uint64_t mad_c(uint32_t x, uint64_t add) {
  uint64_t r, cdummy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cdummy) : "v"(x), "i"(C), "v"(add));
  return r;
}
// acc = x * C + add, add a scalar (SGPR) 64-bit value
template <int C>
__device__ __forceinline__ uint64_t mad_cs(uint32_t x, uint64_t add) {
  uint64_t r, cdummy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cdummy) : "v"(x), "i"(C), "s"(add));
  return r;
}

// value = al + 2^32 ah (al, ah < 2^42)  ->  [0, 2^64), same residue
__device__ __forceinline__ uint64_t reduce_row(uint64_t al, uint64_t ah) {
  uint64_t t, c1, c2;
  uint32_t e;
  // t = al + eps * hi32(ah)   (< 2^43, no overflow)
  asm("v_mad_u64_u32 %0, %1, %2, -1, %3" : "=v"(t), "=s"(c1) : "v"(hi32(ah)), "v"(al));
  // t.hi += lo32(ah), carry c2 (worth 2^64 = eps)
  uint32_t t0 = lo32(t), t1 = hi32(t);
  asm("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(t1), "=s"(c2) : "v"(t1), "v"(lo32(ah)));
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(c2));
  // t + e: when c2, t < 2^42 so no overflow
  const uint64_t tt = ((uint64_t)t1 << 32) | t0;
  uint64_t r;
  asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(c1) : "v"(e), "v"(tt));
  return r;
}

// a * b mod p, a, b in [0, 2^64), result in [0, 2^64)
__device__ __forceinline__ uint64_t mul(uint64_t a, uint64_t b) {
  const uint32_t a0 = lo32(a), a1 = hi32(a), b0 = lo32(b), b1 = hi32(b);
  // middle column as one 65-bit sum: T = a0 b1 + L.hi, U = a1 b0 + T with its
  // carry-out c (worth 2^96), W = a1 b1 + (U.hi | c << 32): one zero-extension
  // and no separate 64-bit add (the textbook four-product form, mul_c below,
  // needs three and a v_lshl_add_u64; profiles/r02_ab_mul_form_dot_halves.log)
  const uint64_t L = (uint64_t)a0 * b0;
  const uint64_t T = (uint64_t)a0 * b1 + hi32(L);
  uint64_t U, cu;
  uint32_t ce;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(U), "=s"(cu) : "v"(a1), "v"(b0), "v"(T));
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(ce) : "s"(cu));
  const uint64_t W = (uint64_t)a1 * b1 + (((uint64_t)ce << 32) | hi32(U));  // < 2^64 (high half)
  const uint64_t X = ((uint64_t)lo32(U) << 32) | lo32(L);
  // 128-bit product = X + 2^64 W, X = (L0, U0);  ≡ X + eps*w2 - w3
  uint64_t t, c1, c2, c3;
  uint32_t e;
  asm("v_mad_u64_u32 %0, %1, %2, -1, %3" : "=v"(t), "=s"(c1) : "v"(lo32(W)), "v"(X));
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(c1));
  // carry: true value t + 2^64 ≡ t + eps; t < 2^64 - 2^33 then, no overflow
  asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(t), "=s"(c2) : "v"(e), "v"(t));
  // t - w3, borrow b (worth -2^64 ≡ -eps)
  uint32_t r0 = lo32(t), r1 = hi32(t);
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c3) : "v"(r0), "v"(hi32(W)));
  asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r1), "=s"(c3) : "v"(r1), "s"(c3));
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(c3));
  // borrow: t - w3 + 2^64 >= 2^64 - 2^32, minus eps stays >= 0
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c3) : "v"(r0), "v"(e));
  asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r1), "=s"(c3) : "v"(r1), "s"(c3));
  return ((uint64_t)r1 << 32) | r0;
}

// C forms of the same (compiler-chosen carries)
__device__ __forceinline__ uint64_t reduce_row_c(uint64_t al, uint64_t ah) {
  const uint64_t t = al + (ah >> 32) * EPS;
  const uint32_t t1 = hi32(t) + lo32(ah);
  const uint64_t r = ((uint64_t)t1 << 32) | lo32(t);
  return t1 < lo32(ah) ? r + EPS : r;
}
__device__ __forceinline__ uint64_t mul_c(uint64_t a, uint64_t b) {
  const uint32_t a0 = lo32(a), a1 = hi32(a), b0 = lo32(b), b1 = hi32(b);
  const uint64_t L = (uint64_t)a0 * b0;
  const uint64_t T = (uint64_t)a0 * b1 + hi32(L);
  const uint64_t U = (uint64_t)a1 * b0 + lo32(T);
  const uint64_t V = (uint64_t)a1 * b1 + hi32(T);
  const uint64_t W = V + hi32(U);
  const uint64_t X = ((uint64_t)lo32(U) << 32) | lo32(L);
  uint64_t t = X + (uint64_t)lo32(W) * EPS;
  t = t < X ? t + EPS : t;
  const uint64_t w3 = hi32(W);
  const uint64_t r = t - w3;
  return t < w3 ? r - EPS : r;
}
__device__ __forceinline__ uint64_t sbox_c(uint64_t x) {
  const uint64_t x2 = mul_c(x, x);
  const uint64_t x3 = mul_c(x2, x);
  const uint64_t x4 = mul_c(x2, x2);
  return mul_c(x3, x4);
}

// ---- K independent products with their carry steps interleaved (K = 2, 3):
// each asm statement below issues one step of every product, so a carry SGPR
// written by product i's instruction is read K - 1 instructions (plus the
// compiler's one-state pad after an asm statement) later — the gfx950 carry
// hazard's two wait states are met by the other products' work instead of
// s_nop (one product alone needs ~14 pad states).  Same arithmetic as mul():
// U = a1 b0 + T with carry, W = a1 b1 + (U.hi | c << 32), X = (U.lo, L.lo),
// then the 8-step reduction.  The NTT passes use it (nt::mul_rows); in the
// Poseidon S-boxes it measured slower (leaf hash +4 %, e2e -2 %,
// profiles/r02_ab_mulk.log): at 7 waves/SIMD the pads it removes (8.0k -> 2.9k
// s_nop per permutation) were nearly free and it adds ~500 register-pair
// moves, so the S-boxes keep one product at a time.
#define QP_W2 QP_CWAIT  // K = 2: one explicit wait state before each carry read
template <int K>
__device__ __forceinline__ void mulk(const uint64_t *a, const uint64_t *b, uint64_t *r) {
  static_assert(K == 2 || K == 3, "K");
  uint64_t T[K], U[K], W[K], X[K], t[K], cs[K];
  uint32_t ce[K], e[K], r0[K], r1[K];
#pragma unroll
  for (int i = 0; i < K; i++) {
    const uint64_t L = (uint64_t)lo32(a[i]) * lo32(b[i]);
    T[i] = (uint64_t)lo32(a[i]) * hi32(b[i]) + hi32(L);
    X[i] = lo32(L);
  }
  if constexpr (K == 3) {
    asm("v_mad_u64_u32 %0, %3, %6, %9, %12\n\t"
        "v_mad_u64_u32 %1, %4, %7, %10, %13\n\t"
        "v_mad_u64_u32 %2, %5, %8, %11, %14"
        : "=&v"(U[0]), "=&v"(U[1]), "=&v"(U[2]), "=&s"(cs[0]), "=&s"(cs[1]), "=&s"(cs[2])
        : "v"(hi32(a[0])), "v"(hi32(a[1])), "v"(hi32(a[2])), "v"(lo32(b[0])), "v"(lo32(b[1])), "v"(lo32(b[2])),
          "v"(T[0]), "v"(T[1]), "v"(T[2]));
    asm("v_cndmask_b32_e64 %0, 0, 1, %3\n\t"
        "v_cndmask_b32_e64 %1, 0, 1, %4\n\t"
        "v_cndmask_b32_e64 %2, 0, 1, %5"
        : "=v"(ce[0]), "=v"(ce[1]), "=v"(ce[2]) : "s"(cs[0]), "s"(cs[1]), "s"(cs[2]));
  } else {
    asm("v_mad_u64_u32 %0, %2, %4, %6, %8\n\t"
        "v_mad_u64_u32 %1, %3, %5, %7, %9"
        : "=&v"(U[0]), "=&v"(U[1]), "=&s"(cs[0]), "=&s"(cs[1])
        : "v"(hi32(a[0])), "v"(hi32(a[1])), "v"(lo32(b[0])), "v"(lo32(b[1])), "v"(T[0]), "v"(T[1]));
    asm(QP_W2 "v_cndmask_b32_e64 %0, 0, 1, %2\n\t"
        "v_cndmask_b32_e64 %1, 0, 1, %3"
        : "=v"(ce[0]), "=v"(ce[1]) : "s"(cs[0]), "s"(cs[1]));
  }
#pragma unroll
  for (int i = 0; i < K; i++) {
    W[i] = (uint64_t)hi32(a[i]) * hi32(b[i]) + (((uint64_t)ce[i] << 32) | hi32(U[i]));
    X[i] |= (uint64_t)lo32(U[i]) << 32;
  }
  if constexpr (K == 3) {
    // t = X + eps w2 (carry c1); e = c1 ? eps : 0; t += e
    asm("v_mad_u64_u32 %0, %3, %6, -1, %9\n\t"
        "v_mad_u64_u32 %1, %4, %7, -1, %10\n\t"
        "v_mad_u64_u32 %2, %5, %8, -1, %11"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&s"(cs[0]), "=&s"(cs[1]), "=&s"(cs[2])
        : "v"(lo32(W[0])), "v"(lo32(W[1])), "v"(lo32(W[2])), "v"(X[0]), "v"(X[1]), "v"(X[2]));
    asm("v_cndmask_b32_e64 %0, 0, -1, %3\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, %4\n\t"
        "v_cndmask_b32_e64 %2, 0, -1, %5"
        : "=v"(e[0]), "=v"(e[1]), "=v"(e[2]) : "s"(cs[0]), "s"(cs[1]), "s"(cs[2]));
    asm("v_mad_u64_u32 %0, vcc, %3, 1, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %4, 1, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %5, 1, %2"
        : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]) : "v"(e[0]), "v"(e[1]), "v"(e[2]) : "vcc");
    // r = t - w3 (borrow b); e = b ? eps : 0; r -= e
    asm("v_sub_co_u32_e64 %0, %3, %6, %9\n\t"
        "v_sub_co_u32_e64 %1, %4, %7, %10\n\t"
        "v_sub_co_u32_e64 %2, %5, %8, %11"
        : "=&v"(r0[0]), "=&v"(r0[1]), "=&v"(r0[2]), "=&s"(cs[0]), "=&s"(cs[1]), "=&s"(cs[2])
        : "v"(lo32(t[0])), "v"(lo32(t[1])), "v"(lo32(t[2])), "v"(hi32(W[0])), "v"(hi32(W[1])), "v"(hi32(W[2])));
    asm("v_subb_co_u32_e64 %0, %3, %6, 0, %3\n\t"
        "v_subb_co_u32_e64 %1, %4, %7, 0, %4\n\t"
        "v_subb_co_u32_e64 %2, %5, %8, 0, %5"
        : "=&v"(r1[0]), "=&v"(r1[1]), "=&v"(r1[2]), "+s"(cs[0]), "+s"(cs[1]), "+s"(cs[2])
        : "v"(hi32(t[0])), "v"(hi32(t[1])), "v"(hi32(t[2])));
    asm("v_cndmask_b32_e64 %0, 0, -1, %3\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, %4\n\t"
        "v_cndmask_b32_e64 %2, 0, -1, %5"
        : "=v"(e[0]), "=v"(e[1]), "=v"(e[2]) : "s"(cs[0]), "s"(cs[1]), "s"(cs[2]));
    asm("v_sub_co_u32_e64 %0, %3, %0, %6\n\t"
        "v_sub_co_u32_e64 %1, %4, %1, %7\n\t"
        "v_sub_co_u32_e64 %2, %5, %2, %8"
        : "+v"(r0[0]), "+v"(r0[1]), "+v"(r0[2]), "=&s"(cs[0]), "=&s"(cs[1]), "=&s"(cs[2])
        : "v"(e[0]), "v"(e[1]), "v"(e[2]));
    asm("v_subb_co_u32_e64 %0, vcc, %0, 0, %3\n\t"
        "v_subb_co_u32_e64 %1, vcc, %1, 0, %4\n\t"
        "v_subb_co_u32_e64 %2, vcc, %2, 0, %5"
        : "+v"(r1[0]), "+v"(r1[1]), "+v"(r1[2]) : "s"(cs[0]), "s"(cs[1]), "s"(cs[2]) : "vcc");
  } else {
    asm("v_mad_u64_u32 %0, %2, %4, -1, %6\n\t"
        "v_mad_u64_u32 %1, %3, %5, -1, %7"
        : "=&v"(t[0]), "=&v"(t[1]), "=&s"(cs[0]), "=&s"(cs[1])
        : "v"(lo32(W[0])), "v"(lo32(W[1])), "v"(X[0]), "v"(X[1]));
    asm(QP_W2 "v_cndmask_b32_e64 %0, 0, -1, %2\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, %3"
        : "=v"(e[0]), "=v"(e[1]) : "s"(cs[0]), "s"(cs[1]));
    asm("v_mad_u64_u32 %0, vcc, %2, 1, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %3, 1, %1"
        : "+v"(t[0]), "+v"(t[1]) : "v"(e[0]), "v"(e[1]) : "vcc");
    asm("v_sub_co_u32_e64 %0, %2, %4, %6\n\t"
        "v_sub_co_u32_e64 %1, %3, %5, %7"
        : "=&v"(r0[0]), "=&v"(r0[1]), "=&s"(cs[0]), "=&s"(cs[1])
        : "v"(lo32(t[0])), "v"(lo32(t[1])), "v"(hi32(W[0])), "v"(hi32(W[1])));
    asm(QP_W2 "v_subb_co_u32_e64 %0, %2, %4, 0, %2\n\t"
        "v_subb_co_u32_e64 %1, %3, %5, 0, %3"
        : "=&v"(r1[0]), "=&v"(r1[1]), "+s"(cs[0]), "+s"(cs[1])
        : "v"(hi32(t[0])), "v"(hi32(t[1])));
    asm(QP_W2 "v_cndmask_b32_e64 %0, 0, -1, %2\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, %3"
        : "=v"(e[0]), "=v"(e[1]) : "s"(cs[0]), "s"(cs[1]));
    asm("v_sub_co_u32_e64 %0, %2, %0, %4\n\t"
        "v_sub_co_u32_e64 %1, %3, %1, %5"
        : "+v"(r0[0]), "+v"(r0[1]), "=&s"(cs[0]), "=&s"(cs[1])
        : "v"(e[0]), "v"(e[1]));
    asm(QP_W2 "v_subb_co_u32_e64 %0, vcc, %0, 0, %2\n\t"
        "v_subb_co_u32_e64 %1, vcc, %1, 0, %3"
        : "+v"(r1[0]), "+v"(r1[1]) : "s"(cs[0]), "s"(cs[1]) : "vcc");
  }
#pragma unroll
  for (int i = 0; i < K; i++) r[i] = ((uint64_t)r1[i] << 32) | r0[i];
}

__device__ __forceinline__ uint64_t sbox(uint64_t x) {
  const uint64_t x2 = mul(x, x);
  const uint64_t x3 = mul(x2, x);
  const uint64_t x4 = mul(x2, x2);
  return mul(x3, x4);
}

// the 12 S-boxes of a full round
__device__ __forceinline__ void sbox12(uint64_t s[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = sbox(s[i]);
}

// a + c, a in [0, 2^64), c < p
__device__ __forceinline__ uint64_t add_c(uint64_t a, uint64_t c) {
  const uint64_t s = a + c;
  return s + (s < c ? EPS : 0);
}

__device__ __forceinline__ uint64_t canon(uint64_t x) { return x >= P ? x - P : x; }

// MDS row R with the next round's constant k folded in (k < p, as SGPR halves)
template <int M, int R, int I>
__device__ __forceinline__ void row_terms(uint64_t &al, uint64_t &ah, const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (I < 12) {
    constexpr int C = (int)ps::mds_circ(I) + ((R == 0 && I == 0) ? 8 : 0);
    if constexpr (M == 0) {
      al = mad_c<C>(lo[(I + R) % 12], al);
      ah = mad_c<C>(hi[(I + R) % 12], ah);
    } else {
      const uint32_t c = opaque<C>();
      al += (uint64_t)lo[(I + R) % 12] * c;
      ah += (uint64_t)hi[(I + R) % 12] * c;
    }
    row_terms<M, R, I + 1>(al, ah, lo, hi);
  }
}

// runtime-constant variant: s <- MDS(s) + k (k[12] wave-uniform, < p)
template <int R>
__device__ __forceinline__ void mds_rows_k(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12],
                                           const uint64_t k[12]) {
  if constexpr (R < 12) {
    constexpr int C0 = (int)ps::mds_circ(0) + (R == 0 ? 8 : 0);
    uint64_t al = mad_cs<C0>(lo[R], k[R] & EPS);
    uint64_t ah = mad_cs<C0>(hi[R], k[R] >> 32);
    row_terms<0, R, 1>(al, ah, lo, hi);
    s[R] = reduce_row(al, ah);
    mds_rows_k<R + 1>(s, lo, hi, k);
  }
}

__device__ __forceinline__ void mds_k(uint64_t s[12], const uint64_t k[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = lo32(s[i]);
    hi[i] = hi32(s[i]);
  }
  mds_rows_k<0>(s, lo, hi, k);
}

template <int M, int R, int RC>
__device__ __forceinline__ void mds_rows(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (R < 12) {
    constexpr int C0 = (int)ps::mds_circ(0) + (R == 0 ? 8 : 0);
    uint64_t al, ah;
    constexpr uint64_t k = RC >= 0 ? ps::rc_cx(RC * 12 + R) : 0;
    if constexpr (M == 0) {
      // constant of the next round folded into the accumulators' start
      if constexpr (RC >= 0) {
        al = mad_cs<C0>(lo[R], k & EPS);
        ah = mad_cs<C0>(hi[R], k >> 32);
      } else {
        al = mad_c<C0>(lo[R], 0);
        ah = mad_c<C0>(hi[R], 0);
      }
    } else {
      const uint32_t c = opaque<C0>();
      al = (uint64_t)lo[R] * c + (k & EPS);
      ah = (uint64_t)hi[R] * c + (k >> 32);
    }
    row_terms<M, R, 1>(al, ah, lo, hi);
    s[R] = M == 2 ? reduce_row_c(al, ah) : reduce_row(al, ah);
    mds_rows<M, R + 1, RC>(s, lo, hi);
  }
}

// One MDS row as a single asm block: 24 v_mad_u64_u32 on the rotated halves
// (x[i] = half[(i+R)%12]) with the circulant constants inline, starting from
// the folded round-constant halves kl/kh.  Inside one asm statement the
// compiler's conservative inline-asm hazard padding (an s_nop after every
// SGPR-writing asm VALU op) disappears; the mads only write the dead carry
// SGPR pair and read none, so no wait state is needed between them.
#define QP_MDS_ROW_ASM(C0)                                                                                  \
  asm("v_mad_u64_u32 %0, %2, %3, " #C0 ", %27\n\t"                                                     \
      "v_mad_u64_u32 %1, %2, %15, " #C0 ", %28\n\t"                                                    \
      "v_mad_u64_u32 %0, %2, %4, 15, %0\n\t"                                                           \
      "v_mad_u64_u32 %1, %2, %16, 15, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %5, 41, %0\n\t"                                                           \
      "v_mad_u64_u32 %1, %2, %17, 41, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %6, 16, %0\n\t"                                                           \
      "v_mad_u64_u32 %1, %2, %18, 16, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %7, 2, %0\n\t"                                                            \
      "v_mad_u64_u32 %1, %2, %19, 2, %1\n\t"                                                           \
      "v_mad_u64_u32 %0, %2, %8, 28, %0\n\t"                                                           \
      "v_mad_u64_u32 %1, %2, %20, 28, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %9, 13, %0\n\t"                                                           \
      "v_mad_u64_u32 %1, %2, %21, 13, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %10, 13, %0\n\t"                                                          \
      "v_mad_u64_u32 %1, %2, %22, 13, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %11, 39, %0\n\t"                                                          \
      "v_mad_u64_u32 %1, %2, %23, 39, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %12, 18, %0\n\t"                                                          \
      "v_mad_u64_u32 %1, %2, %24, 18, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %13, 34, %0\n\t"                                                          \
      "v_mad_u64_u32 %1, %2, %25, 34, %1\n\t"                                                          \
      "v_mad_u64_u32 %0, %2, %14, 20, %0\n\t"                                                          \
      "v_mad_u64_u32 %1, %2, %26, 20, %1"                                                                \
      : "=&v"(al), "=&v"(ah), "=&s"(cd)                                                                  \
      : "v"(lo[(0 + R) % 12]), "v"(lo[(1 + R) % 12]), "v"(lo[(2 + R) % 12]), "v"(lo[(3 + R) % 12]),     \
        "v"(lo[(4 + R) % 12]), "v"(lo[(5 + R) % 12]), "v"(lo[(6 + R) % 12]), "v"(lo[(7 + R) % 12]),     \
        "v"(lo[(8 + R) % 12]), "v"(lo[(9 + R) % 12]), "v"(lo[(10 + R) % 12]), "v"(lo[(11 + R) % 12]),   \
        "v"(hi[(0 + R) % 12]), "v"(hi[(1 + R) % 12]), "v"(hi[(2 + R) % 12]), "v"(hi[(3 + R) % 12]),     \
        "v"(hi[(4 + R) % 12]), "v"(hi[(5 + R) % 12]), "v"(hi[(6 + R) % 12]), "v"(hi[(7 + R) % 12]),     \
        "v"(hi[(8 + R) % 12]), "v"(hi[(9 + R) % 12]), "v"(hi[(10 + R) % 12]), "v"(hi[(11 + R) % 12]),   \
        "s"(kl), "s"(kh))

template <int R>
__device__ __forceinline__ void mds_row_block(uint64_t &al, uint64_t &ah, const uint32_t lo[12],
                                              const uint32_t hi[12], uint64_t kl, uint64_t kh) {
  static_assert(ps::mds_circ(0) == 17 && ps::mds_circ(1) == 15 && ps::mds_circ(11) == 20, "MDS constants");
  uint64_t cd;
  if constexpr (R == 0) {
    QP_MDS_ROW_ASM(25);  // circulant 17 + diagonal 8
  } else {
    QP_MDS_ROW_ASM(17);
  }
  (void)cd;
}

template <int R, int RC, uint32_t OUT = 0xFFFu>
__device__ __forceinline__ void mds_rows_block(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (R < 12) {
    if constexpr ((OUT >> R) & 1) {  // rows nobody reads (OUT) are skipped
      constexpr uint64_t k = RC >= 0 ? ps::rc_cx(RC * 12 + R) : 0;
      uint64_t al, ah;
      mds_row_block<R>(al, ah, lo, hi, k & EPS, k >> 32);
      s[R] = reduce_row(al, ah);
    }
    mds_rows_block<R + 1, RC, OUT>(s, lo, hi);
  }
}

// modes 6-9: blocks of NR = 2, 3, 4, 6 rows, their 2*NR accumulate chains
// interleaved in one asm block (poseidon_mds_asm.h) so a wave keeps 2*NR
// independent v_mad_u64_u32 chains in flight instead of 2
template <int M>
constexpr int mds_block_rows() { return M == 6 ? 2 : M == 7 ? 3 : M == 8 ? 4 : 6; }

template <int NR, int R>
__device__ __forceinline__ void mds_asm_rows(uint64_t acc[2 * NR], const uint32_t lo[12], const uint32_t hi[12],
                                             const uint64_t k[2 * NR]) {
  if constexpr (NR == 2) mds_asm_rows2<R>(acc, lo, hi, k);
  else if constexpr (NR == 3) mds_asm_rows3<R>(acc, lo, hi, k);
  else if constexpr (NR == 4) mds_asm_rows4<R>(acc, lo, hi, k);
  else mds_asm_rows6<R>(acc, lo, hi, k);
}

template <int NR, int R, int RC>
__device__ __forceinline__ void mds_rows_multi(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (R < 12) {
    uint64_t k[2 * NR], acc[2 * NR];
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const uint64_t kk = RC >= 0 ? ps::rc_cx(RC * 12 + R + r) : 0;
      k[2 * r] = kk & EPS;
      k[2 * r + 1] = kk >> 32;
    }
    mds_asm_rows<NR, R>(acc, lo, hi, k);
#pragma unroll
    for (int r = 0; r < NR; r++) s[R + r] = reduce_row(acc[2 * r], acc[2 * r + 1]);
    mds_rows_multi<NR, R + NR, RC>(s, lo, hi);
  }
}

// s <- MDS(s) + RC[next] (next < 0: no constant); OUT: the output rows needed
template <int M, int NEXT, uint32_t OUT = 0xFFFu>
__device__ __forceinline__ void mds(uint64_t s[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = lo32(s[i]);
    hi[i] = hi32(s[i]);
  }
  if constexpr (M >= 6) mds_rows_multi<mds_block_rows<M>(), 0, NEXT>(s, lo, hi);
  else if constexpr (M >= 3) mds_rows_block<0, NEXT, OUT>(s, lo, hi);
  else mds_rows<M, 0, NEXT>(s, lo, hi);
}

// block-asm MDS with the next round's constants read at run time (uniform
// index: scalar loads into SGPRs) — the body of the rolled partial-round loop
template <int R>
__device__ __forceinline__ void mds_rows_block_dyn(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12],
                                                   const uint64_t *__restrict__ k) {
  if constexpr (R < 12) {
    const uint64_t kr = k[R];
    uint64_t al, ah;
    mds_row_block<R>(al, ah, lo, hi, kr & EPS, kr >> 32);
    s[R] = reduce_row(al, ah);
    mds_rows_block_dyn<R + 1>(s, lo, hi, k);
  }
}

// one full round (12 S-boxes + MDS folding the next round's constants, read at
// run time) — the body of the rolled full-round loops of mode 5
__device__ __forceinline__ void full_round_dyn(uint64_t s[12], const uint64_t *__restrict__ knext) {
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = sbox(s[i]);
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = lo32(s[i]);
    hi[i] = hi32(s[i]);
  }
  mds_rows_block_dyn<0>(s, lo, hi, knext);
}

// ---- sparse partial rounds (tools/gen_poseidon_partial.py): round 3's MDS
// merged with D_4 (rows 1..11 dense), then per partial round one S-box, one
// dot product for lane 0 and 11 scalar multiply-adds.  Dense constants act on
// 22-bit limbs (x = l0 + 2^22 l1 + 2^44 l2) through precomputed c 2^(22k) mod
// p halves, so every accumulator stays < 2^60 and reduces in 4 instructions.
// Same permutation as the plain rounds (modes 3 and 10 take this form).

__device__ __forceinline__ void limbs22(uint64_t x, uint32_t l[3]) {
  const uint32_t lo = lo32(x), hi = hi32(x);
  l[0] = lo & 0x3FFFFFu;
  l[1] = __builtin_amdgcn_alignbit(hi, lo, 22) & 0x3FFFFFu;
  l[2] = hi >> 12;
}

// the generated tables as compile-time values (every product below has a
// literal constant operand; zero halves emit nothing)
enum { PT_INIT, PT_AHAT, PT_BV, PT_S0C, PT_GAM };
template <int TB, int OFF>
__device__ __forceinline__ constexpr uint32_t ptab() {
  return TB == PT_INIT ? pfp::INIT[OFF] : TB == PT_AHAT ? pfp::AHAT[OFF] : TB == PT_BV ? pfp::BV[OFF]
       : TB == PT_GAM ? pfp::GAM[OFF] : pfp::S0C[OFF];
}

// al/ah += sum_k l[k] * (halves of the constant at table TB, words OFF..OFF+5)
template <int TB, int OFF, int K = 0>
__device__ __forceinline__ void mac_limbs(uint64_t &al, uint64_t &ah, const uint32_t l[3]) {
  if constexpr (K < 3) {
    constexpr uint32_t cl = ptab<TB, OFF + 2 * K>(), ch = ptab<TB, OFF + 2 * K + 1>();
    // explicit mads with the (dead) carry-out sunk into VCC: as C the compiler
    // hands the carry the SGPR pair holding the constant, and the next
    // constant's s_mov into it then costs a hazard s_nop per product
    if constexpr (cl != 0) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(al) : "v"(l[K]), "s"(cl) : "vcc");
    if constexpr (ch != 0) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(ah) : "v"(l[K]), "s"(ch) : "vcc");
    mac_limbs<TB, OFF, K + 1>(al, ah, l);
  }
}

// row I (1..11) of D_4 M over the limbs of all 12 lanes
template <int I, int J = 0>
__device__ __forceinline__ void init_row(uint64_t &al, uint64_t &ah, const uint32_t L[12][3]) {
  if constexpr (J < 12) {
    mac_limbs<PT_INIT, ((I - 1) * 12 + J) * 6>(al, ah, L[J]);
    init_row<I, J + 1>(al, ah, L);
  }
}
template <int I = 1>
__device__ __forceinline__ void init_rows(uint64_t out[12], const uint32_t L[12][3]) {
  if constexpr (I < 12) {
    uint64_t al = pfp::INIT_K[2 * I], ah = pfp::INIT_K[2 * I + 1];
    init_row<I>(al, ah, L);
    out[I] = reduce_row(al, ah);
    init_rows<I + 1>(out, L);
  }
}

// s <- D_4 M s + D_4 c_4  (s = the S-box outputs of round 3)
__device__ __forceinline__ void mds_init_sparse(uint64_t s[12]) {
  uint32_t lo[12], hi[12], L[12][3];
#pragma unroll
  for (int j = 0; j < 12; j++) {
    lo[j] = lo32(s[j]);
    hi[j] = hi32(s[j]);
    limbs22(s[j], L[j]);
  }
  uint64_t out[12];
  {
    uint64_t al, ah;
    mds_row_block<0>(al, ah, lo, hi, pfp::INIT_K[0], pfp::INIT_K[1]);
    out[0] = reduce_row(al, ah);
  }
  init_rows(out, L);
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = out[i];
}

template <int T, int I = 1>
__device__ __forceinline__ void sparse_col0(uint64_t s[12], const uint32_t l0[3]) {
  if constexpr (I < 12) {
    uint64_t bl = (uint64_t)lo32(s[I]) + (T == 21 ? pfp::KLAST[2 * I] : 0u);
    uint64_t bh = (uint64_t)hi32(s[I]) + (T == 21 ? pfp::KLAST[2 * I + 1] : 0u);
    mac_limbs<PT_BV, (T * 11 + I - 1) * 6>(bl, bh, l0);
    s[I] = reduce_row(bl, bh);
    sparse_col0<T, I + 1>(s, l0);
  }
}

// lane-0 dot product on the 32-bit halves of lanes 1..11 (AH2 pieces of
// weights 1, 2^22, 2^44; each accumulator < 2^59)
template <int T, int J = 1, int H = 0, int K = 0>
__device__ __forceinline__ void sparse_row0_h(uint64_t S[3], const uint64_t s[12]) {
  if constexpr (J < 12) {
    constexpr uint32_t c = pfp::AH2[((T * 11 + J - 1) * 2 + H) * 3 + K];
    const uint32_t v = H ? hi32(s[J]) : lo32(s[J]);
    if constexpr (c != 0) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(S[K]) : "v"(v), "s"(c) : "vcc");
    if constexpr (K < 2) sparse_row0_h<T, J, H, K + 1>(S, s);
    else if constexpr (H == 0) sparse_row0_h<T, J, 1, 0>(S, s);
    else sparse_row0_h<T, J + 1, 0, 0>(S, s);
  }
}

// r - y for y < 2^40: a borrow means r - y + 2^64 (>= 2^64 - 2^40) was kept,
// so subtracting eps = 2^64 mod p cannot borrow again
__device__ __forceinline__ uint64_t sub_small(uint64_t r, uint32_t y0, uint32_t y1) {
  uint32_t r0 = lo32(r), r1 = hi32(r), e;
  uint64_t c;
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c) : "v"(r0), "v"(y0));
  asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r1), "=s"(c) : "v"(r1), "v"(y1), "s"(c));
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(c));
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c) : "v"(r0), "v"(e));
  asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r1), "=s"(c) : "v"(r1), "s"(c));
  return ((uint64_t)r1 << 32) | r0;
}

// partial round 4 + T in sparse form (the next round's constants folded in)
template <int T>
__device__ __forceinline__ void partial_sparse(uint64_t s[12]) {
  const uint64_t x0 = sbox(s[0]);
  uint32_t l0[3];
  limbs22(x0, l0);
  // lane 0's dot product on the S-box output's 32-bit halves (the 22-bit limb
  // form measured slower: profiles/r02_ab_mul_form_dot_halves.log)
  // V = S0 + 2^22 S1 + 2^44 S2 + k,  25 x0 = 25 lo + (25 2^10) 2^22 hi
  constexpr uint32_t kl = pfp::K0[2 * T], kh = pfp::K0[2 * T + 1];
  uint64_t S[3];
  asm("v_mad_u64_u32 %0, vcc, %1, 25, %2" : "=v"(S[0]) : "v"(lo32(x0)), "s"((uint64_t)kl) : "vcc");
  S[1] = (uint64_t)hi32(x0) * 25600u;
  S[2] = 0;
  sparse_row0_h<T>(S, s);
  sparse_col0<T>(s, l0);
  // al + 2^32 ah - y:  2^22 S1 = 2^22 S1.lo + 2^32 (2^22 S1.hi);
  // 2^44 S2 = 2^32 (2^12 S2.lo) + 2^76 S2.hi, 2^76 = 2^32 2^12 - 2^12 (mod p)
  const uint64_t al = S[0] + (uint64_t)lo32(S[1]) * (1u << 22);
  uint64_t ah = (uint64_t)kh + (uint64_t)hi32(S[1]) * (1u << 22);
  ah += (uint64_t)lo32(S[2]) * (1u << 12);
  ah += (uint64_t)hi32(S[2]) * (1u << 12);
  s[0] = sub_small(reduce_row(al, ah), hi32(S[2]) << 12, hi32(S[2]) >> 20);
}

// ---- groups of G partial rounds (tools/gen_poseidon_partial.py
// permute_fast_grouped): lanes 1..11 only change by b_i x0 per round, so their
// updates are deferred to the end of the group (one reduction per lane per
// group instead of per round); round t's lane-0 dot then reads the group-start
// lanes and adds gamma[t][l] x_l for the group's earlier S-box outputs x_l.
constexpr int PF_GROUP = 4;  // partial rounds per group (profiles/r02_ab_poseidon_group4.log)
struct NoHook {
  __device__ __forceinline__ uint64_t operator()(int, uint64_t v) const { return v; }
};

template <int T0, int M, int L = 0>
__device__ __forceinline__ void group_gammas(uint64_t &al, uint64_t &ah, const uint32_t (*l)[3]) {
  if constexpr (L < M) {
    mac_limbs<PT_GAM, ((T0 + M) * 22 + T0 + L) * 6>(al, ah, l[L]);
    group_gammas<T0, M, L + 1>(al, ah, l);
  }
}

template <int T0, int G, int M = 0, class HK>
__device__ __forceinline__ void group_lane0(const uint64_t s[12], uint64_t &s0, uint32_t (*l)[3], const HK &hook) {
  if constexpr (M < G) {
    constexpr int T = T0 + M;
    const uint64_t x = sbox(hook(T, s0));
    limbs22(x, l[M]);
    constexpr uint32_t kl = pfp::K0[2 * T], kh = pfp::K0[2 * T + 1];
    uint64_t S[3];
    asm("v_mad_u64_u32 %0, vcc, %1, 25, %2" : "=v"(S[0]) : "v"(lo32(x)), "s"((uint64_t)kl) : "vcc");
    S[1] = (uint64_t)hi32(x) * 25600u;
    S[2] = 0;
    sparse_row0_h<T>(S, s);
    uint64_t al = S[0] + (uint64_t)lo32(S[1]) * (1u << 22);
    uint64_t ah = (uint64_t)kh + (uint64_t)hi32(S[1]) * (1u << 22);
    ah += (uint64_t)lo32(S[2]) * (1u << 12);
    ah += (uint64_t)hi32(S[2]) * (1u << 12);
    group_gammas<T0, M>(al, ah, l);
    s0 = sub_small(reduce_row(al, ah), hi32(S[2]) << 12, hi32(S[2]) >> 20);
    group_lane0<T0, G, M + 1>(s, s0, l, hook);
  }
}

template <int T0, int G, int I, int M>
__device__ __forceinline__ void group_col_macs(uint64_t &bl, uint64_t &bh, const uint32_t (*l)[3]) {
  if constexpr (M < G) {
    mac_limbs<PT_BV, ((T0 + M) * 11 + I - 1) * 6>(bl, bh, l[M]);
    group_col_macs<T0, G, I, M + 1>(bl, bh, l);
  }
}

template <int T0, int G, int I = 1>
__device__ __forceinline__ void group_cols(uint64_t s[12], const uint32_t (*l)[3]) {
  if constexpr (I < 12) {
    constexpr bool last = T0 + G == 22;
    uint64_t bl = (uint64_t)lo32(s[I]) + (last ? pfp::KLAST[2 * I] : 0u);
    uint64_t bh = (uint64_t)hi32(s[I]) + (last ? pfp::KLAST[2 * I + 1] : 0u);
    group_col_macs<T0, G, I, 0>(bl, bh, l);
    s[I] = reduce_row(bl, bh);
    group_cols<T0, G, I + 1>(s, l);
  }
}

template <int T0, int G, class HK = NoHook>
__device__ __forceinline__ void partial_group(uint64_t s[12], const HK &hook = HK{}) {
  uint32_t l[G][3];
  uint64_t s0 = s[0];
  group_lane0<T0, G>(s, s0, l, hook);
  group_cols<T0, G>(s, l);
  s[0] = s0;
}

// OUT: bit mask of the output lanes the caller reads (the last MDS computes
// only those rows; digests need lanes 0..3, the PoW lane 7)
template <int M, int R, uint32_t OUT = 0xFFFu>
__device__ __forceinline__ void rounds(uint64_t s[12]) {
  if constexpr (M == 10 && R == 0) {
    // mode 10: mode 3 with the full rounds 0-2 and 26-28 rolled (a third of
    // the code; round constants from memory)
#pragma unroll 1
    for (int r = 0; r < 3; r++) full_round_dyn(s, ps::RC_DEV + (r + 1) * 12);
    rounds<M, 3, OUT>(s);
  } else if constexpr (M == 10 && R == 26) {
#pragma unroll 1
    for (int r = 26; r < 29; r++) full_round_dyn(s, ps::RC_DEV + (r + 1) * 12);
    rounds<3, 29, OUT>(s);
  } else if constexpr ((M == 3 || M == 10) && R == 3) {
    sbox12(s);
    mds_init_sparse(s);
    rounds<M, 4, OUT>(s);
  } else if constexpr ((M == 3 || M == 10) && R >= 4 && R < 26) {
    constexpr int T0 = R - 4, G = (22 - T0) < PF_GROUP ? (22 - T0) : PF_GROUP;
    if constexpr (G > 1) partial_group<T0, G>(s);
    else partial_sparse<T0>(s);
    rounds<M, R + G, OUT>(s);
  } else if constexpr (M == 5 && R == 0) {
    // every round rolled: a ~4k-instruction permutation
#pragma unroll 1
    for (int r = 0; r < 4; r++) full_round_dyn(s, ps::RC_DEV + (r + 1) * 12);
    rounds<5, 4>(s);  // rolled partial rounds, then the rolled tail
  } else if constexpr (M == 5 && R == 26) {
#pragma unroll 1
    for (int r = 26; r < 29; r++) full_round_dyn(s, ps::RC_DEV + (r + 1) * 12);
    rounds<3, 29>(s);  // the last round: MDS without a next constant
  } else if constexpr ((M == 4 || M == 5) && R == 4) {
    // 22 partial rounds as a loop: ~9k fewer instructions of code (the
    // unrolled permutation is several times the instruction cache)
#pragma unroll 1
    for (int r = 4; r < 26; r++) {
      s[0] = sbox(s[0]);
      uint32_t lo[12], hi[12];
#pragma unroll
      for (int i = 0; i < 12; i++) {
        lo[i] = lo32(s[i]);
        hi[i] = hi32(s[i]);
      }
      mds_rows_block_dyn<0>(s, lo, hi, ps::RC_DEV + (r + 1) * 12);
    }
    rounds<M, 26>(s);
  } else if constexpr (R < 30) {
    constexpr bool full = R < 4 || R >= 26;
    if constexpr (full && M == 3) {
      sbox12(s);
    } else if constexpr (full) {
#pragma unroll
      for (int i = 0; i < 12; i++) s[i] = M == 2 ? sbox_c(s[i]) : sbox(s[i]);
    } else {
      s[0] = M == 2 ? sbox_c(s[0]) : sbox(s[0]);
    }
    if constexpr (R == 29) mds<M, -1, OUT>(s);
    else mds<M, R + 1>(s);
    rounds<M, R + 1, OUT>(s);
  }
}

// round 0 of a state whose lanes 8..11 enter as zero (two_to_one, the first
// absorption of a sponge): their S-box outputs are constants, so only lanes
// 0..7 are S-boxed and each MDS row takes 16 mads on them, starting from the
// folded constant CAPZ_K[r] = RC[1][r] + sum_(j>=8) M[r][j] sbox(RC[0][j])
template <int R, int I = 0>
__device__ __forceinline__ void capz_row_terms(uint64_t &al, uint64_t &ah, const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (I < 12) {
    constexpr int J = (I + R) % 12;
    if constexpr (J < 8) {
      constexpr int C = (int)ps::mds_circ(I) + ((R == 0 && I == 0) ? 8 : 0);
      al = mad_c<C>(lo[J], al);
      ah = mad_c<C>(hi[J], ah);
    }
    capz_row_terms<R, I + 1>(al, ah, lo, hi);
  }
}
template <int R = 0>
__device__ __forceinline__ void capz_mds(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (R < 12) {
    uint64_t al = pfp::CAPZ_K[2 * R], ah = pfp::CAPZ_K[2 * R + 1];
    capz_row_terms<R>(al, ah, lo, hi);
    s[R] = reduce_row(al, ah);
    capz_mds<R + 1>(s, lo, hi);
  }
}

// permute_nc for s[8..11] == 0 on entry (mode 3), reading only lanes OUT
// (profiles/r02_ab_capz.log)
template <uint32_t OUT = 0xFFFu>
__device__ __forceinline__ void permute_nc_capz(uint64_t s[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    s[i] = sbox(add_c(s[i], ps::rc_cx(i)));
    lo[i] = lo32(s[i]);
    hi[i] = hi32(s[i]);
  }
  capz_mds(s, lo, hi);
  rounds<3, 1, OUT>(s);
}

// permutation; inputs in [0, 2^64), outputs in [0, 2^64) (canon() lanes read out)
// M: 0 = asm mads, 1 = compiler mads on opaque constants, 2 = 1 + C reductions,
//    3 = 0 with each MDS row's 24 mads in one asm block, 4 = 3 with the
//    partial rounds rolled into a loop, 5 = every round rolled,
//    6..9 = MDS in blocks of 2 / 3 / 4 / 6 rows with interleaved chains
template <int M = 1>
__device__ __forceinline__ void permute_nc(uint64_t s[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = add_c(s[i], ps::rc_cx(i));
  rounds<M, 0>(s);
}

template <int M = 1>
__device__ __forceinline__ void permute(uint64_t s[12]) {
  permute_nc<M>(s);
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = canon(s[i]);
}

}  // namespace pf
