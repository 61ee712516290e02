// ntt16.h — register-blocked radix-16 DIF NTT core for gfx950.
//
// Every transform the prover runs is a size-n (n <= 2^14) NTT held in one
// workgroup's LDS.  This core replaces the radix-2 stage loop with passes of
// radix 16: each thread pulls 16 elements of one sub-problem (stride S/16) into
// registers, runs a 16-point DFT whose internal twiddles are powers of
// w_16 = 2^12 in Goldilocks (multiplication by a power of two = shifts + one
// short reduction, no 64x64 product), then applies one general twiddle
// w_S^{t*p} per element (table lookup + one product) and writes back in place.
// 13 radix-2 levels become 3 radix-16 passes + 1 radix-2 pass: ~4x fewer LDS
// round trips and barriers, and 15/16 general products per element per 4
// levels instead of 2.  Arithmetic stays non-canonical in [0, 2^64)
// (plonky2's own representation); callers canonicalise on store.
// Output order is the standard in-place DIF order: a[q] = X[bitrev(q)].
//
// LDS layout: element i lives at slot lp(i) = i + i/32 (one pad slot per 32
// elements, lds_words(n) slots).  Without it the stride-2 accesses of the
// S = 32 radix-16 pass put all 64 lanes of a wave on two 8-byte bank pairs
// (a 32-way conflict); padded, lane sp of that pass lands on bank pair
// (sp + ...) mod 32 and every pass is conflict-free.  For the addresses the
// passes generate, lp(b0 + m*q) = lp(b0) + lp(m*q) (q | 32 or 32 | q), so the
// per-element offsets stay wave-uniform.
#pragma once
#include "field.h"
#include "kernels.h"
#include "poseidon_fast.h"
#include "field_nc.h"

namespace nt {

constexpr uint64_t EPS = 0xFFFFFFFFull;

// Branch-free 32-bit carry chains (field_nc.h) rather than 64-bit
// compare-and-branch forms; additions with the wrap corrections as
// v_mad_u64_u32 with carry-out (s + e, e = eps on a wrap): 6 instructions
// instead of the 8-step carry chain, LDE -4.4 %, iNTT -8 %
// (profiles/r03_ab_ntt_add_mad.log)
__device__ __forceinline__ uint64_t add_mad(uint64_t a, uint64_t b) {
  uint32_t c0, c1;
  const uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  const uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
  const uint64_t s = ((uint64_t)hi << 32) | lo;
  const uint32_t e = 0u - c1;  // a + b wrapped: 2^64 = eps
  uint64_t s2, c2, s3, cd;
  uint32_t e2;
  asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(s2), "=s"(c2) : "v"(e), "v"(s));
  // wrapped again (both inputs in [p, 2^64)): s2 < eps, + eps cannot wrap
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e2) : "s"(c2));
  asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(s3), "=s"(cd) : "v"(e2), "v"(s2));
  return s3;
}

__device__ __forceinline__ uint64_t add(uint64_t a, uint64_t b) { return add_mad(a, b); }

__device__ __forceinline__ uint64_t sub(uint64_t a, uint64_t b) { return gfn::sub(a, b); }

__device__ __forceinline__ uint64_t reduce(uint64_t lo, uint64_t hi) {
  const uint64_t hh = hi >> 32, hl = hi & EPS;
  uint64_t t0 = lo - hh;
  t0 -= (lo < hh) ? EPS : 0;
  const uint64_t t1 = (hl << 32) - hl;
  const uint64_t r = t0 + t1;
  return r + (r < t1 ? EPS : 0);
}

// general product: the asm form (5 mads + 8-op reduction, poseidon_fast.h)
__device__ __forceinline__ uint64_t mul(uint64_t a, uint64_t b) { return pf::mul(a, b); }

// r[m] *= tw(m) for m = 1..15 (a group's twiddles); K = true (the LDS passes)
// issues them as five interleaved triples (pf::mulk<3>: each carry is read two
// products later instead of after hazard pads), K = false one at a time (the
// coset LDE's first pass, at its register cap)
template <bool K = true, class TW>
__device__ __forceinline__ void mul_rows(uint64_t r[16], const TW &tw) {
  if constexpr (K) {
#pragma unroll
    for (int m = 1; m < 16; m += 3) {
      const uint64_t a[3] = {r[m], r[m + 1], r[m + 2]}, b[3] = {tw(m), tw(m + 1), tw(m + 2)};
      uint64_t o[3];
      pf::mulk<3>(a, b, o);
      r[m] = o[0];
      r[m + 1] = o[1];
      r[m + 2] = o[2];
    }
  } else {
#pragma unroll
    for (int m = 1; m < 16; m++) r[m] = mul(r[m], tw(m));
  }
}

__device__ __forceinline__ uint64_t canon(uint64_t x) { return x >= gl::P ? x - gl::P : x; }

__device__ __forceinline__ uint64_t neg(uint64_t x) {
  x = canon(x);
  return x ? gl::P - x : 0;
}

// r - (b ? eps : 0) for a borrow b of a subtraction whose wrapped result is
// >= 2^64 - 2^63 (so subtracting eps cannot borrow again); r = (r0, r1)
__device__ __forceinline__ uint64_t sub_borrow_eps(uint32_t r0, uint32_t r1, uint64_t b) {
  uint32_t e;
  uint64_t c;
  asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(b));
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c) : "v"(r0), "v"(e));
  asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r1), "=s"(c) : "v"(r1), "s"(c));
  return ((uint64_t)r1 << 32) | r0;
}

// mad-based reductions for shifts E in [32, 96) (10 and 9 instructions
// against 14 and 23 for the reduce()-based forms, which the small shifts keep)

// x * 2^E for a compile-time E in [0, 192) (2^96 = -1, 2^192 = 1)
template <int E>
__device__ __forceinline__ uint64_t mul_pow2(uint64_t x) {
  if constexpr (E >= 96) {
    return neg(mul_pow2<E - 96>(x));
  } else if constexpr (E == 0) {
    return x;
  } else if constexpr (E >= 32 && E < 64) {
    // x 2^E = lo + 2^64 (h0 + 2^32 h1) = lo + h0 eps - h1  (h1 < 2^31)
    const uint64_t lo = x << E, hi = x >> (64 - E);
    uint64_t t, c;
    uint32_t e;
    asm("v_mad_u64_u32 %0, %1, %2, -1, %3" : "=v"(t), "=s"(c) : "v"((uint32_t)hi), "v"(lo));
    asm(QP_CWAIT "v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(e) : "s"(c));
    // carry: the wrapped t < 2^64 - 2^33 + 1, so + eps stays below 2^64
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(t), "=s"(c) : "v"(e), "v"(t));
    uint32_t r0, r1;
    asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r0), "=s"(c) : "v"((uint32_t)t), "v"((uint32_t)(hi >> 32)));
    asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r1), "=s"(c) : "v"((uint32_t)(t >> 32)), "s"(c));
    return sub_borrow_eps(r0, r1, c);
  } else if constexpr (E >= 64) {
    // E = 64 + F: x 2^E = x0 2^F 2^64 + x1 2^F 2^96 = u eps - v with
    // u = x0 2^F, v = x1 2^F (< 2^63); u eps = u0 2^32 - u0 - u1, so
    // x 2^E = (u0 << 32) - S, S = u0 + u1 + v < 2^64
    constexpr int F = E - 64;
    const uint64_t u = (uint64_t)(uint32_t)x << F, v = (x >> 32) << F;
    const uint64_t S = v + (uint32_t)u + (uint32_t)(u >> 32);
    uint32_t r0, r1;
    uint64_t c;
    asm("v_sub_co_u32_e64 %0, %1, 0, %2" : "=v"(r0), "=s"(c) : "v"((uint32_t)S));
    asm(QP_CWAIT "v_subb_co_u32_e64 %0, %1, %2, %3, %1" : "=v"(r1), "+s"(c) : "v"((uint32_t)u), "v"((uint32_t)(S >> 32)));
    // borrow: the wrapped A - S + 2^64 >= 2^64 - S > 2^63
    return sub_borrow_eps(r0, r1, c);
  } else {
    return reduce(x << E, x >> (64 - E));
  }
}

// twiddle w_16^j (forward) or w_16^-j (inverse): w_16 = 2^12
template <bool INV, int J>
__device__ __forceinline__ uint64_t mul_w16(uint64_t x) {
  if constexpr (J == 0) return x;
  else if constexpr (!INV) return mul_pow2<(12 * J) % 192>(x);
  else return mul_pow2<(192 - 12 * J) % 192>(x);
}

// A stage's butterflies four at a time, their adds and subs interleaved in one
// asm block each (add4 / sub4): every carry is read four instructions after it
// is written, so the gfx950 carry hazard needs no s_nop (a 16-point DFT: 694
// VALU + 387 s_nop -> 660 VALU + 113 s_nop, static)
// 4 independent Goldilocks adds (non-canonical in and out, as nt::add),
// interleaved in one asm block: every carry is read 4 instructions after it
// is written, so no hazard pads
__device__ __forceinline__ void add4(const uint64_t a[4], const uint64_t b[4], uint64_t s[4]) {
  uint64_t c0, c1, c2, c3;
  uint32_t e0, e1, e2, e3;
  asm("v_lshl_add_u64 %0, %12, 0, %16\n\t"
      "v_lshl_add_u64 %1, %13, 0, %17\n\t"
      "v_lshl_add_u64 %2, %14, 0, %18\n\t"
      "v_lshl_add_u64 %3, %15, 0, %19\n\t"
      "v_cmp_lt_u64_e64 %8, %0, %16\n\t"
      "v_cmp_lt_u64_e64 %9, %1, %17\n\t"
      "v_cmp_lt_u64_e64 %10, %2, %18\n\t"
      "v_cmp_lt_u64_e64 %11, %3, %19\n\t"
      "v_cndmask_b32_e64 %4, 0, -1, %8\n\t"
      "v_cndmask_b32_e64 %5, 0, -1, %9\n\t"
      "v_cndmask_b32_e64 %6, 0, -1, %10\n\t"
      "v_cndmask_b32_e64 %7, 0, -1, %11\n\t"
      "v_mad_u64_u32 %0, %8, %4, 1, %0\n\t"
      "v_mad_u64_u32 %1, %9, %5, 1, %1\n\t"
      "v_mad_u64_u32 %2, %10, %6, 1, %2\n\t"
      "v_mad_u64_u32 %3, %11, %7, 1, %3\n\t"
      "v_cndmask_b32_e64 %4, 0, -1, %8\n\t"
      "v_cndmask_b32_e64 %5, 0, -1, %9\n\t"
      "v_cndmask_b32_e64 %6, 0, -1, %10\n\t"
      "v_cndmask_b32_e64 %7, 0, -1, %11\n\t"
      "v_mad_u64_u32 %0, %8, %4, 1, %0\n\t"
      "v_mad_u64_u32 %1, %9, %5, 1, %1\n\t"
      "v_mad_u64_u32 %2, %10, %6, 1, %2\n\t"
      "v_mad_u64_u32 %3, %11, %7, 1, %3"
      : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(e0), "=&v"(e1), "=&v"(e2), "=&v"(e3),
        "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}

// 4 independent Goldilocks subs (as nt::sub): d = a - b; on a borrow d - eps,
// and on a second borrow (b > a + p) d - eps again
__device__ __forceinline__ void sub4(const uint64_t a[4], const uint64_t b[4], uint64_t d[4]) {
  uint32_t l0, l1, l2, l3, h0, h1, h2, h3, e0, e1, e2, e3;
  uint64_t c0, c1, c2, c3;
  asm("v_sub_co_u32_e64 %0, %12, %16, %24\n\t"
      "v_sub_co_u32_e64 %1, %13, %17, %25\n\t"
      "v_sub_co_u32_e64 %2, %14, %18, %26\n\t"
      "v_sub_co_u32_e64 %3, %15, %19, %27\n\t"
      "v_subb_co_u32_e64 %4, %12, %20, %28, %12\n\t"
      "v_subb_co_u32_e64 %5, %13, %21, %29, %13\n\t"
      "v_subb_co_u32_e64 %6, %14, %22, %30, %14\n\t"
      "v_subb_co_u32_e64 %7, %15, %23, %31, %15\n\t"
      "v_cndmask_b32_e64 %8, 0, -1, %12\n\t"
      "v_cndmask_b32_e64 %9, 0, -1, %13\n\t"
      "v_cndmask_b32_e64 %10, 0, -1, %14\n\t"
      "v_cndmask_b32_e64 %11, 0, -1, %15\n\t"
      "v_sub_co_u32_e64 %0, %12, %0, %8\n\t"
      "v_sub_co_u32_e64 %1, %13, %1, %9\n\t"
      "v_sub_co_u32_e64 %2, %14, %2, %10\n\t"
      "v_sub_co_u32_e64 %3, %15, %3, %11\n\t"
      "v_subb_co_u32_e64 %4, %12, %4, 0, %12\n\t"
      "v_subb_co_u32_e64 %5, %13, %5, 0, %13\n\t"
      "v_subb_co_u32_e64 %6, %14, %6, 0, %14\n\t"
      "v_subb_co_u32_e64 %7, %15, %7, 0, %15\n\t"
      "v_cndmask_b32_e64 %8, 0, -1, %12\n\t"
      "v_cndmask_b32_e64 %9, 0, -1, %13\n\t"
      "v_cndmask_b32_e64 %10, 0, -1, %14\n\t"
      "v_cndmask_b32_e64 %11, 0, -1, %15\n\t"
      "v_sub_co_u32_e64 %0, %12, %0, %8\n\t"
      "v_sub_co_u32_e64 %1, %13, %1, %9\n\t"
      "v_sub_co_u32_e64 %2, %14, %2, %10\n\t"
      "v_sub_co_u32_e64 %3, %15, %3, %11\n\t"
      "v_subb_co_u32_e64 %4, %12, %4, 0, %12\n\t"
      "v_subb_co_u32_e64 %5, %13, %5, 0, %13\n\t"
      "v_subb_co_u32_e64 %6, %14, %6, 0, %14\n\t"
      "v_subb_co_u32_e64 %7, %15, %7, 0, %15"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(e0),
        "=&v"(e1), "=&v"(e2), "=&v"(e3), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"((uint32_t)a[0]), "v"((uint32_t)a[1]), "v"((uint32_t)a[2]), "v"((uint32_t)a[3]),
        "v"((uint32_t)(a[0] >> 32)), "v"((uint32_t)(a[1] >> 32)), "v"((uint32_t)(a[2] >> 32)),
        "v"((uint32_t)(a[3] >> 32)), "v"((uint32_t)b[0]), "v"((uint32_t)b[1]), "v"((uint32_t)b[2]),
        "v"((uint32_t)b[3]), "v"((uint32_t)(b[0] >> 32)), "v"((uint32_t)(b[1] >> 32)), "v"((uint32_t)(b[2] >> 32)),
        "v"((uint32_t)(b[3] >> 32)));
  d[0] = ((uint64_t)h0 << 32) | l0;
  d[1] = ((uint64_t)h1 << 32) | l1;
  d[2] = ((uint64_t)h2 << 32) | l2;
  d[3] = ((uint64_t)h3 << 32) | l3;
}

// radix-2 DIF stage of half-width H on a register array of size 16
template <bool INV, int H>
__device__ __forceinline__ void stage16(uint64_t a[16]) {
#pragma unroll
  for (int g = 0; g < 8; g += 4) {
    // butterflies g..g+3: index pairs (lo_i, lo_i + H)
    int lo[4];
#pragma unroll
    for (int i = 0; i < 4; i++) lo[i] = ((g + i) / H) * 2 * H + (g + i) % H;
    uint64_t u[4], v[4], s[4], d[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      u[i] = a[lo[i]];
      v[i] = a[lo[i] + H];
    }
    add4(u, v, s);
    sub4(u, v, d);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      a[lo[i]] = s[i];
      switch ((lo[i] % H) * (8 / H)) {
        case 0: a[lo[i] + H] = d[i]; break;
        case 1: a[lo[i] + H] = mul_w16<INV, 1>(d[i]); break;
        case 2: a[lo[i] + H] = mul_w16<INV, 2>(d[i]); break;
        case 3: a[lo[i] + H] = mul_w16<INV, 3>(d[i]); break;
        case 4: a[lo[i] + H] = mul_w16<INV, 4>(d[i]); break;
        case 5: a[lo[i] + H] = mul_w16<INV, 5>(d[i]); break;
        case 6: a[lo[i] + H] = mul_w16<INV, 6>(d[i]); break;
        default: a[lo[i] + H] = mul_w16<INV, 7>(d[i]); break;
      }
    }
  }
}

template <bool INV>
__device__ __forceinline__ void dft16(uint64_t a[16]) {
  stage16<INV, 8>(a);
  stage16<INV, 4>(a);
  stage16<INV, 2>(a);
  stage16<INV, 1>(a);
}

// w_S^e from the power table of w_{2^TW_LOG} (even/odd layout: kernels.h tw_get)
__device__ __forceinline__ uint64_t tw_pow(const uint64_t *__restrict__ tw, uint32_t e, uint32_t log_S) {
  return qpk::tw_get(tw, e << (qpk::TW_LOG - log_S));
}

// LDS index with one pad word per 32 (bank-conflict-free strided passes)
__host__ __device__ __forceinline__ constexpr uint32_t lp(uint32_t i) { return i + (i >> 5); }

__device__ __forceinline__ uint32_t brev4(uint32_t m) { return __builtin_bitreverse32(m) >> 28; }

// radix-2^LOGS DIF on each group of S = 2^LOGS contiguous LDS elements
// (the last levels of ntt_lds); twiddles are powers of w_S = w_16^(16/S)
template <bool INV, int H, int S>
__device__ __forceinline__ void stage_small(uint64_t r[S]) {
#pragma unroll
  for (int k = 0; k < S; k += 2 * H) {
#pragma unroll
    for (int j = 0; j < H; j++) {
      const uint64_t u = r[k + j], v = r[k + j + H];
      r[k + j] = add(u, v);
      const uint64_t d = sub(u, v);
      switch (j * (8 / H)) {
        case 0: r[k + j + H] = d; break;
        case 1: r[k + j + H] = mul_w16<INV, 1>(d); break;
        case 2: r[k + j + H] = mul_w16<INV, 2>(d); break;
        case 3: r[k + j + H] = mul_w16<INV, 3>(d); break;
        case 4: r[k + j + H] = mul_w16<INV, 4>(d); break;
        case 5: r[k + j + H] = mul_w16<INV, 5>(d); break;
        case 6: r[k + j + H] = mul_w16<INV, 6>(d); break;
        default: r[k + j + H] = mul_w16<INV, 7>(d); break;
      }
    }
  }
}

template <bool INV, int LOGS>
__device__ __forceinline__ void tail(uint64_t *a, uint32_t n) {
  constexpr int S = 1 << LOGS;
  for (uint32_t g = threadIdx.x; g < (n >> LOGS); g += blockDim.x) {
    uint64_t *base = a + lp(g << LOGS);
    uint64_t r[S];
#pragma unroll
    for (int m = 0; m < S; m++) r[m] = base[m];
    if constexpr (S >= 8) stage_small<INV, S / 2, S>(r);
    if constexpr (S >= 4) stage_small<INV, 2, S>(r);
    stage_small<INV, 1, S>(r);
#pragma unroll
    for (int m = 0; m < S; m++) base[m] = r[m];
  }
  __syncthreads();
}

// x * w_32^j (forward) or w_32^-j (inverse), w_32 = 2^6; j folds to a constant
// after unrolling, so each case is a shift + short reduction
template <bool INV>
__device__ __forceinline__ uint64_t mul_w32(uint64_t x, int j) {
#define QP_W32(J) \
  case J: return INV ? mul_pow2<(192 - 6 * J) % 192>(x) : mul_pow2<(6 * J) % 192>(x);
  switch (j) {
    QP_W32(1) QP_W32(2) QP_W32(3) QP_W32(4) QP_W32(5) QP_W32(6) QP_W32(7) QP_W32(8)
    QP_W32(9) QP_W32(10) QP_W32(11) QP_W32(12) QP_W32(13) QP_W32(14) QP_W32(15)
    default: return x;
  }
#undef QP_W32
}

// The S = 32 radix-16 pass (q = 2): its twiddles w_32^{t brev4(m)}, t in {0,1},
// are powers of two.  Groups are assigned so t is uniform per wave (t = bit 6
// of g): t = 0 waves skip the twiddles, t = 1 waves shift instead of
// multiplying.  Needs n/16 to be a multiple of 128.
template <bool INV>
__device__ __forceinline__ void pass32(uint64_t *a, uint32_t n) {
  for (uint32_t g = threadIdx.x; g < (n >> 4); g += blockDim.x) {
    const uint32_t t = (g >> 6) & 1, sp = ((g >> 7) << 6) | (g & 63);
    uint64_t *base = a + lp((sp << 5) + t);
    uint64_t r[16];
#pragma unroll
    for (int m = 0; m < 16; m++) r[m] = base[lp(2 * m)];
    dft16<INV>(r);
    if (t) {
#pragma unroll
      for (int m = 1; m < 16; m++) r[m] = mul_w32<INV>(r[m], (int)brev4(m));
    }
#pragma unroll
    for (int m = 0; m < 16; m++) base[lp(2 * m)] = r[m];
  }
  __syncthreads();
}

// In-place DIF over LDS a[lp(0..2^log_n)), all threads of the block participate,
// starting at sub-problem size 2^log_S (log_S = log_n: the whole transform;
// smaller: the levels above were already done, e.g. from registers).
// pt = the pass twiddles (Twiddles::pt_fwd or pt_inv, matching INV): a pass's
// 15 twiddles per group are read as [m][t] rows, so the lanes of a wave
// (consecutive t) read consecutive words instead of a gather with stride
// brev4(m) through the power table.  Ends with a barrier.
// TAIL = false: stop before the last radix-2^log_S (log_S < 4) levels and
// return log_S (after the barrier of the last pass), for callers that fold
// those levels into their output loop (tail_group)
__host__ __device__ constexpr bool use_pass32(uint32_t log_S, uint32_t n, uint32_t T) {
  return log_S == 5 && (n >> 4) % 128 == 0 && T % 64 == 0;
}
// the log_S ntt_lds_from<.., false> returns for a block of T threads
__host__ __device__ constexpr uint32_t lds_levels_left(uint32_t log_n, uint32_t log_S, uint32_t T) {
  while (log_S >= 4) log_S = use_pass32(log_S, 1u << log_n, T) ? 1 : log_S - 4;
  return log_S;
}
// K: the pass twiddles as interleaved triples (mul_rows); the coset LDE uses
// single products
template <bool INV, bool TAIL = true, bool K = true>
__device__ __forceinline__ uint32_t ntt_lds_from(uint64_t *a, uint32_t log_n, uint32_t log_S, const uint64_t *__restrict__ pt) {
  const uint32_t n = 1u << log_n;
  const uint32_t T = blockDim.x;
  // radix-16 passes
  while (log_S >= 4) {
    if (use_pass32(log_S, n, T)) {
      pass32<INV>(a, n);
      log_S = 1;
      continue;
    }
    const uint32_t S = 1u << log_S, q = S >> 4, log_q = log_S - 4;
    for (uint32_t g = threadIdx.x; g < (n >> 4); g += T) {
      const uint32_t sp = g >> log_q, t = g & (q - 1);
      uint64_t *base = a + lp((sp << log_S) + t);
      uint64_t r[16];
#pragma unroll
      for (int m = 0; m < 16; m++) r[m] = base[lp(m * q)];
      dft16<INV>(r);
      if (t) {
        const uint64_t *ptS = pt + qpk::pt_offset(log_S) + t;
        mul_rows<K>(r, [&](int m) { return ptS[m * q]; });
      }
#pragma unroll
      for (int m = 0; m < 16; m++) base[lp(m * q)] = r[m];
    }
    __syncthreads();
    log_S -= 4;
  }
  // remaining radix-2^log_S levels (log_S < 4): groups of S contiguous elements
  if (!TAIL) return log_S;
  if (log_S == 1) tail<INV, 1>(a, n);
  else if (log_S == 2) tail<INV, 2>(a, n);
  else if (log_S == 3) tail<INV, 3>(a, n);
  return 0;
}

// the last LOGS levels of a DIF on one group of S = 2^LOGS contiguous values
template <bool INV, int LOGS>
__device__ __forceinline__ void tail_group(uint64_t r[1 << LOGS]) {
  constexpr int S = 1 << LOGS;
  if constexpr (S >= 8) stage_small<INV, S / 2, S>(r);
  if constexpr (S >= 4) stage_small<INV, 2, S>(r);
  if constexpr (S >= 2) stage_small<INV, 1, S>(r);
}

template <bool INV>
__device__ __forceinline__ void ntt_lds(uint64_t *a, uint32_t log_n, const uint64_t *__restrict__ pt) {
  ntt_lds_from<INV, true>(a, log_n, log_n, pt);
}

// ---- radix-8 variant: 8 elements per thread (n/8 threads per transform), so
// a size-2^13 transform is a 1024-thread workgroup whose LDS (67.6 KB) still
// fits twice per CU: 8 waves per SIMD instead of 4 (VALU issue at 8 waves/SIMD
// measured 2.56 vs 3.12 cycles per instruction, tools/isa_rates.hip).

__device__ __forceinline__ uint32_t brev3(uint32_t m) { return __builtin_bitreverse32(m) >> 29; }

template <bool INV>
__device__ __forceinline__ void dft8(uint64_t a[8]) {
  stage_small<INV, 4, 8>(a);
  stage_small<INV, 2, 8>(a);
  stage_small<INV, 1, 8>(a);
}

// x * w_16^j (forward) or w_16^-j (inverse) for a runtime j < 16 that folds to
// a constant after unrolling
template <bool INV>
__device__ __forceinline__ uint64_t mul_w16_rt(uint64_t x, int j) {
#define QP_W16(J) \
  case J: return mul_w16<INV, J>(x);
  switch (j) {
    QP_W16(1) QP_W16(2) QP_W16(3) QP_W16(4) QP_W16(5) QP_W16(6) QP_W16(7)
    default: return x;
  }
#undef QP_W16
}

// radix-8 DIF passes over LDS from sub-problem size 2^log_S down to 2, then the
// last radix-2 level; every thread of the block participates (n/8 groups per
// pass).  The S = 16 pass (twiddles w_16^{t brev3(m)}, t in {0,1}: shifts) maps
// t to bit 6 of the group index so it is wave-uniform.  Ends with a barrier.
template <bool INV>
__device__ __forceinline__ void ntt8_lds_from(uint64_t *a, uint32_t log_n, uint32_t log_S,
                                              const uint64_t *__restrict__ tw) {
  const uint32_t n = 1u << log_n;
  const uint32_t T = blockDim.x;
  while (log_S >= 3) {
    if (log_S == 4 && (n >> 3) % 128 == 0 && T % 64 == 0) {
      for (uint32_t g = threadIdx.x; g < (n >> 3); g += T) {
        const uint32_t t = (g >> 6) & 1, sp = ((g >> 7) << 6) | (g & 63);
        uint64_t *base = a + lp((sp << 4) + t);
        uint64_t r[8];
#pragma unroll
        for (int m = 0; m < 8; m++) r[m] = base[lp(2 * m)];
        dft8<INV>(r);
        if (t) {
#pragma unroll
          for (int m = 1; m < 8; m++) r[m] = mul_w16_rt<INV>(r[m], (int)brev3(m));
        }
#pragma unroll
        for (int m = 0; m < 8; m++) base[lp(2 * m)] = r[m];
      }
      __syncthreads();
      log_S = 1;
      break;
    }
    const uint32_t q = 1u << (log_S - 3), log_q = log_S - 3;
    for (uint32_t g = threadIdx.x; g < (n >> 3); g += T) {
      const uint32_t sp = g >> log_q, t = g & (q - 1);
      uint64_t *base = a + lp((sp << log_S) + t);
      uint64_t r[8];
#pragma unroll
      for (int m = 0; m < 8; m++) r[m] = base[lp(m * q)];
      dft8<INV>(r);
      if (t) {
#pragma unroll
        for (int m = 1; m < 8; m++) r[m] = mul(r[m], tw_pow(tw, t * brev3(m), log_S));
      }
#pragma unroll
      for (int m = 0; m < 8; m++) base[lp(m * q)] = r[m];
    }
    __syncthreads();
    log_S -= 3;
  }
  if (log_S == 1) tail<INV, 1>(a, n);
  else if (log_S == 2) tail<INV, 2>(a, n);
}

}  // namespace nt
