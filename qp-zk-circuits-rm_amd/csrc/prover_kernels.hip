// prover_kernels.hip — gfx950 kernels for the proof stages after the
// commitments, batched over
// proofs of one circuit (blockIdx.y / .z = proof index, per-proof strides).
//
//   k_pp_rows / k_z_scan   wires_permutation_partial_products_and_zs (a9)
//   k_quotient             compute_quotient_polys: vanishing poly at every
//                          LDE point, alpha-reduced, / Z_H (a8)
//   k_qintt_blocks/_radix  coset_ifft of size N as 2^r size-n LDS iNTTs + a
//                          radix-2^r cross-block pass (a8, second half)
//   k_openings             OpeningSet::new: Horner at zeta / g*zeta (a10)
//   k_fri_compose/_divide  prove_openings: alpha-reduce + divide by (X - z) (a11)
//   k_fri_leaf, k_fold     fri_committed_trees: leaves of 2^a ext, folding (a11)
//   k_pow_scan             fri_proof_of_work: minimal witness (a12)
//   k_gather_*             query-round openings (a11)
#include "field.h"
#include "poseidon.h"
#include "poseidon_dev.h"
#include "poseidon_coop.h"
#include "prover_kernels.h"
#include "paths.h"
#include <stdlib.h>
#include <algorithm>
#include "ntt16.h"

namespace qpk {

using gl::ext;

__device__ __forceinline__ uint64_t wpow_N(const uint64_t *__restrict__ tw, uint32_t j, uint32_t logN) {
  // w_N^j from the half table of w_{2^TW_LOG}: w_N^j = w_T^{j << (TW_LOG-logN)}
  return tw_get(tw, j << (TW_LOG - logN));
}

// ---------------------------------------------------------------- a9

// per row: P_j = prod_{k<=j} num_k/den_k over chunks of qdf routed wires
__global__ void __launch_bounds__(256) k_pp_rows(const uint64_t *__restrict__ wires, const uint64_t *__restrict__ sigmas,
                                                 const uint64_t *__restrict__ k_is, const uint64_t *__restrict__ chal,
                                                 uint64_t *__restrict__ prods, uint32_t log_n, uint32_t R, uint32_t qdf,
                                                 uint32_t nc, uint64_t w_bstride, uint64_t p_bstride,
                                                 const uint64_t *__restrict__ tw) {
  const uint32_t n = 1u << log_n;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = blockIdx.y;
  wires += b * w_bstride;
  prods += b * p_bstride;
  const uint64_t *ch = chal + b * CHAL_STRIDE;
  const uint64_t x = wpow_N(tw, i, log_n);
  const uint32_t nchunks = (R + qdf - 1) / qdf;
  for (uint32_t c = 0; c < nc; c++) {
    const uint64_t beta = ch[CH_BETA + c], gamma = ch[CH_GAMMA + c];
    uint64_t num[16], den[16];
    for (uint32_t k = 0; k < nchunks; k++) {
      uint64_t nn = 1, dd = 1;
      for (uint32_t j = k * qdf; j < (k + 1) * qdf && j < R; j++) {
        uint64_t wv = wires[(uint64_t)j * n + i];
        nn = gl::mul(nn, gl::add(gl::add(wv, gl::mul(beta, gl::mul(k_is[j], x))), gamma));
        dd = gl::mul(dd, gl::add(gl::add(wv, gl::mul(beta, sigmas[(uint64_t)j * n + i])), gamma));
      }
      num[k] = nn;
      den[k] = dd;
    }
    // batch inversion of den[0..nchunks)
    uint64_t pre[16], acc = 1;
    for (uint32_t k = 0; k < nchunks; k++) {
      pre[k] = acc;
      acc = gl::mul(acc, den[k]);
    }
    uint64_t inv = gl::inv(acc);
    for (uint32_t k = nchunks; k-- > 0;) {
      uint64_t t = gl::mul(inv, pre[k]);
      inv = gl::mul(inv, den[k]);
      den[k] = t;
    }
    uint64_t run = 1;
    for (uint32_t k = 0; k < nchunks; k++) {
      run = gl::mul(run, gl::mul(num[k], den[k]));
      prods[((uint64_t)c * nchunks + k) * n + i] = run;
    }
  }
}

// a^(p-2) by the addition chain of p - 2 = (2^32 - 2) 2^32 + (2^32 - 1):
// 63 squarings + 8 products (the generic gl::inv runs a 64-step
// square-and-multiply loop with a product per set bit: 125 products)
__device__ __forceinline__ uint64_t inv_chain(uint64_t x) {
  auto sq = [](uint64_t v, int k) {
#pragma unroll
    for (int i = 0; i < k; i++) v = gfn::mul(v, v);
    return v;
  };
  const uint64_t t1 = x;
  const uint64_t t2 = gfn::mul(sq(t1, 1), t1);   // x^(2^2-1)
  const uint64_t t3 = gfn::mul(sq(t2, 1), t1);   // x^(2^3-1)
  const uint64_t t6 = gfn::mul(sq(t3, 3), t3);   // x^(2^6-1)
  const uint64_t t12 = gfn::mul(sq(t6, 6), t6);  // x^(2^12-1)
  const uint64_t t24 = gfn::mul(sq(t12, 12), t12);
  const uint64_t t30 = gfn::mul(sq(t24, 6), t6);
  const uint64_t t31 = gfn::mul(sq(t30, 1), t1);  // x^(2^31-1)
  const uint64_t t32 = gfn::mul(sq(t31, 1), t1);  // x^(2^32-1)
  // x^(2^32-2) = (x^(2^31-1))^2; then shift up 32 and add 2^32-1
  return gfn::mul(sq(sq(t31, 1), 32), t32);
}

// k_pp_rows for the leaf circuits' shape (R routed wires in chunks of QDF,
// 2 challenges), compile-time so the per-row chunk values stay in registers:
// the numerator term is w + gamma + k_j (beta x) (beta x once per row), and
// the running quotient is kept as a fraction N_k / D_k (prefix products of
// the chunk numerators and denominators), so one inversion of D_last per
// challenge gives every D_k^-1 walking back (D_(k-1)^-1 = D_k^-1 den_k).
// Non-canonical arithmetic inside (field_nc.h), canonical products out.  Same
// values as k_pp_rows (plonky2 wires_permutation_partial_products_and_zs).
template <int R, int QDF>
__global__ void __launch_bounds__(256) k_pp_rows_t(const uint64_t *__restrict__ wires,
                                                   const uint64_t *__restrict__ sigmas,
                                                   const uint64_t *__restrict__ k_is,
                                                   const uint64_t *__restrict__ chal, uint64_t *__restrict__ prods,
                                                   uint32_t log_n, uint64_t w_bstride, uint64_t p_bstride,
                                                   const uint64_t *__restrict__ tw) {
  constexpr int NCH = (R + QDF - 1) / QDF;
  const uint32_t n = 1u << log_n;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = blockIdx.y;
  wires += b * w_bstride;
  prods += b * p_bstride;
  const uint64_t *ch = chal + b * CHAL_STRIDE;
  const uint64_t x = wpow_N(tw, i, log_n);
#pragma unroll 1
  for (int c = 0; c < 2; c++) {
    const uint64_t beta = ch[CH_BETA + c], gamma = ch[CH_GAMMA + c];
    const uint64_t bx = gfn::mul(beta, x);
    uint64_t N[NCH], den[NCH], D = 1;
#pragma unroll
    for (int k = 0; k < NCH; k++) {
      uint64_t nn = 1, dd = 1;
#pragma unroll
      for (int jj = 0; jj < QDF; jj++) {
        const int j = k * QDF + jj;
        if (j < R) {
          const uint64_t wg = gfn::add(wires[(uint64_t)j * n + i], gamma);
          const uint64_t nj = gfn::add(wg, gfn::mul(k_is[j], bx));
          const uint64_t dj = gfn::add(wg, gfn::mul(beta, sigmas[(uint64_t)j * n + i]));
          nn = jj ? gfn::mul(nn, nj) : nj;
          dd = jj ? gfn::mul(dd, dj) : dj;
        }
      }
      N[k] = k ? gfn::mul(N[k - 1], nn) : nn;
      den[k] = dd;
      D = k ? gfn::mul(D, dd) : dd;
    }
    uint64_t dinv = inv_chain(D);
    uint64_t *out = prods + (uint64_t)c * NCH * n + i;
#pragma unroll
    for (int k = NCH - 1; k >= 0; k--) {
      out[(uint64_t)k * n] = gfn::canon(gfn::mul(N[k], dinv));
      if (k) dinv = gfn::mul(dinv, den[k]);
    }
  }
}
template __global__ void k_pp_rows_t<80, 8>(const uint64_t *, const uint64_t *, const uint64_t *, const uint64_t *,
                                            uint64_t *, uint32_t, uint64_t, uint64_t, const uint64_t *);

// exclusive prefix product of the full-row products -> Z; pp_j = Z * P_j.
// The row products go through LDS (coalesced in, each thread's contiguous
// chunk scanned from LDS, Z written back over them), so every HBM access is a
// coalesced row sweep: n reads of the full products, (npp) reads of the
// partial products, (1 + npp) n writes per challenge.
// STAGE = true: the row products are staged in LDS (n <= 2^14); false: read
// from HBM (the degree-2^15/2^16 top aggregation circuits), Z written there
template <bool STAGE>
__global__ void __launch_bounds__(1024) k_z_scan(const uint64_t *__restrict__ prods, uint64_t *__restrict__ zs,
                                                 uint32_t log_n, uint32_t nc, uint32_t nchunks, uint64_t p_bstride,
                                                 uint64_t z_bstride) {
  extern __shared__ __attribute__((aligned(16))) uint64_t zbuf[];  // [lp(n)] rows (STAGE), then [T] partials
  const uint32_t n = 1u << log_n;
  const uint32_t c = blockIdx.x, b = blockIdx.y;
  prods += b * p_bstride + (uint64_t)c * nchunks * n;
  zs += b * z_bstride;
  const uint64_t *full = prods + (uint64_t)(nchunks - 1) * n;
  const uint32_t T = blockDim.x, t = threadIdx.x, per = (n + T - 1) / T;
  uint64_t *part = STAGE ? zbuf + nt::lp(n) : zbuf;
  // staged: row i at zbuf[lp(i)]; unstaged: Z itself is built in zs column c
  uint64_t *zc = zs + (uint64_t)c * n;
  auto row = [&](uint32_t i) -> uint64_t { return STAGE ? zbuf[nt::lp(i)] : full[i]; };
  if constexpr (STAGE) {
    for (uint32_t i = t; i < n; i += T) zbuf[nt::lp(i)] = full[i];
    __syncthreads();
  }
  const uint32_t lo = min(t * per, n), hi = min(lo + per, n);
  uint64_t local = 1;
  for (uint32_t i = lo; i < hi; i++) local = gl::mul(local, row(i));
  part[t] = local;
  __syncthreads();
  // inclusive Hillis-Steele scan over T partial products
  for (uint32_t off = 1; off < T; off <<= 1) {
    uint64_t v = t >= off ? part[t - off] : 1;
    __syncthreads();
    part[t] = gl::mul(part[t], v);
    __syncthreads();
  }
  uint64_t z = t ? part[t - 1] : 1;
  for (uint32_t i = lo; i < hi; i++) {
    const uint64_t f = row(i);
    if constexpr (STAGE) zbuf[nt::lp(i)] = z;
    else zc[i] = z;
    z = gl::mul(z, f);
  }
  __syncthreads();
  const uint32_t npp = nchunks - 1;
  for (uint32_t i = t; i < n; i += T) {
    const uint64_t zi = STAGE ? zbuf[nt::lp(i)] : zc[i];
    if constexpr (STAGE) zc[i] = zi;
    for (uint32_t j = 0; j < npp; j++) zs[((uint64_t)nc + c * npp + j) * n + i] = gl::mul(zi, prods[(uint64_t)j * n + i]);
  }
}
template __global__ void k_z_scan<true>(const uint64_t *, uint64_t *, uint32_t, uint32_t, uint32_t, uint64_t, uint64_t);
template __global__ void k_z_scan<false>(const uint64_t *, uint64_t *, uint32_t, uint32_t, uint32_t, uint64_t, uint64_t);

// ---------------------------------------------------------------- a8
//
// One lane per LDE point.  Terms are alpha-reduced as sum_i t_i alpha_c^i
// with per-proof power tables (apow, uniform across the workgroup -> scalar
// loads); a gate's constraints are summed first and multiplied by the gate's
// selector filter once.  Arithmetic is non-canonical (field_nc.h).

#define WV(j) wl[(uint64_t)(j) * N]

// two independent products (an interleaved pf::mulk<2> form measured no
// change, profiles/r03_ab_quotient_mulk.log)
__device__ __forceinline__ void mul2(uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1, uint64_t &r0, uint64_t &r1) {
  r0 = gfn::mul(a0, b0);
  r1 = gfn::mul(a1, b1);
}

// sum_i t_i alpha_c^i for both challenges, lazily reduced (gfn::Acc3: one
// reduction per sum instead of per term)
struct TermAcc {
  const uint64_t *__restrict__ p0;  // alpha_0^i
  const uint64_t *__restrict__ p1;  // alpha_1^i
  gfn::Acc3 s0, s1;
  uint32_t i;
  __device__ __forceinline__ void emit(uint64_t t) {
    s0.mac(t, p0[i]);
    s1.mac(t, p1[i]);
    i++;
  }
  __device__ __forceinline__ uint64_t sum0() const { return s0.value(); }
  __device__ __forceinline__ uint64_t sum1() const { return s1.value(); }
};

// Poseidon gate constraints (plonky2 PoseidonGate): the MDS of
// round r adds round r+1's constants (poseidon_fast.h folding), so each round
// starts with its constants already in the state.
__device__ __forceinline__ void rc_row(uint64_t k[12], int r) {
#pragma unroll
  for (int i = 0; i < 12; i++) k[i] = ps::RC_DEV[r * 12 + i];
}

// wire reader of the Poseidon gate: wires below `nstash` come from an LDS copy
// made while they streamed by (k_quotient_1r), the rest from HBM
struct WireRead {
  const uint64_t *__restrict__ wl;
  uint64_t N;
  const uint64_t *stash;  // [nstash][blockDim.x], this lane's column at stash + threadIdx.x
  uint32_t nstash;
  __device__ __forceinline__ uint64_t operator()(uint32_t j) const {
    return j < nstash ? stash[j * blockDim.x + threadIdx.x] : wl[(uint64_t)j * N];
  }
};

template <class RD>
__device__ __forceinline__ void poseidon_gate_rd(const RD &WR, TermAcc &A);

// the partial-round wire check as the grouped rounds' pre-S-box hook: lane 0
// is checked against the gate's S-box input wire and replaced by it
template <class RD>
struct QposHook {
  const RD &WR;
  TermAcc &A;
  __device__ __forceinline__ uint64_t operator()(int T, uint64_t s0) const {
    const uint64_t sb = WR(65 + T);
    A.emit(gfn::sub(s0, sb));
    return sb;
  }
};

template <int T, class RD>
__device__ __forceinline__ void qpos_partial(const RD &WR, TermAcc &A, uint64_t s[12]) {
  if constexpr (T < 22) {
    constexpr int G = (22 - T) < pf::PF_GROUP ? (22 - T) : pf::PF_GROUP;
    if constexpr (G > 1) {
      pf::partial_group<T, G>(s, QposHook<RD>{WR, A});
    } else {
      const uint64_t sb = WR(65 + T);
      A.emit(gfn::sub(s[0], sb));
      s[0] = sb;
      pf::partial_sparse<T>(s);
    }
    qpos_partial<T + G>(WR, A, s);
  }
}

__device__ __forceinline__ void poseidon_gate(const uint64_t *__restrict__ wl, uint64_t N, TermAcc &A) {
  WireRead rd{wl, N, nullptr, 0};
  poseidon_gate_rd(rd, A);
}
template <class RD>
__device__ __forceinline__ void poseidon_gate_rd(const RD &WR, TermAcc &A) {
#undef WV
#define WV(j) WR(j)
  const uint64_t swap = WV(24);
  A.emit(gfn::mul(swap, gfn::sub(swap, 1)));
  uint64_t s[12], k[12];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t delta = WV(25 + i), a = WV(i), c = WV(i + 4);
    A.emit(gfn::sub(gfn::mul(swap, gfn::sub(c, a)), delta));
    s[i] = gfn::add_c(a, delta);
    s[i + 4] = gfn::sub(c, delta);
  }
#pragma unroll
  for (int i = 8; i < 12; i++) s[i] = WV(i);
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = gfn::add_c(s[i], ps::RC_DEV[i]);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    if (r) {
#pragma unroll
      for (int i = 0; i < 12; i++) {
        const uint64_t sb = WV(29 + (r - 1) * 12 + i);
        A.emit(gfn::sub(s[i], sb));
        s[i] = sb;
      }
    }
    pf::sbox12(s);
    if (r == 3) {
      pf::mds_init_sparse(s);
    } else {
      rc_row(k, r + 1);
      pf::mds_k(s, k);
    }
  }
  // sparse partial rounds (poseidon_fast.h): lane 0 before each S-box is the
  // plain form's S-box input, so the wire checks are unchanged
  qpos_partial<0>(WR, A, s);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint64_t sb = WV(87 + r * 12 + i);
      A.emit(gfn::sub(s[i], sb));
      s[i] = sb;
    }
    pf::sbox12(s);
    if (r < 3) {
      rc_row(k, 27 + r);
      pf::mds_k(s, k);
    } else {
      pf::mds<0, -1>(s);
    }
  }
#pragma unroll
  for (int i = 0; i < 12; i++) A.emit(gfn::sub(s[i], WV(12 + i)));
#undef WV
#define WV(j) wl[(uint64_t)(j) * N]
}

// Recursive-verifier gates (the aggregator circuits, tree.rs:106-143), evaluated
// in the order of upstream plonky2's eval_unfiltered (oracle/gates_impl.h
// gate_recursion restates the same; parity unpinned).  Extension-algebra
// values are wire pairs (c0, c1) over F[Y]/(Y^2 - 7).  Generic and read-as-
// you-go: these circuits are off the Wormhole hot path.
__device__ __forceinline__ void alg_mul(uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1, uint64_t &r0,
                                        uint64_t &r1) {
  r0 = gfn::add(gfn::mul(a0, b0), gfn::mul(7, gfn::mul(a1, b1)));
  r1 = gfn::add(gfn::mul(a0, b1), gfn::mul(a1, b0));
}

// (inlined into the per-gate kernel, so TermAcc stays in registers and the
// alpha-power reads are uniform scalar loads)
__device__ __forceinline__ void recursion_gate_body(uint32_t kind, uint32_t q0, uint32_t q1, uint32_t q2,
                                                    const uint64_t *__restrict__ wl,
                                                    const uint64_t *__restrict__ gc, uint64_t N, TermAcc &A) {
  switch (kind) {
    case GK_ARITH_EXT:  // per op: multiplicand_0, multiplicand_1, addend, output
      for (uint32_t i = 0; i < q0; i++) {
        const uint32_t o = 8 * i;
        uint64_t p0, p1;
        alg_mul(WV(o), WV(o + 1), WV(o + 2), WV(o + 3), p0, p1);
        const uint64_t c0 = gc[0], c1 = gc[N];
        A.emit(gfn::sub(WV(o + 6), gfn::add(gfn::mul(p0, c0), gfn::mul(WV(o + 4), c1))));
        A.emit(gfn::sub(WV(o + 7), gfn::add(gfn::mul(p1, c0), gfn::mul(WV(o + 5), c1))));
      }
      break;
    case GK_MUL_EXT:  // per op: multiplicand_0, multiplicand_1, output
      for (uint32_t i = 0; i < q0; i++) {
        const uint32_t o = 6 * i;
        uint64_t p0, p1;
        alg_mul(WV(o), WV(o + 1), WV(o + 2), WV(o + 3), p0, p1);
        A.emit(gfn::sub(WV(o + 4), gfn::mul(p0, gc[0])));
        A.emit(gfn::sub(WV(o + 5), gfn::mul(p1, gc[0])));
      }
      break;
    case GK_REDUCING:
    case GK_REDUCING_EXT: {
      // output 0..2, alpha 2..4, old_acc 4..6, coeffs from 6, then accumulators;
      // a chunk's coefficients and accumulators are loaded before its Horner
      // steps (eight steps' reads in flight instead of one)
      const uint32_t cw = kind == GK_REDUCING ? 1 : 2, start_accs = 6 + cw * q0;
      uint64_t a0 = WV(4), a1 = WV(5);
      const uint64_t al0 = WV(2), al1 = WV(3);
      constexpr uint32_t CH = 8;
      for (uint32_t i0 = 0; i0 < q0; i0 += CH) {
        const uint32_t n = q0 - i0 < CH ? q0 - i0 : CH;
        uint64_t c0[CH], c1[CH], x0[CH], x1[CH];
#pragma unroll
        for (uint32_t k = 0; k < CH; k++)
          if (k < n) {
            const uint32_t i = i0 + k, ai = i == q0 - 1 ? 0 : start_accs + 2 * i;
            c0[k] = WV(6 + cw * i);
            c1[k] = cw == 2 ? WV(7 + 2 * i) : 0;
            x0[k] = WV(ai);
            x1[k] = WV(ai + 1);
          }
#pragma unroll
        for (uint32_t k = 0; k < CH; k++)
          if (k < n) {
            uint64_t m0, m1;
            alg_mul(a0, a1, al0, al1, m0, m1);
            m0 = gfn::add(m0, c0[k]);
            if (cw == 2) m1 = gfn::add(m1, c1[k]);
            a0 = x0[k];
            a1 = x1[k];
            A.emit(gfn::sub(m0, a0));
            A.emit(gfn::sub(m1, a1));
          }
      }
      break;
    }
    case GK_EXPONENTIATION: {  // base 0, power bits 1.. (LE), output 1+nb, intermediates 2+nb..
      const uint64_t base = WV(0);
      uint64_t prev = 1;
      for (uint32_t i = 0; i < q0; i++) {
        const uint64_t bit = WV(1 + q0 - 1 - i);
        const uint64_t comp = gfn::mul(prev, gfn::add(gfn::mul(bit, base), gfn::sub(1, bit)));
        const uint64_t iv = WV(2 + q0 + i);
        A.emit(gfn::sub(comp, iv));
        prev = gfn::mul(iv, iv);
      }
      A.emit(gfn::sub(WV(1 + q0), WV(2 + q0 + q0 - 1)));
      break;
    }
    case GK_POSEIDON_MDS: {  // inputs 0..24, outputs 24..48 (ext pairs)
      // the permutation's MDS layer (circulant + diagonal) on each coordinate
      // of the 12 extension inputs, each input read once
      uint64_t a[12], b[12];
#pragma unroll
      for (int i = 0; i < 12; i++) {
        a[i] = WV(2 * i);
        b[i] = WV(2 * i + 1);
      }
      pf::mds<0, -1>(a);
      pf::mds<0, -1>(b);
#pragma unroll
      for (int r = 0; r < 12; r++) {
        A.emit(gfn::sub(WV(24 + 2 * r), a[r]));
        A.emit(gfn::sub(WV(25 + 2 * r), b[r]));
      }
      break;
    }
    case GK_RANDOM_ACCESS: {  // q0 bits, q1 copies, q2 extra constants
      const uint32_t vec = 1u << q0, routed = (2 + vec) * q1 + q2;
      for (uint32_t cp = 0; cp < q1; cp++) {
        const uint32_t base = (2 + vec) * cp, bw = routed + cp * q0;
        for (uint32_t i = 0; i < q0; i++) {
          const uint64_t b = WV(bw + i);
          A.emit(gfn::mul(b, gfn::sub(b, 1)));
        }
        uint64_t idx = 0;
        for (uint32_t i = q0; i-- > 0;) idx = gfn::add(gfn::add(idx, idx), WV(bw + i));
        A.emit(gfn::sub(idx, WV(base)));
        // the list folded bit by bit (random_access.rs): list[i] <- b (list[2i+1] - list[2i]) + list[2i]
        uint64_t sel;
        if (q0 == RA_QBITS) {
          uint64_t list[1u << RA_QBITS];
#pragma unroll
          for (uint32_t i = 0; i < (1u << RA_QBITS); i++) list[i] = WV(base + 2 + i);
#pragma unroll
          for (uint32_t k = 0; k < RA_QBITS; k++) {
            const uint64_t b = WV(bw + k);
#pragma unroll
            for (uint32_t i = 0; i < (1u << RA_QBITS) >> (k + 1); i++)
              list[i] = gfn::add(gfn::mul(b, gfn::sub(list[2 * i + 1], list[2 * i])), list[2 * i]);
          }
          sel = list[0];
        } else {
          // other widths: sum_i item_i prod_k (bit_k(i) ? b_k : 1 - b_k), the same value
          sel = 0;
          for (uint32_t i = 0; i < vec; i++) {
            uint64_t wgt = 1;
            for (uint32_t k = 0; k < q0; k++) {
              const uint64_t b = WV(bw + k);
              wgt = gfn::mul(wgt, (i >> k) & 1 ? b : gfn::sub(1, b));
            }
            sel = gfn::add(sel, gfn::mul(wgt, WV(base + 2 + i)));
          }
        }
        A.emit(gfn::sub(sel, WV(base + 1)));
      }
      for (uint32_t i = 0; i < q2; i++) A.emit(gfn::sub(gc[(uint64_t)i * N], WV((2 + vec) * q1 + i)));
      break;
    }
    case GK_COSET_INTERP: {  // q0 subgroup bits, q1 degree
      const uint32_t np = 1u << q0, deg = q1, nint = (np - 2) / (deg - 1);
      const uint32_t sv = 1, sep = sv + 2 * np, sev = sep + 2, si = sev + 2, ssh = si + 4 * nint;
      // w_16 = 2^12 (the subgroup of the FRI arity-16 cosets), 1 / 2^k = p - (p - 1) / 2^k
      const uint64_t om = q0 == 4 ? 4096 : gl::root_of_unity(q0), inv_n = gl::P - ((gl::P - 1) >> q0);
      const uint64_t shift = WV(0), sp0 = WV(ssh), sp1 = WV(ssh + 1);
      A.emit(gfn::sub(WV(sep), gfn::mul(sp0, shift)));
      A.emit(gfn::sub(WV(sep + 1), gfn::mul(sp1, shift)));
      uint64_t e0 = 0, e1 = 0, p0 = 1, p1 = 0, x = 1;
      uint32_t lo = 0, hi = deg;
      for (uint32_t it = 0;; it++) {
        for (uint32_t i = lo; i < hi; i++) {
          // barycentric weight over the whole subgroup: 1 / prod_{j != i}(x_i - x_j) = x_i / n
          const uint64_t wt = gfn::mul(x, inv_n);
          const uint64_t t0 = gfn::sub(sp0, x), t1 = sp1;
          const uint64_t v0 = gfn::mul(WV(sv + 2 * i), wt), v1 = gfn::mul(WV(sv + 2 * i + 1), wt);
          uint64_t a0, a1, b0, b1, n0, n1;
          alg_mul(e0, e1, t0, t1, a0, a1);
          alg_mul(v0, v1, p0, p1, b0, b1);
          alg_mul(p0, p1, t0, t1, n0, n1);
          e0 = gfn::add(a0, b0);
          e1 = gfn::add(a1, b1);
          p0 = n0;
          p1 = n1;
          x = gfn::mul(x, om);
        }
        if (it == nint) break;
        const uint64_t ie0 = WV(si + 2 * it), ie1 = WV(si + 2 * it + 1);
        const uint64_t ip0 = WV(si + 2 * (nint + it)), ip1 = WV(si + 2 * (nint + it) + 1);
        A.emit(gfn::sub(ie0, e0));
        A.emit(gfn::sub(ie1, e1));
        A.emit(gfn::sub(ip0, p0));
        A.emit(gfn::sub(ip1, p1));
        e0 = ie0;
        e1 = ie1;
        p0 = ip0;
        p1 = ip1;
        lo = 1 + (deg - 1) * (it + 1);
        hi = lo + deg - 1 < np ? lo + deg - 1 : np;
      }
      A.emit(gfn::sub(WV(sev), e0));
      A.emit(gfn::sub(WV(sev + 1), e1));
      break;
    }
    default:
      break;
  }
}


// Single-read form (the default): every LDE column is read once per point,
// wires 0..23 a second time by the Poseidon gate (its inputs and outputs).
// While wires 0..R-1 stream by, the permutation checks of BOTH challenges
// (sigma columns read once), and the Constant, PublicInput, BaseSum and
// Arithmetic constraints accumulate, each term at its own alpha power (the
// alpha-weighted sums do not depend on evaluation order); then the Poseidon
// gate.  Per point: 135 + 24 wire, 84 constants/sigmas and 20 + 2 zs reads
// against 241 distinct values (a one-pass generic form that re-read the wires
// per challenge and per gate moved 3.0x the algorithmic HBM bytes,
// profiles/r01_v5_pmc_hbm_b128.json).
__device__ __forceinline__ void emit_at(const uint64_t *__restrict__ p0, const uint64_t *__restrict__ p1, uint32_t i,
                                        uint64_t t, uint64_t &s0, uint64_t &s1) {
  uint64_t m0, m1;
  mul2(t, p0[i], t, p1[i], m0, m1);
  s0 = gfn::add(s0, m0);
  s1 = gfn::add(s1, m1);
}

__device__ __forceinline__ void emit_at(const uint64_t *__restrict__ p0, const uint64_t *__restrict__ p1, uint32_t i,
                                        uint64_t t, gfn::Acc3 &s0, gfn::Acc3 &s1) {
  s0.mac(t, p0[i]);
  s1.mac(t, p1[i]);
}

// x * 2^e, 0 <= e < 64, x in [0, 2^64) -> [0, 2^64)
__device__ __forceinline__ uint64_t mul_pow2_rt(uint64_t x, uint32_t e) {
  return e ? gfn::reduce(x << e, x >> (64 - e)) : x;
}

// wires kept in LDS for the Poseidon gate: 16 x 256 lanes x 8 B = 32 KB per
// workgroup, 5 workgroups per CU (4 waves/SIMD need 4)
constexpr uint32_t QSTASH = 16, QPREFETCH = 4;
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_quotient_1r(QuotientArgs a) {
  const uint32_t logN = a.log_n + a.rate_bits;
  const uint64_t N = 1ull << logN;
  // proof index fastest in the grid: the workgroups of one block of points
  // over all proofs run together, so that block's constants/sigmas rows
  // (shared by every proof) come from L2 after the first read on each XCD
  // rather than from HBM once per proof (quotient HBM fetch -25 %, headline
  // +1.2 %: profiles/r06_ab_quotient_point_major.log)
  const uint32_t t = blockIdx.y * blockDim.x + threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (t >= N) return;
  const uint64_t *ch = a.chal + b * CHAL_STRIDE;
  const uint64_t *cs = a.cs_lde + t;                       // [ncs][N]
  const uint64_t *wl = a.w_lde + b * a.w_bstride + t;      // [W][N]
  const uint64_t *zl = a.z_lde + b * a.z_bstride;          // [nzs][N]
  const uint32_t j = gl::rev_bits(t, logN);
  uint64_t *q = a.q_out + b * a.q_bstride;
  const uint64_t *p0 = a.apow + (uint64_t)b * 2 * APOW_STRIDE, *p1 = p0 + APOW_STRIDE;
  const uint32_t R = a.R, qdf = a.qdf, nchunks = (R + qdf - 1) / qdf, npp = nchunks - 1;
  const uint32_t tn = gl::rev_bits((j + (1u << a.rate_bits)) & (uint32_t)(N - 1), logN);
  const uint32_t nsel = a.g.nsel;
  const uint64_t *gc = cs + (uint64_t)nsel * N;  // gate-constant columns
  // gates of the circuit by kind (kernel arguments: uniform)
  int g_const = -1, g_pi = -1, g_bs = -1, g_ar = -1, g_pos = -1, g_ra = -1;
  for (uint32_t gi = 0; gi < a.g.ngates; gi++) {
    switch (a.g.kind[gi]) {
      case GK_CONSTANT: g_const = (int)gi; break;
      case GK_PUBLIC_INPUT: g_pi = (int)gi; break;
      case GK_BASE_SUM: g_bs = (int)gi; break;
      case GK_ARITHMETIC: g_ar = (int)gi; break;
      case GK_POSEIDON: g_pos = (int)gi; break;
      case GK_RANDOM_ACCESS: g_ra = (int)gi; break;
      default: break;
    }
  }
  const uint32_t pre = 2 * (1 + nchunks);
  const uint32_t n_const = g_const >= 0 ? a.g.param[g_const] : 0;
  const uint32_t n_pi = g_pi >= 0 ? 4 : 0;
  const uint32_t L = g_bs >= 0 ? a.g.param[g_bs] : 0;
  const uint32_t n_ar = g_ar >= 0 ? a.g.param[g_ar] : 0;
  // vanishing terms 0..pre-1 go straight into the totals (lazily reduced sums:
  // gfn::Acc3, one reduction per sum)
  gfn::Acc3 pz0, pz1;
  const uint64_t x = a.xtab[t], l0 = a.l0tab[t];
  uint64_t z[2], prev[2];
  for (uint32_t c = 0; c < 2; c++) {
    z[c] = zl[(uint64_t)c * N + t];
    prev[c] = z[c];
    emit_at(p0, p1, c, gfn::mul(l0, gfn::sub(z[c], 1)), pz0, pz1);
  }
  // permutation factors divided by beta_c: w / beta_c + gamma_c / beta_c + s
  // (s = k_j x or sigma_j), the chunk's beta_c^len restored once per chunk
  // (CH_BETA_INV..CH_BETA_LAST): the k_j x steps are shared by both challenges
  // and the sigma values need no product (7 products per wire, not 8)
  const uint64_t binv0 = ch[CH_BETA_INV], binv1 = ch[CH_BETA_INV + 1];
  const uint64_t gamb0 = ch[CH_GAMMA_B], gamb1 = ch[CH_GAMMA_B + 1];
  uint64_t kx = x;  // k_j x, k_j = g^j
  uint64_t num0 = 1, den0 = 1, num1 = 1, den1 = 1;
  // per-gate alpha sums (multiplied by the gate's filter at the end)
  uint64_t sc0 = 0, sc1 = 0, sp0 = 0, sp1 = 0;  // 2 and 4 terms: reduced as they come
  gfn::Acc3 sb0, sb1, sa0, sa1;  // the BaseSum and Arithmetic gates' terms
  uint64_t w0 = 0, wa0 = 0, wa1 = 0, wa2 = 0;
  gfn::Acc3 bs_acc;  // sum of limb_i 2^i as a wide integer, reduced once
  // the Poseidon gate reads wires 0..23 again after the sweep: the first
  // QSTASH of them are kept in LDS (per lane, conflict-free [j][lane])
  __shared__ uint64_t stash[QSTASH * 256];
  const uint32_t nst = g_pos >= 0 ? (R < QSTASH ? R : QSTASH) : 0;
  // QPREFETCH wires and sigmas loaded ahead of the sweep (the loads of
  // iteration jj + QPREFETCH are issued before iteration jj's arithmetic)
  constexpr uint32_t PF = QPREFETCH;
  uint64_t wbuf[PF ? PF : 1], sbuf[PF ? PF : 1];
  if constexpr (PF > 0) {
#pragma unroll
    for (uint32_t i = 0; i < PF; i++) {
      wbuf[i] = i < R ? WV(i) : 0;
      sbuf[i] = i < R ? cs[(uint64_t)(a.num_constants + i) * N] : 0;
    }
  }
  for (uint32_t jj = 0; jj < R; jj++) {
    uint64_t w, sg;
    if constexpr (PF > 0) {
      w = wbuf[0];
      sg = sbuf[0];
#pragma unroll
      for (uint32_t i = 0; i + 1 < PF; i++) {
        wbuf[i] = wbuf[i + 1];
        sbuf[i] = sbuf[i + 1];
      }
      const uint32_t jn = jj + PF;
      wbuf[PF - 1] = jn < R ? WV(jn) : 0;
      sbuf[PF - 1] = jn < R ? cs[(uint64_t)(a.num_constants + jn) * N] : 0;
    } else {
      w = WV(jj);
      sg = cs[(uint64_t)(a.num_constants + jj) * N];
    }
    if (jj < nst) stash[jj * blockDim.x + threadIdx.x] = w;
    // permutation argument, both challenges
    {
      uint64_t wb0, wb1;
      mul2(w, binv0, w, binv1, wb0, wb1);
      const uint64_t wg0 = gfn::add_c(wb0, gamb0), wg1 = gfn::add_c(wb1, gamb1);
      mul2(num0, gfn::add(wg0, kx), den0, gfn::add(wg0, sg), num0, den0);
      mul2(num1, gfn::add(wg1, kx), den1, gfn::add(wg1, sg), num1, den1);
      kx = gfn::mul(kx, gl::GEN);
    }
    if ((jj + 1) % qdf == 0 || jj + 1 == R) {
      const uint32_t k = jj / qdf;
      const uint32_t bw = k == nchunks - 1 ? CH_BETA_LAST : CH_BETA_QDF;
      for (uint32_t c = 0; c < 2; c++) {
        const uint64_t nx = k == nchunks - 1 ? zl[(uint64_t)c * N + tn] : zl[((uint64_t)2 + c * npp + k) * N + t];
        const uint64_t num = c ? num1 : num0, den = c ? den1 : den0;
        const uint64_t d = gfn::sub(gfn::mul(prev[c], num), gfn::mul(nx, den));
        emit_at(p0, p1, 2 + c * nchunks + k, gfn::mul(d, ch[bw + c]), pz0, pz1);
        prev[c] = nx;
      }
      num0 = den0 = num1 = den1 = 1;
    }
    if (jj < n_const) emit_at(p0, p1, pre + jj, gfn::sub(gc[(uint64_t)jj * N], w), sc0, sc1);
    if (jj < n_pi) emit_at(p0, p1, pre + jj, gfn::sub(w, ch[CH_PIH + jj]), sp0, sp1);
    if (L) {
      if (jj == 0) {
        w0 = w;
      } else if (jj <= L) {
        bs_acc.add_shifted(w, jj - 1);
        {
          const uint64_t tb = gfn::mul(w, gfn::sub(w, 1));
          sb0.mac(tb, p0[pre + jj]);
          sb1.mac(tb, p1[pre + jj]);
        }
        if (jj == L) {
          const uint64_t tb = gfn::sub(bs_acc.value(), w0);
          sb0.mac(tb, p0[pre]);
          sb1.mac(tb, p1[pre]);
        }
      }
    }
    if (jj < 4 * n_ar) {
      switch (jj & 3) {
        case 0: wa0 = w; break;
        case 1: wa1 = w; break;
        case 2: wa2 = w; break;
        default: {
          const uint64_t comp = gfn::add(gfn::mul(gfn::mul(wa0, wa1), gc[0]), gfn::mul(wa2, gc[N]));
          emit_at(p0, p1, pre + jj / 4, gfn::sub(w, comp), sa0, sa1);
        }
      }
    }
  }
  uint64_t acc0 = pz0.value(), acc1 = pz1.value();
  // selector filters: prod_{j in group, j != gate}(j - s) * (UNUSED - s)
  auto filter = [&](int gi) -> uint64_t {
    const uint32_t si = a.g.sel_index[gi];
    const uint64_t sv = cs[(uint64_t)si * N];
    uint64_t f = 1;
    for (uint32_t jg = a.g.grp_lo[si]; jg < a.g.grp_hi[si]; jg++)
      if (jg != (uint32_t)gi) f = gfn::mul(f, gfn::sub(jg, sv));
    if (nsel > 1) f = gfn::mul(f, gfn::sub(0xFFFFFFFFull, sv));
    return f;
  };
  if (g_const >= 0) {
    const uint64_t f = filter(g_const);
    acc0 = gfn::add(acc0, gfn::mul(f, sc0));
    acc1 = gfn::add(acc1, gfn::mul(f, sc1));
  }
  if (g_pi >= 0) {
    const uint64_t f = filter(g_pi);
    acc0 = gfn::add(acc0, gfn::mul(f, sp0));
    acc1 = gfn::add(acc1, gfn::mul(f, sp1));
  }
  if (g_bs >= 0) {
    const uint64_t f = filter(g_bs);
    acc0 = gfn::add(acc0, gfn::mul(f, sb0.value()));
    acc1 = gfn::add(acc1, gfn::mul(f, sb1.value()));
  }
  if (g_ar >= 0) {
    const uint64_t f = filter(g_ar);
    acc0 = gfn::add(acc0, gfn::mul(f, sa0.value()));
    acc1 = gfn::add(acc1, gfn::mul(f, sa1.value()));
  }
  if (g_ra >= 0) {
    // RandomAccessGate (the aggregation circuits' recursive verifier): per copy
    // the bits' boolean checks, the index recomposition and the claimed
    // element against the list folded bit by bit (plonky2 random_access.rs
    // eval_unfiltered: list[i] <- b (list[2i+1] - list[2i]) + list[2i]; the
    // same multilinear value the generic kernel forms as sum_i item_i weight_i),
    // then the extra constants.  Terms in the generic kernel's order.
    // (bits = RA_QBITS: the host picks this kernel only for that width)
    constexpr uint32_t q0 = RA_QBITS, vec = 1u << RA_QBITS;
    const uint32_t q1 = a.g.param2[g_ra], q2 = a.g.param3[g_ra];
    const uint32_t routed = (2 + vec) * q1 + q2;
    uint64_t sr0 = 0, sr1 = 0;
    uint32_t k = pre;
    for (uint32_t cp = 0; cp < q1; cp++) {
      const uint32_t base = (2 + vec) * cp, bw = routed + cp * q0;
      uint64_t bits[q0];
      uint64_t idx = 0;
#pragma unroll
      for (uint32_t i = 0; i < q0; i++) {
        bits[i] = WV(bw + i);
        emit_at(p0, p1, k++, gfn::mul(bits[i], gfn::sub(bits[i], 1)), sr0, sr1);
      }
#pragma unroll
      for (int i = q0 - 1; i >= 0; i--) idx = gfn::add(gfn::add(idx, idx), bits[i]);
      emit_at(p0, p1, k++, gfn::sub(idx, WV(base)), sr0, sr1);
      uint64_t list[vec];
#pragma unroll
      for (uint32_t i = 0; i < vec; i++) list[i] = WV(base + 2 + i);
#pragma unroll
      for (uint32_t lb = 0; lb < q0; lb++) {
#pragma unroll
        for (uint32_t i = 0; i < (vec >> (lb + 1)); i++)
          list[i] = gfn::add(gfn::mul(bits[lb], gfn::sub(list[2 * i + 1], list[2 * i])), list[2 * i]);
      }
      emit_at(p0, p1, k++, gfn::sub(list[0], WV(base + 1)), sr0, sr1);
    }
    for (uint32_t i = 0; i < q2; i++) emit_at(p0, p1, k++, gfn::sub(gc[(uint64_t)i * N], WV(routed - q2 + i)), sr0, sr1);
    const uint64_t f = filter(g_ra);
    acc0 = gfn::add(acc0, gfn::mul(f, sr0));
    acc1 = gfn::add(acc1, gfn::mul(f, sr1));
  }
  if (g_pos >= 0) {
    TermAcc A;
    A.p0 = p0;
    A.p1 = p1;
    A.i = pre;
    WireRead rd{wl, N, stash, nst};
    poseidon_gate_rd(rd, A);
    const uint64_t f = filter(g_pos);
    acc0 = gfn::add(acc0, gfn::mul(f, A.sum0()));
    acc1 = gfn::add(acc1, gfn::mul(f, A.sum1()));
  }
  const uint64_t zh_inv = a.zh_inv[j & ((1u << a.rate_bits) - 1)];
  q[t] = gfn::canon(gfn::mul(acc0, zh_inv));
  q[N + t] = gfn::canon(gfn::mul(acc1, zh_inv));
}

// ---- per-gate form of the generic quotient (the default for gate lists
// outside the leaf set, i.e. the aggregation circuits).  A one-pass kernel
// evaluating every gate per point (removed; measured in round 4) re-reads the
// wires gate after gate: with 135 wires x 8 B per point and 1,024 points in
// flight per CU the working set is far beyond L2, so every gate's reads come
// from HBM again (30 GB per 32-proof level-1 launch, 6.6x the distinct
// values, 432 B of spill per lane; profiles/r04_pmc_hbm_b128.json).  Here one
// launch writes the L_0 and partial-product terms, then one launch per gate
// streams only that gate's columns and adds its filtered alpha sum to the
// point's accumulators; the last one multiplies by 1/Z_H.  Same sums (the
// alpha-weighted terms do not depend on evaluation order), so the output is
// bit-identical.  PART 0: permutation terms; 1: one non-Poseidon gate; 2: the
// Poseidon gate.
template <int PART>
__global__ void __launch_bounds__(256) k_quotient_part(QuotientArgs a, uint32_t gi, uint32_t last) {
  const uint32_t logN = a.log_n + a.rate_bits;
  const uint64_t N = 1ull << logN;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const uint32_t b = blockIdx.y;
  const uint64_t *ch = a.chal + b * CHAL_STRIDE;
  const uint64_t *cs = a.cs_lde + t;
  const uint64_t *wl = a.w_lde + b * a.w_bstride + t;
  const uint64_t *zl = a.z_lde + b * a.z_bstride;
  uint64_t *q = a.q_out + b * a.q_bstride;
  TermAcc A;
  A.p0 = a.apow + (uint64_t)b * 2 * APOW_STRIDE;
  A.p1 = A.p0 + APOW_STRIDE;
  A.i = 0;
  const uint32_t R = a.R, qdf = a.qdf, nchunks = (R + qdf - 1) / qdf, npp = nchunks - 1;
  uint64_t acc0, acc1;
  if constexpr (PART == 0) {
    const uint32_t j = gl::rev_bits(t, logN);
    const uint32_t tn = gl::rev_bits((j + (1u << a.rate_bits)) & (uint32_t)(N - 1), logN);
    const uint64_t x = a.xtab[t];
    const uint64_t l0 = a.l0tab[t];
    for (uint32_t c = 0; c < 2; c++) A.emit(gfn::mul(l0, gfn::sub(zl[(uint64_t)c * N + t], 1)));
    for (uint32_t c = 0; c < 2; c++) {
      const uint64_t beta = ch[CH_BETA + c], gamma = ch[CH_GAMMA + c];
      uint64_t bkx = gfn::mul(beta, x);
      for (uint32_t k = 0; k < nchunks; k++) {
        uint64_t num = 1, den = 1;
        for (uint32_t jj = k * qdf; jj < (k + 1) * qdf && jj < R; jj++) {
          const uint64_t wv = WV(jj);
          const uint64_t wg = gfn::add_c(wv, gamma);
          num = gfn::mul(num, gfn::add(wg, bkx));
          den = gfn::mul(den, gfn::add(wg, gfn::mul(beta, cs[(uint64_t)(a.num_constants + jj) * N])));
          bkx = gfn::mul(bkx, gl::GEN);
        }
        const uint64_t prev = k == 0 ? zl[(uint64_t)c * N + t] : zl[((uint64_t)2 + c * npp + k - 1) * N + t];
        const uint64_t next = k == nchunks - 1 ? zl[(uint64_t)c * N + tn] : zl[((uint64_t)2 + c * npp + k) * N + t];
        A.emit(gfn::sub(gfn::mul(prev, num), gfn::mul(next, den)));
      }
    }
    acc0 = A.sum0();
    acc1 = A.sum1();
  } else {
    const uint32_t kind = a.g.kind[gi];
    const uint32_t si = a.g.sel_index[gi], nsel = a.g.nsel;
    const uint64_t sv = cs[(uint64_t)si * N];
    uint64_t f = 1;
    for (uint32_t jj = a.g.grp_lo[si]; jj < a.g.grp_hi[si]; jj++)
      if (jj != gi) f = gfn::mul(f, gfn::sub(jj, sv));
    if (nsel > 1) f = gfn::mul(f, gfn::sub(0xFFFFFFFFull, sv));
    A.i = 2 * (1 + nchunks);
    const uint64_t *gc = cs + (uint64_t)nsel * N;
    if constexpr (PART == 2) {
      poseidon_gate(wl, N, A);
    } else {
      switch (kind) {
        case GK_CONSTANT:
          for (uint32_t i = 0; i < a.g.param[gi]; i++) A.emit(gfn::sub(gc[(uint64_t)i * N], WV(i)));
          break;
        case GK_PUBLIC_INPUT:
          for (uint32_t i = 0; i < 4; i++) A.emit(gfn::sub(WV(i), ch[CH_PIH + i]));
          break;
        case GK_BASE_SUM: {
          // each limb read once, high limb first in chunks: the sum by Horner
          // and the limb's boolean check at its own alpha index (i0 + 1 + i)
          const uint32_t L = a.g.param[gi], i0 = A.i;
          constexpr uint32_t CH = 8;
          uint64_t acc = 0;
          for (uint32_t hi = L; hi > 0;) {
            const uint32_t n = hi < CH ? hi : CH;
            uint64_t l[CH];
#pragma unroll
            for (uint32_t k = 0; k < CH; k++)
              if (k < n) l[k] = WV(hi - k);  // limb hi - 1 - k is wire hi - k
#pragma unroll
            for (uint32_t k = 0; k < CH; k++)
              if (k < n) {
                acc = gfn::add(gfn::add(acc, acc), l[k]);
                A.i = i0 + hi - k;
                A.emit(gfn::mul(l[k], gfn::sub(l[k], 1)));
              }
            hi -= n;
          }
          A.i = i0;
          A.emit(gfn::sub(acc, WV(0)));
          A.i = i0 + 1 + L;
          break;
        }
        case GK_ARITHMETIC:
          for (uint32_t i = 0; i < a.g.param[gi]; i++) {
            const uint64_t comp = gfn::add(gfn::mul(gfn::mul(WV(4 * i), WV(4 * i + 1)), gc[0]),
                                           gfn::mul(WV(4 * i + 2), gc[N]));
            A.emit(gfn::sub(WV(4 * i + 3), comp));
          }
          break;
        default:
          recursion_gate_body(kind, a.g.param[gi], a.g.param2[gi], a.g.param3[gi], wl, gc, N, A);
          break;
      }
    }
    acc0 = gfn::add(q[t], gfn::mul(f, A.sum0()));
    acc1 = gfn::add(q[N + t], gfn::mul(f, A.sum1()));
  }
  if (last) {
    const uint32_t j = gl::rev_bits(t, logN);
    const uint64_t zh_inv = a.zh_inv[j & ((1u << a.rate_bits) - 1)];
    q[t] = gfn::canon(gfn::mul(acc0, zh_inv));
    q[N + t] = gfn::canon(gfn::mul(acc1, zh_inv));
  } else {
    q[t] = acc0;
    q[N + t] = acc1;
  }
}
// ---- k_quotient_prefix: the permutation terms and every gate of gmask that
// reads routed wires only (Constant, PublicInput, BaseSum, Arithmetic,
// ArithmeticExtension, MulExtension) in ONE pass over windows of QP_WIN routed
// wires held in registers, where k_quotient_part<0> and one launch per gate read
// the routed wires up to seven times and round-trip both accumulators through
// HBM per gate.  Each term keeps its own alpha index and each gate's sum is
// multiplied by its filter, so the result is the same field element (the sums
// do not depend on evaluation order): bit-identical.  The other gates follow
// as k_quotient_part launches.  QDF: the permutation chunk (quotient degree
// factor), a divisor of QP_WIN, so windows hold whole chunks and whole ops.
constexpr uint32_t QP_WIN = 24;  // multiple of 4 (Arithmetic), 6 (MulExtension), 8 (ArithmeticExtension, chunks)
template <int QDF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_quotient_prefix(QuotientArgs a, uint32_t gmask, uint32_t last) {
  static_assert(QP_WIN % QDF == 0, "windows hold whole permutation chunks");
  const uint32_t logN = a.log_n + a.rate_bits;
  const uint64_t N = 1ull << logN;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const uint32_t b = blockIdx.y;
  const uint64_t *ch = a.chal + b * CHAL_STRIDE;
  const uint64_t *cs = a.cs_lde + t;
  const uint64_t *wl = a.w_lde + b * a.w_bstride + t;
  const uint64_t *zl = a.z_lde + b * a.z_bstride;
  uint64_t *q = a.q_out + b * a.q_bstride;
  const uint64_t *__restrict__ p0 = a.apow + (uint64_t)b * 2 * APOW_STRIDE;
  const uint64_t *__restrict__ p1 = p0 + APOW_STRIDE;
  const uint32_t R = a.R, nchunks = (R + QDF - 1) / QDF, npp = nchunks - 1;
  const uint32_t gb = 2 * (1 + nchunks);  // alpha index of every gate's constraint 0
  int gi_c = -1, gi_pi = -1, gi_bs = -1, gi_ar = -1, gi_ae = -1, gi_me = -1;
  for (uint32_t gi = 0; gi < a.g.ngates; gi++)
    if ((gmask >> gi) & 1) switch (a.g.kind[gi]) {
        case GK_CONSTANT: gi_c = (int)gi; break;
        case GK_PUBLIC_INPUT: gi_pi = (int)gi; break;
        case GK_BASE_SUM: gi_bs = (int)gi; break;
        case GK_ARITHMETIC: gi_ar = (int)gi; break;
        case GK_ARITH_EXT: gi_ae = (int)gi; break;
        case GK_MUL_EXT: gi_me = (int)gi; break;
        default: break;
      }
  const uint32_t n_c = gi_c >= 0 ? a.g.param[gi_c] : 0, n_bs = gi_bs >= 0 ? a.g.param[gi_bs] : 0;
  const uint32_t n_ar = gi_ar >= 0 ? a.g.param[gi_ar] : 0, n_ae = gi_ae >= 0 ? a.g.param[gi_ae] : 0;
  const uint32_t n_me = gi_me >= 0 ? a.g.param[gi_me] : 0;
  // one accumulator pair: a gate's terms enter multiplied by its selector
  // filter, prod over the gate's group of (j - s), j != gate, times (UNUSED -
  // s) with several groups (per-gate sums would hold 12 more registers)
  gfn::Acc3 lz0, lz1;  // lazily reduced (gfn::Acc3)
  auto emit = [&](uint32_t i, uint64_t term) {
    lz0.mac(term, p0[i]);
    lz1.mac(term, p1[i]);
  };
  auto filter = [&](int gi) -> uint64_t {
    if (gi < 0) return 0;
    const uint32_t si = a.g.sel_index[gi];
    const uint64_t sv = cs[(uint64_t)si * N];
    uint64_t f = 1;
    for (uint32_t jj = a.g.grp_lo[si]; jj < a.g.grp_hi[si]; jj++)
      if (jj != (uint32_t)gi) f = gfn::mul(f, gfn::sub(jj, sv));
    if (a.g.nsel > 1) f = gfn::mul(f, gfn::sub(0xFFFFFFFFull, sv));
    return f;
  };
  const uint64_t f_c = filter(gi_c), f_pi = filter(gi_pi), f_bs = filter(gi_bs), f_ar = filter(gi_ar),
                 f_ae = filter(gi_ae), f_me = filter(gi_me);
  const uint32_t jn = gl::rev_bits(t, logN);
  const uint32_t tn = gl::rev_bits((jn + (1u << a.rate_bits)) & (uint32_t)(N - 1), logN);
  const uint64_t x = a.xtab[t], l0 = a.l0tab[t];
  emit(0, gfn::mul(l0, gfn::sub(zl[t], 1)));
  emit(1, gfn::mul(l0, gfn::sub(zl[N + t], 1)));
  const uint64_t *gc = cs + (uint64_t)a.g.nsel * N;
  const bool need_k0 = gi_c >= 0 || gi_ar >= 0 || gi_ae >= 0 || gi_me >= 0;
  const bool need_k1 = (gi_c >= 0 && n_c > 1) || gi_ar >= 0 || gi_ae >= 0;
  const uint64_t k0 = need_k0 ? gc[0] : 0, k1 = need_k1 ? gc[N] : 0;
  // permutation factors divided by beta_c, as k_quotient_1r (CH_BETA_INV..)
  const uint64_t binv0 = ch[CH_BETA_INV], binv1 = ch[CH_BETA_INV + 1];
  const uint64_t gam0 = ch[CH_GAMMA_B], gam1 = ch[CH_GAMMA_B + 1];
  uint64_t kx = x;
  uint64_t bs_acc = 0, bs_pw = 1, wire0 = 0, bss0 = 0, bss1 = 0;
  for (uint32_t base = 0; base < R; base += QP_WIN) {
    const uint32_t nw = R - base < QP_WIN ? R - base : QP_WIN;
    uint64_t w[QP_WIN];
#pragma unroll
    for (uint32_t k = 0; k < QP_WIN; k++) w[k] = k < nw ? WV(base + k) : 0;
    if (base == 0) {
      wire0 = w[0];
      if (gi_c >= 0 && n_c > 0) emit(gb, gfn::mul(f_c, gfn::sub(k0, w[0])));
      if (gi_c >= 0 && n_c > 1) emit(gb + 1, gfn::mul(f_c, gfn::sub(k1, w[1])));
      if (gi_pi >= 0) {
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) emit(gb + i, gfn::mul(f_pi, gfn::sub(w[i], ch[CH_PIH + i])));
      }
    }
    // permutation: the window's chunks of QDF wires
#pragma unroll
    for (uint32_t c = 0; c < QP_WIN; c += QDF) {
      if (c >= nw) break;
      const uint32_t k = (base + c) / QDF;
      uint64_t num0 = 1, den0 = 1, num1 = 1, den1 = 1;
#pragma unroll
      for (uint32_t i = 0; i < QDF; i++) {
        if (c + i >= nw) break;
        const uint64_t s = cs[(uint64_t)(a.num_constants + base + c + i) * N];
        const uint64_t wg0 = gfn::add_c(gfn::mul(w[c + i], binv0), gam0);
        const uint64_t wg1 = gfn::add_c(gfn::mul(w[c + i], binv1), gam1);
        num0 = gfn::mul(num0, gfn::add(wg0, kx));
        num1 = gfn::mul(num1, gfn::add(wg1, kx));
        den0 = gfn::mul(den0, gfn::add(wg0, s));
        den1 = gfn::mul(den1, gfn::add(wg1, s));
        kx = gfn::mul(kx, gl::GEN);
      }
      const uint32_t bw = k == nchunks - 1 ? CH_BETA_LAST : CH_BETA_QDF;
#pragma unroll
      for (uint32_t cc = 0; cc < 2; cc++) {
        const uint64_t prev = k == 0 ? zl[(uint64_t)cc * N + t] : zl[((uint64_t)2 + cc * npp + k - 1) * N + t];
        const uint64_t next = k == nchunks - 1 ? zl[(uint64_t)cc * N + tn] : zl[((uint64_t)2 + cc * npp + k) * N + t];
        emit(2 + cc * nchunks + k,
             gfn::mul(gfn::sub(gfn::mul(prev, cc ? num1 : num0), gfn::mul(next, cc ? den1 : den0)), ch[bw + cc]));
      }
    }
    // Arithmetic ops (4 wires), ArithmeticExtension ops (8), MulExtension ops (6)
#pragma unroll
    for (uint32_t o = 0; o < QP_WIN; o += 4) {
      const uint32_t op = (base + o) / 4;
      if (o < nw && op < n_ar)
        emit(gb + op, gfn::mul(f_ar, gfn::sub(w[o + 3], gfn::add(gfn::mul(gfn::mul(w[o], w[o + 1]), k0),
                                                                  gfn::mul(w[o + 2], k1)))));
    }
#pragma unroll
    for (uint32_t o = 0; o < QP_WIN; o += 8) {
      const uint32_t op = (base + o) / 8;
      if (o < nw && op < n_ae) {
        uint64_t m0, m1;
        alg_mul(w[o], w[o + 1], w[o + 2], w[o + 3], m0, m1);
        emit(gb + 2 * op, gfn::mul(f_ae, gfn::sub(w[o + 6], gfn::add(gfn::mul(m0, k0), gfn::mul(w[o + 4], k1)))));
        emit(gb + 2 * op + 1,
             gfn::mul(f_ae, gfn::sub(w[o + 7], gfn::add(gfn::mul(m1, k0), gfn::mul(w[o + 5], k1)))));
      }
    }
#pragma unroll
    for (uint32_t o = 0; o < QP_WIN; o += 6) {
      const uint32_t op = (base + o) / 6;
      if (o < nw && op < n_me) {
        uint64_t m0, m1;
        alg_mul(w[o], w[o + 1], w[o + 2], w[o + 3], m0, m1);
        emit(gb + 2 * op, gfn::mul(f_me, gfn::sub(w[o + 4], gfn::mul(m0, k0))));
        emit(gb + 2 * op + 1, gfn::mul(f_me, gfn::sub(w[o + 5], gfn::mul(m1, k0))));
      }
    }
    // BaseSum limbs (wires 1..n_bs): range checks at 1 + limb into their own
    // sum (one filter product at the end), the limb sum by Horner over the
    // window's limbs from the top, then scaled by 2^(the window's lowest limb)
    if (gi_bs >= 0 && base < n_bs + 1) {
      uint64_t h = 0;
#pragma unroll
      for (int k = QP_WIN - 1; k >= 0; k--) {
        const uint32_t wi = base + k;
        if ((uint32_t)k < nw && wi >= 1 && wi <= n_bs) {
          uint64_t m0, m1;
          const uint64_t tm = gfn::mul(w[k], gfn::sub(w[k], 1));
          mul2(tm, p0[gb + wi], tm, p1[gb + wi], m0, m1);
          bss0 = gfn::add(bss0, m0);
          bss1 = gfn::add(bss1, m1);
          h = gfn::add(gfn::add(h, h), w[k]);
        }
      }
      bs_acc = gfn::add(bs_acc, gfn::mul(h, bs_pw));
      bs_pw = gfn::mul(bs_pw, 1ull << (base == 0 ? QP_WIN - 1 : QP_WIN));  // 2^(first limb of the next window)
    }
  }
  uint64_t acc0 = lz0.value(), acc1 = lz1.value();
  if (gi_bs >= 0) {
    uint64_t m0, m1, d = gfn::sub(bs_acc, wire0);
    mul2(d, p0[gb], d, p1[gb], m0, m1);
    acc0 = gfn::add(acc0, gfn::mul(f_bs, gfn::add(bss0, m0)));
    acc1 = gfn::add(acc1, gfn::mul(f_bs, gfn::add(bss1, m1)));
  }
  if (last) {
    const uint64_t zh_inv = a.zh_inv[jn & ((1u << a.rate_bits) - 1)];
    q[t] = gfn::canon(gfn::mul(acc0, zh_inv));
    q[N + t] = gfn::canon(gfn::mul(acc1, zh_inv));
  } else {
    q[t] = acc0;
    q[N + t] = acc1;
  }
}
template __global__ void k_quotient_prefix<8>(QuotientArgs, uint32_t, uint32_t);

template __global__ void k_quotient_part<0>(QuotientArgs, uint32_t, uint32_t);
template __global__ void k_quotient_part<1>(QuotientArgs, uint32_t, uint32_t);
template __global__ void k_quotient_part<2>(QuotientArgs, uint32_t, uint32_t);

#undef WV

// coset iNTT, stage 1: block s' holds coset s = rev_r(s') values in bit-reversed
// order; produce C^s_k = iNTT_n(block)_k * (g w_N^s)^-k   (scaled by 1/n)
__global__ void __launch_bounds__(512) k_qintt_blocks(const uint64_t *__restrict__ vals, uint64_t *__restrict__ out,
                                                      uint32_t log_n, uint32_t rate_bits, uint64_t v_bstride,
                                                      uint64_t o_bstride, const uint64_t *__restrict__ tw,
                                                      const uint64_t *__restrict__ pt_inv, uint64_t n_inv,
                                                      uint64_t ginv) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t n = 1u << log_n, logN = log_n + rate_bits;
  const uint32_t sp = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
  const uint32_t s = gl::rev_bits(sp, rate_bits);
  const uint64_t N = (uint64_t)n << rate_bits;
  const uint64_t *src = vals + b * v_bstride + c * N + ((uint64_t)sp << log_n);
  for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) lds[nt::lp(gl::rev_bits(p, log_n))] = src[p];
  __syncthreads();
  nt::ntt_lds<true>(lds, log_n, pt_inv);
  // base^-1 = g^-1 w_N^-s
  const uint64_t wNs = wpow_N(tw, s, logN);
  const uint64_t binv = gl::mul(ginv, gl::inv(wNs));
  uint64_t f = gl::mul(gl::pow(binv, threadIdx.x), n_inv);
  const uint64_t step = gl::pow(binv, blockDim.x);
  uint64_t *dst = out + b * o_bstride + ((uint64_t)c << rate_bits) * n + (uint64_t)s * n;
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
    dst[k] = gl::mul(lds[nt::lp(gl::rev_bits(k, log_n))], f);
    f = gl::mul(f, step);
  }
}

// coset iNTT stage 1 for n > 2^14: block sp (coset s = rev_r(sp), values in
// bit-reversed order) gathered into natural order at block s of out; the
// caller then runs the inverse DIF in place (dif_big) and the bit-reversal
// scaled by base^-k / n (bitrev_scale), as k_qintt_blocks does in LDS
__global__ void __launch_bounds__(256) k_qintt_gather_big(const uint64_t *__restrict__ vals, uint64_t *__restrict__ out,
                                                          uint32_t log_n, uint32_t rate_bits, uint64_t v_bstride,
                                                          uint64_t o_bstride) {
  const uint32_t n = 1u << log_n, B = 1u << rate_bits, c = blockIdx.y / B, sp = blockIdx.y % B;
  const uint32_t s = gl::rev_bits(sp, rate_bits);
  const uint64_t N = (uint64_t)n << rate_bits;
  const uint64_t *src = vals + blockIdx.z * v_bstride + c * N + ((uint64_t)sp << log_n);
  uint64_t *dst = out + blockIdx.z * o_bstride + ((uint64_t)c << rate_bits) * n + (uint64_t)s * n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    dst[i] = src[gl::rev_bits(i, log_n)];
}

// coset iNTT, stage 2: e_j = (1/2^r) sum_s C^s_k w_{2^r}^{-sj}; a_{k+jn} = e_j g^{-jn}
__global__ void __launch_bounds__(256) k_qintt_radix(const uint64_t *__restrict__ cbuf, uint64_t *__restrict__ coeffs,
                                                     uint32_t log_n, uint32_t rate_bits, uint64_t c_bstride,
                                                     uint64_t o_bstride, uint64_t winv_r, uint64_t r_inv,
                                                     uint64_t gninv) {
  const uint32_t n = 1u << log_n, B = 1u << rate_bits;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t c = blockIdx.y, b = blockIdx.z;
  const uint64_t *src = cbuf + b * c_bstride + (uint64_t)c * B * n + k;
  uint64_t C[16];
  for (uint32_t s = 0; s < B; s++) C[s] = src[(uint64_t)s * n];
  uint64_t *dst = coeffs + b * o_bstride + (uint64_t)c * B * n + k;
  uint64_t gj = r_inv;  // (1/B) g^{-jn}
  uint64_t wj = 1;      // w_B^{-j}
  for (uint32_t jj = 0; jj < B; jj++) {
    uint64_t e = 0, wsj = 1;
    for (uint32_t s = 0; s < B; s++) {
      e = gl::add(e, gl::mul(C[s], wsj));
      wsj = gl::mul(wsj, wj);
    }
    dst[(uint64_t)jj * n] = gl::mul(e, gj);
    gj = gl::mul(gj, gninv);
    wj = gl::mul(wj, winv_r);
  }
}

// ---- compute_quotient_polys as launches, shared by the prover's stage 3 and
// the qp_quotient seam (any 2^6 <= n <= 2^15: the coset iNTT takes its LDS or
// its large-n form by size)
void quotient_values(const QuotientArgs &a, QuotientKernel k, uint32_t nb, hipStream_t s) {
  const uint64_t N = 1ull << (a.log_n + a.rate_bits);
  const dim3 qg((unsigned)((N + 255) / 256), nb);
  switch (k) {
    case QK_PARTS: {
      // the permutation terms with the gates that read only routed wires
      // (k_quotient_prefix: one pass; path hook qprefix=0 turns it off), then
      // one launch per other gate (each streams only its gate's columns), the
      // last multiplying by 1/Z_H
      uint32_t gmask = 0;
      if (a.qdf == 8 && path_opt("qprefix", 1))
        for (uint32_t gi = 0; gi < a.g.ngates; gi++) {
          const uint32_t p = a.g.param[gi];
          uint64_t wires = ~0ull;
          switch (a.g.kind[gi]) {
            case GK_CONSTANT: wires = p <= 2 ? p : ~0ull; break;
            case GK_PUBLIC_INPUT: wires = 4; break;
            case GK_BASE_SUM: wires = 1ull + p; break;
            case GK_ARITHMETIC: wires = 4ull * p; break;
            case GK_ARITH_EXT: wires = 8ull * p; break;
            case GK_MUL_EXT: wires = 6ull * p; break;
            default: break;
          }
          if (wires <= a.R) gmask |= 1u << gi;
        }
      int lastg = -1;
      for (uint32_t gi = 0; gi < a.g.ngates; gi++)
        if (a.g.kind[gi] != GK_NOOP && !((gmask >> gi) & 1)) lastg = (int)gi;
      if (gmask) k_quotient_prefix<8><<<qg, 256, 0, s>>>(a, gmask, lastg < 0);
      else k_quotient_part<0><<<qg, 256, 0, s>>>(a, 0, lastg < 0);
      for (uint32_t gi = 0; gi < a.g.ngates; gi++) {
        if (a.g.kind[gi] == GK_NOOP || ((gmask >> gi) & 1)) continue;
        const uint32_t l = (int)gi == lastg;
        if (a.g.kind[gi] == GK_POSEIDON) k_quotient_part<2><<<qg, 256, 0, s>>>(a, gi, l);
        else k_quotient_part<1><<<qg, 256, 0, s>>>(a, gi, l);
      }
      break;
    }
    case QK_1R: k_quotient_1r<<<dim3(nb, qg.x), 256, 0, s>>>(a); break;
  }
}

void quotient_coeffs(const Twiddles &tw, const uint64_t *qvals, uint64_t *cbuf, uint64_t *coeffs, uint32_t log_n,
                     uint32_t rate_bits, uint32_t nc, uint32_t nb, uint64_t v_bstride, uint64_t c_bstride,
                     uint64_t o_bstride, hipStream_t s) {
  const uint64_t n = 1ull << log_n;
  const uint32_t B = 1u << rate_bits;
  const uint64_t n_inv = gl::inv(n), ginv = gl::inv(gl::GEN);
  if (log_n <= LDS_LOG_MAX) {
    k_qintt_blocks<<<dim3(B, nc, nb), 512, 8u * ntt_lds_words(1u << log_n), s>>>(qvals, cbuf, log_n, rate_bits,
                                                                                v_bstride, c_bstride, tw.fwd,
                                                                                tw.pt_inv, n_inv, ginv);
  } else {
    // n > 2^14: gather each coset block into natural order, inverse DIF in
    // place, then per coset the bit-reversal scaled by (g w_N^s)^-k / n
    k_qintt_gather_big<<<dim3(64, nc * B, nb), 256, 0, s>>>(qvals, cbuf, log_n, rate_bits, v_bstride, c_bstride);
    dif_big(tw, cbuf, (uint64_t)B * n, nc, B, n, log_n, true, nb, c_bstride, s);
    const uint64_t wN = gl::root_of_unity(log_n + rate_bits);
    for (uint32_t sc = 0; sc < B; sc++)
      bitrev_scale(cbuf + (uint64_t)sc * n, (uint64_t)B * n, nc, log_n, n_inv, gl::mul(ginv, gl::inv(gl::pow(wN, sc))),
                   nb, c_bstride, s);
  }
  k_qintt_radix<<<dim3((unsigned)((n + 255) / 256), nc, nb), 256, 0, s>>>(
      cbuf, coeffs, log_n, rate_bits, c_bstride, o_bstride, gl::inv(gl::root_of_unity(rate_bits)), gl::inv(B),
      gl::inv(gl::pow(gl::GEN, n)));
}

// ---------------------------------------------------------------- a10

// value of each coefficient column at an extension point: out[b][poly].
// A block evaluates OPEN_PB polys of one proof: thread t walks k = t + jT with
// one running power z^k shared by the OPEN_PB columns (2 base products per
// coefficient instead of 6), then a tree reduction per poly.  blockDim = T
// (host: 256, or n/4 >= 64 for small circuits so z^t's pow stays amortised).
__global__ void __launch_bounds__(256) k_openings(const uint64_t *__restrict__ coeffs, uint64_t c_bstride,
                                                  uint32_t npolys, uint32_t log_n, const uint64_t *__restrict__ pts,
                                                  uint32_t pt_off, uint64_t *__restrict__ out, uint32_t out_off) {
  __shared__ ext red[OPEN_PB][256];
  const uint32_t n = 1u << log_n, T = blockDim.x, t = threadIdx.x;
  const uint32_t p0 = blockIdx.x * OPEN_PB, b = blockIdx.y;
  const uint32_t np = min((uint32_t)OPEN_PB, npolys - p0);
  const uint64_t *cf = coeffs + b * c_bstride + (uint64_t)p0 * n;
  const ext z = ext{pts[b * CHAL_STRIDE + pt_off], pts[b * CHAL_STRIDE + pt_off + 1]};
  ext zp = gl::ext_pow(z, t);
  const ext zs = gl::ext_pow(z, T);
  ext acc[OPEN_PB];
#pragma unroll
  for (int j = 0; j < OPEN_PB; j++) acc[j] = ext{0, 0};
  for (uint32_t k = t; k < n; k += T) {
#pragma unroll
    for (int j = 0; j < OPEN_PB; j++)
      if ((uint32_t)j < np) acc[j] = gl::ext_add(acc[j], gl::ext_scale(zp, cf[(uint64_t)j * n + k]));
    zp = gl::ext_mul(zp, zs);
  }
#pragma unroll
  for (int j = 0; j < OPEN_PB; j++) red[j][t] = acc[j];
  __syncthreads();
  for (uint32_t o = T / 2; o; o >>= 1) {
    if (t < o)
      for (uint32_t j = 0; j < np; j++) red[j][t] = gl::ext_add(red[j][t], red[j][t + o]);
    __syncthreads();
  }
  if (t < np) {
    uint64_t *dst = out + b * OPEN_STRIDE + 2 * (out_off + p0 + t);
    dst[0] = red[t][0].c0;
    dst[1] = red[t][0].c1;
  }
}

// all of a proof's opening batches in one launch: segment j's polys form
// groups of OPEN_PB from group g0; each group's coefficient range splits into
// S slices of n / S (a small batch otherwise leaves most CUs idle: one proof
// has ~33 groups), whose partial sums k_openings_reduce adds (S > 1)
__global__ void __launch_bounds__(256) k_openings_seg(OpeningsArgs a) {
  __shared__ ext red[OPEN_PB][256];
  const uint32_t n = 1u << a.log_n, T = blockDim.x, t = threadIdx.x;
  const uint32_t g = blockIdx.x / a.S, slice = blockIdx.x % a.S, b = blockIdx.y;
  uint32_t j = 0;
  while (j + 1 < a.nseg && g >= a.seg[j + 1].g0) j++;
  const OpenSeg sg = a.seg[j];
  const uint32_t p0 = (g - sg.g0) * OPEN_PB;
  const uint32_t np = min((uint32_t)OPEN_PB, sg.npolys - p0);
  const uint32_t len = n / a.S, lo = slice * len;
  const uint64_t *cf = sg.coeffs + b * sg.c_bstride + (uint64_t)p0 * n;
  const ext z = ext{a.pts[b * CHAL_STRIDE + sg.pt_off], a.pts[b * CHAL_STRIDE + sg.pt_off + 1]};
  ext zp = gl::ext_pow(z, lo + t);
  const ext zs = gl::ext_pow(z, T);
  ext acc[OPEN_PB];
#pragma unroll
  for (int q = 0; q < OPEN_PB; q++) acc[q] = ext{0, 0};
  for (uint32_t k = lo + t; k < lo + len; k += T) {
#pragma unroll
    for (int q = 0; q < OPEN_PB; q++)
      if ((uint32_t)q < np) acc[q] = gl::ext_add(acc[q], gl::ext_scale(zp, cf[(uint64_t)q * n + k]));
    zp = gl::ext_mul(zp, zs);
  }
#pragma unroll
  for (int q = 0; q < OPEN_PB; q++) red[q][t] = acc[q];
  __syncthreads();
  for (uint32_t o = T / 2; o; o >>= 1) {
    if (t < o)
      for (uint32_t q = 0; q < np; q++) red[q][t] = gl::ext_add(red[q][t], red[q][t + o]);
    __syncthreads();
  }
  if (t < np) {
    const uint32_t idx = sg.out_off + p0 + t;
    uint64_t *dst = a.S == 1 ? a.out + b * OPEN_STRIDE + 2 * idx
                             : a.part + ((uint64_t)(b * a.S + slice) * OPEN_STRIDE + 2 * idx);
    dst[0] = red[t][0].c0;
    dst[1] = red[t][0].c1;
  }
}

__global__ void __launch_bounds__(256) k_openings_reduce(const uint64_t *__restrict__ part, uint64_t *__restrict__ out,
                                                         uint32_t ntot, uint32_t S) {
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (idx >= ntot) return;
  ext acc{0, 0};
  for (uint32_t sl = 0; sl < S; sl++) {
    const uint64_t *p = part + (uint64_t)(b * S + sl) * OPEN_STRIDE + 2 * idx;
    acc = gl::ext_add(acc, ext{p[0], p[1]});
  }
  out[b * OPEN_STRIDE + 2 * idx] = acc.c0;
  out[b * OPEN_STRIDE + 2 * idx + 1] = acc.c1;
}

void openings(OpeningsArgs a, uint32_t nb, hipStream_t s) {
  const uint32_t n = 1u << a.log_n;
  const unsigned T = (unsigned)std::min<uint32_t>(256, std::max<uint32_t>(64, n / 4));
  a.ngroups = 0;
  a.ntot = 0;
  for (uint32_t j = 0; j < a.nseg; j++) {
    a.seg[j].g0 = a.ngroups;
    a.ngroups += (a.seg[j].npolys + OPEN_PB - 1) / OPEN_PB;
    a.ntot = std::max(a.ntot, a.seg[j].out_off + a.seg[j].npolys);
  }
  // path hook open_slices=1: one block per group (the shape of the large batches)
  const uint32_t smax = (uint32_t)std::min<long>(std::max<long>(path_opt("open_slices", OPEN_MAX_SLICES), 1),
                                                 OPEN_MAX_SLICES);
  a.S = 1;
  while (a.S * 2 <= smax && a.S * 2 * T * 8 <= n && (uint64_t)a.ngroups * nb * a.S < 1024) a.S *= 2;
  k_openings_seg<<<dim3(a.ngroups * a.S, nb), T, 0, s>>>(a);
  if (a.S > 1) k_openings_reduce<<<dim3((a.ntot + 255) / 256, nb), 256, 0, s>>>(a.part, a.out, a.ntot, a.S);
}

// ---------------------------------------------------------------- a11

// comp[k] = sum_j alpha^j c_j[k] over the listed oracles (Horner, reverse order)
__global__ void __launch_bounds__(256) k_fri_compose(FriComposeArgs a) {
  const uint32_t n = 1u << a.log_n;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t b = blockIdx.y;
  const uint64_t *ch = a.chal + b * CHAL_STRIDE;
  const ext al{ch[CH_FRI_ALPHA], ch[CH_FRI_ALPHA + 1]};
  ext acc{0, 0};
  for (int o = (int)a.noracles - 1; o >= 0; o--) {
    const uint64_t *base = a.coeffs[o] + b * a.bstride[o] + k;
    for (uint32_t p = a.npolys[o]; p-- > 0;) acc = gl::ext_add(gl::ext_mul(acc, al), ext{base[(uint64_t)p * n], 0});
  }
  ext acc2{0, 0};
  const uint64_t *zb = a.coeffs[2] + b * a.bstride[2] + k;
  for (uint32_t p = a.nnext; p-- > 0;) acc2 = gl::ext_add(gl::ext_mul(acc2, al), ext{zb[(uint64_t)p * n], 0});
  uint64_t *o1 = a.comp + b * (4ull * n);
  o1[k] = acc.c0;
  o1[n + k] = acc.c1;
  o1[2 * n + k] = acc2.c0;
  o1[3 * n + k] = acc2.c1;
}

// suffix-scan form of divide_by_linear: q_{k-1} = sum_{i>=k} c_i z^{i-k}
//   = z^{-k} S_k with S_k = sum_{i>=k} c_i z^i; final = alpha^nc Q1 + Q2
// MAXPER: n / blockDim.x values per thread (16 up to n = 2^14; 64 for the
// degree-2^15/2^16 top aggregation circuits, whose arrays live in scratch)
template <int MAXPER>
__global__ void __launch_bounds__(1024) k_fri_divide(const uint64_t *__restrict__ comp, uint64_t *__restrict__ fin,
                                                     uint32_t log_n, const uint64_t *__restrict__ chal,
                                                     uint64_t f_bstride, uint64_t f_cstride) {
  __shared__ ext sh[1024];
  const uint32_t n = 1u << log_n, b = blockIdx.x;
  const uint64_t *ch = chal + b * CHAL_STRIDE;
  const uint32_t T = blockDim.x, per = n / T;
  const uint32_t lo = threadIdx.x * per;
  ext res[MAXPER];
  for (int pass = 0; pass < 2; pass++) {
    const uint64_t *cc = comp + b * (4ull * n) + (uint64_t)pass * 2 * n;
    const ext z{ch[pass ? CH_ZETA_NEXT : CH_ZETA], ch[(pass ? CH_ZETA_NEXT : CH_ZETA) + 1]};
    const ext zi{ch[pass ? CH_ZETA_NEXT_INV : CH_ZETA_INV], ch[(pass ? CH_ZETA_NEXT_INV : CH_ZETA_INV) + 1]};
    // local suffix sums within [lo, lo+per) of d_i = c_i z^i
    ext zp = gl::ext_pow(z, lo);
    ext d[MAXPER];
    for (uint32_t i = 0; i < per; i++) {
      d[i] = gl::ext_mul(ext{cc[lo + i], cc[n + lo + i]}, zp);
      zp = gl::ext_mul(zp, z);
    }
    ext tot{0, 0};
    for (uint32_t i = per; i-- > 0;) {
      tot = gl::ext_add(tot, d[i]);
      d[i] = tot;
    }
    sh[threadIdx.x] = tot;
    __syncthreads();
    // inclusive suffix scan across threads
    for (uint32_t off = 1; off < T; off <<= 1) {
      ext v = threadIdx.x + off < T ? sh[threadIdx.x + off] : ext{0, 0};
      __syncthreads();
      sh[threadIdx.x] = gl::ext_add(sh[threadIdx.x], v);
      __syncthreads();
    }
    const ext after = threadIdx.x + 1 < T ? sh[threadIdx.x + 1] : ext{0, 0};
    __syncthreads();
    // q_{k-1} = z^{-k} (S_k) for k >= 1; output index m = k-1; q_{n-1} = 0 (padding)
    ext zk = gl::ext_pow(zi, lo);
    for (uint32_t i = 0; i < per; i++) {
      const uint32_t k = lo + i;
      ext q = gl::ext_mul(gl::ext_add(d[i], after), zk);  // S_k z^-k = q_{k-1}
      zk = gl::ext_mul(zk, zi);
      if (pass == 0) {
        res[i] = q;
      } else {
        res[i] = gl::ext_add(res[i], q);
      }
      (void)k;
    }
    if (pass == 0) {
      const ext ap{ch[CH_ALPHA_POW_NC], ch[CH_ALPHA_POW_NC + 1]};
      for (uint32_t i = 0; i < per; i++) res[i] = gl::ext_mul(res[i], ap);
    }
  }
  // res[i] at k = lo+i holds q_{k-1}; shift down by one, q_{n-1} = 0
  uint64_t *o = fin + b * f_bstride;
  for (uint32_t i = 0; i < per; i++) {
    const uint32_t k = lo + i;
    if (k == 0) continue;
    o[k - 1] = res[i].c0;
    o[f_cstride + k - 1] = res[i].c1;
  }
  if (threadIdx.x == T - 1) {
    o[n - 1] = 0;
    o[f_cstride + n - 1] = 0;
  }
}
template __global__ void k_fri_divide<16>(const uint64_t *, uint64_t *, uint32_t, const uint64_t *, uint64_t, uint64_t);
template __global__ void k_fri_divide<64>(const uint64_t *, uint64_t *, uint32_t, const uint64_t *, uint64_t, uint64_t);

// FRI layer leaves: leaf i = 2^ab consecutive leaf-order ext values, interleaved c0,c1
__global__ void __launch_bounds__(256) k_fri_leaf(const uint64_t *__restrict__ vals, uint64_t *__restrict__ dig,
                                                  uint32_t log_len, uint32_t ab, uint64_t v_bstride, uint64_t d_bstride) {
  const uint32_t nleaves = 1u << (log_len - ab);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nleaves) return;
  const uint32_t b = blockIdx.y;
  const uint64_t L = 1ull << log_len;
  const uint64_t *c0 = vals + b * v_bstride + ((uint64_t)i << ab);
  const uint64_t *c1 = c0 + L;
  const uint32_t W = 2u << ab;
  uint64_t *o = dig + b * d_bstride + (uint64_t)i * 4;
  if (W <= 4) {  // hash_or_noop: a leaf of <= 4 elements is its own digest (arity 2)
    o[0] = psd::canon(c0[0]); o[1] = psd::canon(c1[0]); o[2] = psd::canon(c0[1]); o[3] = psd::canon(c1[1]);
    return;
  }
  uint64_t s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t off = 0; off < W; off += 8) {
#pragma unroll
    for (uint32_t k = 0; k < 8; k += 2) {
      const uint32_t e = (off + k) >> 1;
      if (off + k < W) {
        s[k] = c0[e];
        s[k + 1] = c1[e];
      }
    }
    psd::permute_nc(s);
  }
  o[0] = psd::canon(s[0]); o[1] = psd::canon(s[1]); o[2] = psd::canon(s[2]); o[3] = psd::canon(s[3]);
}

// k_fri_leaf with one 16-lane row per leaf (pc::permute_row): a layer of few
// leaves (small batches, the upper FRI layers) otherwise costs a one-lane
// permutation's latency per absorbed chunk whatever its width
__global__ void __launch_bounds__(256) k_fri_leaf_row(const uint64_t *__restrict__ vals, uint64_t *__restrict__ dig,
                                                      uint32_t log_len, uint32_t ab, uint64_t v_bstride,
                                                      uint64_t d_bstride) {
  const uint32_t i = blockIdx.x * 16 + (threadIdx.x >> 4), l16 = threadIdx.x & 15;
  if (i >= (1u << (log_len - ab))) return;
  const uint32_t b = blockIdx.y;
  const uint64_t L = 1ull << log_len;
  const uint64_t *c0 = vals + b * v_bstride + ((uint64_t)i << ab);
  const uint32_t W = 2u << ab;  // > 4 (the launcher sends arity 2 to k_fri_leaf)
  uint64_t x = 0;
  for (uint32_t off = 0; off < W; off += 8) {
    const uint32_t e = off + l16;  // element e: c0/c1 of value e >> 1
    if (l16 < 8 && e < W) x = (e & 1 ? c0 + L : c0)[e >> 1];
    x = pc::permute_row(x);
  }
  if (l16 < 4) dig[b * d_bstride + (uint64_t)i * 4 + l16] = psd::canon(x);
}

// leaves of a FRI layer: the row form up to FRI_ROW_MAX leaves over the
// batch (path hook fri_row), the one-lane form above
constexpr long FRI_ROW_MAX = 16384;
void fri_leaf(const uint64_t *vals, uint64_t *dig, uint32_t log_len, uint32_t ab, uint64_t v_bstride,
              uint64_t d_bstride, uint32_t nb, hipStream_t s) {
  const uint64_t lim = (uint64_t)path_opt("fri_row", FRI_ROW_MAX);
  const uint64_t nl = 1ull << (log_len - ab);
  if ((2u << ab) > 4 && nl * nb <= lim)
    k_fri_leaf_row<<<dim3((unsigned)((nl + 15) / 16), nb), 256, 0, s>>>(vals, dig, log_len, ab, v_bstride, d_bstride);
  else
    k_fri_leaf<<<dim3((unsigned)((nl + 255) / 256), nb), 256, 0, s>>>(vals, dig, log_len, ab, v_bstride, d_bstride);
}

// fold: out[k] = sum_{i<2^ab} beta^i c[2^ab k + i]  (coefficients, ext as 2 columns).
// Only the first 2^log_nz input coefficients can be nonzero (the layer-0
// polynomial has degree < n in a length-N buffer): outputs past them are
// written as zeros without reading the zero tail.
__global__ void __launch_bounds__(256) k_fold(const uint64_t *__restrict__ cin, uint64_t *__restrict__ cout,
                                              uint32_t log_len, uint32_t ab, uint32_t layer,
                                              const uint64_t *__restrict__ chal, uint64_t i_bstride,
                                              uint64_t o_bstride, uint32_t log_nz) {
  const uint32_t nout = 1u << (log_len - ab);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nout) return;
  const uint32_t b = blockIdx.y;
  uint64_t *o = cout + b * o_bstride;
  if (((uint64_t)k << ab) >= (1ull << log_nz)) {
    o[k] = 0;
    o[nout + k] = 0;
    return;
  }
  const uint64_t *ch = chal + b * CHAL_STRIDE;
  const ext beta{ch[CH_FRI_BETA + 2 * layer], ch[CH_FRI_BETA + 2 * layer + 1]};
  const uint64_t L = 1ull << log_len;
  const uint64_t *c0 = cin + b * i_bstride, *c1 = c0 + L;
  ext acc{0, 0};
  for (uint32_t i = 1u << ab; i-- > 0;) {
    const uint64_t idx = ((uint64_t)k << ab) + i;
    acc = gl::ext_add(gl::ext_mul(acc, beta), ext{c0[idx], c1[idx]});
  }
  o[k] = acc.c0;
  o[nout + k] = acc.c1;
}

// ---------------------------------------------------------------- a12

// Minimal witness, one launch for all proofs.  Candidates of proof b are
// claimed in blocks of 256 from a per-proof counter (next[b], increasing), so
// every block below the best hit is claimed while that hit is still unknown
// and gets tested: the final found[b] is the minimal witness.  A workgroup
// keeps claiming blocks of one proof until the claimed block starts at or
// above found[b] (or at limit), then moves to the next proof, so the stragglers
// of the geometric search get every workgroup of the grid.  limit bounds every
// loop (16 PoW bits: no hit below 2^36 has probability exp(-2^20)).
__device__ __forceinline__ bool pow_hit(const uint64_t *__restrict__ pre, uint32_t pos, uint64_t cand, uint32_t bits) {
  const uint64_t y = pf::sbox(pf::add_c(cand, ps::RC_DEV[pos]));
  const uint32_t y0 = pf::lo32(y), y1 = pf::hi32(y);
  uint64_t s[12];
#pragma unroll
  for (int r = 0; r < 12; r++) {
    const uint32_t c = (uint32_t)pre[12 + r];
    s[r] = pf::reduce_row((uint64_t)y0 * c + (pre[r] & pf::EPS), (uint64_t)y1 * c + (pre[r] >> 32));
  }
  pf::rounds<QP_POSEIDON_MODE, 1, 0x80u>(s);  // only lane 7 is read
  return (psd::canon(s[7]) >> (64 - bits)) == 0;
}

// one candidate per thread per claimed block of 256 (2 or 4 per thread and
// per-wave claims measured no better: profiles/r05_ab_pow_cpt.log,
// r05_ab_pow_wave.log)
__global__ void __launch_bounds__(256) k_pow_scan(const uint64_t *__restrict__ states, const uint32_t *__restrict__ pos,
                                                  uint64_t *__restrict__ found, uint64_t *__restrict__ next, uint32_t nb,
                                                  uint32_t bits, uint64_t limit) {
  constexpr uint64_t BLK = 256;
  __shared__ uint64_t blk;
  __shared__ uint32_t done;
  for (uint32_t i = 0; i < nb; i++) {
    const uint32_t b = (blockIdx.x + i) % nb;
    const uint64_t *pre = states + b * 24;
    for (;;) {
      if (threadIdx.x == 0) {
        const uint64_t k = atomicAdd((unsigned long long *)(next + b), 1ull);
        blk = k;
        done = k * BLK >= limit || k * BLK >= *(const volatile uint64_t *)(found + b);
      }
      __syncthreads();
      const uint64_t k = blk;
      const uint32_t d = done;
      __syncthreads();  // every lane has read blk / done before lane 0 rewrites them
      if (d) break;
      const uint64_t cand = k * BLK + threadIdx.x;
      if (pow_hit(pre, pos[b], cand, bits)) atomicMin((unsigned long long *)(found + b), (unsigned long long)cand);
    }
  }
}
// ---------------------------------------------------------------- gathers

// out[b][q][c] = cols[b*bstride + c*stride + idx[b][q] >> shift]
__global__ void k_gather_rows_b(const uint64_t *__restrict__ cols, uint64_t stride, uint64_t bstride, uint32_t ncols,
                                const uint32_t *__restrict__ idx, uint32_t nq, uint32_t shift,
                                uint64_t *__restrict__ out, uint64_t o_bstride) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = blockIdx.y;
  if (t >= ncols * nq) return;
  const uint32_t q = t / ncols, c = t % ncols;
  out[b * o_bstride + t] = cols[b * bstride + (uint64_t)c * stride + (idx[b * nq + q] >> shift)];
}

// out[b][q][k][4] = sibling digest at level k of leaf idx[b][q] >> shift
__global__ void k_gather_paths_b(const uint64_t *__restrict__ dig, uint64_t d_bstride, uint32_t log_leaves,
                                 uint32_t cap_h, const uint32_t *__restrict__ idx, uint32_t nq, uint32_t shift,
                                 uint64_t *__restrict__ out, uint64_t o_bstride) {
  const uint32_t depth = log_leaves - cap_h;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = blockIdx.y;
  if (t >= nq * depth * 4) return;
  const uint32_t q = t / (depth * 4), r = t % (depth * 4), k = r / 4, e = r % 4;
  uint64_t off = 0;
  for (uint32_t j = 0; j < k; j++) off += (uint64_t)1 << (log_leaves - j);
  const uint64_t leaf = idx[b * nq + q] >> shift;
  const uint64_t sib = (leaf >> k) ^ 1u;
  out[b * o_bstride + t] = dig[b * d_bstride + (off + sib) * 4 + e];
}

// FRI layer leaves for queries: out[b][q][2*arity] interleaved from 2 columns
__global__ void k_gather_fri_leaf(const uint64_t *__restrict__ vals, uint64_t v_bstride, uint32_t log_len, uint32_t ab,
                                  const uint32_t *__restrict__ idx, uint32_t nq, uint32_t shift,
                                  uint64_t *__restrict__ out, uint64_t o_bstride) {
  const uint32_t W = 2u << ab;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = blockIdx.y;
  if (t >= nq * W) return;
  const uint32_t q = t / W, e = t % W;
  const uint64_t leaf = idx[b * nq + q] >> shift;
  const uint64_t L = 1ull << log_len;
  out[b * o_bstride + t] = vals[b * v_bstride + (e & 1) * L + (leaf << ab) + (e >> 1)];
}

}  // namespace qpk
