// ntt.hip — Goldilocks radix-2 NTT kernels for gfx950 (plonky2 field/fft.rs
// semantics: ifft / coset LDE).
//
// Design (MI355X): every transform the prover needs is built from size-n
// (n <= 2^14) NTTs that live entirely in one workgroup's LDS (n*8 <= 128 KiB
// of the 160 KiB), so HBM sees each element once in and once out:
//   * LDE n -> N = n*2^r is 2^r independent size-n NTTs of the coefficients
//     scaled by (g*w_N^s)^k, s < 2^r (no zero-padded size-N transform);
//     DIF leaves block s in bit-reversed order, which is exactly Merkle-leaf
//     order at rows rev_r(s)*n + p.
//   * ifft is a DIF with inverse twiddles and a bit-reversed LDS read on store.
#include <stdlib.h>
#include <vector>
#include "field.h"
#include "kernels.h"
#include "ntt_device.h"
#include "ntt16.h"
#include "paths.h"

// occupancy target of the LDS NTT kernels (64 KiB LDS per size-2^13 workgroup
// allows 2 workgroups = 4 waves per SIMD; uncapped, the compiler spends ~165
// VGPRs and only one workgroup fits per CU)
#define QP_NTT_OCC __attribute__((amdgpu_waves_per_eu(4)))

namespace qpk {

__global__ void k_twiddles(uint64_t *fwd, uint64_t *inv, uint64_t w, uint64_t wi, uint32_t half) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < half) {
    // see kernels.h tw_get: even powers first, then odd ones
    const uint32_t e = j < half / 2 ? 2 * j : 2 * (j - half / 2) + 1;
    fwd[j] = gl::pow(w, e);
    inv[j] = gl::pow(wi, e);
  }
}

// pass twiddles (kernels.h Twiddles::pt_*): entry i of the concatenated
// tables, looked up in the power table so the values are the ones the
// gathers read before
__global__ void k_pass_twiddles(uint64_t *pt, const uint64_t *__restrict__ tw, uint32_t total) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint32_t L = 31 - __builtin_clz(i + 16u), loc = i + 16u - (1u << L), log_q = L - 4;
  const uint32_t m = loc >> log_q, t = loc & ((1u << log_q) - 1);
  pt[i] = nt::tw_pow(tw, t * nt::brev4(m), L);
}

// merged first-pass twiddles of k_lde_cosets for one (log_n, rate)
__global__ void k_merged_twiddles(uint64_t *mtw, const uint64_t *__restrict__ tw, uint32_t log_n, uint32_t rate_bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, log_T = log_n - 4, logN = log_n + rate_bits;
  if (i >= (1u << logN)) return;
  const uint32_t t = i & ((1u << log_T) - 1), sm = i >> log_T, s = sm >> 4, m = sm & 15;
  mtw[i] = nt::tw_pow(tw, t * (s + (nt::brev4(m) << rate_bits)), logN);
}

hipError_t twiddles_init(Twiddles &t, hipStream_t s) {
  uint32_t half = 1u << (TW_LOG - 1);
  hipError_t e = hipMalloc(&t.fwd, half * 8ull);
  if (e) return e;
  e = hipMalloc(&t.inv, half * 8ull);
  if (e) return e;
  uint64_t w = gl::root_of_unity(TW_LOG);
  k_twiddles<<<(half + 255) / 256, 256, 0, s>>>(t.fwd, t.inv, w, gl::inv(w), half);
  e = hipGetLastError();
  if (e) return e;
  // coset pre-twists of k_lde_cosets
  std::vector<uint64_t> ptw(ptw_offset(LDE_MAX_RATE + 1));
  for (uint32_t r = 1; r <= LDE_MAX_RATE; r++) {
    const uint64_t wr = gl::root_of_unity(4 + r);
    for (uint32_t sc = 0; sc < (1u << r); sc++)
      for (uint32_t m = 0; m < 16; m++) ptw[ptw_offset(r) + 16 * sc + m] = gl::pow(wr, (uint64_t)sc * m);
  }
  e = hipMalloc(&t.ptw, ptw.size() * 8);
  if (e) return e;
  e = hipMemcpyAsync(t.ptw, ptw.data(), ptw.size() * 8, hipMemcpyHostToDevice, s);
  if (e) return e;
  const uint32_t npt = pt_offset(TW_LOG + 1);
  if ((e = hipMalloc(&t.pt_fwd, npt * 8ull)) || (e = hipMalloc(&t.pt_inv, npt * 8ull))) return e;
  k_pass_twiddles<<<(npt + 255) / 256, 256, 0, s>>>(t.pt_fwd, t.fwd, npt);
  k_pass_twiddles<<<(npt + 255) / 256, 256, 0, s>>>(t.pt_inv, t.inv, npt);
  uint64_t nm = 0;
  for (uint32_t ln = LDE_COSETS_MIN_LOG; ln <= LDE_COSETS_MAX_LOG; ln++)
    for (uint32_t r = 1; r <= LDE_MAX_RATE && ln + r <= TW_LOG; r++) {
      t.mtw_off[ln][r] = nm;
      nm += 1ull << (ln + r);
    }
  if ((e = hipMalloc(&t.mtw, nm * 8))) return e;
  for (uint32_t ln = LDE_COSETS_MIN_LOG; ln <= LDE_COSETS_MAX_LOG; ln++)
    for (uint32_t r = 1; r <= LDE_MAX_RATE && ln + r <= TW_LOG; r++)
      k_merged_twiddles<<<((1u << (ln + r)) + 255) / 256, 256, 0, s>>>(t.mtw + t.mtw_off[ln][r], t.fwd, ln, r);
  if ((e = hipGetLastError())) return e;
  return hipStreamSynchronize(s);
}

void twiddles_free(Twiddles &t) {
  if (t.fwd) (void)hipFree(t.fwd);
  if (t.inv) (void)hipFree(t.inv);
  if (t.ptw) (void)hipFree(t.ptw);
  if (t.pt_fwd) (void)hipFree(t.pt_fwd);
  if (t.pt_inv) (void)hipFree(t.pt_inv);
  if (t.mtw) (void)hipFree(t.mtw);
  t.fwd = t.inv = t.ptw = t.pt_fwd = t.pt_inv = t.mtw = nullptr;
}

__global__ void __launch_bounds__(512) QP_NTT_OCC k_intt(const uint64_t *__restrict__ in, uint64_t in_stride,
                                              uint64_t *__restrict__ out, uint64_t out_stride, uint32_t log_n,
                                              uint64_t n_inv, const uint64_t *__restrict__ pt_inv,
                                              uint64_t in_bstride, uint64_t out_bstride) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t n = 1u << log_n;
  const uint64_t *src = in + blockIdx.y * in_bstride + (uint64_t)blockIdx.x * in_stride;
  uint64_t *dst = out + blockIdx.y * out_bstride + (uint64_t)blockIdx.x * out_stride;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) lds[nt::lp(i)] = src[i];
  __syncthreads();
  nt::ntt_lds<true>(lds, log_n, pt_inv);
  for (uint32_t m = threadIdx.x; m < n; m += blockDim.x) dst[m] = gl::mul(lds[nt::lp(gl::rev_bits(m, log_n))], n_inv);
}

__global__ void __launch_bounds__(512) QP_NTT_OCC k_lde(const uint64_t *__restrict__ coeffs, uint64_t c_stride,
                                             uint64_t *__restrict__ out, uint64_t o_stride, uint32_t log_n,
                                             uint32_t rate_bits, uint64_t shift, const uint64_t *__restrict__ tw,
                                             const uint64_t *__restrict__ pt, uint64_t c_bstride, uint64_t o_bstride) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t n = 1u << log_n;
  const uint32_t s = blockIdx.x;        // coset index
  const uint32_t col = blockIdx.y;
  const uint64_t *src = coeffs + blockIdx.z * c_bstride + (uint64_t)col * c_stride;
  uint64_t *dst = out + blockIdx.z * o_bstride + (uint64_t)col * o_stride +
                  ((uint64_t)gl::rev_bits(s, rate_bits) << log_n);
  // base = shift * w_N^s ; element k scaled by base^k
  const uint64_t wN = tw_get(tw, s << (TW_LOG - log_n - rate_bits));
  const uint64_t base = gl::mul(shift, wN);
  uint64_t f = gl::pow(base, threadIdx.x);
  const uint64_t step = gl::pow(base, blockDim.x);
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
    lds[nt::lp(k)] = gl::mul(src[k], f);
    f = gl::mul(f, step);
  }
  __syncthreads();
  nt::ntt_lds<false>(lds, log_n, pt);
  for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) dst[p] = nt::canon(lds[nt::lp(p)]);
}

// Coset-fused LDE: one workgroup per column produces all B = 2^r cosets, so
// the n coefficients are read from HBM once (the per-coset kernel above reads
// them B times) and scaled by shift^k once.  n = 16 T (T = 2^LOG_T threads):
// thread t holds a_m = c_{t+Tm} shift^{t+Tm}, m < 16, in registers -- exactly
// the inputs of its first radix-16 DIF butterfly.  For coset s the inputs are
// a_m w_N^{s(t+Tm)} = a_m w_N^{st} w_{16B}^{sm}: the registers are multiplied
// by w_{16B}^{sm} (ptw) before the 16-point DFT and by the merged twiddle
// w_N^{t(s + B brev4(m))} (mtw: N words per (log_n, r), read from L2 by every
// column's workgroup) after it.  The remaining levels run in LDS; output rows
// in leaf order.
//   * twiddle products one at a time (nt::mul_rows<0>), not as interleaved
//     triples: fewer live temporaries at the 128-VGPR cap (72 -> 48 B of spill
//     per lane; 4.33 -> 4.18 ms per 86-proof launch, profiles/r04_lde_ab.log)
//   * the last LDE_ALDS shifted coefficients in LDS past the transform
//     (12 KB per 8192-point workgroup: 2 still fit per CU); spill 48 -> 12 B
//     per lane, 4.11 -> 4.06 ms per 86-proof launch (profiles/r04_lde_ab.log)
//   * n = 2^13: the last two passes wave-local (two workgroup barriers per
//     coset instead of four), the closing barrier after the next coset's
//     register work (profiles/r05_ab_lde_wavelocal.log)
//   * factored first-pass tables (coset steps and pass twiddles, held in
//     registers or re-read) measured slower: 701 vs 548 us per 64-column
//     launch at n = 2^13 (profiles/r04_lde_ab.log); so did a radix-8 form at
//     twice the threads (4.63 vs 4.48 ms per 64-proof launch: LDS stalls,
//     profiles/r02_ab_lde_radix8.log)
constexpr int LDE_ALDS = 3;
template <int LOG_T>
__global__ void __launch_bounds__(1 << LOG_T) QP_NTT_OCC k_lde_cosets(const uint64_t *__restrict__ coeffs, uint64_t c_stride,
                                                          uint64_t c_bstride, uint64_t *__restrict__ out,
                                                          uint64_t o_stride, uint64_t o_bstride, uint32_t rate_bits,
                                                          uint64_t shift, uint64_t shift_T,
                                                          const uint64_t *__restrict__ mtw,
                                                          const uint64_t *__restrict__ pt,
                                                          const uint64_t *__restrict__ ptw) {
  constexpr uint32_t T = 1u << LOG_T, LOG_N = LOG_T + 4;
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t t = threadIdx.x;
  const uint64_t *src = coeffs + blockIdx.y * c_bstride + (uint64_t)blockIdx.x * c_stride;
  uint64_t *dst0 = out + blockIdx.y * o_bstride + (uint64_t)blockIdx.x * o_stride;
  uint64_t a[16];
#pragma unroll
  for (int m = 0; m < 16; m++) a[m] = src[t + T * m];
  {
    uint64_t f = gl::pow(shift, t);
#pragma unroll
    for (int m = 0; m < 16; m++) {
      a[m] = nt::mul(a[m], f);
      f = nt::mul(f, shift_T);
    }
  }
  const uint32_t B = 1u << rate_bits;
  const uint64_t *pw = ptw + ptw_offset(rate_bits);
  // the last LDE_ALDS shifted coefficients live in LDS past the transform's
  // words instead of VGPRs across the coset loop (the launch adds their bytes)
  uint64_t *alds = lds + ntt_lds_words(1u << LOG_N);
  if constexpr (LDE_ALDS > 0) {
#pragma unroll
    for (int m = 16 - LDE_ALDS; m < 16; m++) alds[(m - (16 - LDE_ALDS)) * T + t] = a[m];
  }
  for (uint32_t s = 0; s < B; s++) {
    uint64_t r[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      r[m] = m >= 16 - LDE_ALDS ? alds[(m - (16 - LDE_ALDS)) * T + t] : a[m];
    nt::mul_rows<0>(r, [&](int m) { return pw[16 * s + m]; });
    nt::dft16<false>(r);
    // merged twiddles w_N^{t(s + B brev4(m))}: row (s, m) of the table, lane t
    // (a product by w^0 = 1 returns its input unchanged)
    const uint64_t *ms = mtw + (uint64_t)16 * T * s + t;
    if (s) r[0] = nt::mul(r[0], ms[0]);
    nt::mul_rows<0>(r, [&](int m) { return ms[T * m]; });
    // wave-local tail: the barrier that keeps this coset's writes from
    // overtaking other waves' reads of the previous coset's words sits here,
    // after this wave's registers are ready, so a wave that finished its
    // stores early transforms the next coset's 16 values instead of idling
    if constexpr (LOG_N == 13 && LOG_T == 9)
      if (s) __syncthreads();
#pragma unroll
    for (int m = 0; m < 16; m++) lds[nt::lp(t) + nt::lp(T * m)] = r[m];
    __syncthreads();
    if constexpr (LOG_N == 13 && LOG_T == 9) {
      // n = 2^13, T = 512: after the cross-wave pass (stride-32 groups of each
      // 512-element block) wave w holds elements [1024 w, 1024 w + 1024), so the
      // stride-2 pass and the last radix-2 level run on the wave's own LDS
      // words: in-order LDS within a wave, no workgroup barrier between them
      const uint32_t lane = t & 63, w = t >> 6;
      {
        const uint32_t sp = t >> 5, tt = t & 31;  // n / 16 == T groups: one per thread
        uint64_t *base = lds + nt::lp((sp << 9) + tt);
        uint64_t q[16];
#pragma unroll
        for (int m = 0; m < 16; m++) q[m] = base[nt::lp(m * 32)];
        nt::dft16<false>(q);
        if (tt) {
          const uint64_t *ptS = pt + pt_offset(9) + tt;
          nt::mul_rows<0>(q, [&](int m) { return ptS[m * 32]; });
        }
#pragma unroll
        for (int m = 0; m < 16; m++) base[nt::lp(m * 32)] = q[m];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      {
        // the stride-2 pass (twiddles w_32^{tt brev4(m)}: shifts) on the wave's 32
        // blocks of 32, lanes 0..31 the even halves, 32..63 the odd ones
        const uint32_t b32 = 32 * w + (lane & 31), tt = lane >> 5;
        uint64_t *base = lds + nt::lp((b32 << 5) + tt);
        uint64_t q[16];
#pragma unroll
        for (int m = 0; m < 16; m++) q[m] = base[nt::lp(2 * m)];
        nt::dft16<false>(q);
        if (tt) {
#pragma unroll
          for (int m = 1; m < 16; m++) q[m] = nt::mul_w32<false>(q[m], (int)nt::brev4(m));
        }
#pragma unroll
        for (int m = 0; m < 16; m++) base[nt::lp(2 * m)] = q[m];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint64_t *dst = dst0 + ((uint64_t)gl::rev_bits(s, rate_bits) << LOG_N);
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        const uint32_t g0 = 1024 * w + 2 * (lane + 64 * k);
        uint64_t q[2] = {lds[nt::lp(g0)], lds[nt::lp(g0 + 1)]};
        nt::tail_group<false, 1>(q);
        dst[g0] = nt::canon(q[0]);
        dst[g0 + 1] = nt::canon(q[1]);
      }
      continue;
    }
    // the last radix-2^g levels (g = LOG_N mod 4) run in the store loop: each
    // thread takes 16 / 2^g groups of 2^g contiguous values, transforms them in
    // registers and stores them contiguously (leaf order = DIF order)
    constexpr uint32_t G = LOG_N % 4;
    // the LDS passes (launched with T threads) leave exactly the G levels the
    // store loop runs
    static_assert(nt::lds_levels_left(LOG_N, LOG_T, T) == G, "LDS passes and the store loop disagree");
    nt::ntt_lds_from<false, false, 0>(lds, LOG_N, LOG_T, pt);
    uint64_t *dst = dst0 + ((uint64_t)gl::rev_bits(s, rate_bits) << LOG_N);
    if constexpr (G == 0) {
#pragma unroll
      for (int m = 0; m < 16; m++) dst[t + T * m] = nt::canon(lds[nt::lp(t) + nt::lp(T * m)]);
    } else {
      constexpr uint32_t S = 1u << G;
#pragma unroll
      for (uint32_t k = 0; k < 16 / S; k++) {
        const uint32_t g0 = (t + T * k) * S;  // group start: n / S groups over T threads
        uint64_t r[S];
#pragma unroll
        for (uint32_t e = 0; e < S; e++) r[e] = lds[nt::lp(g0 + e)];
        nt::tail_group<false, G>(r);
#pragma unroll
        for (uint32_t e = 0; e < S; e++) dst[g0 + e] = nt::canon(r[e]);
      }
    }
    __syncthreads();
  }
}

// ---- transforms beyond one workgroup's LDS (n = 2^15, 2^16: the top levels
// of a 2048-leaf aggregation tree register every leaf's public inputs and
// need 2^15 rows).  A DIF's levels of half-width H >= 2^LDS_LOG_MAX pair
// elements across 2^14-blocks: those run as one HBM pass each
// (x_j, x_{j+H} -> x_j + x_{j+H}, (x_j - x_{j+H}) w_{2H}^{j mod H}); the
// remaining 14 levels are the blocks' own size-2^14 DIFs, in LDS with the
// same pass tables as every other NTT.  Off the Wormhole hot path (one or two
// proofs per tree), so the HBM levels are plain radix-2.

// one radix-2 DIF level of half-width 2^log_h over columns of 2^log_n values
__global__ void __launch_bounds__(256) k_dif_level(uint64_t *x, uint64_t c_stride, uint32_t nsub, uint64_t nsub_stride,
                                                   uint64_t bstride, uint32_t log_n, uint32_t log_h,
                                                   const uint64_t *__restrict__ tw) {
  const uint32_t col = blockIdx.y / nsub, sub = blockIdx.y % nsub;
  uint64_t *v = x + blockIdx.z * bstride + (uint64_t)col * c_stride + (uint64_t)sub * nsub_stride;
  const uint64_t half = 1ull << (log_n - 1), H = 1ull << log_h;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < half; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t off = j & (H - 1), i0 = ((j >> log_h) << (log_h + 1)) + off, i1 = i0 + H;
    const uint64_t a = v[i0], b = v[i1];
    v[i0] = gl::add(a, b);
    v[i1] = gl::mul(gl::sub(a, b), nt::tw_pow(tw, (uint32_t)off, log_h + 1));
  }
}

// the size-2^LDS_LOG_MAX DIF of every block, in place (canonical out)
template <bool INV>
__global__ void __launch_bounds__(512) QP_NTT_OCC k_dif_blocks(uint64_t *x, uint64_t c_stride, uint32_t nsub,
                                                               uint64_t nsub_stride, uint64_t bstride,
                                                               const uint64_t *__restrict__ pt) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  constexpr uint32_t M = 1u << LDS_LOG_MAX;
  const uint32_t col = blockIdx.y / nsub, sub = blockIdx.y % nsub;
  uint64_t *v = x + blockIdx.z * bstride + (uint64_t)col * c_stride + (uint64_t)sub * nsub_stride +
                ((uint64_t)blockIdx.x << LDS_LOG_MAX);
  for (uint32_t i = threadIdx.x; i < M; i += blockDim.x) lds[nt::lp(i)] = v[i];
  __syncthreads();
  nt::ntt_lds<INV>(lds, LDS_LOG_MAX, pt);
  for (uint32_t i = threadIdx.x; i < M; i += blockDim.x) v[i] = nt::canon(lds[nt::lp(i)]);
}

// in place: x[k] <- x[rev(k)] * c0 * base^k (pairs k < rev(k) swapped by one thread)
__global__ void __launch_bounds__(256) k_bitrev_scale(uint64_t *x, uint64_t stride, uint32_t log_n, uint64_t c0,
                                                      uint64_t base, uint64_t bstride) {
  uint64_t *v = x + blockIdx.z * bstride + (uint64_t)blockIdx.y * stride;
  const uint32_t n = 1u << log_n, gs = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gs) {
    const uint32_t r = gl::rev_bits(k, log_n);
    if (r < k) continue;
    const uint64_t fk = base == 1 ? c0 : gl::mul(c0, gl::pow(base, k));
    const uint64_t a = v[k], b = v[r];
    v[k] = gl::mul(b, fk);
    if (r != k) v[r] = gl::mul(a, base == 1 ? c0 : gl::mul(c0, gl::pow(base, r)));
  }
}

// LDE input of coset block y % B of column y / B: c_k (shift w_N^s)^k, s = rev_r(y % B)
__global__ void __launch_bounds__(256) k_coset_scale(const uint64_t *__restrict__ coeffs, uint64_t c_stride,
                                                     uint64_t *__restrict__ out, uint64_t o_stride, uint32_t log_n,
                                                     uint32_t rate_bits, uint64_t shift,
                                                     const uint64_t *__restrict__ tw, uint64_t c_bstride,
                                                     uint64_t o_bstride) {
  const uint32_t B = 1u << rate_bits, col = blockIdx.y / B, sp = blockIdx.y % B;
  const uint32_t s = gl::rev_bits(sp, rate_bits);
  const uint64_t *a = coeffs + blockIdx.z * c_bstride + (uint64_t)col * c_stride;
  uint64_t *o = out + blockIdx.z * o_bstride + (uint64_t)col * o_stride + ((uint64_t)sp << log_n);
  const uint64_t base = gl::mul(shift, nt::tw_pow(tw, s, log_n + rate_bits));
  const uint32_t n = 1u << log_n, stride = gridDim.x * blockDim.x;
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t f = gl::pow(base, k);
  const uint64_t step = gl::pow(base, stride);
  for (; k < n; k += stride) {
    o[k] = gl::mul(a[k], f);
    f = gl::mul(f, step);
  }
}

void dif_big(const Twiddles &t, uint64_t *x, uint64_t c_stride, uint32_t ncols, uint32_t nsub, uint64_t nsub_stride,
             uint32_t log_n, bool inv, uint32_t nbat, uint64_t bstride, hipStream_t s) {
  if (!ncols || !nbat || log_n <= LDS_LOG_MAX || log_n > BIG_LOG_MAX) return;
  const dim3 g((unsigned)std::min<uint64_t>((1ull << (log_n - 1)) / 256, 256), ncols * nsub, nbat);
  for (uint32_t lh = log_n - 1; lh >= LDS_LOG_MAX; lh--)
    k_dif_level<<<g, 256, 0, s>>>(x, c_stride, nsub, nsub_stride, bstride, log_n, lh, inv ? t.inv : t.fwd);
  const dim3 gb(1u << (log_n - LDS_LOG_MAX), ncols * nsub, nbat);
  const size_t lds = 8u * qpk::ntt_lds_words(1u << LDS_LOG_MAX);
  if (inv)
    k_dif_blocks<true><<<gb, 512, lds, s>>>(x, c_stride, nsub, nsub_stride, bstride, t.pt_inv);
  else
    k_dif_blocks<false><<<gb, 512, lds, s>>>(x, c_stride, nsub, nsub_stride, bstride, t.pt_fwd);
}

void bitrev_scale(uint64_t *x, uint64_t stride, uint32_t ncols, uint32_t log_n, uint64_t c0, uint64_t base,
                  uint32_t nbat, uint64_t bstride, hipStream_t s) {
  if (!ncols || !nbat) return;
  const dim3 g((unsigned)std::min<uint64_t>(((1ull << log_n) + 255) / 256, 64), ncols, nbat);
  k_bitrev_scale<<<g, 256, 0, s>>>(x, stride, log_n, c0, base, bstride);
}

static unsigned ntt_threads(uint32_t log_n) {
  uint32_t half = log_n ? (1u << (log_n - 1)) : 1;
  return half < 64 ? 64 : (half > 512 ? 512 : half);
}

void intt(const Twiddles &t, const uint64_t *in, uint64_t in_stride, uint64_t *out, uint64_t out_stride,
          uint32_t ncols, uint32_t log_n, uint32_t nbat, uint64_t in_bstride, uint64_t out_bstride, hipStream_t s) {
  if (!ncols || !nbat) return;
  uint64_t n_inv = gl::inv((uint64_t)1 << log_n);
  if (log_n > LDS_LOG_MAX) {
    // the values into out, an in-place inverse DIF, then the in-place
    // bit-reversal scaled by 1/n
    const uint64_t n = 1ull << log_n;
    for (uint32_t b = 0; b < nbat; b++)
      if (out + b * out_bstride != in + b * in_bstride)
        (void)hipMemcpy2DAsync(out + b * out_bstride, out_stride * 8, in + b * in_bstride, in_stride * 8, n * 8,
                               (size_t)ncols, hipMemcpyDeviceToDevice, s);
    dif_big(t, out, out_stride, ncols, 1, 0, log_n, true, nbat, out_bstride, s);
    bitrev_scale(out, out_stride, ncols, log_n, n_inv, 1, nbat, out_bstride, s);
    return;
  }
  dim3 grid(ncols, nbat);
  k_intt<<<grid, ntt_threads(log_n), 8u * qpk::ntt_lds_words(1u << log_n), s>>>(in, in_stride, out, out_stride, log_n, n_inv, t.pt_inv,
                                                         in_bstride, out_bstride);
}

constexpr long LDE_FEW = 256;
void lde(const Twiddles &t, const uint64_t *coeffs, uint64_t c_stride, uint64_t *out, uint64_t o_stride,
         uint32_t ncols, uint32_t log_n, uint32_t rate_bits, uint64_t shift, uint32_t nbat, uint64_t c_bstride,
         uint64_t o_bstride, hipStream_t s) {
  if (!ncols || !nbat) return;
  if (log_n > LDS_LOG_MAX) {
    // every coset block of the output: the scaled coefficients, then an
    // in-place DIF (bit-reversed = Merkle-leaf order within the block)
    const uint32_t B = 1u << rate_bits;
    const dim3 g((unsigned)std::min<uint64_t>((1ull << log_n) / 256, 64), ncols * B, nbat);
    k_coset_scale<<<g, 256, 0, s>>>(coeffs, c_stride, out, o_stride, log_n, rate_bits, shift, t.fwd, c_bstride,
                                    o_bstride);
    dif_big(t, out, o_stride, ncols, B, 1ull << log_n, log_n, false, nbat, o_bstride, s);
    return;
  }
  // n = 2^14 (the aggregation circuits): 1024 threads x 16 and 135 KB of LDS,
  // one workgroup per CU
  // fewer columns x proofs than LDE_FEW (path hook lde_few, 0 = never): one
  // workgroup per coset (k_lde), since one per column would leave most CUs
  // idle while each walks its 2^rate cosets in turn (small aggregation
  // batches, FRI layers)
  const uint64_t few = (uint64_t)path_opt("lde_few", LDE_FEW);
  if (rate_bits >= 1 && rate_bits <= LDE_MAX_RATE && log_n >= LDE_COSETS_MIN_LOG && log_n <= LDE_COSETS_MAX_LOG &&
      log_n + rate_bits <= TW_LOG && (uint64_t)ncols * nbat >= few) {
    dim3 g(ncols, nbat);
    const size_t lds_bytes = (size_t)8 * (qpk::ntt_lds_words(1u << log_n) + LDE_ALDS * (1u << (log_n - 4)));
    const uint32_t T = 1u << (log_n - 4);
    const uint64_t shift_T = gl::pow(shift, T);
    const uint64_t *mtw = t.mtw + t.mtw_off[log_n][rate_bits];
#define QP_LDE_COSETS(LT)                                                                                   \
  k_lde_cosets<LT><<<g, 1u << LT, lds_bytes, s>>>(coeffs, c_stride, c_bstride, out, o_stride, o_bstride, \
                                                  rate_bits, shift, shift_T, mtw, t.pt_fwd, t.ptw)
    switch (log_n) {
      case 10: QP_LDE_COSETS(6); break;
      case 11: QP_LDE_COSETS(7); break;
      case 12: QP_LDE_COSETS(8); break;
      case 13: QP_LDE_COSETS(9); break;
      default: QP_LDE_COSETS(10); break;
    }
#undef QP_LDE_COSETS
    return;
  }
  dim3 grid(1u << rate_bits, ncols, nbat);
  k_lde<<<grid, ntt_threads(log_n), 8u * qpk::ntt_lds_words(1u << log_n), s>>>(coeffs, c_stride, out, o_stride, log_n, rate_bits, shift,
                                                        t.fwd, t.pt_fwd, c_bstride, o_bstride);
}

}  // namespace qpk
