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
#include "field.h"
#include "kernels.h"
#include "ntt_device.h"
#include "ntt16.h"

namespace qpk {

__global__ void k_twiddles(uint64_t *fwd, uint64_t *inv, uint64_t w, uint64_t wi, uint32_t half) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < half) {
    fwd[j] = gl::pow(w, j);
    inv[j] = gl::pow(wi, j);
  }
}

hipError_t twiddles_init(Twiddles &t, hipStream_t s) {
  uint32_t half = 1u << (TW_LOG - 1);
  hipError_t e = hipMalloc(&t.fwd, half * 8ull);
  if (e) return e;
  e = hipMalloc(&t.inv, half * 8ull);
  if (e) return e;
  uint64_t w = gl::root_of_unity(TW_LOG);
  k_twiddles<<<(half + 255) / 256, 256, 0, s>>>(t.fwd, t.inv, w, gl::inv(w), half);
  return hipGetLastError();
}

void twiddles_free(Twiddles &t) {
  if (t.fwd) (void)hipFree(t.fwd);
  if (t.inv) (void)hipFree(t.inv);
  t.fwd = t.inv = nullptr;
}

__global__ void __launch_bounds__(512) k_intt(const uint64_t *__restrict__ in, uint64_t in_stride,
                                              uint64_t *__restrict__ out, uint64_t out_stride, uint32_t log_n,
                                              uint64_t n_inv, const uint64_t *__restrict__ tw_inv,
                                              uint64_t in_bstride, uint64_t out_bstride) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t n = 1u << log_n;
  const uint64_t *src = in + blockIdx.y * in_bstride + (uint64_t)blockIdx.x * in_stride;
  uint64_t *dst = out + blockIdx.y * out_bstride + (uint64_t)blockIdx.x * out_stride;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) lds[i] = src[i];
  __syncthreads();
  nt::ntt_lds<true>(lds, log_n, tw_inv);
  for (uint32_t m = threadIdx.x; m < n; m += blockDim.x) dst[m] = gl::mul(lds[gl::rev_bits(m, log_n)], n_inv);
}

__global__ void __launch_bounds__(512) k_lde(const uint64_t *__restrict__ coeffs, uint64_t c_stride,
                                             uint64_t *__restrict__ out, uint64_t o_stride, uint32_t log_n,
                                             uint32_t rate_bits, uint64_t shift, const uint64_t *__restrict__ tw,
                                             uint64_t c_bstride, uint64_t o_bstride) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const uint32_t n = 1u << log_n;
  const uint32_t s = blockIdx.x;        // coset index
  const uint32_t col = blockIdx.y;
  const uint64_t *src = coeffs + blockIdx.z * c_bstride + (uint64_t)col * c_stride;
  uint64_t *dst = out + blockIdx.z * o_bstride + (uint64_t)col * o_stride +
                  ((uint64_t)gl::rev_bits(s, rate_bits) << log_n);
  // base = shift * w_N^s ; element k scaled by base^k
  const uint64_t wN = tw[(uint64_t)s << (TW_LOG - log_n - rate_bits)];
  const uint64_t base = gl::mul(shift, wN);
  uint64_t f = gl::pow(base, threadIdx.x);
  const uint64_t step = gl::pow(base, blockDim.x);
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
    lds[k] = gl::mul(src[k], f);
    f = gl::mul(f, step);
  }
  __syncthreads();
  nt::ntt_lds<false>(lds, log_n, tw);
  for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) dst[p] = nt::canon(lds[p]);
}

static unsigned ntt_threads(uint32_t log_n) {
  uint32_t half = log_n ? (1u << (log_n - 1)) : 1;
  return half < 64 ? 64 : (half > 512 ? 512 : half);
}

void intt(const Twiddles &t, const uint64_t *in, uint64_t in_stride, uint64_t *out, uint64_t out_stride,
          uint32_t ncols, uint32_t log_n, uint32_t nbat, uint64_t in_bstride, uint64_t out_bstride, hipStream_t s) {
  if (!ncols || !nbat) return;
  uint64_t n_inv = gl::inv((uint64_t)1 << log_n);
  dim3 grid(ncols, nbat);
  k_intt<<<grid, ntt_threads(log_n), (8u << log_n), s>>>(in, in_stride, out, out_stride, log_n, n_inv, t.inv,
                                                         in_bstride, out_bstride);
}

void lde(const Twiddles &t, const uint64_t *coeffs, uint64_t c_stride, uint64_t *out, uint64_t o_stride,
         uint32_t ncols, uint32_t log_n, uint32_t rate_bits, uint64_t shift, uint32_t nbat, uint64_t c_bstride,
         uint64_t o_bstride, hipStream_t s) {
  if (!ncols || !nbat) return;
  dim3 grid(1u << rate_bits, ncols, nbat);
  k_lde<<<grid, ntt_threads(log_n), (8u << log_n), s>>>(coeffs, c_stride, out, o_stride, log_n, rate_bits, shift,
                                                        t.fwd, c_bstride, o_bstride);
}

}  // namespace qpk
