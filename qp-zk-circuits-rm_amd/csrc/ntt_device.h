// ntt_device.h — the in-LDS radix-2 DIF used by every NTT-shaped kernel.
#pragma once
#include "field.h"
#include "kernels.h"

namespace qpk {

// DIF over LDS a[0..2^log_n): afterwards a[p] = sum_k x_k w^{rev(p) k}, with
// w = the 2^log_n-th root whose powers are read from tw (w_{2^TW_LOG} table).
__device__ __forceinline__ void dif_lds(uint64_t *a, uint32_t log_n, const uint64_t *__restrict__ tw) {
  const uint32_t half_n = 1u << (log_n - 1);
  for (int s = (int)log_n - 1; s >= 0; s--) {
    const uint32_t h = 1u << s;
    const uint32_t tsh = TW_LOG - 1 - s;
    for (uint32_t b = threadIdx.x; b < half_n; b += blockDim.x) {
      uint32_t j = b & (h - 1);
      uint32_t k = ((b >> s) << (s + 1)) + j;
      uint64_t u = a[k], v = a[k + h];
      a[k] = gl::add(u, v);
      a[k + h] = gl::mul(gl::sub(u, v), tw_get(tw, j << tsh));
    }
    __syncthreads();
  }
}

}  // namespace qpk
