// leaf_ubench.hip — development micro-benchmark of the wires leaf hash
// (k_leaf_hash's shape: one lane per leaf, 135 columns absorbed 8 at a time,
// column-major [col][leaf] input) in variants that separate memory from
// issue effects.  Not shipped.
//   L0  production shape: load a chunk of 8 columns, permute
//   L1  as L0, but every chunk reads columns 0..7 (L2-resident input)
//   L2  as L0 with the next chunk's loads issued before the permutation
//   L3  no loads: the chunk is derived from the lane index (pure issue)
//   L4  as L0 with the first absorption on the zero-capacity permutation
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qp-zk-circuits-rm_amd/csrc tools/leaf_ubench.hip -o tools/leaf_ubench
// Run:   tools/leaf_ubench [proofs=16] [iters=5]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "poseidon.h"
#include "poseidon_dev.h"
#include "poseidon_fast.h"

constexpr uint32_t NCOLS = 135;

template <int V>
__global__ void __launch_bounds__(256) k_leaf(const uint64_t *__restrict__ cols, uint64_t stride,
                                              uint64_t *__restrict__ dig, uint32_t N) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  cols += (uint64_t)blockIdx.y * NCOLS * stride;
  uint64_t s[12];
#pragma unroll
  for (int k = 0; k < 12; k++) s[k] = 0;
  if constexpr (V == 2) {
    uint64_t nx[8];
#pragma unroll
    for (int k = 0; k < 8; k++) nx[k] = cols[(uint64_t)k * stride + i];
    for (uint32_t off = 0; off < NCOLS; off += 8) {
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (off + k < NCOLS) s[k] = nx[k];
      if (off + 8 < NCOLS) {
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (off + 8 + k < NCOLS) nx[k] = cols[(uint64_t)(off + 8 + k) * stride + i];
      }
      psd::permute_nc(s);
    }
  } else {
    for (uint32_t off = 0; off < NCOLS; off += 8) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t c = off + k;
        if (c < NCOLS) {
          if constexpr (V == 1) s[k] = cols[(uint64_t)k * stride + i];
          else if constexpr (V == 3) s[k] = (uint64_t)(i * 0x9E3779B9u + c) * 0x100000001B3ull;
          else s[k] = cols[(uint64_t)c * stride + i];
        }
      }
      if constexpr (V == 4) {
        if (off == 0) pf::permute_nc_capz(s);
        else psd::permute_nc(s);
      } else {
        psd::permute_nc(s);
      }
    }
  }
  uint64_t *o = dig + ((uint64_t)blockIdx.y * N + i) * 4;
#pragma unroll
  for (int k = 0; k < 4; k++) o[k] = psd::canon(s[k]);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_) {                                                              \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int V>
static double run(const uint64_t *cols, uint64_t *dig, uint32_t N, uint32_t nb, int iters) {
  dim3 g((N + 255) / 256, nb);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_leaf<V><<<g, 256>>>(cols, N, dig, N);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  for (int it = 0; it < iters; it++) k_leaf<V><<<g, 256>>>(cols, N, dig, N);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char **argv) {
  const uint32_t nb = argc > 1 ? atoi(argv[1]) : 16, iters = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t N = 1u << 16;
  const size_t words = (size_t)nb * NCOLS * N;
  uint64_t *cols, *dig;
  CK(hipMalloc(&cols, words * 8));
  CK(hipMalloc(&dig, (size_t)nb * N * 32));
  uint64_t *h = (uint64_t *)malloc(words * 8);
  uint64_t x = 0x1234567;
  for (size_t k = 0; k < words; k++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[k] = x % 0xFFFFFFFF00000001ull;
  }
  CK(hipMemcpy(cols, h, words * 8, hipMemcpyHostToDevice));
  const double perms = (double)nb * N * 17;
  double t[5] = {run<0>(cols, dig, N, nb, iters), run<1>(cols, dig, N, nb, iters), run<2>(cols, dig, N, nb, iters),
                 run<3>(cols, dig, N, nb, iters), run<4>(cols, dig, N, nb, iters)};
  const char *names[5] = {"L0 production", "L1 cached cols", "L2 prefetch", "L3 no loads", "L4 capz first"};
  for (int v = 0; v < 5; v++)
    printf("%-16s %8.3f ms per %u-proof launch  %.3f Gperm/s\n", names[v], t[v], nb, perms / (t[v] * 1e-3) / 1e9);
  return 0;
}
