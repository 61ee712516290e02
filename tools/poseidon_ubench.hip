// poseidon_ubench.hip — permutations/s of Poseidon code-shape variants on
// gfx950 (state in registers, one lane per state, n independent states).
//   V0: ps::permute (canonical arithmetic, round loop)
//   V1: psd::permute_nc fully unrolled (the kernels' current form)
//   V2: psd arithmetic, full rounds unrolled, partial rounds rolled (loop)
//   V3: psd arithmetic, all rounds rolled
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qp-zk-circuits-rm_amd/csrc tools/poseidon_ubench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "poseidon.h"
#include "poseidon_dev.h"

namespace v2 {
__device__ __noinline__ void dummy() {}
__device__ __forceinline__ void permute(uint64_t s[12]) {
#pragma unroll
  for (int r = 0; r < 4; r++) psd::full_round(s, r);
#pragma nounroll
  for (int r = 4; r < 26; r++) psd::partial_round(s, r);
#pragma unroll
  for (int r = 26; r < 30; r++) psd::full_round(s, r);
}
}  // namespace v2

namespace v3 {
__device__ __forceinline__ void permute(uint64_t s[12]) {
#pragma nounroll
  for (int r = 0; r < 4; r++) psd::full_round(s, r);
#pragma nounroll
  for (int r = 4; r < 26; r++) psd::partial_round(s, r);
#pragma nounroll
  for (int r = 26; r < 30; r++) psd::full_round(s, r);
}
}  // namespace v3

template <int V, int REPS>
__global__ void __launch_bounds__(256) kperm(uint64_t *st, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  uint64_t s[12];
  for (int k = 0; k < 12; k++) s[k] = st[k * n + i];
  for (int r = 0; r < REPS; r++) {
    if (V == 0) ps::permute(s);
    if (V == 1) psd::permute_nc(s);
    if (V == 2) v2::permute(s);
    if (V == 3) v3::permute(s);
  }
  for (int k = 0; k < 12; k++) st[k * n + i] = V == 0 ? s[k] : psd::canon(s[k]);
}

template <int V>
float run(uint64_t *d, uint64_t n) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  kperm<V, 8><<<(unsigned)(n / 256), 256>>>(d, n);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(a);
    kperm<V, 8><<<(unsigned)(n / 256), 256>>>(d, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  const uint64_t n = 1ull << 22;
  uint64_t *d;
  (void)hipMalloc(&d, n * 96);
  (void)hipMemset(d, 7, n * 96);
  float t[4] = {run<0>(d, n), run<1>(d, n), run<2>(d, n), run<3>(d, n)};
  // check all variants agree
  uint64_t *h = new uint64_t[12 * 4];
  for (int v = 0; v < 4; v++) {
    (void)hipMemset(d, 7, n * 96);
    if (v == 0) kperm<0, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 1) kperm<1, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 2) kperm<2, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 3) kperm<3, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    (void)hipDeviceSynchronize();
    for (int k = 0; k < 12; k++) (void)hipMemcpy(h + v * 12 + k, d + k * n, 8, hipMemcpyDeviceToHost);
  }
  for (int v = 0; v < 4; v++) {
    bool same = true;
    for (int k = 0; k < 12; k++) same &= h[v * 12 + k] == h[k];
    printf("V%d: %8.3f ms  %.3f Gperm/s  %s\n", v, t[v], n * 8 / (t[v] * 1e-3) / 1e9, same ? "agree" : "MISMATCH");
  }
  return 0;
}
