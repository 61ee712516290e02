// poseidon_occ.hip — Poseidon permutations/s at forced occupancy: the pf
// modes of poseidon_fast.h compiled with and without
// amdgpu_waves_per_eu(8) (VGPR budget 64 instead of the natural 76).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qp-zk-circuits-rm_amd/csrc tools/poseidon_occ.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "poseidon_fast.h"

template <int M>
__global__ void __launch_bounds__(256) kp(uint64_t *st, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  uint64_t s[12];
  for (int k = 0; k < 12; k++) s[k] = st[k * n + i];
  for (int r = 0; r < 8; r++) pf::permute_nc<M>(s);
  for (int k = 0; k < 12; k++) st[k * n + i] = pf::canon(s[k]);
}
template <int M>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) kp8(uint64_t *st, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  uint64_t s[12];
  for (int k = 0; k < 12; k++) s[k] = st[k * n + i];
  for (int r = 0; r < 8; r++) pf::permute_nc<M>(s);
  for (int k = 0; k < 12; k++) st[k * n + i] = pf::canon(s[k]);
}

template <typename K>
float run(K k, uint64_t *d, uint64_t n) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k<<<(unsigned)(n / 256), 256>>>(d, n);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(a);
    k<<<(unsigned)(n / 256), 256>>>(d, n);
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
  struct { const char *name; void (*k)(uint64_t *, uint64_t); } ks[] = {
      {"mode0", kp<0>}, {"mode0 w8", kp8<0>}, {"mode3", kp<3>}, {"mode3 w8", kp8<3>},
      {"mode6", kp<6>}, {"mode6 w8", kp8<6>}, {"mode4 w8", kp8<4>}};
  uint64_t ref[12];
  for (auto &k : ks) {
    (void)hipMemset(d, 7, n * 96);
    float t = run(k.k, d, n);
    (void)hipMemset(d, 7, n * 96);
    k.k<<<(unsigned)(n / 256), 256>>>(d, n);
    uint64_t h[12];
    for (int j = 0; j < 12; j++) (void)hipMemcpy(h + j, d + j * n, 8, hipMemcpyDeviceToHost);
    if (&k == &ks[0]) for (int j = 0; j < 12; j++) ref[j] = h[j];
    bool same = true;
    for (int j = 0; j < 12; j++) same &= h[j] == ref[j];
    printf("%-10s %8.3f ms  %.3f Gperm/s  %s\n", k.name, t, n * 8 / (t * 1e-3) / 1e9, same ? "agree" : "MISMATCH");
  }
  return 0;
}
