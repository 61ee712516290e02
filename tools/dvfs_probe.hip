// dvfs_probe.hip — does a one-workgroup kernel run slower when the rest of the
// GPU is idle?  A fixed dependent VALU chain (one workgroup of 256 threads) is
// timed with HIP events alone, then while a "load" kernel keeps the other CUs
// busy with independent work on a second stream, and finally at 32 and 256
// copies (one per CU).  Equal per-workgroup work in every case, so a longer
// alone-time means a lower clock (DVFS), not more work.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dvfs_probe.hip -o tools/dvfs_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) k_chain(uint64_t *out, uint32_t iters) {
  uint64_t x = threadIdx.x + 1, y = blockIdx.x + 3;
  for (uint32_t i = 0; i < iters; i++) {
    x = x * 0x9E3779B97F4A7C15ull + y;
    y = y * 0xC2B2AE3D27D4EB4Full + x;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y;
}

// independent work on every other CU (bounded: fixed iteration count)
__global__ void __launch_bounds__(256) k_load(uint64_t *out, uint32_t iters) {
  uint64_t a = threadIdx.x, b = blockIdx.x, c = 7, d = 11;
  for (uint32_t i = 0; i < iters; i++) {
    a = a * 3 + b;
    b = b * 5 + c;
    c = c * 7 + d;
    d = d * 9 + a;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}

static float time_chain(hipStream_t s, uint64_t *out, int blocks, uint32_t iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  k_chain<<<blocks, 256, 0, s>>>(out, iters);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

int main() {
  uint64_t *out, *lout;
  CK(hipMalloc(&out, 256 * 256 * 8));
  CK(hipMalloc(&lout, 4096 * 256 * 8));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const uint32_t iters = 1u << 20;
  time_chain(s0, out, 1, iters / 8);  // warm-up
  for (int rep = 0; rep < 3; rep++) {
    const float alone = time_chain(s0, out, 1, iters);
    // the load: 1020 workgroups (4 per CU on the other CUs' share), long enough to cover the probe
    k_load<<<1020, 256, 0, s1>>>(lout, iters * 4);
    const float loaded = time_chain(s0, out, 1, iters);
    CK(hipStreamSynchronize(s1));
    const float b32 = time_chain(s0, out, 32, iters);
    const float b256 = time_chain(s0, out, 256, iters);
    printf("{\"rep\": %d, \"alone_ms\": %.3f, \"with_load_ms\": %.3f, \"blocks32_ms\": %.3f, \"blocks256_ms\": %.3f}\n",
           rep, alone, loaded, b32, b256);
  }
  CK(hipFree(out));
  CK(hipFree(lout));
  return 0;
}
