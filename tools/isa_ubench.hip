// isa_ubench.hip — throughput of the VALU instructions a Goldilocks field
// kernel is built from, on gfx950 (measured, not guessed).  Each lane runs 8
// independent chains of one instruction; report wave-instructions per cycle
// per CU at the measured clock-free rate (instr/s per CU / 2.4e9).
// Build: hipcc --offload-arch=gfx950 -O3 tools/isa_ubench.hip -o tools/isa_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 256

#define BODY8(ins) ins(0) ins(1) ins(2) ins(3) ins(4) ins(5) ins(6) ins(7)

__global__ void k_mad_u64_u32(uint64_t *out, uint32_t seed) {
  uint64_t a[8];
  uint32_t x = seed + threadIdx.x, y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y) : "vcc");
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_u32(uint64_t *out, uint32_t seed) {
  uint32_t a[8];
  uint32_t y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(y));
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint64_t *out, uint32_t seed) {
  uint32_t a[8];
  uint32_t y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(y));
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint64_t *out, uint32_t seed) {
  uint32_t a[8];
  uint32_t x = seed + threadIdx.x, y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y));
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t *out, uint32_t seed) {
  double a[8];
  double x = 1.0000001 * (seed + threadIdx.x), y = 0.999999;
  for (int i = 0; i < 8; i++) a[i] = seed + i;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y));
    BODY8(I)
#undef I
  }
  double s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_add_co(uint64_t *out, uint32_t seed) {
  uint32_t a[8];
  uint32_t y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(y) : "vcc");
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_lshl_add_u64(uint64_t *out, uint32_t seed) {
  uint64_t a[8];
  uint64_t y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(a[k]) : "v"(y));
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_u32(uint64_t *out, uint32_t seed) {
  uint32_t a[8];
  uint32_t y = seed * 3 + 1;
  for (int i = 0; i < 8; i++) a[i] = seed + i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(y));
    BODY8(I)
#undef I
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_cvt_f64_u32(uint64_t *out, uint32_t seed) {
  double a[8];
  uint32_t x = seed + threadIdx.x;
  for (int i = 0; i < 8; i++) a[i] = seed + i;
  for (int it = 0; it < ITERS; it++) {
#define I(k) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[k]) : "v"(x + k));
    BODY8(I)
#undef I
  }
  double s = 0;
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t *, uint32_t);

int main() {
  struct {
    const char *name;
    kfn f;
  } ks[] = {{"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_hi_u32", k_mul_hi_u32},
            {"v_mad_u32_u24", k_mad_u32_u24}, {"v_fma_f64", k_fma_f64},       {"v_add_co_u32", k_add_co},
            {"v_lshl_add_u64", k_lshl_add_u64}, {"v_add_u32", k_add_u32},     {"v_cvt_f64_u32", k_cvt_f64_u32}};
  const int blocks = 256 * 16, threads = 256;
  uint64_t *out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (auto &k : ks) {
    k.f<<<blocks, threads>>>(out, 1);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      (void)hipEventRecord(a);
      k.f<<<blocks, threads>>>(out, r + 2);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    double wave_instr = (double)blocks * threads / 64 * ITERS * 8;
    double per_cu_per_s = wave_instr / (best * 1e-3) / 256;
    printf("%-16s %8.3f ms  %.3f wave-instr/cycle/CU @2.4GHz  (%.2f cycles per wave-instr per SIMD)\n", k.name, best,
           per_cu_per_s / 2.4e9, 4 / (per_cu_per_s / 2.4e9));
  }
  return 0;
}
