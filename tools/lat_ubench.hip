// lat_ubench.hip — dependent-chain latency vs throughput of the VALU patterns
// Goldilocks arithmetic is built from, on gfx950.  Each lane runs CH
// independent dependent chains; launched at 1 wave/SIMD (latency) and at
// 8 waves/SIMD (throughput).  Reports cycles per wave-instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lat_ubench.hip -o tools/lat_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 512

// one "op" of each pattern; instructions per op in NI
template <int P, int CH>
__global__ void kchain(uint64_t *out, uint32_t seed) {
  uint64_t a[CH];
  uint32_t x = seed + threadIdx.x, y = seed * 3 + 1;
  for (int i = 0; i < CH; i++) a[i] = seed + i * 77 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < CH; k++) {
      if (P == 0) {  // v_mad_u64_u32 dependent through the 64-bit addend
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y) : "vcc");
      } else if (P == 1) {  // 32-bit carry pair through vcc
        uint32_t lo = (uint32_t)a[k], hi = (uint32_t)(a[k] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc"
                     : "+v"(lo), "+v"(hi) : "v"(x) : "vcc");
        a[k] = ((uint64_t)hi << 32) | lo;
      } else if (P == 2) {  // v_lshl_add_u64 (64-bit add)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[k]) : "v"((uint64_t)y));
      } else if (P == 3) {  // cmp_u64 -> vcc -> cndmask (carry detect + select)
        uint32_t lo = (uint32_t)a[k], hi = (uint32_t)(a[k] >> 32);
        asm volatile("v_cmp_lt_u64 vcc, %2, %3\n\tv_cndmask_b32 %0, %0, %1, vcc"
                     : "+v"(lo), "+v"(hi) : "v"(a[k]), "v"((uint64_t)x) : "vcc");
        a[k] = ((uint64_t)hi << 32) | lo;
      } else if (P == 4) {  // v_add_u32
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(x));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      } else if (P == 5) {  // v_mov_b32 pair
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "v"(lo + 0u));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      } else if (P == 6) {  // v_mad_u64_u32 with carry-out to an SGPR pair read by cndmask
        uint32_t c;
        asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_cndmask_b32_e64 %1, 0, -1, s[40:41]"
                     : "+v"(a[k]), "=v"(c) : "v"(x), "v"(y) : "s40", "s41");
        a[k] += c;
      } else if (P == 7) {  // v_mul_lo_u32 + v_mul_hi_u32 independent pair
        uint32_t lo = (uint32_t)a[k], hi = (uint32_t)(a[k] >> 32);
        asm volatile("v_mul_lo_u32 %0, %0, %2\n\tv_mul_hi_u32 %1, %1, %2" : "+v"(lo), "+v"(hi) : "v"(y));
        a[k] = ((uint64_t)hi << 32) | lo;
      } else if (P == 8) {  // v_add3_u32
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(lo) : "v"(x), "v"(y));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      } else if (P == 9) {  // v_mad_u32_u24
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_mad_u32_u24 %0, %1, 13, %0" : "+v"(lo) : "v"(x));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      } else if (P == 10) {  // v_lshlrev_b32 + v_or
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(lo) : "v"(x));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      } else if (P == 11) {  // v_dot4_u32_u8
        uint32_t lo = (uint32_t)a[k];
        asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(lo) : "v"(x), "v"(y));
        a[k] = (a[k] & ~0xFFFFFFFFull) | lo;
      }
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < CH; i++) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char *NAMES[] = {"mad_u64_u32",     "add_co+addc(vcc)", "lshl_add_u64",   "cmp_u64+cndmask",
                              "add_u32",         "mov_b32",          "mad+cndmask(sgpr)", "mul_lo+mul_hi",
                              "add3_u32",        "mad_u32_u24",      "lshl_or_b32",    "dot4_u32_u8"};
static const int NI[] = {1, 2, 1, 2, 1, 1, 2, 2, 1, 1, 1, 1};

template <int P, int CH>
void run(uint64_t *out, int waves_per_simd) {
  // 256 CUs x 4 SIMDs; blocks of 64 threads = 1 wave
  const int blocks = 256 * 4 * waves_per_simd;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  kchain<P, CH><<<blocks, 64>>>(out, 1);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(a);
    kchain<P, CH><<<blocks, 64>>>(out, r + 2);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  // cycles per wave-instruction per SIMD at 2.4 GHz
  const double instr_per_simd = (double)waves_per_simd * ITERS * CH * NI[P];
  printf("%-20s CH=%d waves/SIMD=%d  %7.3f ms  %6.2f cyc/instr/SIMD\n", NAMES[P], CH, waves_per_simd, best,
         best * 1e-3 * 2.4e9 / instr_per_simd);
}

template <int P>
void runall(uint64_t *out) {
  run<P, 1>(out, 1);
  run<P, 1>(out, 8);
  run<P, 8>(out, 1);
  run<P, 8>(out, 8);
}

int main() {
  uint64_t *out;
  (void)hipMalloc(&out, (size_t)256 * 4 * 8 * 64 * 8);
  runall<0>(out);
  runall<1>(out);
  runall<2>(out);
  runall<3>(out);
  runall<4>(out);
  runall<5>(out);
  runall<6>(out);
  runall<7>(out);
  runall<8>(out);
  runall<9>(out);
  runall<10>(out);
  runall<11>(out);
  return 0;
}
