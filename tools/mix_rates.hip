// mix_rates.hip — are VALU class costs additive?  tools/issue_ceiling.py
// prices k_leaf_hash's instruction mix with per-class costs measured on
// single-class streams (tools/gen_isa_rates.py BLOCKS).  Here the same classes
// run alone and interleaved in the leaf hash's proportions (per 9 VALU:
// 5 v_mad_u64_u32, 1 v_cndmask_b32_e64, 1 v_sub_co_u32_e64, 1 v_subb_co_u32_e64,
// 1 v_mov_b32; static mix of the kernel: 9044 / 1634 / 988 / 988 / 1721 of
// 15.3 k), 8 independent chains per wave, 8 waves per SIMD (256 CUs x 8 x 256
// lanes), timed with HIP events: ns per wave-instruction per SIMD.  If the
// mixed stream costs less than the sum of its parts, the additive ceiling is
// too low and a kernel can run above it.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mix_rates.hip -o tools/mix_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 131072
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// chain k: 64-bit accumulator a[k] (mads), 32-bit b[k] (carry ops, moves)
#define MAD(k) "v_mad_u64_u32 %" #k ", s[40:41], %16, 13, %" #k "\n\t"
#define CND(k) "v_cndmask_b32_e64 %" #k ", %" #k ", %16, s[42:43]\n\t"
#define SUB(k) "v_sub_co_u32_e64 %" #k ", s[44:45], %" #k ", %16\n\t"
#define SBB(k) "v_subb_co_u32_e64 %" #k ", s[46:47], %" #k ", %16, s[42:43]\n\t"
#define MOV(k) "v_mov_b32_e32 %" #k ", %16\n\t"

template <int KIND>
__global__ void __launch_bounds__(256) k_mix(uint64_t *out, uint32_t seed) {
  uint64_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  uint32_t b0 = seed ^ threadIdx.x, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6,
           b7 = b0 + 7;
  const uint32_t x = seed * 3 + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
    if constexpr (KIND == 0) {  // 8 mads
      asm volatile(MAD(0) MAD(1) MAD(2) MAD(3) MAD(4) MAD(5) MAD(6) MAD(7)
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                   : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    } else if constexpr (KIND == 1) {  // 8 carry-class ops (cndmask, sub, subb, cndmask ...)
      asm volatile(CND(8) SUB(9) SBB(10) CND(11) SUB(12) SBB(13) CND(14) SUB(15)
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                   : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    } else if constexpr (KIND == 2) {  // 8 moves
      asm volatile(MOV(8) MOV(9) MOV(10) MOV(11) MOV(12) MOV(13) MOV(14) MOV(15)
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                   : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    } else {  // the leaf hash's proportions: 5 mad, 1 cndmask, 1 sub, 1 subb, 1 mov (x2 = 18 per iteration)
      asm volatile(MAD(0) CND(8) MAD(1) SUB(9) MAD(2) SBB(10) MAD(3) MOV(11) MAD(4)
                   MAD(5) CND(12) MAD(6) SUB(13) MAD(7) SBB(14) MAD(0) MOV(15) MAD(1)
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                   : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^
                                               b6 ^ b7;
}

template <int KIND>
static float run(uint64_t *out, hipStream_t s) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_mix<KIND><<<256 * 8, 256, 0, s>>>(out, 1);  // warm
  (void)hipEventRecord(e0, s);
  k_mix<KIND><<<256 * 8, 256, 0, s>>>(out, 2);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint64_t *out;
  CK(hipMalloc(&out, 256ull * 8 * 256 * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  // wave-instructions per SIMD: 2048 workgroups x 4 waves / 1024 SIMDs = 8 waves per SIMD
  const double waves_per_simd = 2048.0 * 4 / 1024;
  const char *names[4] = {"mad x8", "carry-class x8 (cndmask/sub/subb)", "mov x8", "mix 10 mad : 2 cndmask : 2 sub : 2 subb : 2 mov"};
  const int per_it[4] = {8, 8, 8, 18};
  for (int rep = 0; rep < 2; rep++) {
    float ms[4] = {run<0>(out, s), run<1>(out, s), run<2>(out, s), run<3>(out, s)};
    double ns[4];
    for (int k = 0; k < 4; k++) {
      ns[k] = ms[k] * 1e6 / (waves_per_simd * ITERS * per_it[k]);
      printf("{\"rep\": %d, \"stream\": \"%s\", \"ms\": %.3f, \"ns_per_wave_instr_per_simd\": %.4f}\n", rep, names[k], ms[k], ns[k]);
    }
    // additive prediction for the mix from the single-class streams
    const double pred = (10 * ns[0] + 6 * ns[1] + 2 * ns[2]) / 18;
    printf("{\"rep\": %d, \"mix_measured_ns\": %.4f, \"mix_additive_prediction_ns\": %.4f, \"ratio\": %.3f}\n", rep, ns[3],
           pred, ns[3] / pred);
  }
  CK(hipFree(out));
  return 0;
}
