// poseidon_ubench.hip — permutations/s of Poseidon code-shape variants on
// gfx950 (state in registers, one lane per state, n independent states).
//   V0: ps::permute (canonical arithmetic, round loop)
//   V1: psd::permute_nc_v1 (first-generation carry-chain form)
//   V2: psd arithmetic, full rounds unrolled, partial rounds rolled (loop)
//   V3: psd arithmetic, all rounds rolled
//   V4: 64-bit C arithmetic (compare-based carries), unrolled
//   V5: V4 arithmetic, MDS as 24 explicit v_mad_u64_u32 per row + mad reduction
//   V6: psd (carry-chain) sbox, V5 MDS
//   V7: pf:: (poseidon_fast.h) mode 0: asm mads, asm reductions, folded round constants
//   V8: pf mode 1: compiler mads on opaque constants, asm reductions
//   V9: pf mode 2: mode 1 with C reductions
//   V10: pf mode 3: mode 0 with each MDS row's 24 mads in one asm block
//   V11: pf mode 4: mode 3 with the partial rounds rolled into a loop
//   V12: pf mode 5: every round rolled
//   V13-V16: pf modes 6-9: MDS rows in interleaved asm blocks of 2 / 3 / 4 / 6 rows
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qp-zk-circuits-rm_amd/csrc tools/poseidon_ubench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "poseidon.h"
#include "poseidon_dev.h"
#include "poseidon_fast.h"

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

namespace p64 {
constexpr uint64_t EPS = 0xFFFFFFFFull;
__device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t c) {
  uint64_t s = a + c;
  return s + (s < c ? EPS : 0);
}
__device__ __forceinline__ uint64_t reduce_nc(uint64_t lo, uint64_t hi) {
  const uint64_t hh = hi >> 32, hl = hi & EPS;
  uint64_t t0 = lo - hh;
  t0 -= (lo < hh) ? EPS : 0;
  const uint64_t t1 = (hl << 32) - hl;
  const uint64_t r = t0 + t1;
  return r + (r < t1 ? EPS : 0);
}
__device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  gl::mul_wide(a, b, lo, hi);
  return reduce_nc(lo, hi);
}
__device__ __forceinline__ uint64_t sbox_nc(uint64_t x) {
  const uint64_t x2 = mul_nc(x, x);
  const uint64_t x3 = mul_nc(x2, x);
  const uint64_t x4 = mul_nc(x2, x2);
  return mul_nc(x3, x4);
}
__device__ __forceinline__ void mds_nc(uint64_t s[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = (uint32_t)s[i];
    hi[i] = (uint32_t)(s[i] >> 32);
  }
#pragma unroll
  for (int r = 0; r < 12; r++) {
    uint64_t al = 0, ah = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      al += (uint64_t)lo[(i + r) % 12] * ps::mds_circ(i);
      ah += (uint64_t)hi[(i + r) % 12] * ps::mds_circ(i);
    }
    if (r == 0) {
      al += (uint64_t)lo[0] * 8u;
      ah += (uint64_t)hi[0] * 8u;
    }
    const uint64_t l = al + (ah << 32);
    const uint64_t H = (ah >> 32) + (l < al ? 1 : 0);
    const uint64_t t1 = (H << 32) - H;
    const uint64_t v = l + t1;
    s[r] = v + (v < t1 ? EPS : 0);
  }
}
// explicit mads: acc += x * C (C inline constant <= 64)
template <int C>
__device__ __forceinline__ void mac(uint64_t &acc, uint32_t x) {
  uint64_t d;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(d) : "v"(x), "i"(C));
}
template <int R, int I>
__device__ __forceinline__ void row_terms(uint64_t &al, uint64_t &ah, const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (I < 12) {
    constexpr int C = (int)ps::mds_circ(I) + ((R == 0 && I == 0) ? 8 : 0);
    mac<C>(al, lo[(I + R) % 12]);
    mac<C>(ah, hi[(I + R) % 12]);
    row_terms<R, I + 1>(al, ah, lo, hi);
  }
}
template <int R>
__device__ __forceinline__ void mds_row(uint64_t s[12], const uint32_t lo[12], const uint32_t hi[12]) {
  if constexpr (R < 12) {
    uint64_t al = 0, ah = 0;
    row_terms<R, 0>(al, ah, lo, hi);
    // V = al + ah 2^32, al, ah < 2^41; ah = ah0 + 2^32 ah1
    const uint32_t ah0 = (uint32_t)ah, ah1 = (uint32_t)(ah >> 32);
    const uint64_t t = al + (uint64_t)ah1 * EPS;  // < 2^42
    const uint32_t t0 = (uint32_t)t, t1 = (uint32_t)(t >> 32);
    const uint32_t u = t1 + ah0;
    const uint64_t r = ((uint64_t)u << 32) | t0;
    s[R] = u < ah0 ? r + EPS : r;
    mds_row<R + 1>(s, lo, hi);
  }
}
__device__ __forceinline__ void mds_mad(uint64_t s[12]) {
  uint32_t lo[12], hi[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    lo[i] = (uint32_t)s[i];
    hi[i] = (uint32_t)(s[i] >> 32);
  }
  mds_row<0>(s, lo, hi);
}
template <int MODE>  // 0: p64 mds, 1: mad mds, p64 sbox, 2: mad mds, psd sbox
__device__ __forceinline__ void permute(uint64_t s[12]) {
  auto sb = [](uint64_t x) { return MODE == 2 ? psd::sbox_nc(x) : sbox_nc(x); };
  auto ad = [](uint64_t x, uint64_t c) { return MODE == 2 ? psd::add_nc(x, c) : add_nc(x, c); };
#pragma unroll
  for (int r = 0; r < 30; r++) {
    if (r < 4 || r >= 26) {
#pragma unroll
      for (int i = 0; i < 12; i++) s[i] = sb(ad(s[i], ps::RC_DEV[r * 12 + i]));
    } else {
#pragma unroll
      for (int i = 1; i < 12; i++) s[i] = ad(s[i], ps::RC_DEV[r * 12 + i]);
      s[0] = sb(ad(s[0], ps::RC_DEV[r * 12]));
    }
    if (MODE == 0) mds_nc(s);
    else mds_mad(s);
  }
}
}  // namespace p64

template <int V, int REPS>
__global__ void __launch_bounds__(256) kperm(uint64_t *st, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  uint64_t s[12];
  for (int k = 0; k < 12; k++) s[k] = st[k * n + i];
  for (int r = 0; r < REPS; r++) {
    if (V == 0) ps::permute(s);
    if (V == 1) psd::permute_nc_v1(s);
    if (V == 2) v2::permute(s);
    if (V == 3) v3::permute(s);
    if (V == 4) p64::permute<0>(s);
    if (V == 5) p64::permute<1>(s);
    if (V == 6) p64::permute<2>(s);
    if (V == 7) pf::permute_nc<0>(s);
    if (V == 8) pf::permute_nc<1>(s);
    if (V == 9) pf::permute_nc<2>(s);
    if (V == 10) pf::permute_nc<3>(s);
    if (V == 11) pf::permute_nc<4>(s);
    if (V == 12) pf::permute_nc<5>(s);
    if (V == 13) pf::permute_nc<6>(s);
    if (V == 14) pf::permute_nc<7>(s);
    if (V == 15) pf::permute_nc<8>(s);
    if (V == 16) pf::permute_nc<9>(s);
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
  constexpr int NV = 17;
  float t[NV] = {run<0>(d, n), run<1>(d, n), run<2>(d, n), run<3>(d, n), run<4>(d, n), run<5>(d, n), run<6>(d, n), run<7>(d, n), run<8>(d, n), run<9>(d, n), run<10>(d, n), run<11>(d, n), run<12>(d, n),
                 run<13>(d, n), run<14>(d, n), run<15>(d, n), run<16>(d, n)};
  // check all variants agree
  uint64_t *h = new uint64_t[12 * NV];
  for (int v = 0; v < NV; v++) {
    (void)hipMemset(d, 7, n * 96);
    if (v == 0) kperm<0, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 1) kperm<1, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 2) kperm<2, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 3) kperm<3, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 4) kperm<4, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 5) kperm<5, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 6) kperm<6, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 7) kperm<7, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 8) kperm<8, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 9) kperm<9, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 10) kperm<10, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 11) kperm<11, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 12) kperm<12, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 13) kperm<13, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 14) kperm<14, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 15) kperm<15, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    if (v == 16) kperm<16, 1><<<(unsigned)(n / 256), 256>>>(d, n);
    (void)hipDeviceSynchronize();
    for (int k = 0; k < 12; k++) (void)hipMemcpy(h + v * 12 + k, d + k * n, 8, hipMemcpyDeviceToHost);
  }
  for (int v = 0; v < NV; v++) {
    bool same = true;
    for (int k = 0; k < 12; k++) same &= h[v * 12 + k] == h[k];
    printf("V%d: %8.3f ms  %.3f Gperm/s  %s\n", v, t[v], n * 8 / (t[v] * 1e-3) / 1e9, same ? "agree" : "MISMATCH");
  }
  return 0;
}
