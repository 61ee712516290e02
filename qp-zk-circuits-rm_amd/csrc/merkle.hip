// merkle.hip — Poseidon leaf hashing, Merkle tree/cap, query gathers (gfx950).
// plonky2 hash/merkle_tree.rs semantics: leaf digest =
// hash_or_noop(leaf), node = two_to_one(L, R), cap = 2^h subtree roots.
// VALU-bound: one lane per leaf / node, the 12-element state in registers;
// column-major LDE input makes each absorbed column a coalesced 512-B
// wave load.
#include "field.h"
#include "poseidon.h"
#include "poseidon_dev.h"
#include "kernels.h"

namespace qpk {

__global__ void __launch_bounds__(256) k_leaf_hash(const uint64_t *__restrict__ cols, uint64_t stride, uint32_t ncols,
                                                   const uint64_t *__restrict__ salt, uint32_t nsalt,
                                                   uint64_t *__restrict__ dig, uint32_t N, uint64_t c_bstride,
                                                   uint64_t s_bstride, uint64_t d_bstride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  cols += blockIdx.y * c_bstride;
  if (salt) salt += blockIdx.y * s_bstride;
  dig += blockIdx.y * d_bstride;
  const uint32_t W = ncols + nsalt;
  uint64_t s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (W <= 4) {
    for (uint32_t c = 0; c < W; c++) s[c] = c < ncols ? cols[(uint64_t)c * stride + i] : salt[(uint64_t)i * nsalt + c - ncols];
  } else {
    for (uint32_t off = 0; off < W; off += 8) {
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        uint32_t c = off + k;
        if (c < ncols) s[k] = cols[(uint64_t)c * stride + i];
        else if (c < W) s[k] = salt[(uint64_t)i * nsalt + (c - ncols)];
      }
      psd::permute_nc(s);
    }
  }
  uint64_t *o = dig + (uint64_t)i * 4;
  o[0] = psd::canon(s[0]); o[1] = psd::canon(s[1]); o[2] = psd::canon(s[2]); o[3] = psd::canon(s[3]);
}

__global__ void __launch_bounds__(256) k_merkle_level(const uint64_t *__restrict__ prev, uint64_t *__restrict__ next,
                                                      uint32_t count, uint64_t d_bstride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  prev += blockIdx.y * d_bstride;
  next += blockIdx.y * d_bstride;
  uint64_t s[12];
  const uint64_t *l = prev + (uint64_t)i * 8;
#pragma unroll
  for (int k = 0; k < 8; k++) s[k] = l[k];
  s[8] = s[9] = s[10] = s[11] = 0;
  psd::permute_nc(s);
  uint64_t *o = next + (uint64_t)i * 4;
  o[0] = psd::canon(s[0]); o[1] = psd::canon(s[1]); o[2] = psd::canon(s[2]); o[3] = psd::canon(s[3]);
}

void leaf_hash(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
               uint64_t *digests, uint32_t N, uint32_t nbat, uint64_t c_bstride, uint64_t s_bstride,
               uint64_t d_bstride, hipStream_t s) {
  dim3 grid((N + 255) / 256, nbat);
  k_leaf_hash<<<grid, 256, 0, s>>>(cols, stride, ncols, salt, nsalt, digests, N, c_bstride, s_bstride, d_bstride);
}

void merkle_tree(uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t d_bstride,
                 hipStream_t s) {
  uint64_t off = 0;
  for (uint32_t k = 1; k <= log_N - cap_h; k++) {
    uint32_t count = 1u << (log_N - k);
    uint64_t *prev = digests + off * 4;
    off += (uint64_t)1 << (log_N - k + 1);
    uint64_t *next = digests + off * 4;
    dim3 grid((count + 255) / 256, nbat);
    k_merkle_level<<<grid, 256, 0, s>>>(prev, next, count, d_bstride);
  }
}

__global__ void k_gather_rows(const uint64_t *__restrict__ cols, uint64_t stride, uint32_t ncols,
                              const uint32_t *__restrict__ idx, uint32_t nidx, uint64_t *__restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ncols * nidx) return;
  const uint32_t q = t / ncols, c = t % ncols;
  out[t] = cols[(uint64_t)c * stride + idx[q]];
}

void gather_rows(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint32_t *idx, uint32_t nidx,
                 uint64_t *out, hipStream_t s) {
  uint32_t tot = ncols * nidx;
  if (!tot) return;
  k_gather_rows<<<(tot + 255) / 256, 256, 0, s>>>(cols, stride, ncols, idx, nidx, out);
}

__global__ void k_gather_paths(const uint64_t *__restrict__ dig, uint32_t log_N, uint32_t cap_h,
                               const uint32_t *__restrict__ idx, uint32_t nidx, uint64_t *__restrict__ out) {
  const uint32_t depth = log_N - cap_h;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nidx * depth * 4) return;
  const uint32_t q = t / (depth * 4), r = t % (depth * 4), k = r / 4, e = r % 4;
  uint64_t off = 0;
  for (uint32_t j = 0; j < k; j++) off += (uint64_t)1 << (log_N - j);
  const uint64_t sib = (uint64_t)((idx[q] >> k) ^ 1u);
  out[t] = dig[(off + sib) * 4 + e];
}

void gather_paths(const uint64_t *digests, uint32_t log_N, uint32_t cap_h, const uint32_t *idx, uint32_t nidx,
                  uint64_t *out, hipStream_t s) {
  uint32_t tot = nidx * (log_N - cap_h) * 4;
  if (!tot) return;
  k_gather_paths<<<(tot + 255) / 256, 256, 0, s>>>(digests, log_N, cap_h, idx, nidx, out);
}

__global__ void __launch_bounds__(256) k_permute(uint64_t *states, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s[12];
#pragma unroll
  for (int k = 0; k < 12; k++) s[k] = states[i * 12 + k];
  psd::permute(s);
#pragma unroll
  for (int k = 0; k < 12; k++) states[i * 12 + k] = s[k];
}

void permute_batch(uint64_t *states, uint64_t n, hipStream_t s) {
  if (!n) return;
  k_permute<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(states, n);
}

}  // namespace qpk
