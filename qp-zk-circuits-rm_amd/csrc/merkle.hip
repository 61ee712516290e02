// merkle.hip — Poseidon leaf hashing, Merkle tree/cap, query gathers (gfx950).
// plonky2 hash/merkle_tree.rs semantics: leaf digest =
// hash_or_noop(leaf), node = two_to_one(L, R), cap = 2^h subtree roots.
// VALU-bound: one lane per leaf / node, the 12-element state in registers;
// column-major LDE input makes each absorbed column a coalesced 512-B
// wave load.
#include "field.h"
#include "poseidon.h"
#include "poseidon_dev.h"
#include "poseidon_coop.h"
#include <stdlib.h>
#include "kernels.h"
#include "paths.h"

// Leaf digests and the first tree level are separate launches: one kernel
// doing both (three inlined permutations per lane) measured slower, 919.8 /
// 924.9 vs 930.0 / 933.0 proofs/s (profiles/r02_ab_leaf_pairs.log).  The
// hashing kernels run at the compiler's occupancy (72 VGPRs = 7 waves/SIMD).

namespace qpk {

// leaf digest of row i: hash_or_noop over the ncols column values (+ salt)
__device__ __forceinline__ void leaf_digest(const uint64_t *__restrict__ cols, uint64_t stride, uint32_t ncols,
                                            const uint64_t *__restrict__ salt, uint32_t nsalt, uint32_t i,
                                            uint64_t s[12]) {
  const uint32_t W = ncols + nsalt;
#pragma unroll
  for (int k = 0; k < 12; k++) s[k] = 0;
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
#pragma unroll
  for (int k = 0; k < 4; k++) s[k] = psd::canon(s[k]);
}

__global__ void __launch_bounds__(256) k_leaf_hash(const uint64_t *__restrict__ cols, uint64_t stride, uint32_t ncols,
                                                   const uint64_t *__restrict__ salt, uint32_t nsalt,
                                                   uint64_t *__restrict__ dig, uint32_t N, uint64_t c_bstride,
                                                   uint64_t s_bstride, uint64_t d_bstride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  cols += blockIdx.y * c_bstride;
  if (salt) salt += blockIdx.y * s_bstride;
  dig += blockIdx.y * d_bstride;
  uint64_t s[12];
  leaf_digest(cols, stride, ncols, salt, nsalt, i, s);
  uint64_t *o = dig + (uint64_t)i * 4;
  o[0] = s[0]; o[1] = s[1]; o[2] = s[2]; o[3] = s[3];
}

// k_leaf_hash for a compile-time column count and no salt (the prover's
// commitments: wires 135, Z/partial products 20, quotient chunks 16): the
// absorb loop's bounds and load predicates fold away.  The run-time form ran
// 7 % below the same loop with a constant count (tools/leaf_ubench L0: 2.87
// vs 2.67 Gperm/s per 86-proof wires launch)
template <uint32_t NC>
__global__ void __launch_bounds__(256) k_leaf_hash_t(const uint64_t *__restrict__ cols, uint64_t stride,
                                                                 uint64_t *__restrict__ dig, uint32_t N,
                                                                 uint64_t c_bstride, uint64_t d_bstride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  cols += blockIdx.y * c_bstride;
  uint64_t s[12];
#pragma unroll
  for (int k = 0; k < 12; k++) s[k] = 0;
  for (uint32_t off = 0; off < NC; off += 8) {
#pragma unroll
    for (uint32_t k = 0; k < 8; k++)
      if (off + k < NC) s[k] = cols[(uint64_t)(off + k) * stride + i];
    psd::permute_nc(s);
  }
  uint64_t *o = dig + blockIdx.y * d_bstride + (uint64_t)i * 4;
#pragma unroll
  for (int k = 0; k < 4; k++) o[k] = psd::canon(s[k]);
}


// 1..9 tree levels per launch: a block takes B = min(256, count) nodes of
// level k0 (their 2B children read from HBM), then folds them level by level
// through LDS down to one node, writing every level's digests out.  Level k
// of a tree sits at node offset 2^(log_N+1) - 2^(log_N-k+1) (level 0 = the
// leaf digests).  The upper levels of a tree are launch-bound (16..256 nodes
// per proof), so they share one launch.
__global__ void __launch_bounds__(256) k_merkle_levels(uint64_t *__restrict__ digests, uint32_t log_N, uint32_t k0,
                                                       uint32_t nl, uint64_t d_bstride) {
  __shared__ uint64_t sh[256 * 4];
  digests += blockIdx.y * d_bstride;
  const uint32_t t = threadIdx.x;
  const uint32_t cnt = 1u << (log_N - k0);
  const uint32_t B = cnt < 256u ? cnt : 256u;
  const uint32_t base = blockIdx.x * B;
  const uint64_t top = (uint64_t)1 << (log_N + 1);
  for (uint32_t l = 0; l < nl; l++) {
    const uint32_t k = k0 + l;
    const uint32_t nb = B >> l;
    uint64_t s[12];
    if (t < nb) {
      if (l == 0) {
        const uint64_t *c = digests + (top - ((uint64_t)1 << (log_N - k + 2))) * 4 + (uint64_t)(base + t) * 8;
#pragma unroll
        for (int j = 0; j < 8; j++) s[j] = c[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) s[j] = sh[t * 8 + j];
      }
      s[8] = s[9] = s[10] = s[11] = 0;
      psd::permute_nc_node(s);
#pragma unroll
      for (int j = 0; j < 4; j++) s[j] = psd::canon(s[j]);
      uint64_t *o = digests + (top - ((uint64_t)1 << (log_N - k + 1))) * 4 + (uint64_t)((base >> l) + t) * 4;
#pragma unroll
      for (int j = 0; j < 4; j++) o[j] = s[j];
    }
    __syncthreads();
    if (t < nb) {
#pragma unroll
      for (int j = 0; j < 4; j++) sh[t * 4 + j] = s[j];
    }
    __syncthreads();
  }
}

// one wide tree level: lane t hashes children 2t, 2t+1 of level k-1 into node t
// of level k (no LDS, no level loop: 69 VGPRs = 7 waves/SIMD against the
// folding kernel's 103 = 4)
__global__ void __launch_bounds__(256) k_merkle_level(uint64_t *__restrict__ digests, uint32_t log_N, uint32_t k,
                                                      uint64_t d_bstride) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (1u << (log_N - k))) return;
  digests += blockIdx.y * d_bstride;
  const uint64_t top = (uint64_t)1 << (log_N + 1);
  const uint64_t *c = digests + (top - ((uint64_t)1 << (log_N - k + 2))) * 4 + (uint64_t)t * 8;
  uint64_t s[12];
#pragma unroll
  for (int j = 0; j < 8; j++) s[j] = c[j];
  s[8] = s[9] = s[10] = s[11] = 0;
  psd::permute_nc_node(s);
  uint64_t *o = digests + (top - ((uint64_t)1 << (log_N - k + 1))) * 4 + (uint64_t)t * 4;
#pragma unroll
  for (int j = 0; j < 4; j++) o[j] = psd::canon(s[j]);
}

// one tree level of a small batch: one wave per node (pc::permute, the
// cooperative permutation).  A level whose nodes x proofs fill a few waves per
// SIMD at most costs the one-lane form the latency of one permutation
// (≈70 us: a wave issues its ~15k instructions one per ≈8.5 cycles) whatever
// its width; this form's chain is ≈125 instructions per round.  Exits are
// wave-uniform (no barriers).
__global__ void __launch_bounds__(256) k_merkle_level_coop(uint64_t *__restrict__ digests, uint32_t log_N, uint32_t k,
                                                           uint64_t d_bstride) {
  const uint32_t node = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (node >= (1u << (log_N - k))) return;
  digests += blockIdx.y * d_bstride;
  const uint64_t top = (uint64_t)1 << (log_N + 1);
  const uint64_t *c = digests + (top - ((uint64_t)1 << (log_N - k + 2))) * 4 + (uint64_t)node * 8;
  uint64_t x = lane < 8 ? c[lane] : 0;
  x = pc::permute(x);
  uint64_t *o = digests + (top - ((uint64_t)1 << (log_N - k + 1))) * 4 + (uint64_t)node * 4;
  if (lane < 4) o[lane] = psd::canon(x);
}

// the row form: one 16-lane row per node (pc::permute_row), 16 nodes per
// block; rows past the level's end exit together
__global__ void __launch_bounds__(256) k_merkle_level_row(uint64_t *__restrict__ digests, uint32_t log_N, uint32_t k,
                                                          uint64_t d_bstride) {
  const uint32_t node = blockIdx.x * 16 + (threadIdx.x >> 4), l16 = threadIdx.x & 15;
  if (node >= (1u << (log_N - k))) return;
  digests += blockIdx.y * d_bstride;
  const uint64_t top = (uint64_t)1 << (log_N + 1);
  const uint64_t *c = digests + (top - ((uint64_t)1 << (log_N - k + 2))) * 4 + (uint64_t)node * 8;
  uint64_t x = l16 < 8 ? c[l16] : 0;
  x = pc::permute_row(x);
  uint64_t *o = digests + (top - ((uint64_t)1 << (log_N - k + 1))) * 4 + (uint64_t)node * 4;
  if (l16 < 4) o[l16] = psd::canon(x);
}

// levels of at most this many nodes (over all proofs of the launch) run one
// wave per node (k_merkle_level_coop) in launches of at most
// MERKLE_COOP_NBAT proofs: the latency-bound small batches of the
// aggregation tree's upper levels (one aggregation proof 12.5 -> 10.8 ms,
// 256-leaf subtree 0.42 -> 0.405 s); the leaf bench's 86-proof launches, which
// share a saturated GPU, keep the one-lane and fused forms (1184 vs 1200
// proofs/s with coop there; profiles/r05_ab_merkle_coop.log).
// The row form (k_merkle_level_row: four nodes per wave, DPP broadcasts) takes
// levels up to MERKLE_ROW_MAX nodes: 256-leaf subtree 0.387 -> 0.361-0.365 s
// with the row forms of the FRI leaves, the sliced openings and the per-coset
// LDE of few columns (profiles/r05_ab_small_batch.log).
// (path hook merkle_coop overrides the node bound, 0 = never)
constexpr long MERKLE_COOP_MAX = 8192, MERKLE_COOP_NBAT = 32, MERKLE_ROW_MAX = 32768;
// trees narrower than 2^MERKLE_FUSE_LOG nodes per level finish in one launch
// (one wave per block at 6, so no wave idles at the level barriers)
constexpr uint32_t MERKLE_FUSE_LOG = 6;
// path hook merkle_row=0: the one-wave-per-node form instead of the row form
// (read per tree: tests switch it in one process)
static bool merkle_row() { return path_opt("merkle_row", 1) != 0; }
static uint64_t merkle_coop_max(bool row) {
  return (uint64_t)path_opt("merkle_coop", row ? MERKLE_ROW_MAX : MERKLE_COOP_MAX);
}

void leaf_hash(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
               uint64_t *digests, uint32_t N, uint32_t nbat, uint64_t c_bstride, uint64_t s_bstride,
               uint64_t d_bstride, hipStream_t s) {
  dim3 grid((N + 255) / 256, nbat);
  const bool generic = path_opt("leaf_t", 1) == 0;  // path hook: the any-width form
  if (!nsalt && !generic) {
    switch (ncols) {
      case 135: k_leaf_hash_t<135><<<grid, 256, 0, s>>>(cols, stride, digests, N, c_bstride, d_bstride); return;
      case 20: k_leaf_hash_t<20><<<grid, 256, 0, s>>>(cols, stride, digests, N, c_bstride, d_bstride); return;
      case 16: k_leaf_hash_t<16><<<grid, 256, 0, s>>>(cols, stride, digests, N, c_bstride, d_bstride); return;
      default: break;
    }
  }
  k_leaf_hash<<<grid, 256, 0, s>>>(cols, stride, ncols, salt, nsalt, digests, N, c_bstride, s_bstride, d_bstride);
}

void merkle_tree_from(uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t d_bstride,
                      uint32_t first_level, hipStream_t s) {
  const uint32_t K = log_N - cap_h;  // levels above the leaves
  const bool row = merkle_row();
  const uint64_t coop_max = merkle_coop_max(row);
  // the batch size up to which the cooperative forms apply (path hook merkle_nbat)
  const uint64_t coop_nbat = (uint64_t)path_opt("merkle_nbat", MERKLE_COOP_NBAT);
  for (uint32_t k0 = first_level; k0 <= K;) {
    const uint32_t lc = log_N - k0;  // log2(nodes at level k0)
    if (nbat <= coop_nbat && ((uint64_t)nbat << lc) <= coop_max) {
      if (row)
        k_merkle_level_row<<<dim3(((1u << lc) + 15) / 16, nbat), 256, 0, s>>>(digests, log_N, k0, d_bstride);
      else
        k_merkle_level_coop<<<dim3(((1u << lc) + 3) / 4, nbat), 256, 0, s>>>(digests, log_N, k0, d_bstride);
      k0++;
      continue;
    }
    const uint32_t lb = lc < 8 ? lc : 8;
    // wide levels one launch each (a fused block would idle all but one
    // wave through its lower levels: measured 165 -> 222 ms per bench run);
    // from 2^MERKLE_FUSE_LOG nodes per tree down, the rest of the tree in one launch
    const uint32_t nl = lc > MERKLE_FUSE_LOG ? 1 : ((lb + 1) < (K - k0 + 1) ? (lb + 1) : (K - k0 + 1));
    dim3 grid(1u << (lc - lb), nbat);
    if (nl == 1)  // one level: the single-level kernel
      k_merkle_level<<<grid, 1u << lb, 0, s>>>(digests, log_N, k0, d_bstride);
    else
      k_merkle_levels<<<grid, 1u << lb, 0, s>>>(digests, log_N, k0, nl, d_bstride);
    k0 += nl;
  }
}

void merkle_tree(uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t d_bstride,
                 hipStream_t s) {
  merkle_tree_from(digests, log_N, cap_h, nbat, d_bstride, 1, s);
}

uint32_t leaf_hash_first(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
                         uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t c_bstride,
                         uint64_t s_bstride, uint64_t d_bstride, hipStream_t s) {
  (void)cap_h;
  leaf_hash(cols, stride, ncols, salt, nsalt, digests, 1u << log_N, nbat, c_bstride, s_bstride, d_bstride, s);
  return 1;
}

void leaf_hash_tree(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
                    uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t c_bstride,
                    uint64_t s_bstride, uint64_t d_bstride, hipStream_t s) {
  const uint32_t first = leaf_hash_first(cols, stride, ncols, salt, nsalt, digests, log_N, cap_h, nbat, c_bstride,
                                         s_bstride, d_bstride, s);
  merkle_tree_from(digests, log_N, cap_h, nbat, d_bstride, first, s);
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
