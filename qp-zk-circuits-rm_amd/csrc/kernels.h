// kernels.h — launchers for the gfx950 kernels of the prover hot path.
// Layouts (device, all canonical u64):
//   polynomial matrices are column-major [col][len] with a column stride;
//   an LDE matrix holds column c at rows in Merkle-leaf order: row i is the
//   evaluation at g*w_N^{rev(i)} (plonky2 fri/oracle.rs reverse_index_bits);
//   digests of a tree: level 0 (N leaf digests) followed by each parent level
//   down to the 2^cap_h cap, 4 felts per digest.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qpk {

constexpr unsigned TW_LOG = 18;  // twiddle tables cover sizes up to 2^18 (degree-2^15 circuits at rate 3)
// Twiddle table layout (2^17 words per direction): [0, 2^16) holds w_{2^17}^j
// (= w_{2^18}^{2j}), [2^16, 2^17) holds w_{2^18}^{2j+1}.  Every size <= 2^17
// reads only the first half; the odd powers serve size-2^18 transforms
// (tw_get below: E = the w_{2^18} exponent).
__host__ __device__ __forceinline__ uint64_t tw_get(const uint64_t *__restrict__ tw, uint32_t E) {
  constexpr uint32_t Q = 1u << (TW_LOG - 2);  // 2^16
  const uint32_t j = E >> 1;
  const uint64_t *t = tw + ((E & 1) ? Q : 0);
  if (j < Q) return t[j];
  const uint64_t v = t[j - Q];
  return v ? 0xFFFFFFFF00000001ull - v : 0;  // w^(2^17) = -1
}
// the largest transform one workgroup holds in LDS (2^14 words: 135 KB with
// padding); larger ones (the degree-2^15 top levels of an aggregation tree)
// run their first log_n - 14 radix-2 levels in HBM, then 2^14-point blocks
// in LDS (ntt.hip "transforms beyond one workgroup's LDS")
constexpr uint32_t LDS_LOG_MAX = 14, BIG_LOG_MAX = 16;
// LDS slots of a size-n NTT workgroup: one pad slot per 32 elements (ntt16.h lp())
__host__ __device__ constexpr uint32_t ntt_lds_words(uint32_t n) { return n + (n >> 5); }
#define QP_HAVE_LDS_WORDS 1

constexpr unsigned LDE_MAX_RATE = 4;  // coset-fused LDE kernel: up to 16 cosets

struct Twiddles {
  // power tables of w = w_{2^TW_LOG} (fwd) and w^-1 (inv), 2^(TW_LOG-1) words
  // each in the even/odd layout above: read them only through tw_get / tw_pow
  // (a direct index tw[E] is NOT w^E)
  uint64_t *fwd = nullptr;
  uint64_t *inv = nullptr;
  // coset pre-twists of the fused LDE: for rate r (1..LDE_MAX_RATE), at
  // offset 16*(2^r - 2): ptw[16 s + m] = w_{16*2^r}^(s*m), s < 2^r, m < 16
  uint64_t *ptw = nullptr;
  // twiddles of the radix-16 LDS passes laid out per pass so a wave's lanes
  // (consecutive t) read consecutive words: for S = 2^L, 4 <= L <= TW_LOG, at
  // pt_offset(L): pt[m (S/16) + t] = w_S^(+-t brev4(m)), t < S/16, m < 16
  uint64_t *pt_fwd = nullptr, *pt_inv = nullptr;
  // merged first-pass twiddles of k_lde_cosets per (log_n, r), n = 16 T,
  // N = n 2^r: at mtw_off[log_n][r], mtw[(16 s + m) T + t] = w_N^(t (s + 2^r brev4(m)))
  // (N words per (log_n, r) re-read by every column's workgroup, from L2;
  // factored tables' extra vector loads cost more, profiles/r04_lde_ab.log)
  uint64_t *mtw = nullptr;
  uint64_t mtw_off[TW_LOG + 1][LDE_MAX_RATE + 1] = {};
};
__host__ __device__ constexpr uint32_t pt_offset(uint32_t log_S) { return (1u << log_S) - 16u; }
constexpr uint32_t LDE_COSETS_MIN_LOG = 10, LDE_COSETS_MAX_LOG = 14;  // k_lde_cosets sizes
__host__ __device__ inline uint32_t ptw_offset(uint32_t rate_bits) { return 16u * ((1u << rate_bits) - 2u); }

hipError_t twiddles_init(Twiddles &t, hipStream_t s);
void twiddles_free(Twiddles &t);

// values -> coefficients (plonky2 PolynomialValues::ifft), natural order in/out.
// batch: nbat independent matrices at in + b*in_bstride etc.
void intt(const Twiddles &t, const uint64_t *in, uint64_t in_stride, uint64_t *out, uint64_t out_stride,
          uint32_t ncols, uint32_t log_n, uint32_t nbat, uint64_t in_bstride, uint64_t out_bstride, hipStream_t s);

// in-place radix-2 DIF over each column (natural in, bit-reversed out, values
// canonical), any 2^log_n <= 2^BIG_LOG_MAX: HBM levels down to 2^LDS_LOG_MAX
// blocks, then the blocks in LDS.  nsub columns per (col, batch) group, nsub_stride apart
void dif_big(const Twiddles &t, uint64_t *x, uint64_t c_stride, uint32_t ncols, uint32_t nsub, uint64_t nsub_stride,
             uint32_t log_n, bool inv, uint32_t nbat, uint64_t bstride, hipStream_t s);
// in place per column: x[k] <- x[rev_n(k)] * c0 * base^k (the bit-reversal of a DIF result)
void bitrev_scale(uint64_t *x, uint64_t stride, uint32_t ncols, uint32_t log_n, uint64_t c0, uint64_t base,
                  uint32_t nbat, uint64_t bstride, hipStream_t s);

// coefficients (n) -> coset LDE (N = n << rate_bits) at shift*w_N^j, written in
// Merkle-leaf (bit-reversed) order.  (plonky2 PolynomialBatch::lde_values)
void lde(const Twiddles &t, const uint64_t *coeffs, uint64_t c_stride, uint64_t *out, uint64_t o_stride,
         uint32_t ncols, uint32_t log_n, uint32_t rate_bits, uint64_t shift, uint32_t nbat,
         uint64_t c_bstride, uint64_t o_bstride, hipStream_t s);

// leaf digests: hash_or_noop(row i of [ncols] ++ salt[i][nsalt])
void leaf_hash(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
               uint64_t *digests, uint32_t N, uint32_t nbat, uint64_t c_bstride, uint64_t s_bstride,
               uint64_t d_bstride, hipStream_t s);

// parent levels down to the cap (two_to_one), appended after the N leaf digests
void merkle_tree(uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t d_bstride,
                 hipStream_t s);
// leaf digests; returns the first level merkle_tree_from still builds (1)
uint32_t leaf_hash_first(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
                         uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t c_bstride,
                         uint64_t s_bstride, uint64_t d_bstride, hipStream_t s);
void merkle_tree_from(uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t d_bstride,
                      uint32_t first_level, hipStream_t s);
// leaf digests + the whole tree
void leaf_hash_tree(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint64_t *salt, uint32_t nsalt,
                    uint64_t *digests, uint32_t log_N, uint32_t cap_h, uint32_t nbat, uint64_t c_bstride,
                    uint64_t s_bstride, uint64_t d_bstride, hipStream_t s);

inline uint64_t tree_digest_count(uint32_t log_N, uint32_t cap_h) {
  uint64_t n = 0;
  for (uint32_t k = 0; k <= log_N - cap_h; k++) n += (uint64_t)1 << (log_N - k);
  return n;
}
inline uint64_t tree_level_offset(uint32_t log_N, uint32_t level) {  // in digests
  uint64_t o = 0;
  for (uint32_t k = 0; k < level; k++) o += (uint64_t)1 << (log_N - k);
  return o;
}

// row gather for query openings: out[q][c] = cols[c*stride + idx[q]]
void gather_rows(const uint64_t *cols, uint64_t stride, uint32_t ncols, const uint32_t *idx, uint32_t nidx,
                 uint64_t *out, hipStream_t s);
// Merkle paths: out[q][k][4] = sibling digest at level k of leaf idx[q]
void gather_paths(const uint64_t *digests, uint32_t log_N, uint32_t cap_h, const uint32_t *idx, uint32_t nidx,
                  uint64_t *out, hipStream_t s);

// bulk Poseidon permutations (states [n][12], in place)
void permute_batch(uint64_t *states, uint64_t n, hipStream_t s);

}  // namespace qpk
