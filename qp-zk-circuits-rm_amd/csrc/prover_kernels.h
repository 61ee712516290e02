// prover_kernels.h — argument layouts and launchers of prover_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"
#include "ntt_device.h"

#include <vector>

namespace qpk {

// host helpers shared by the prover and the routine-level seams (prover.cpp)
std::vector<uint64_t> quotient_point_tables(uint32_t log_n, uint32_t rate_bits);
void pow_prestate(const uint64_t st12[12], uint32_t pos, uint64_t pre[24]);

// per-proof challenge block (device, u64 words)
enum : uint32_t {
  CH_BETA = 0, CH_GAMMA = 2, CH_ALPHA = 4, CH_PIH = 6, CH_ZETA = 10, CH_ZETA_NEXT = 12, CH_ZETA_INV = 14,
  CH_ZETA_NEXT_INV = 16, CH_FRI_ALPHA = 18, CH_ALPHA_POW_NC = 20, CH_FRI_BETA = 22,
  // the permutation argument scaled by 1 / beta (k_quotient_1r): (w + gamma +
  // beta s) = beta (w / beta + gamma / beta + s), the beta^len of a chunk's
  // products applied once per chunk (len = qdf, or the last chunk's R mod qdf)
  CH_BETA_INV = 32, CH_GAMMA_B = 34, CH_BETA_QDF = 36, CH_BETA_LAST = 38, CHAL_STRIDE = 40
};
constexpr uint32_t MAX_FRI_LAYERS = (CH_BETA_INV - CH_FRI_BETA) / 2;
// the permutation-argument words of the challenge block for challenges beta, gamma
void perm_challenges(uint64_t *ch, const uint64_t *beta, const uint64_t *gamma, uint32_t nc, uint32_t R, uint32_t qdf);
constexpr uint32_t OPEN_STRIDE = 520;  // 257 ext openings per proof (+pad)
constexpr uint32_t APOW_STRIDE = 256;  // alpha_c^i, i < #vanishing terms (per challenge)

// = QP_GATE_* (include/qpgpu.h)
enum GateKindDev : uint32_t {
  GK_NOOP = 0, GK_CONSTANT, GK_PUBLIC_INPUT, GK_BASE_SUM, GK_ARITHMETIC, GK_POSEIDON,
  GK_ARITH_EXT, GK_MUL_EXT, GK_RANDOM_ACCESS, GK_EXPONENTIATION, GK_REDUCING, GK_REDUCING_EXT, GK_POSEIDON_MDS,
  GK_COSET_INTERP, GK_COUNT
};
// RandomAccessGate width k_quotient_1r evaluates (the recursive verifier's
// RandomAccessGate::new_from_config shape); other widths take the per-gate
// launches (k_quotient_part)
constexpr uint32_t RA_QBITS = 4;
constexpr uint32_t MAX_GATES_DEV = 16;

struct GateDesc {
  uint32_t ngates = 0, nsel = 0;
  uint32_t kind[MAX_GATES_DEV] = {0}, param[MAX_GATES_DEV] = {0}, param2[MAX_GATES_DEV] = {0},
           param3[MAX_GATES_DEV] = {0}, sel_index[MAX_GATES_DEV] = {0}, grp_lo[MAX_GATES_DEV] = {0},
           grp_hi[MAX_GATES_DEV] = {0};
};

struct QuotientArgs {
  const uint64_t *cs_lde, *w_lde, *z_lde;
  uint64_t w_bstride, z_bstride;
  const uint64_t *chal, *tw, *apow;
  const uint64_t *xtab, *l0tab;  // [N] leaf order: x = g w_N^rev(t), L_0(x)
  uint64_t zh[16], zh_inv[16];
  uint64_t *q_out;
  uint64_t q_bstride;
  uint32_t log_n, rate_bits, R, qdf, num_constants;
  GateDesc g;
};

struct FriComposeArgs {
  const uint64_t *coeffs[4];
  uint64_t bstride[4];
  uint32_t npolys[4];
  uint32_t noracles, nnext, log_n;
  const uint64_t *chal;
  uint64_t *comp;
};

__global__ void k_pp_rows(const uint64_t *wires, const uint64_t *sigmas, const uint64_t *k_is, const uint64_t *chal,
                          uint64_t *prods, uint32_t log_n, uint32_t R, uint32_t qdf, uint32_t nc, uint64_t w_bstride,
                          uint64_t p_bstride, const uint64_t *tw);
template <int R, int QDF>
__global__ void k_pp_rows_t(const uint64_t *wires, const uint64_t *sigmas, const uint64_t *k_is, const uint64_t *chal,
                            uint64_t *prods, uint32_t log_n, uint64_t w_bstride, uint64_t p_bstride,
                            const uint64_t *tw);
template <bool STAGE>
__global__ void k_z_scan(const uint64_t *prods, uint64_t *zs, uint32_t log_n, uint32_t nc, uint32_t nchunks,
                         uint64_t p_bstride, uint64_t z_bstride);
__global__ void k_quotient_1r(QuotientArgs a);
template <int PART>
__global__ void k_quotient_part(QuotientArgs a, uint32_t gi, uint32_t last);
// the permutation terms + the gates of gmask that read routed wires only, one pass
template <int QDF>
__global__ void k_quotient_prefix(QuotientArgs a, uint32_t gmask, uint32_t last);
__global__ void k_qintt_gather_big(const uint64_t *vals, uint64_t *out, uint32_t log_n, uint32_t rate_bits,
                                   uint64_t v_bstride, uint64_t o_bstride);
__global__ void k_qintt_blocks(const uint64_t *vals, uint64_t *out, uint32_t log_n, uint32_t rate_bits,
                               uint64_t v_bstride, uint64_t o_bstride, const uint64_t *tw, const uint64_t *pt_inv,
                               uint64_t n_inv, uint64_t ginv);
__global__ void k_qintt_radix(const uint64_t *cbuf, uint64_t *coeffs, uint32_t log_n, uint32_t rate_bits,
                              uint64_t c_bstride, uint64_t o_bstride, uint64_t winv_r, uint64_t r_inv, uint64_t gninv);
// compute_quotient_polys (plonk/prover.rs) as launches, shared by the prover's
// stage 3 and the qp_quotient seam: the vanishing-polynomial values at every
// LDE point of nb proofs with the chosen kernel(s) ...
enum QuotientKernel : uint32_t {
  QK_1R,    // k_quotient_1r: the leaf gate set, every column read once
  QK_PARTS  // k_quotient_part: permutation terms, then one launch per gate (any gate list)
};
void quotient_values(const QuotientArgs &a, QuotientKernel k, uint32_t nb, hipStream_t s);
// ... and their coset iNTT into nc * qdf * n coefficients per proof (qvals
// [nb][nc][N] leaf order -> coeffs [nb][nc][qdf * n]; cbuf: scratch of the
// size of qvals); LDS form up to n = 2^LDS_LOG_MAX, HBM levels above
void quotient_coeffs(const Twiddles &tw, const uint64_t *qvals, uint64_t *cbuf, uint64_t *coeffs, uint32_t log_n,
                     uint32_t rate_bits, uint32_t nc, uint32_t nb, uint64_t v_bstride, uint64_t c_bstride,
                     uint64_t o_bstride, hipStream_t s);
constexpr int OPEN_PB = 8;  // polys per k_openings block
__global__ void k_openings(const uint64_t *coeffs, uint64_t c_bstride, uint32_t npolys, uint32_t log_n,
                           const uint64_t *pts, uint32_t pt_off, uint64_t *out, uint32_t out_off);
// every opening batch of a proof (OpeningSet::new's zeta and g*zeta
// evaluations) in one launch (+ a reduction when the coefficient range is
// split over S slices); out[b][OPEN_STRIDE] as k_openings writes it
constexpr int OPEN_MAX_SEG = 6, OPEN_MAX_SLICES = 16;
struct OpenSeg {
  const uint64_t *coeffs;
  uint64_t c_bstride;
  uint32_t npolys, pt_off, out_off, g0;
};
struct OpeningsArgs {
  OpenSeg seg[OPEN_MAX_SEG];
  uint32_t nseg = 0, ngroups = 0, log_n = 0, S = 1, ntot = 0;
  const uint64_t *pts = nullptr;
  uint64_t *out = nullptr, *part = nullptr;  // part: nb * OPEN_MAX_SLICES * OPEN_STRIDE words
};
__global__ void k_openings_seg(OpeningsArgs a);
__global__ void k_openings_reduce(const uint64_t *part, uint64_t *out, uint32_t ntot, uint32_t S);
void openings(OpeningsArgs a, uint32_t nb, hipStream_t s);
__global__ void k_fri_compose(FriComposeArgs a);
template <int MAXPER>
__global__ void k_fri_divide(const uint64_t *comp, uint64_t *fin, uint32_t log_n, const uint64_t *chal,
                             uint64_t f_bstride, uint64_t f_cstride);
__global__ void k_fri_leaf(const uint64_t *vals, uint64_t *dig, uint32_t log_len, uint32_t ab, uint64_t v_bstride,
                           uint64_t d_bstride);
__global__ void k_fri_leaf_row(const uint64_t *vals, uint64_t *dig, uint32_t log_len, uint32_t ab, uint64_t v_bstride,
                               uint64_t d_bstride);
// the leaf digests of a FRI layer for nb proofs (row or one-lane form by size)
void fri_leaf(const uint64_t *vals, uint64_t *dig, uint32_t log_len, uint32_t ab, uint64_t v_bstride,
              uint64_t d_bstride, uint32_t nb, hipStream_t s);
__global__ void k_fold(const uint64_t *cin, uint64_t *cout, uint32_t log_len, uint32_t ab, uint32_t layer,
                       const uint64_t *chal, uint64_t i_bstride, uint64_t o_bstride, uint32_t log_nz);
__global__ void k_pow_scan(const uint64_t *states, const uint32_t *pos, uint64_t *found, uint64_t *next, uint32_t nb,
                           uint32_t bits, uint64_t limit);
__global__ void k_gather_rows_b(const uint64_t *cols, uint64_t stride, uint64_t bstride, uint32_t ncols,
                                const uint32_t *idx, uint32_t nq, uint32_t shift, uint64_t *out, uint64_t o_bstride);
__global__ void k_gather_paths_b(const uint64_t *dig, uint64_t d_bstride, uint32_t log_leaves, uint32_t cap_h,
                                 const uint32_t *idx, uint32_t nq, uint32_t shift, uint64_t *out, uint64_t o_bstride);
__global__ void k_gather_fri_leaf(const uint64_t *vals, uint64_t v_bstride, uint32_t log_len, uint32_t ab,
                                  const uint32_t *idx, uint32_t nq, uint32_t shift, uint64_t *out, uint64_t o_bstride);

}  // namespace qpk
