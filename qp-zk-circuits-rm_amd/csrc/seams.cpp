// seams.cpp — routine-level entry points of the C ABI: the
// pieces of plonky2's prove() a patched qp-plonky2 routes to the GPU for ANY
// circuit over the supported gate set, not only the built-in ones (the
// aggregator's CircuitData::prove, wormhole/aggregator/src/circuits/tree.rs:136):
//   qp_quotient          plonk/prover.rs compute_quotient_polys (leaf gates: the
//                        single-read kernel; any gate list: the generic one)
//   qp_fri_layer_commit  fri/prover.rs fri_committed_trees, one reduction layer
//   qp_fri_fold          the same loop's coefficient fold with beta
//   qp_pow_grind         fri/prover.rs fri_proof_of_work (minimal witness)
// The transcript stays with the caller: each seam consumes the challenges the
// caller's Challenger drew and returns what it must observe next.
#include <stdlib.h>
#include <string.h>
#include <string>
#include <algorithm>
#include <new>
#include <vector>
#include "../../include/qpgpu.h"
#include "circuit_obj.h"
#include "ctx.h"
#include "field.h"
#include "kernels.h"
#include "prover_kernels.h"
#include "paths.h"

namespace {

struct DMem {  // device allocation owned by one call
  uint64_t *p = nullptr;
  hipError_t alloc(size_t words) { return hipMalloc(&p, (words ? words : 1) * 8); }
  ~DMem() {
    if (p) (void)hipFree(p);
  }
};

inline unsigned cdiv(uint64_t a, unsigned b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

struct qp_fri_layer {
  qp_ctx *ctx = nullptr;
  uint32_t log_values = 0, arity_bits = 0, cap_h = 0;
  uint64_t *d_vals = nullptr;  // [2][2^log_values] leaf order (c0 row, c1 row)
  uint64_t *d_dig = nullptr;   // tree digests over 2^(log_values - arity_bits) leaves
  ~qp_fri_layer() {
    if (d_vals) (void)hipFree(d_vals);
    if (d_dig) (void)hipFree(d_dig);
  }
};

extern "C" {

int qp_circuit_gate_desc(const qp_circuit *c, qp_gate_desc *g) {
  if (!c || !g) return QP_ERR_ARG;
  const qc::CircuitData &cd = c->cd;
  memset(g, 0, sizeof(*g));
  if (cd.gate_kinds.size() > QP_MAX_GATES || cd.groups.size() > QP_MAX_GATES) return QP_ERR_ARG;
  g->num_gates = (uint32_t)cd.gate_kinds.size();
  for (uint32_t i = 0; i < g->num_gates; i++) {
    switch (cd.gate_kinds[i]) {
      case qc::G_NOOP: g->kind[i] = QP_GATE_NOOP; break;
      case qc::G_CONSTANT: g->kind[i] = QP_GATE_CONSTANT; break;
      case qc::G_PUBLIC_INPUT: g->kind[i] = QP_GATE_PUBLIC_INPUT; break;
      case qc::G_BASE_SUM: g->kind[i] = QP_GATE_BASE_SUM; break;
      case qc::G_ARITHMETIC: g->kind[i] = QP_GATE_ARITHMETIC; break;
      case qc::G_POSEIDON: g->kind[i] = QP_GATE_POSEIDON; break;
      case qc::G_RANDOM_ACCESS: g->kind[i] = QP_GATE_RANDOM_ACCESS; break;
      case qc::G_ARITH_EXT: g->kind[i] = QP_GATE_ARITHMETIC_EXTENSION; break;
      case qc::G_MUL_EXT: g->kind[i] = QP_GATE_MUL_EXTENSION; break;
      case qc::G_REDUCING: g->kind[i] = QP_GATE_REDUCING; break;
      case qc::G_REDUCING_EXT: g->kind[i] = QP_GATE_REDUCING_EXTENSION; break;
      case qc::G_POSEIDON_MDS: g->kind[i] = QP_GATE_POSEIDON_MDS; break;
      case qc::G_COSET_INTERP: g->kind[i] = QP_GATE_COSET_INTERPOLATION; break;
      default: return QP_ERR_ARG;
    }
    g->param[i] = cd.gate_params[i];
    g->param2[i] = i < cd.gate_params2.size() ? cd.gate_params2[i] : 0;
    g->param3[i] = i < cd.gate_params3.size() ? cd.gate_params3[i] : 0;
    g->selector_index[i] = cd.selector_indices[i];
  }
  g->num_selectors = (uint32_t)cd.groups.size();
  for (uint32_t s = 0; s < g->num_selectors; s++) {
    g->group_lo[s] = cd.groups[s].first;
    g->group_hi[s] = cd.groups[s].second;
  }
  g->num_constants = cd.num_constants;
  g->num_routed_wires = cd.config.num_routed_wires;
  g->num_wires = cd.config.num_wires;
  g->quotient_degree_factor = cd.quotient_degree_factor;
  g->num_challenges = cd.config.num_challenges;
  g->num_gate_constraints = cd.num_gate_constraints;
  return QP_OK;
}

int qp_quotient(qp_ctx *ctx, const qp_batch *cs, const qp_batch *wires, const qp_batch *zs_pp, const qp_gate_desc *g,
                const uint64_t *betas, const uint64_t *gammas, const uint64_t *alphas, const uint64_t pi_hash[4],
                uint64_t *quotient_coeffs_out) {
  if (!ctx || !cs || !wires || !zs_pp || !g || !betas || !gammas || !alphas || !pi_hash || !quotient_coeffs_out)
    return QP_ERR_ARG;
  const uint32_t log_n = cs->log_n, rb = cs->rate_bits, logN = log_n + rb;
  const uint32_t R = g->num_routed_wires, qdf = g->quotient_degree_factor, nc = g->num_challenges;
  const uint32_t nchunks = qdf ? (R + qdf - 1) / qdf : 0;
  const uint32_t nterms = nc + nc * nchunks + g->num_gate_constraints;
  if (nc != 2 || g->num_gates == 0 || g->num_gates > QP_MAX_GATES || g->num_selectors == 0 ||
      g->num_selectors > QP_MAX_GATES || qdf != (1u << rb) || logN > qpk::TW_LOG || log_n < 6 ||
      log_n > qpk::BIG_LOG_MAX - 1 ||
      nterms > qpk::APOW_STRIDE || wires->log_n != log_n || zs_pp->log_n != log_n || wires->rate_bits != rb ||
      zs_pp->rate_bits != rb || cs->nbat != 1 || wires->nbat != 1 || zs_pp->nbat != 1 ||
      cs->npolys != g->num_constants + R || wires->npolys != g->num_wires || zs_pp->npolys != nc * nchunks ||
      wires->nsalt || zs_pp->nsalt || cs->nsalt || R > g->num_wires || rb > 4 ||
      g->num_constants < g->num_selectors) {
    ctx->err = "qp_quotient: unsupported shape (2 challenges, qdf = 2^rate_bits <= 16, 2^6 <= n <= 2^15, unsalted batches of one)";
    return QP_ERR_ARG;
  }
  // per-gate checks: known kind, selector in range, parameters inside the
  // kernels' bounds, every wire a gate reads < num_wires, every gate constant
  // < num_constants - num_selectors, constraint count <= num_gate_constraints
  const uint32_t W = g->num_wires, n_gc = g->num_constants - g->num_selectors;
  for (uint32_t s = 0; s < g->num_selectors; s++)
    if (g->group_lo[s] > g->group_hi[s] || g->group_hi[s] > g->num_gates) {
      ctx->err = "qp_quotient: selector group " + std::to_string(s) + " out of range";
      return QP_ERR_ARG;
    }
  bool fast = g->num_gates <= 8 && !qpk::path_opt("quotient_parts", 0);
  uint32_t seen = 0;
  for (uint32_t i = 0; i < g->num_gates; i++) {
    const uint32_t k = g->kind[i], p = g->param[i], p2 = g->param2[i], p3 = g->param3[i];
    uint64_t wires_used = 0, consts_used = 0, ncons = 0;
    // plonky2 places each gate in the selector group it belongs to
    bool ok = g->selector_index[i] < g->num_selectors && g->group_lo[g->selector_index[i]] <= i &&
              i < g->group_hi[g->selector_index[i]];
    switch (k) {
      case QP_GATE_NOOP: break;
      case QP_GATE_CONSTANT: wires_used = p; consts_used = p; ncons = p; break;
      case QP_GATE_PUBLIC_INPUT: wires_used = 4; ncons = 4; break;
      case QP_GATE_BASE_SUM: wires_used = 1ull + p; ncons = 1ull + p; break;
      case QP_GATE_ARITHMETIC: wires_used = 4ull * p; consts_used = 2; ncons = p; break;
      case QP_GATE_POSEIDON: wires_used = 135; ncons = 123; break;
      case QP_GATE_ARITHMETIC_EXTENSION: wires_used = 8ull * p; consts_used = 2; ncons = 2ull * p; break;
      case QP_GATE_MUL_EXTENSION: wires_used = 6ull * p; consts_used = 1; ncons = 2ull * p; break;
      case QP_GATE_RANDOM_ACCESS:
        ok = ok && p >= 1 && p <= 6;
        wires_used = (2ull + (1ull << (p & 63))) * p2 + p3 + (uint64_t)p2 * p;
        consts_used = p3;
        ncons = (p + 2ull) * p2 + p3;
        break;
      case QP_GATE_EXPONENTIATION: ok = ok && p >= 1; wires_used = 2ull + 2ull * p; ncons = p + 1ull; break;
      case QP_GATE_REDUCING: ok = ok && p >= 1; wires_used = 6ull + p + 2ull * (p - 1); ncons = 2ull * p; break;
      case QP_GATE_REDUCING_EXTENSION:
        ok = ok && p >= 1;
        wires_used = 6ull + 2ull * p + 2ull * (p - 1);
        ncons = 2ull * p;
        break;
      case QP_GATE_POSEIDON_MDS: wires_used = 48; ncons = 24; break;
      case QP_GATE_COSET_INTERPOLATION: {
        ok = ok && p >= 2 && p <= 6 && p2 >= 2 && p2 <= (1u << p);
        const uint64_t np = 1ull << (p & 63), nint = ok ? (np - 2) / (p2 - 1) : 0;
        wires_used = 1 + 2 * np + 4 + 4 * nint + 2;
        ncons = 4 + 4 * nint;
        break;
      }
      default: ok = false; break;
    }
    if (!ok || wires_used > W || consts_used > n_gc || ncons > g->num_gate_constraints) {
      ctx->err = "qp_quotient: gate " + std::to_string(i) + ": unknown gate kind, selector or parameters";
      return QP_ERR_ARG;
    }
    // the single-read kernel: the six leaf-circuit kinds, each at most once, the
    // non-Poseidon ones inside the routed wires it sweeps
    if (k > QP_GATE_POSEIDON || (seen >> k) & 1 || (k != QP_GATE_POSEIDON && wires_used > R)) fast = false;
    seen |= 1u << k;
  }
  const uint64_t n = 1ull << log_n, N = 1ull << logN;
  QP_HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  try {
    std::vector<uint64_t> tab = qpk::quotient_point_tables(log_n, rb);
    std::vector<uint64_t> chal(qpk::CHAL_STRIDE, 0), apow(2 * qpk::APOW_STRIDE, 0);
    for (uint32_t c = 0; c < 2; c++) {
      chal[qpk::CH_BETA + c] = gl::canon(betas[c]);
      chal[qpk::CH_GAMMA + c] = gl::canon(gammas[c]);
      uint64_t p = 1;
      for (uint32_t i = 0; i < nterms; i++) {
        apow[c * qpk::APOW_STRIDE + i] = p;
        p = gl::mul(p, gl::canon(alphas[c]));
      }
    }
    qpk::perm_challenges(chal.data(), chal.data() + qpk::CH_BETA, chal.data() + qpk::CH_GAMMA, 2, R, qdf);
    for (int i = 0; i < 4; i++) chal[qpk::CH_PIH + i] = gl::canon(pi_hash[i]);
    DMem d_tab, d_chal, d_apow, d_q, d_cbuf, d_out;
    QP_HIP_TRY(ctx, d_tab.alloc(tab.size()));
    QP_HIP_TRY(ctx, d_chal.alloc(chal.size()));
    QP_HIP_TRY(ctx, d_apow.alloc(apow.size()));
    QP_HIP_TRY(ctx, d_q.alloc(2 * N));
    QP_HIP_TRY(ctx, d_cbuf.alloc(2 * N));
    QP_HIP_TRY(ctx, d_out.alloc((uint64_t)nc * qdf * n));
    QP_HIP_TRY(ctx, hipMemcpyAsync(d_tab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, s));
    QP_HIP_TRY(ctx, hipMemcpyAsync(d_chal.p, chal.data(), chal.size() * 8, hipMemcpyHostToDevice, s));
    QP_HIP_TRY(ctx, hipMemcpyAsync(d_apow.p, apow.data(), apow.size() * 8, hipMemcpyHostToDevice, s));
    qpk::QuotientArgs a;
    a.cs_lde = cs->d_lde;
    a.w_lde = wires->d_lde;
    a.z_lde = zs_pp->d_lde;
    a.w_bstride = a.z_bstride = 0;
    a.chal = d_chal.p;
    a.tw = ctx->tw.fwd;
    a.apow = d_apow.p;
    a.xtab = d_tab.p;
    a.l0tab = d_tab.p + N;
    const uint32_t B = 1u << rb;
    const uint64_t wN = gl::root_of_unity(logN);
    for (uint32_t k = 0; k < B; k++) {
      const uint64_t xn = gl::pow(gl::mul(gl::GEN, gl::pow(wN, k)), n);
      a.zh[k] = gl::sub(xn, 1);
      a.zh_inv[k] = gl::inv(a.zh[k]);
    }
    a.q_out = d_q.p;
    a.q_bstride = 2 * N;
    a.log_n = log_n;
    a.rate_bits = rb;
    a.R = R;
    a.qdf = qdf;
    a.num_constants = g->num_constants;
    a.g.ngates = g->num_gates;
    a.g.nsel = g->num_selectors;
    for (uint32_t i = 0; i < g->num_gates; i++) {
      a.g.kind[i] = g->kind[i];
      a.g.param[i] = g->param[i];
      a.g.param2[i] = g->param2[i];
      a.g.param3[i] = g->param3[i];
      a.g.sel_index[i] = g->selector_index[i];
    }
    for (uint32_t i = 0; i < g->num_selectors; i++) {
      a.g.grp_lo[i] = g->group_lo[i];
      a.g.grp_hi[i] = g->group_hi[i];
    }
    // the prover's kernels: the single-read one for the leaf gate set, else
    // the permutation terms and one launch per gate
    const qpk::QuotientKernel qk = fast ? qpk::QK_1R : qpk::QK_PARTS;
    qpk::quotient_values(a, qk, 1, s);
    qpk::quotient_coeffs(ctx->tw, d_q.p, d_cbuf.p, d_out.p, log_n, rb, nc, 1, 2 * N, 2 * N, (uint64_t)nc * qdf * n, s);
    QP_HIP_TRY(ctx, hipGetLastError());
    QP_HIP_TRY(ctx, hipMemcpyAsync(quotient_coeffs_out, d_out.p, (uint64_t)nc * qdf * n * 8, hipMemcpyDeviceToHost, s));
    QP_HIP_TRY(ctx, hipStreamSynchronize(s));
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
  return QP_OK;
}

int qp_fri_layer_commit(qp_ctx *ctx, const uint64_t *coeffs, uint32_t log_coeffs, uint32_t log_values, uint64_t shift,
                        uint32_t arity_bits, uint32_t cap_height, uint64_t *cap_out, qp_fri_layer **out) {
  if (!ctx || !coeffs || !cap_out) return QP_ERR_ARG;
  if (out) *out = nullptr;
  if (log_values > qpk::TW_LOG || log_coeffs > log_values || log_coeffs < 1 || arity_bits < 1 || arity_bits > 4 ||
      log_values < arity_bits + cap_height) {
    ctx->err = "qp_fri_layer_commit: unsupported sizes";
    return QP_ERR_ARG;
  }
  // The reference keeps the folded coefficient vector at full length (zero
  // tail, fri/prover.rs fri_committed_trees); transform only the nonzero
  // prefix, rounded up to a power of two.
  uint64_t nz = 0;
  for (uint64_t i = 1ull << log_coeffs; i-- > 0;)
    if (gl::canon(coeffs[i]) | gl::canon(coeffs[(1ull << log_coeffs) + i])) {
      nz = i + 1;
      break;
    }
  uint32_t lc = 1;
  while ((1ull << lc) < nz) lc++;
  if (lc > qpk::BIG_LOG_MAX) {  // the coset LDE's sizes
    ctx->err = "qp_fri_layer_commit: more than 2^16 nonzero coefficients";
    return QP_ERR_ARG;
  }
  lc = std::min(lc, log_coeffs);
  const uint64_t Lin = 1ull << log_coeffs;
  QP_HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const uint64_t Lc = 1ull << lc, Lv = 1ull << log_values;
  const uint32_t log_leaves = log_values - arity_bits;
  qp_fri_layer *L = new (std::nothrow) qp_fri_layer();
  if (!L) return QP_ERR_OOM;
  L->ctx = ctx;
  L->log_values = log_values;
  L->arity_bits = arity_bits;
  L->cap_h = cap_height;
  DMem d_c;
  const uint64_t dbs = qpk::tree_digest_count(log_leaves, cap_height) * 4;
  hipError_t e = d_c.alloc(2 * Lc);
  if (!e) e = hipMalloc(&L->d_vals, 2 * Lv * 8);
  if (!e) e = hipMalloc(&L->d_dig, dbs * 8);
  if (e) {
    delete L;
    ctx->err = std::string("qp_fri_layer_commit: ") + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? QP_ERR_OOM : QP_ERR_HIP;
  }
  e = hipMemcpy2DAsync(d_c.p, Lc * 8, coeffs, Lin * 8, Lc * 8, 2, hipMemcpyHostToDevice, s);
  if (!e) {
    // values = coset_fft(coeffs, shift), leaf (bit-reversed) order
    qpk::lde(ctx->tw, d_c.p, Lc, L->d_vals, Lv, 2, lc, log_values - lc, shift, 1, 2 * Lc, 2 * Lv, s);
    qpk::fri_leaf(L->d_vals, L->d_dig, log_values, arity_bits, 2 * Lv, dbs, 1, s);
    qpk::merkle_tree(L->d_dig, log_leaves, cap_height, 1, dbs, s);
    e = hipGetLastError();
  }
  if (!e)
    e = hipMemcpyAsync(cap_out, L->d_dig + qpk::tree_level_offset(log_leaves, log_leaves - cap_height) * 4,
                       (size_t)32 << cap_height, hipMemcpyDeviceToHost, s);
  if (!e) e = hipStreamSynchronize(s);
  if (e) {
    delete L;
    ctx->err = std::string("qp_fri_layer_commit: ") + hipGetErrorString(e);
    return QP_ERR_HIP;
  }
  if (out) *out = L;
  else delete L;
  return QP_OK;
}

int qp_fri_layer_open(qp_fri_layer *L, const uint32_t *idx, uint32_t nidx, uint64_t *evals_out, uint64_t *siblings_out) {
  if (!L || (!idx && nidx) || (nidx && (!evals_out || !siblings_out))) return QP_ERR_ARG;
  if (!nidx) return QP_OK;
  qp_ctx *ctx = L->ctx;
  const uint32_t log_leaves = L->log_values - L->arity_bits;
  for (uint32_t i = 0; i < nidx; i++)
    if (idx[i] >> log_leaves) {
      ctx->err = "qp_fri_layer_open: leaf index out of range";
      return QP_ERR_ARG;
    }
  QP_HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const uint32_t W = 2u << L->arity_bits, depth = log_leaves - L->cap_h;
  DMem d_idx, d_ev, d_sib;
  QP_HIP_TRY(ctx, d_idx.alloc((nidx + 1) / 2));
  QP_HIP_TRY(ctx, d_ev.alloc((uint64_t)nidx * W));
  QP_HIP_TRY(ctx, d_sib.alloc((uint64_t)nidx * depth * 4));
  QP_HIP_TRY(ctx, hipMemcpyAsync(d_idx.p, idx, nidx * 4ull, hipMemcpyHostToDevice, s));
  const uint64_t dbs = qpk::tree_digest_count(log_leaves, L->cap_h) * 4;
  qpk::k_gather_fri_leaf<<<dim3(cdiv((uint64_t)nidx * W, 256), 1), 256, 0, s>>>(
      L->d_vals, 2ull << L->log_values, L->log_values, L->arity_bits, (const uint32_t *)d_idx.p, nidx, 0, d_ev.p, 0);
  if (depth)
    qpk::k_gather_paths_b<<<dim3(cdiv((uint64_t)nidx * depth * 4, 256), 1), 256, 0, s>>>(
        L->d_dig, dbs, log_leaves, L->cap_h, (const uint32_t *)d_idx.p, nidx, 0, d_sib.p, 0);
  QP_HIP_TRY(ctx, hipGetLastError());
  QP_HIP_TRY(ctx, hipMemcpyAsync(evals_out, d_ev.p, (uint64_t)nidx * W * 8, hipMemcpyDeviceToHost, s));
  if (depth)
    QP_HIP_TRY(ctx, hipMemcpyAsync(siblings_out, d_sib.p, (uint64_t)nidx * depth * 32, hipMemcpyDeviceToHost, s));
  QP_HIP_TRY(ctx, hipStreamSynchronize(s));
  return QP_OK;
}

void qp_fri_layer_free(qp_fri_layer *L) { delete L; }

int qp_fri_fold(qp_ctx *ctx, const uint64_t *coeffs, uint32_t log_coeffs, uint32_t arity_bits, const uint64_t beta[2],
                uint64_t *coeffs_out) {
  if (!ctx || !coeffs || !beta || !coeffs_out || arity_bits < 1 || arity_bits > log_coeffs || log_coeffs > 20)
    return QP_ERR_ARG;
  QP_HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const uint64_t L = 1ull << log_coeffs, Lo = L >> arity_bits;
  std::vector<uint64_t> chal(qpk::CHAL_STRIDE, 0);
  chal[qpk::CH_FRI_BETA] = gl::canon(beta[0]);
  chal[qpk::CH_FRI_BETA + 1] = gl::canon(beta[1]);
  DMem d_in, d_out, d_chal;
  QP_HIP_TRY(ctx, d_in.alloc(2 * L));
  QP_HIP_TRY(ctx, d_out.alloc(2 * Lo));
  QP_HIP_TRY(ctx, d_chal.alloc(chal.size()));
  QP_HIP_TRY(ctx, hipMemcpyAsync(d_in.p, coeffs, 2 * L * 8, hipMemcpyHostToDevice, s));
  QP_HIP_TRY(ctx, hipMemcpyAsync(d_chal.p, chal.data(), chal.size() * 8, hipMemcpyHostToDevice, s));
  qpk::k_fold<<<dim3(cdiv(Lo, 256), 1), 256, 0, s>>>(d_in.p, d_out.p, log_coeffs, arity_bits, 0, d_chal.p, 2 * L,
                                                     2 * Lo, log_coeffs);
  QP_HIP_TRY(ctx, hipGetLastError());
  QP_HIP_TRY(ctx, hipMemcpyAsync(coeffs_out, d_out.p, 2 * Lo * 8, hipMemcpyDeviceToHost, s));
  QP_HIP_TRY(ctx, hipStreamSynchronize(s));
  return QP_OK;
}

int qp_pow_grind(qp_ctx *ctx, const uint64_t *states, const uint32_t *pos, uint32_t n, uint32_t pow_bits,
                 uint64_t *witness_out) {
  if (!ctx || !states || !pos || !witness_out || !n || pow_bits == 0 || pow_bits > 32) return QP_ERR_ARG;
  for (uint32_t b = 0; b < n; b++)
    if (pos[b] >= 8) {  // Challenger invariant: input_buffer.len() < RATE when the witness is observed
      ctx->err = "qp_pow_grind: witness position must be < 8";
      return QP_ERR_ARG;
    }
  QP_HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  try {
    std::vector<uint64_t> pre((size_t)n * 24), found(n);
    for (uint32_t b = 0; b < n; b++) {
      uint64_t st[12];
      for (int i = 0; i < 12; i++) st[i] = gl::canon(states[(size_t)b * 12 + i]);
      qpk::pow_prestate(st, pos[b], pre.data() + (size_t)b * 24);
    }
    DMem d_pre, d_pos, d_next, d_found;
    QP_HIP_TRY(ctx, d_pre.alloc(pre.size()));
    QP_HIP_TRY(ctx, d_pos.alloc((n + 1) / 2));
    QP_HIP_TRY(ctx, d_next.alloc(n));
    QP_HIP_TRY(ctx, d_found.alloc(n));
    QP_HIP_TRY(ctx, hipMemcpyAsync(d_pre.p, pre.data(), pre.size() * 8, hipMemcpyHostToDevice, s));
    QP_HIP_TRY(ctx, hipMemcpyAsync(d_pos.p, pos, n * 4ull, hipMemcpyHostToDevice, s));
    QP_HIP_TRY(ctx, hipMemsetAsync(d_found.p, 0xFF, n * 8ull, s));
    QP_HIP_TRY(ctx, hipMemsetAsync(d_next.p, 0, n * 8ull, s));
    // the prover's single-launch minimal-witness search (prover.cpp stage 6)
    const uint64_t limit = 1ull << std::min<uint32_t>(pow_bits + 20, 62);
    qpk::k_pow_scan<<<2048, 256, 0, s>>>(d_pre.p, (const uint32_t *)d_pos.p, d_found.p, d_next.p, n, pow_bits, limit);
    QP_HIP_TRY(ctx, hipGetLastError());
    QP_HIP_TRY(ctx, hipMemcpyAsync(found.data(), d_found.p, n * 8ull, hipMemcpyDeviceToHost, s));
    QP_HIP_TRY(ctx, hipStreamSynchronize(s));
    for (uint32_t b = 0; b < n; b++)
      if (found[b] == ~0ull) {
        ctx->err = "qp_pow_grind: no witness below the search limit";
        return QP_ERR_STATE;
      }
    memcpy(witness_out, found.data(), n * 8ull);
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
  return QP_OK;
}

}  // extern "C"
