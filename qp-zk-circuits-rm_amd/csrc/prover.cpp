// prover.cpp — batched Plonky2 prove() on one MI355X (plonky2 plonk/prover.rs
// `prove` + fri/oracle.rs `prove_openings` + fri/prover.rs `fri_proof`,
// SURVEY.md 3.2), called from WormholeProver::prove
// (wormhole/prover/src/lib.rs:233-237) and the aggregator's
// CircuitData::prove (wormhole/aggregator/src/circuits/tree.rs:136).
//
// B proofs of one circuit move through every stage together: each stage is
// one batched kernel launch (blockIdx.y/z = proof), so a 256-proof batch
// fills the chip even where one proof alone would not.  The matrices stay
// resident in HBM between stages; only caps, openings, the final polynomial
// and the query openings cross PCIe.  The transcript (Challenger) runs on the
// host, per proof, on a thread pool, between stages.
#include <string.h>
#include <algorithm>
#include <chrono>
#include <atomic>
#include <memory>
#include <new>
#include <stdexcept>
#include <vector>
#include "../../include/qpgpu.h"
#include "circuit_obj.h"
#include "ctx.h"
#include "field.h"
#include "host_util.h"
#include "kernels.h"
#include "prover_kernels.h"
#include "witness_kernels.h"
#include "paths.h"


namespace {

using gl::ext;

struct DevBuf {
  uint64_t *p = nullptr;
  size_t words = 0;
  hipError_t alloc(size_t w) {
    words = w;
    return hipMalloc(&p, (w ? w : 1) * 8);
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

struct Tree {  // one Merkle-committed matrix per proof
  uint32_t npolys = 0, log_n = 0, rate_bits = 0, cap_h = 0;
  DevBuf vals, coeffs, lde, dig;
  uint64_t n() const { return 1ull << log_n; }
  uint64_t N() const { return 1ull << (log_n + rate_bits); }
  uint64_t ndig() const { return qpk::tree_digest_count(log_n + rate_bits, cap_h); }
  uint64_t cbs() const { return (uint64_t)npolys * n(); }
  uint64_t lbs() const { return (uint64_t)npolys * N(); }
  uint64_t dbs() const { return ndig() * 4; }
  hipError_t alloc(uint32_t np, uint32_t ln, uint32_t rb, uint32_t ch, uint32_t b, bool with_vals) {
    npolys = np; log_n = ln; rate_bits = rb; cap_h = ch;
    hipError_t e = with_vals ? vals.alloc((size_t)b * cbs()) : hipSuccess;
    if (!e) e = coeffs.alloc((size_t)b * cbs());
    if (!e) e = lde.alloc((size_t)b * lbs());
    if (!e) e = dig.alloc((size_t)b * dbs());
    return e;
  }
  // coefficients in `coeffs`: LDE + leaves + tree
  void build(qp_ctx *c, uint32_t nbat) {
    qpk::lde(c->tw, coeffs.p, n(), lde.p, N(), npolys, log_n, rate_bits, gl::GEN, nbat, cbs(), lbs(), c->stream);
    qpk::leaf_hash_tree(lde.p, N(), npolys, nullptr, 0, dig.p, log_n + rate_bits, cap_h, nbat, lbs(), 0, dbs(),
                        c->stream);
  }
  // values in `vals` ([nb][npolys][n]): ifft then build
  void build_from_values(qp_ctx *c, uint32_t nbat) {
    qpk::intt(c->tw, vals.p, n(), coeffs.p, n(), npolys, log_n, nbat, cbs(), cbs(), c->stream);
    build(c, nbat);
  }
};

inline unsigned cdiv(uint64_t a, unsigned b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

struct qp_prover {
  qp_ctx *ctx = nullptr;
  const qp_circuit *circuit = nullptr;
  uint32_t max_batch = 0;
  uint32_t log_n = 0, rate_bits = 0, cap_h = 0, W = 0, R = 0, NC = 0, nc = 0, npp = 0, qdf = 0, nchunks = 0;
  uint32_t nq = 0, pow_bits = 0, npis = 0;
  bool pow_forced = false;  // test-only: qp_prover_debug_force_pow
  uint64_t pow_forced_witness = 0;
  std::vector<uint32_t> arity;
  uint32_t final_len = 0;
  uint64_t cs_cap[64 * 4] = {0};
  uint64_t digest[4] = {0};
  qpk::GateDesc gdesc;
  std::vector<uint8_t> common;
  Tree cs;
  DevBuf sigmas, kis;
  Tree wires, zs, quot;
  DevBuf chal, apow, prods, qvals, cbuf, openings, open_part, comp, fin, pow_state, pow_found, pow_pos, pow_next, qidx,
      qout, qtab;
  std::vector<DevBuf> fvals, fdig, fcoef;
  size_t qout_words = 0;
  std::unique_ptr<qh::ThreadPool> pool;
  std::vector<uint64_t> h_chal, h_apow, h_caps, h_open, h_final, h_qout, h_powst, h_found;
  uint32_t nterms = 0;
  std::vector<uint32_t> h_qidx, h_pos;
  size_t proof_len = 0;
  double stage_ms[16] = {0};
  // optional per-kernel HIP-event timing on the prover's stream
  bool timing = false;
  struct KT {
    hipEvent_t a = nullptr, b = nullptr;
    double ms = 0, units = 0;
    uint64_t launches = 0;
    bool pending = false;
    double pend_units = 0;
  } kt[8];
  // device witness generation (witness.hip): schedule + per-proof slot values
  DevBuf wg_gens, wg_lvl, wg_lpos, wg_wslot, wg_wslot_cm, wg_in_slots, wg_pi_slots, wg_vals, wg_in, wg_err, wg_pis;
  uint32_t wg_nslots = 0, wg_nin = 0, wg_nlev = 0;
  bool has_poseidon_gate = false;
  bool has_random_access = false;
  bool generic_quotient = false;  // a gate outside k_quotient_1r's set (the recursive verifier's RandomAccess)
  uint64_t *h_in = nullptr;  // pinned [max_batch][wg_nin] commit() values
  std::vector<std::vector<uint64_t>> wscratch;  // per-proof slot values when host chains run split
  std::vector<uint32_t> h_werr;
  std::vector<uint64_t> h_wpis;
  ~qp_prover() {
    if (h_in) (void)hipHostFree(h_in);
  }
};

namespace qpk {

void perm_challenges(uint64_t *ch, const uint64_t *beta, const uint64_t *gamma, uint32_t nc, uint32_t R, uint32_t qdf) {
  const uint32_t last = R % qdf ? R % qdf : qdf;
  for (uint32_t c = 0; c < nc && c < 2; c++) {
    const uint64_t bi = gl::inv(beta[c]);
    ch[CH_BETA_INV + c] = bi;
    ch[CH_GAMMA_B + c] = gl::mul(gamma[c], bi);
    ch[CH_BETA_QDF + c] = gl::pow(beta[c], qdf);
    ch[CH_BETA_LAST + c] = gl::pow(beta[c], last);
  }
}

// proof-independent point tables of the quotient, leaf order t (point
// x = g w_N^rev(t)): xtab[t] = x, l0tab[t] = L_0(x) = Z_H(x) / (n (x - 1))
// (one batch inversion here instead of a field inversion per point per proof)
std::vector<uint64_t> quotient_point_tables(uint32_t log_n, uint32_t rate_bits) {
  const uint32_t logN = log_n + rate_bits;
  const uint64_t n = 1ull << log_n, N = 1ull << logN;
  const uint64_t wN = gl::root_of_unity(logN);
  std::vector<uint64_t> tab(2 * N), den(N), pre(N);
  for (uint64_t j = 0, w = 1; j < N; j++, w = gl::mul(w, wN)) {
    const uint64_t t = gl::rev_bits((uint32_t)j, logN);
    tab[t] = gl::mul(gl::GEN, w);
    den[t] = gl::mul(gl::sub(tab[t], 1), n % gl::P);
  }
  uint64_t acc = 1;
  for (uint64_t t = 0; t < N; t++) {
    pre[t] = acc;
    acc = gl::mul(acc, den[t]);
  }
  uint64_t inv = gl::inv(acc);
  for (uint64_t t = N; t-- > 0;) {
    const uint64_t dinv = gl::mul(inv, pre[t]);
    inv = gl::mul(inv, den[t]);
    const uint64_t zh = gl::sub(gl::pow(tab[t], n), 1);
    tab[N + t] = gl::mul(zh, dinv);
  }
  return tab;
}

// PoW search state with the candidate at lane pos; round 0 of the permutation
// is folded here: every lane but pos is candidate-independent, so
//   state after round 0 (+ round-1 constants) = K + coef * sbox(cand + rc_pos)
// with K[r] = sum_{j != pos} M[r][j] sbox(s_j + rc_j) + rc(1)_r and
// coef[r] = M[r][pos] (a small circulant/diagonal entry): pre = K[12] || coef[12]
void pow_prestate(const uint64_t st12[12], uint32_t pos, uint64_t pre[24]) {
  uint64_t y[12];
  for (uint32_t j = 0; j < 12; j++) y[j] = j == pos ? 0 : ps::sbox(gl::add(st12[j], ps::rc(j)));
  for (uint32_t r = 0; r < 12; r++) {
    uint64_t k = ps::rc(12 + r);
    for (uint32_t j = 0; j < 12; j++) {
      const uint64_t m = ps::mds_circ((j + 12 - r) % 12) + (r == 0 && j == 0 ? 8 : 0);
      if (j != pos) k = gl::add(k, gl::mul(m, y[j]));
      else pre[12 + r] = m;
    }
    pre[r] = k;
  }
}

}  // namespace qpk

namespace {

#define TRY(expr)                                                              \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      P->ctx->err = std::string(#expr) + ": " + hipGetErrorString(_e);         \
      return _e == hipErrorOutOfMemory ? QP_ERR_OOM : QP_ERR_HIP;              \
    }                                                                          \
  } while (0)

uint32_t oracle_width(const qp_prover *p, int o) {
  switch (o) {
    case 0: return p->NC + p->R;
    case 1: return p->W;
    case 2: return p->nc * p->nchunks;
    default: return p->nc * p->qdf;
  }
}

size_t proof_size(const qp_prover *p) {
  const size_t caps = ((size_t)4 << p->cap_h) * 8;
  size_t s = 3 * caps;
  s += (size_t)(p->NC + p->R + p->W + p->nc * p->nchunks + p->nc * p->qdf + p->nc) * 16;
  s += p->arity.size() * caps;
  const uint32_t logN = p->log_n + p->rate_bits;
  size_t q = 0;
  for (int o = 0; o < 4; o++) q += oracle_width(p, o) * 8 + 1 + (size_t)(logN - p->cap_h) * 32;
  uint32_t lg = logN;
  for (uint32_t ab : p->arity) {
    lg -= ab;
    q += (16ull << ab) + 1 + (size_t)(lg - p->cap_h) * 32;
  }
  s += q * p->nq;
  s += (size_t)p->final_len * 16 + 8 + 8 + (size_t)p->npis * 8;
  return s;
}

int setup(qp_prover *P) {
  qp_ctx *c = P->ctx;
  const qc::CircuitData &cd = P->circuit->cd;
  P->log_n = cd.degree_bits;
  P->rate_bits = cd.config.rate_bits;
  P->cap_h = cd.config.cap_height;
  P->W = cd.config.num_wires;
  P->R = cd.config.num_routed_wires;
  P->NC = cd.num_constants;
  P->nc = cd.config.num_challenges;
  P->npp = cd.num_partial_products;
  P->qdf = cd.quotient_degree_factor;
  P->nchunks = P->npp + 1;
  P->nq = cd.config.num_query_rounds;
  P->pow_bits = cd.config.pow_bits;
  P->npis = cd.num_public_inputs;
  P->arity = cd.fri_arity_bits;
  if (P->arity.size() > qpk::MAX_FRI_LAYERS) {
    c->err = "more FRI layers than the challenge block holds";
    return QP_ERR_ARG;
  }
  uint32_t tot = 0;
  for (auto a : P->arity) tot += a;
  P->final_len = 1u << (P->log_n - tot);
  P->common = cd.common_bytes();
  // zero_knowledge is accepted: under the reference's `no_random` feature the zk
  // config adds neither blinding rows nor salt columns (see DESIGN.md "zk")
  if (P->nc != 2 || (1u << P->rate_bits) != P->qdf || P->log_n > qpk::BIG_LOG_MAX - 1 || P->log_n < 6 ||
      P->log_n + P->rate_bits > qpk::TW_LOG || P->nchunks > 16 || P->NC > 8 || P->arity.size() > 8 || P->nq > 64) {
    c->err = "unsupported circuit shape for the GPU prover (need 2 challenges, qdf = blowup, 2^6 <= n <= 2^15)";
    return QP_ERR_ARG;
  }
  qpk::GateDesc &g = P->gdesc;
  g.ngates = (uint32_t)cd.gate_kinds.size();
  g.nsel = (uint32_t)cd.groups.size();
  for (uint32_t i = 0; i < g.ngates; i++) {
    switch (cd.gate_kinds[i]) {
      case qc::G_NOOP: g.kind[i] = qpk::GK_NOOP; break;
      case qc::G_CONSTANT: g.kind[i] = qpk::GK_CONSTANT; break;
      case qc::G_PUBLIC_INPUT: g.kind[i] = qpk::GK_PUBLIC_INPUT; break;
      case qc::G_BASE_SUM: g.kind[i] = qpk::GK_BASE_SUM; break;
      case qc::G_ARITHMETIC: g.kind[i] = qpk::GK_ARITHMETIC; break;
      case qc::G_POSEIDON:
        g.kind[i] = qpk::GK_POSEIDON;
        P->has_poseidon_gate = true;
        break;
      case qc::G_RANDOM_ACCESS:
        g.kind[i] = qpk::GK_RANDOM_ACCESS;
        P->has_random_access = true;
        // k_quotient_1r evaluates the RandomAccessGate of the recursive verifier's width
        if (cd.gate_params[i] != qpk::RA_QBITS) P->generic_quotient = true;
        break;
      // the other recursive-verifier gates: the generic (any gate list) kernel
      case qc::G_ARITH_EXT: g.kind[i] = qpk::GK_ARITH_EXT; P->generic_quotient = true; break;
      case qc::G_MUL_EXT: g.kind[i] = qpk::GK_MUL_EXT; P->generic_quotient = true; break;
      case qc::G_REDUCING: g.kind[i] = qpk::GK_REDUCING; P->generic_quotient = true; break;
      case qc::G_REDUCING_EXT: g.kind[i] = qpk::GK_REDUCING_EXT; P->generic_quotient = true; break;
      case qc::G_POSEIDON_MDS: g.kind[i] = qpk::GK_POSEIDON_MDS; P->generic_quotient = true; break;
      case qc::G_COSET_INTERP: g.kind[i] = qpk::GK_COSET_INTERP; P->generic_quotient = true; break;
      default:
        c->err = "unsupported gate kind for the GPU prover";
        return QP_ERR_ARG;
    }
    g.param[i] = cd.gate_params[i];
    g.param2[i] = i < cd.gate_params2.size() ? cd.gate_params2[i] : 0;
    g.param3[i] = i < cd.gate_params3.size() ? cd.gate_params3[i] : 0;
    g.sel_index[i] = cd.selector_indices[i];
  }
  for (uint32_t s = 0; s < g.nsel; s++) {
    g.grp_lo[s] = cd.groups[s].first;
    g.grp_hi[s] = cd.groups[s].second;
  }
  const uint64_t n = 1ull << P->log_n;
  const uint64_t N = n << P->rate_bits;
  TRY(hipSetDevice(c->device));
  // constants || sigmas commitment (CircuitBuilder::build preprocessing) + circuit digest
  TRY(P->cs.alloc(P->NC + P->R, P->log_n, P->rate_bits, P->cap_h, 1, true));
  TRY(hipMemcpyAsync(P->cs.vals.p, cd.constants_sigmas.data(), cd.constants_sigmas.size() * 8, hipMemcpyHostToDevice,
                     c->stream));
  P->cs.build_from_values(c, 1);
  TRY(hipGetLastError());
  TRY(P->sigmas.alloc((size_t)P->R * n));
  TRY(hipMemcpyAsync(P->sigmas.p, cd.constants_sigmas.data() + (size_t)P->NC * n, (size_t)P->R * n * 8,
                     hipMemcpyHostToDevice, c->stream));
  TRY(P->kis.alloc(P->R));
  TRY(hipMemcpyAsync(P->kis.p, cd.k_is.data(), P->R * 8ull, hipMemcpyHostToDevice, c->stream));
  const uint32_t logN = P->log_n + P->rate_bits;
  TRY(hipMemcpyAsync(P->cs_cap, P->cs.dig.p + qpk::tree_level_offset(logN, logN - P->cap_h) * 4,
                     (size_t)32 << P->cap_h, hipMemcpyDeviceToHost, c->stream));
  TRY(hipStreamSynchronize(c->stream));
  {
    std::vector<uint64_t> buf(P->cs_cap, P->cs_cap + (4u << P->cap_h));
    uint64_t dsep[4];
    qh::hash_pad(nullptr, 0, dsep);
    buf.insert(buf.end(), dsep, dsep + 4);
    buf.push_back(P->log_n);
    qh::hash_no_pad(buf.data(), buf.size(), P->digest);
  }
  const uint32_t B = P->max_batch;
  TRY(P->wires.alloc(P->W, P->log_n, P->rate_bits, P->cap_h, B, true));
  TRY(P->zs.alloc(P->nc * P->nchunks, P->log_n, P->rate_bits, P->cap_h, B, true));
  TRY(P->quot.alloc(P->nc * P->qdf, P->log_n, P->rate_bits, P->cap_h, B, false));
  TRY(P->chal.alloc((size_t)B * qpk::CHAL_STRIDE));
  P->nterms = P->nc + P->nc * P->nchunks + cd.num_gate_constraints;
  if (P->nterms > qpk::APOW_STRIDE) {
    c->err = "too many vanishing-polynomial terms for the alpha power table";
    return QP_ERR_ARG;
  }
  TRY(P->apow.alloc((size_t)B * 2 * qpk::APOW_STRIDE));
  P->h_apow.assign((size_t)B * 2 * qpk::APOW_STRIDE, 0);
  TRY(P->prods.alloc((size_t)B * P->nc * P->nchunks * n));
  TRY(P->qvals.alloc((size_t)B * P->nc * N));
  TRY(P->cbuf.alloc((size_t)B * P->nc * N));
  TRY(P->openings.alloc((size_t)B * qpk::OPEN_STRIDE));
  TRY(P->open_part.alloc((size_t)B * qpk::OPEN_MAX_SLICES * qpk::OPEN_STRIDE));
  TRY(P->comp.alloc((size_t)B * 4 * n));
  TRY(P->fin.alloc((size_t)B * 2 * N));
  TRY(hipMemsetAsync(P->fin.p, 0, (size_t)B * 2 * N * 8, c->stream));
  P->fvals.resize(P->arity.size());
  P->fdig.resize(P->arity.size());
  P->fcoef.resize(P->arity.size());
  uint32_t lg = logN;
  for (size_t l = 0; l < P->arity.size(); l++) {
    TRY(P->fvals[l].alloc(((size_t)B * 2) << lg));
    TRY(P->fdig[l].alloc((size_t)B * qpk::tree_digest_count(lg - P->arity[l], P->cap_h) * 4));
    lg -= P->arity[l];
    TRY(P->fcoef[l].alloc(((size_t)B * 2) << lg));
  }
  TRY(P->pow_state.alloc((size_t)B * 24));
  TRY(P->pow_found.alloc(B));
  TRY(P->pow_pos.alloc((B + 1) / 2));
  TRY(P->pow_next.alloc(B));
  {
    std::vector<uint64_t> tab = qpk::quotient_point_tables(P->log_n, P->rate_bits);
    TRY(P->qtab.alloc(tab.size()));
    TRY(hipMemcpy(P->qtab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  }
  TRY(P->qidx.alloc(((size_t)B * P->nq + 1) / 2));
  {
    size_t w = 0;
    for (int o = 0; o < 4; o++) w += (size_t)P->nq * (oracle_width(P, o) + (logN - P->cap_h) * 4);
    uint32_t lg2 = logN;
    for (uint32_t ab : P->arity) {
      lg2 -= ab;
      w += (size_t)P->nq * ((2u << ab) + (lg2 - P->cap_h) * 4);
    }
    P->qout_words = w;
    TRY(P->qout.alloc((size_t)B * w));
  }
  P->h_chal.assign((size_t)B * qpk::CHAL_STRIDE, 0);
  P->h_caps.assign((size_t)B * (4u << P->cap_h), 0);
  P->h_open.assign((size_t)B * qpk::OPEN_STRIDE, 0);
  P->h_final.assign((size_t)B * 2 * P->final_len, 0);
  P->h_qout.assign((size_t)B * P->qout_words, 0);
  P->h_qidx.assign((size_t)B * P->nq, 0);
  P->h_pos.assign(B, 0);
  P->h_powst.assign((size_t)B * 24, 0);
  P->h_found.assign(B, 0);
  {
    // witness tables: the slot -> wire expansion (k_witness_expand: every
    // circuit, also for host-generated witnesses) and, for circuits whose
    // generators all have a device form, the level-scheduled generator list
    auto up32 = [&](DevBuf &d, const std::vector<uint32_t> &v) -> hipError_t {
      hipError_t e = d.alloc((v.size() + 1) / 2);
      if (!e && !v.empty()) e = hipMemcpy(d.p, v.data(), v.size() * 4, hipMemcpyHostToDevice);
      return e;
    };
    P->wg_nslots = cd.num_slots;
    P->wg_nin = (uint32_t)cd.input_slots.size();
    TRY(up32(P->wg_wslot_cm, cd.wire_slot_cm));
    TRY(up32(P->wg_pi_slots, cd.pi_slots));
    TRY(P->wg_vals.alloc((size_t)B * P->wg_nslots));
    TRY(P->wg_pis.alloc((size_t)B * std::max<uint32_t>(P->npis, 1)));
    if (cd.device_witness) {
      P->wg_nlev = (uint32_t)cd.level_off.size() - 1;
      TRY(P->wg_gens.alloc(cd.dev_gens.size() * 5));
      TRY(hipMemcpy(P->wg_gens.p, cd.dev_gens.data(), cd.dev_gens.size() * sizeof(qc::DevGen), hipMemcpyHostToDevice));
      TRY(up32(P->wg_lvl, cd.level_off));
      TRY(up32(P->wg_lpos, cd.level_pos));
      TRY(up32(P->wg_wslot, cd.dev_wslot));
      TRY(up32(P->wg_in_slots, cd.input_slots));
      TRY(P->wg_in.alloc((size_t)B * std::max<uint32_t>(P->wg_nin, 1)));
      TRY(P->wg_err.alloc((B + 1) / 2));
      TRY(hipHostMalloc((void **)&P->h_in, (size_t)B * std::max<uint32_t>(P->wg_nin, 1) * 8, hipHostMallocDefault));
      P->h_werr.assign(B, 0);
    }
    P->h_wpis.assign((size_t)B * std::max<uint32_t>(P->npis, 1), 0);
  }
  TRY(hipStreamSynchronize(c->stream));
  P->proof_len = proof_size(P);
  unsigned hw = std::thread::hardware_concurrency();
  unsigned nthreads = std::min<unsigned>(hw ? hw : 4, 16);
  P->pool.reset(new qh::ThreadPool(nthreads > 1 ? nthreads - 1 : 0));
  return QP_OK;
}

// host threads of this prover's commit()/query pool, the calling thread
// included: several provers in one process split the host cores between them
// (qp_prover_set_host_threads(p, cores / provers)) instead of each taking all
extern "C" int qp_prover_set_host_threads(qp_prover *P, uint32_t nthreads) {
  if (!P || nthreads == 0 || nthreads > 256) return QP_ERR_ARG;
  P->pool.reset(new qh::ThreadPool(nthreads - 1));
  return QP_OK;
}

// kernel timers: 0 = LDE of the wires (NTT), 1 = leaf hashing of the wires,
// 2 = Merkle tree levels of the wires, 3 = quotient evaluation
void kt_begin(qp_prover *P, int k) {
  if (!P->timing) return;
  auto &t = P->kt[k];
  if (!t.a) {
    (void)hipEventCreate(&t.a);
    (void)hipEventCreate(&t.b);
  }
  (void)hipEventRecord(t.a, P->ctx->stream);
}
void kt_end(qp_prover *P, int k, double units) {
  if (!P->timing) return;
  auto &t = P->kt[k];
  (void)hipEventRecord(t.b, P->ctx->stream);
  t.pending = true;
  t.pend_units = units;
}
void kt_collect(qp_prover *P) {  // after a stream sync
  for (auto &t : P->kt)
    if (t.pending) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
        t.ms += ms;
        t.units += t.pend_units;
        t.launches++;
      }
      t.pending = false;
    }
}

int fetch_caps(qp_prover *P, const uint64_t *dig_base, uint64_t dbs, uint32_t log_leaves, uint32_t nb) {
  qp_ctx *c = P->ctx;
  const uint64_t off = qpk::tree_level_offset(log_leaves, log_leaves - P->cap_h) * 4;
  const size_t cw = 4u << P->cap_h;
  TRY(hipMemcpy2DAsync(P->h_caps.data(), cw * 8, dig_base + off, dbs * 8, cw * 8, nb, hipMemcpyDeviceToHost,
                       c->stream));
  TRY(hipStreamSynchronize(c->stream));
  kt_collect(P);
  return QP_OK;
}

int push_chal(qp_prover *P, uint32_t nb) {
  TRY(hipMemcpyAsync(P->chal.p, P->h_chal.data(), (size_t)nb * qpk::CHAL_STRIDE * 8, hipMemcpyHostToDevice,
                     P->ctx->stream));
  return QP_OK;
}

// Every device table a launch sequence reads must exist for this circuit: a
// missing one becomes QP_ERR_STATE naming it instead of a kernel fault (the
// class of 0d3293f: the slot -> wire expansion tables were once skipped for
// host-witness circuits).  which: 0 = prove_batch (d_wires given or not),
// 1 = device witness generation.
int check_tables(qp_prover *P, int which, bool wires_on_device) {
  struct T {
    const char *name;
    const void *p;
  };
  std::vector<T> need;
  if (which == 0) {
    need = {{"tw.fwd", P->ctx->tw.fwd}, {"tw.pt_inv", P->ctx->tw.pt_inv}, {"cs.lde", P->cs.lde.p},
            {"cs.coeffs", P->cs.coeffs.p}, {"sigmas", P->sigmas.p}, {"kis", P->kis.p},
            {"wires.coeffs", P->wires.coeffs.p}, {"wires.lde", P->wires.lde.p}, {"wires.dig", P->wires.dig.p},
            {"zs.vals", P->zs.vals.p}, {"zs.coeffs", P->zs.coeffs.p}, {"zs.lde", P->zs.lde.p},
            {"zs.dig", P->zs.dig.p}, {"quot.coeffs", P->quot.coeffs.p}, {"quot.lde", P->quot.lde.p},
            {"quot.dig", P->quot.dig.p}, {"chal", P->chal.p}, {"apow", P->apow.p}, {"prods", P->prods.p},
            {"qvals", P->qvals.p}, {"cbuf", P->cbuf.p}, {"openings", P->openings.p}, {"comp", P->comp.p},
            {"fin", P->fin.p}, {"pow_state", P->pow_state.p}, {"pow_found", P->pow_found.p},
            {"qidx", P->qidx.p}, {"qout", P->qout.p}, {"qtab", P->qtab.p}};
    if (!wires_on_device) need.push_back({"wires.vals", P->wires.vals.p});
    for (size_t l = 0; l < P->arity.size(); l++) {
      need.push_back({"fri.vals", l < P->fvals.size() ? P->fvals[l].p : nullptr});
      need.push_back({"fri.dig", l < P->fdig.size() ? P->fdig[l].p : nullptr});
      need.push_back({"fri.coeffs", l < P->fcoef.size() ? P->fcoef[l].p : nullptr});
    }
  } else {
    need = {{"wg_gens", P->wg_gens.p}, {"wg_lvl", P->wg_lvl.p}, {"wg_lpos", P->wg_lpos.p}, {"wg_wslot", P->wg_wslot.p},
            {"wg_wslot_cm", P->wg_wslot_cm.p}, {"wg_pi_slots", P->wg_pi_slots.p}, {"wg_vals", P->wg_vals.p},
            {"wg_pis", P->wg_pis.p}, {"wg_err", P->wg_err.p}, {"h_in", P->h_in}};
    if (P->wg_nin) {
      need.push_back({"wg_in_slots", P->wg_in_slots.p});
      need.push_back({"wg_in", P->wg_in.p});
    }
  }
  for (const T &t : need)
    if (!t.p) {
      P->ctx->err = std::string("device table '") + t.name + "' is missing for this circuit (" +
                    (which ? "device witness generation" : "prove") + ")";
      return QP_ERR_STATE;
    }
  return QP_OK;
}

struct ProofState {
  qh::Challenger t;
  uint64_t pih[4];
  std::vector<uint64_t> caps[3];
  std::vector<uint64_t> fri_caps;
  uint64_t pow_witness = 0;
};

using Clock = std::chrono::steady_clock;

// d_wires: device wire matrices [nb][W][n] (caller-resident or generated on
// the device into P->wires.vals), or null to upload wires_host[b]
int prove_batch(qp_prover *P, const uint64_t *d_wires, const uint64_t *const *wires_host,
                const uint64_t *const *pis_host, uint32_t nb, uint8_t *out, size_t stride, size_t *lens) {
  qp_ctx *c = P->ctx;
  hipStream_t s = c->stream;
  const uint64_t n = 1ull << P->log_n;
  const uint32_t logN = P->log_n + P->rate_bits;
  const uint64_t N = 1ull << logN;
  const size_t capw = 4u << P->cap_h;
  const uint32_t nc = P->nc;
  std::vector<ProofState> st(nb);
  auto T0 = Clock::now();
  auto lap = [&](int k) {
    auto t = Clock::now();
    P->stage_ms[k] += std::chrono::duration<double, std::milli>(t - T0).count();
    T0 = t;
  };
  TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = check_tables(P, 0, d_wires != nullptr))) return rc;

  // ---- 1. wires commitment
  const uint64_t *wv = d_wires;
  if (!wv) {
    for (uint32_t b = 0; b < nb; b++)
      TRY(hipMemcpyAsync(P->wires.vals.p + b * P->wires.cbs(), wires_host[b], P->wires.cbs() * 8,
                         hipMemcpyHostToDevice, s));
    wv = P->wires.vals.p;
  }
  {
    Tree &t = P->wires;
    qpk::intt(c->tw, wv, t.n(), t.coeffs.p, t.n(), t.npolys, t.log_n, nb, t.cbs(), t.cbs(), s);
    kt_begin(P, 0);
    qpk::lde(c->tw, t.coeffs.p, t.n(), t.lde.p, t.N(), t.npolys, t.log_n, t.rate_bits, gl::GEN, nb, t.cbs(), t.lbs(), s);
    kt_end(P, 0, (double)nb * t.npolys * 8.0 * (double)(t.n() + t.N()));
    kt_begin(P, 1);
    const uint32_t first = qpk::leaf_hash_first(t.lde.p, t.N(), t.npolys, nullptr, 0, t.dig.p, t.log_n + t.rate_bits,
                                                t.cap_h, nb, t.lbs(), 0, t.dbs(), s);
    // permutations: the leaves' (+ the first level's when fused)
    const double lvl1 = first == 2 ? (double)(t.N() / 2) : 0.0;
    kt_end(P, 1, (double)nb * ((double)t.N() * ((t.npolys + 7) / 8) + lvl1));
    kt_begin(P, 2);
    qpk::merkle_tree_from(t.dig.p, t.log_n + t.rate_bits, t.cap_h, nb, t.dbs(), first, s);
    kt_end(P, 2, (double)nb * ((double)t.N() - (1u << t.cap_h) - lvl1));
  }
  TRY(hipGetLastError());
  if ((rc = fetch_caps(P, P->wires.dig.p, P->wires.dbs(), logN, nb))) return rc;
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    qh::hash_no_pad(pis_host[b], P->npis, S.pih);
    S.caps[0].assign(P->h_caps.begin() + b * capw, P->h_caps.begin() + (b + 1) * capw);
    S.t.observe(P->digest, 4);
    S.t.observe(S.pih, 4);
    S.t.observe(S.caps[0].data(), capw);
    uint64_t *ch = P->h_chal.data() + b * qpk::CHAL_STRIDE;
    for (uint32_t i = 0; i < nc; i++) ch[qpk::CH_BETA + i] = S.t.get();
    for (uint32_t i = 0; i < nc; i++) ch[qpk::CH_GAMMA + i] = S.t.get();
    qpk::perm_challenges(ch, ch + qpk::CH_BETA, ch + qpk::CH_GAMMA, nc, P->R, P->qdf);
    for (int i = 0; i < 4; i++) ch[qpk::CH_PIH + i] = S.pih[i];
  });
  if ((rc = push_chal(P, nb))) return rc;
  lap(0);

  // ---- 2. partial products + Z (a9), commitment
  const uint64_t pbs = (uint64_t)nc * P->nchunks * n;
  if (P->R == 80 && P->qdf == 8 && nc == 2)
    qpk::k_pp_rows_t<80, 8><<<dim3(cdiv(n, 256), nb), 256, 0, s>>>(wv, P->sigmas.p, P->kis.p, P->chal.p, P->prods.p,
                                                                    P->log_n, P->wires.cbs(), pbs, c->tw.fwd);
  else
    qpk::k_pp_rows<<<dim3(cdiv(n, 256), nb), 256, 0, s>>>(wv, P->sigmas.p, P->kis.p, P->chal.p, P->prods.p,
                                                           P->log_n, P->R, P->qdf, nc, P->wires.cbs(), pbs, c->tw.fwd);
  if (P->log_n <= qpk::LDS_LOG_MAX)
    qpk::k_z_scan<true><<<dim3(nc, nb), 1024, 8u * (qpk::ntt_lds_words(n) + 1024), s>>>(
        P->prods.p, P->zs.vals.p, P->log_n, nc, P->nchunks, pbs, P->zs.cbs());
  else
    qpk::k_z_scan<false><<<dim3(nc, nb), 1024, 8u * 1024, s>>>(P->prods.p, P->zs.vals.p, P->log_n, nc, P->nchunks,
                                                              pbs, P->zs.cbs());
  P->zs.build_from_values(c, nb);
  TRY(hipGetLastError());
  if ((rc = fetch_caps(P, P->zs.dig.p, P->zs.dbs(), logN, nb))) return rc;
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    S.caps[1].assign(P->h_caps.begin() + b * capw, P->h_caps.begin() + (b + 1) * capw);
    S.t.observe(S.caps[1].data(), capw);
    uint64_t *ch = P->h_chal.data() + b * qpk::CHAL_STRIDE;
    for (uint32_t i = 0; i < nc; i++) ch[qpk::CH_ALPHA + i] = S.t.get();
    for (uint32_t c2 = 0; c2 < 2; c2++) {
      uint64_t *ap = P->h_apow.data() + (b * 2 + c2) * qpk::APOW_STRIDE, p = 1;
      for (uint32_t i = 0; i < P->nterms; i++) {
        ap[i] = p;
        p = gl::mul(p, ch[qpk::CH_ALPHA + c2]);
      }
    }
  });
  if ((rc = push_chal(P, nb))) return rc;
  TRY(hipMemcpyAsync(P->apow.p, P->h_apow.data(), (size_t)nb * 2 * qpk::APOW_STRIDE * 8, hipMemcpyHostToDevice, s));
  lap(1);

  // ---- 3. quotient polynomials (a8)
  {
    qpk::QuotientArgs a;
    a.cs_lde = P->cs.lde.p;
    a.w_lde = P->wires.lde.p;
    a.z_lde = P->zs.lde.p;
    a.w_bstride = P->wires.lbs();
    a.z_bstride = P->zs.lbs();
    a.chal = P->chal.p;
    a.tw = c->tw.fwd;
    a.apow = P->apow.p;
    a.xtab = P->qtab.p;
    a.l0tab = P->qtab.p + N;
    const uint32_t B = 1u << P->rate_bits;
    const uint64_t wN = gl::root_of_unity(logN);
    for (uint32_t k = 0; k < B; k++) {
      uint64_t xn = gl::pow(gl::mul(gl::GEN, gl::pow(wN, k)), n);
      a.zh[k] = gl::sub(xn, 1);
      a.zh_inv[k] = gl::inv(a.zh[k]);
    }
    a.q_out = P->qvals.p;
    a.q_bstride = (uint64_t)nc * N;
    a.log_n = P->log_n;
    a.rate_bits = P->rate_bits;
    a.R = P->R;
    a.qdf = P->qdf;
    a.num_constants = P->NC;
    a.g = P->gdesc;
    kt_begin(P, 3);
    // the leaf gate set: one single-read pass; any other gate list (and the
    // path hook quotient_parts=1): the per-gate launches
    const qpk::QuotientKernel qk =
        P->generic_quotient || qpk::path_opt("quotient_parts", 0) ? qpk::QK_PARTS : qpk::QK_1R;
    qpk::quotient_values(a, qk, nb, s);
    kt_end(P, 3, (double)nb * N);
    qpk::quotient_coeffs(c->tw, P->qvals.p, P->cbuf.p, P->quot.coeffs.p, P->log_n, P->rate_bits, nc, nb,
                         (uint64_t)nc * N, (uint64_t)nc * N, P->quot.cbs(), s);
    P->quot.build(c, nb);
    TRY(hipGetLastError());
  }
  if ((rc = fetch_caps(P, P->quot.dig.p, P->quot.dbs(), logN, nb))) return rc;
  const uint64_t g_n = gl::root_of_unity(P->log_n);
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    S.caps[2].assign(P->h_caps.begin() + b * capw, P->h_caps.begin() + (b + 1) * capw);
    S.t.observe(S.caps[2].data(), capw);
    ext z = S.t.get_ext();
    ext zn = gl::ext_scale(z, g_n);
    ext zi = gl::ext_inv(z), zni = gl::ext_inv(zn);
    uint64_t *ch = P->h_chal.data() + b * qpk::CHAL_STRIDE;
    ch[qpk::CH_ZETA] = z.c0; ch[qpk::CH_ZETA + 1] = z.c1;
    ch[qpk::CH_ZETA_NEXT] = zn.c0; ch[qpk::CH_ZETA_NEXT + 1] = zn.c1;
    ch[qpk::CH_ZETA_INV] = zi.c0; ch[qpk::CH_ZETA_INV + 1] = zi.c1;
    ch[qpk::CH_ZETA_NEXT_INV] = zni.c0; ch[qpk::CH_ZETA_NEXT_INV + 1] = zni.c1;
  });
  if ((rc = push_chal(P, nb))) return rc;
  lap(2);

  // ---- 4. openings (a10)
  {
    const uint32_t ncs = P->NC + P->R, nzs = nc * P->nchunks, nq = nc * P->qdf;
    // the zeta batch in oracle order (constants+sigmas, wires, Z+partial
    // products, quotient chunks), then the g*zeta batch (the Zs)
    qpk::OpeningsArgs oa;
    const struct { const uint64_t *c; uint64_t bs; uint32_t np, pt; } segs[5] = {
        {P->cs.coeffs.p, 0, ncs, qpk::CH_ZETA},
        {P->wires.coeffs.p, P->wires.cbs(), P->W, qpk::CH_ZETA},
        {P->zs.coeffs.p, P->zs.cbs(), nzs, qpk::CH_ZETA},
        {P->quot.coeffs.p, P->quot.cbs(), nq, qpk::CH_ZETA},
        {P->zs.coeffs.p, P->zs.cbs(), nc, qpk::CH_ZETA_NEXT}};
    uint32_t off = 0;
    for (const auto &g : segs) {
      if (!g.np) continue;
      oa.seg[oa.nseg++] = qpk::OpenSeg{g.c, g.bs, g.np, g.pt, off, 0};
      off += g.np;
    }
    oa.log_n = P->log_n;
    oa.pts = P->chal.p;
    oa.out = P->openings.p;
    oa.part = P->open_part.p;
    qpk::openings(oa, nb, s);
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(P->h_open.data(), P->openings.p, (size_t)nb * qpk::OPEN_STRIDE * 8, hipMemcpyDeviceToHost, s));
    TRY(hipStreamSynchronize(s));
  }
  const uint32_t nopen = P->NC + P->R + P->W + nc * P->nchunks + nc * P->qdf;
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    const uint64_t *o = P->h_open.data() + b * qpk::OPEN_STRIDE;
    S.t.observe(o, 2 * (size_t)nopen);           // zeta batch in oracle order
    S.t.observe(o + 2 * (size_t)nopen, 2 * nc);  // g*zeta batch
    ext al = S.t.get_ext();
    ext ap = gl::ext_pow(al, nc);
    uint64_t *ch = P->h_chal.data() + b * qpk::CHAL_STRIDE;
    ch[qpk::CH_FRI_ALPHA] = al.c0; ch[qpk::CH_FRI_ALPHA + 1] = al.c1;
    ch[qpk::CH_ALPHA_POW_NC] = ap.c0; ch[qpk::CH_ALPHA_POW_NC + 1] = ap.c1;
  });
  if ((rc = push_chal(P, nb))) return rc;
  lap(3);

  // ---- 5. FRI (a11)
  {
    qpk::FriComposeArgs fa;
    fa.coeffs[0] = P->cs.coeffs.p; fa.bstride[0] = 0; fa.npolys[0] = P->NC + P->R;
    fa.coeffs[1] = P->wires.coeffs.p; fa.bstride[1] = P->wires.cbs(); fa.npolys[1] = P->W;
    fa.coeffs[2] = P->zs.coeffs.p; fa.bstride[2] = P->zs.cbs(); fa.npolys[2] = nc * P->nchunks;
    fa.coeffs[3] = P->quot.coeffs.p; fa.bstride[3] = P->quot.cbs(); fa.npolys[3] = nc * P->qdf;
    fa.noracles = 4; fa.nnext = nc; fa.log_n = P->log_n;
    fa.chal = P->chal.p;
    fa.comp = P->comp.p;
    qpk::k_fri_compose<<<dim3(cdiv(n, 256), nb), 256, 0, s>>>(fa);
    if (n / std::min<uint64_t>(1024, n / 8) <= 16)
      qpk::k_fri_divide<16><<<nb, (unsigned)std::min<uint64_t>(1024, n / 8), 0, s>>>(P->comp.p, P->fin.p, P->log_n,
                                                                                   P->chal.p, 2 * N, N);
    else
      qpk::k_fri_divide<64><<<nb, 1024, 0, s>>>(P->comp.p, P->fin.p, P->log_n, P->chal.p, 2 * N, N);
    TRY(hipGetLastError());
  }
  {
    uint32_t lg = logN;
    const uint64_t *coef = P->fin.p;  // layer-0 coefficients: final poly zero-padded to N, [2][N]
    uint64_t coef_bs = 2 * N, coef_cs = N;
    uint32_t coef_log = P->log_n;     // number of (possibly) nonzero coefficients
    uint64_t shift = gl::GEN;
    for (size_t l = 0; l < P->arity.size(); l++) {
      const uint32_t ab = P->arity[l];
      // values of this layer: coset_fft(coef, shift) of size 2^lg, leaf order
      qpk::lde(c->tw, coef, coef_cs, P->fvals[l].p, 1ull << lg, 2, coef_log, lg - coef_log, shift, nb, coef_bs,
               2ull << lg, s);
      const uint64_t dbs = qpk::tree_digest_count(lg - ab, P->cap_h) * 4;
      qpk::fri_leaf(P->fvals[l].p, P->fdig[l].p, lg, ab, 2ull << lg, dbs, nb, s);
      qpk::merkle_tree(P->fdig[l].p, lg - ab, P->cap_h, nb, dbs, s);
      TRY(hipGetLastError());
      if ((rc = fetch_caps(P, P->fdig[l].p, dbs, lg - ab, nb))) return rc;
      P->pool->parallel_for(nb, [&](size_t b) {
        ProofState &S = st[b];
        const uint64_t *cp = P->h_caps.data() + b * capw;
        S.fri_caps.insert(S.fri_caps.end(), cp, cp + capw);
        S.t.observe(cp, capw);
        ext beta = S.t.get_ext();
        uint64_t *ch = P->h_chal.data() + b * qpk::CHAL_STRIDE;
        ch[qpk::CH_FRI_BETA + 2 * l] = beta.c0;
        ch[qpk::CH_FRI_BETA + 2 * l + 1] = beta.c1;
      });
      if ((rc = push_chal(P, nb))) return rc;
      // fold: next coefficients (length 2^(lg-ab)); only the low 2^(coef_log-ab) can be nonzero
      qpk::k_fold<<<dim3(cdiv(1ull << (lg - ab), 256), nb), 256, 0, s>>>(coef, P->fcoef[l].p, lg, ab, (uint32_t)l,
                                                                        P->chal.p, coef_bs, 2ull << (lg - ab),
                                                                        coef_log);
      TRY(hipGetLastError());
      coef = P->fcoef[l].p;
      lg -= ab;
      coef_bs = 2ull << lg;
      coef_cs = 1ull << lg;
      coef_log = coef_log > ab ? coef_log - ab : 0;
      shift = gl::pow(shift, 1ull << ab);
    }
    // final polynomial: the first final_len folded coefficients
    TRY(hipMemcpy2DAsync(P->h_final.data(), (size_t)P->final_len * 8, coef, coef_cs * 8, (size_t)P->final_len * 8,
                         (size_t)2 * nb, hipMemcpyDeviceToHost, s));
    TRY(hipStreamSynchronize(s));
  }
  lap(4);

  // ---- 6. proof of work (a12): minimal witness
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    const uint64_t *f0 = P->h_final.data() + (size_t)b * 2 * P->final_len;
    const uint64_t *f1 = f0 + P->final_len;
    for (uint32_t i = 0; i < P->final_len; i++) {
      S.t.observe(f0[i]);
      S.t.observe(f1[i]);
    }
    // sponge state with the candidate at lane pos (round 0 folded on the host)
    uint64_t st12[12];
    memcpy(st12, S.t.state, 96);
    for (uint32_t i = 0; i < S.t.nin; i++) st12[i] = S.t.in[i];
    const uint32_t pos = S.t.nin;
    qpk::pow_prestate(st12, pos, P->h_powst.data() + b * 24);
    P->h_pos[b] = pos;
  });
  TRY(hipMemcpyAsync(P->pow_state.p, P->h_powst.data(), (size_t)nb * 192, hipMemcpyHostToDevice, s));
  TRY(hipMemcpyAsync(P->pow_pos.p, P->h_pos.data(), (size_t)nb * 4, hipMemcpyHostToDevice, s));
  TRY(hipMemsetAsync(P->pow_found.p, 0xFF, (size_t)nb * 8, s));
  if (P->pow_forced) {
    // test-only: the given witness for every proof (reproducing a reference
    // proof, whose find_any witness is nondeterministic); the transcript and
    // any verifier check it like a ground one
    TRY(hipStreamSynchronize(s));
    for (uint32_t b = 0; b < nb; b++) P->h_found[b] = P->pow_forced_witness;
  } else {
    // Minimal witness per proof in one launch (k_pow_scan): 2048 workgroups
    // claim 256-candidate blocks from per-proof counters, moving on to the
    // next proof once theirs has a hit below the claimed block
    const uint64_t limit = 1ull << std::min<uint32_t>(P->pow_bits + 20, 62);
    TRY(hipMemsetAsync(P->pow_next.p, 0, (size_t)nb * 8, s));
    // (per-wave claims and 2-4 candidates per thread measured no better:
    // profiles/r05_ab_pow_wave.log, r05_ab_pow_cpt.log; a windowed loop with a
    // host check per window was the round-1 form)
    qpk::k_pow_scan<<<2048, 256, 0, s>>>(P->pow_state.p, (const uint32_t *)P->pow_pos.p, P->pow_found.p,
                                         P->pow_next.p, nb, P->pow_bits, limit);
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(P->h_found.data(), P->pow_found.p, (size_t)nb * 8, hipMemcpyDeviceToHost, s));
    TRY(hipStreamSynchronize(s));
    for (uint32_t b = 0; b < nb; b++)
      if (P->h_found[b] == ~0ull) {
        c->err = "proof of work not found";
        return QP_ERR_STATE;
      }
  }
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    S.pow_witness = P->h_found[b];
    S.t.observe(S.pow_witness);
    (void)S.t.get();
    for (uint32_t q = 0; q < P->nq; q++) P->h_qidx[b * P->nq + q] = (uint32_t)(S.t.get() % N);
  });
  lap(5);

  // ---- 7. query rounds: gather leaves + Merkle paths
  TRY(hipMemcpyAsync(P->qidx.p, P->h_qidx.data(), (size_t)nb * P->nq * 4, hipMemcpyHostToDevice, s));
  {
    const uint32_t *qi = (const uint32_t *)P->qidx.p;
    uint64_t off = 0;
    const uint64_t obs = P->qout_words;
    Tree *trees[4] = {&P->cs, &P->wires, &P->zs, &P->quot};
    for (int o = 0; o < 4; o++) {
      Tree *t = trees[o];
      const uint32_t w = t->npolys;
      const uint64_t bs = o == 0 ? 0 : t->lbs(), dbs = o == 0 ? 0 : t->dbs();
      qpk::k_gather_rows_b<<<dim3(cdiv((uint64_t)w * P->nq, 256), nb), 256, 0, s>>>(t->lde.p, N, bs, w, qi, P->nq, 0,
                                                                                   P->qout.p + off, obs);
      off += (uint64_t)w * P->nq;
      const uint32_t depth = logN - P->cap_h;
      qpk::k_gather_paths_b<<<dim3(cdiv((uint64_t)P->nq * depth * 4, 256), nb), 256, 0, s>>>(
          t->dig.p, dbs, logN, P->cap_h, qi, P->nq, 0, P->qout.p + off, obs);
      off += (uint64_t)P->nq * depth * 4;
    }
    uint32_t lg = logN, shift = 0;
    for (size_t l = 0; l < P->arity.size(); l++) {
      const uint32_t ab = P->arity[l];
      shift += ab;
      qpk::k_gather_fri_leaf<<<dim3(cdiv((uint64_t)P->nq * (2u << ab), 256), nb), 256, 0, s>>>(
          P->fvals[l].p, 2ull << lg, lg, ab, qi, P->nq, shift, P->qout.p + off, obs);
      off += (uint64_t)P->nq * (2u << ab);
      const uint32_t depth = lg - ab - P->cap_h;
      const uint64_t dbs = qpk::tree_digest_count(lg - ab, P->cap_h) * 4;
      qpk::k_gather_paths_b<<<dim3(cdiv((uint64_t)P->nq * depth * 4, 256), nb), 256, 0, s>>>(
          P->fdig[l].p, dbs, lg - ab, P->cap_h, qi, P->nq, shift, P->qout.p + off, obs);
      off += (uint64_t)P->nq * depth * 4;
      lg -= ab;
    }
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(P->h_qout.data(), P->qout.p, (size_t)nb * obs * 8, hipMemcpyDeviceToHost, s));
    TRY(hipStreamSynchronize(s));
  }
  lap(6);

  // ---- 8. serialize (ProofWithPublicInputs::to_bytes)
  P->pool->parallel_for(nb, [&](size_t b) {
    ProofState &S = st[b];
    qh::ByteWriter w(out + b * stride);
    for (int k = 0; k < 3; k++) w.u64s(S.caps[k].data(), capw);
    const uint64_t *o = P->h_open.data() + b * qpk::OPEN_STRIDE;
    const uint32_t ncs = P->NC + P->R, nzs = nc * P->nchunks;
    // constants, sigmas, wires, zs, zs_next, partial products, quotient
    w.u64s(o, 2 * (size_t)(ncs + P->W));
    w.u64s(o + 2 * (size_t)(ncs + P->W), 2 * nc);
    w.u64s(o + 2 * (size_t)nopen, 2 * nc);
    w.u64s(o + 2 * (size_t)(ncs + P->W + nc), 2 * (size_t)(nzs - nc));
    w.u64s(o + 2 * (size_t)(ncs + P->W + nzs), 2 * (size_t)(nc * P->qdf));
    w.u64s(S.fri_caps.data(), S.fri_caps.size());
    const uint64_t *qo = P->h_qout.data() + b * P->qout_words;
    const uint32_t depth = logN - P->cap_h;
    std::vector<const uint64_t *> leafp(4), pathp(4);
    uint64_t off = 0;
    for (int oo = 0; oo < 4; oo++) {
      leafp[oo] = qo + off;
      off += (uint64_t)oracle_width(P, oo) * P->nq;
      pathp[oo] = qo + off;
      off += (uint64_t)P->nq * depth * 4;
    }
    std::vector<const uint64_t *> lleaf(P->arity.size()), lpath(P->arity.size());
    std::vector<uint32_t> ldepth(P->arity.size());
    uint32_t lg = logN;
    for (size_t l = 0; l < P->arity.size(); l++) {
      lleaf[l] = qo + off;
      off += (uint64_t)P->nq * (2u << P->arity[l]);
      ldepth[l] = lg - P->arity[l] - P->cap_h;
      lpath[l] = qo + off;
      off += (uint64_t)P->nq * ldepth[l] * 4;
      lg -= P->arity[l];
    }
    for (uint32_t q = 0; q < P->nq; q++) {
      for (int oo = 0; oo < 4; oo++) {
        const uint32_t wd = oracle_width(P, oo);
        w.u64s(leafp[oo] + (size_t)q * wd, wd);
        w.u8((uint8_t)depth);
        w.u64s(pathp[oo] + (size_t)q * depth * 4, (size_t)depth * 4);
      }
      for (size_t l = 0; l < P->arity.size(); l++) {
        const uint32_t lw = 2u << P->arity[l];
        w.u64s(lleaf[l] + (size_t)q * lw, lw);
        w.u8((uint8_t)ldepth[l]);
        w.u64s(lpath[l] + (size_t)q * ldepth[l] * 4, (size_t)ldepth[l] * 4);
      }
    }
    const uint64_t *f0 = P->h_final.data() + (size_t)b * 2 * P->final_len;
    for (uint32_t i = 0; i < P->final_len; i++) {
      w.u64(f0[i]);
      w.u64(f0[P->final_len + i]);
    }
    w.u64(S.pow_witness);
    w.u64(P->npis);
    w.u64s(pis_host[b], P->npis);
    if (lens) lens[b] = w.pos;
  });
  lap(7);
  return QP_OK;
}


// device witness generation for nb proofs whose commit() values are in
// P->h_in ([nb][wg_nin], input-slot order): slot values -> generators level
// by level -> wire matrices in P->wires.vals, public inputs in P->h_wpis
int gen_witness_batch(qp_prover *P, uint32_t nb) {
  qp_ctx *c = P->ctx;
  hipStream_t s = c->stream;
  const uint64_t nw = (uint64_t)P->W << P->log_n;
  if (int rc = check_tables(P, 1, true)) return rc;
  if (P->wg_nin)
    TRY(hipMemcpyAsync(P->wg_in.p, P->h_in, (size_t)nb * P->wg_nin * 8, hipMemcpyHostToDevice, s));
  qpk::k_witness_init<<<dim3(std::min<unsigned>(cdiv(P->wg_nslots, 256), 256), nb), 256, 0, s>>>(
      P->wg_vals.p, P->wg_nslots, P->wg_nslots, nullptr, nullptr, 0);
  if (P->wg_nin)
    qpk::k_witness_inputs<<<dim3(cdiv(P->wg_nin, 256), nb), 256, 0, s>>>(
        P->wg_vals.p, P->wg_nslots, (const uint32_t *)P->wg_in_slots.p, P->wg_in.p, P->wg_nin);
  TRY(hipMemsetAsync(P->wg_err.p, 0, (size_t)nb * 4, s));
  qpk::WitnessGenArgs a;
  a.vals = P->wg_vals.p;
  a.v_bstride = P->wg_nslots;
  a.gens = P->wg_gens.p;
  a.level_off = (const uint32_t *)P->wg_lvl.p;
  a.level_pos = (const uint32_t *)P->wg_lpos.p;
  a.nlevels = P->wg_nlev;
  a.wslot = (const uint32_t *)P->wg_wslot.p;
  a.W = P->W;
  a.limbs = std::min<uint32_t>(63, P->R - 1);
  a.zero_slot = P->circuit->cd.zero_const_slot;
  a.num_consts = P->circuit->cd.config.num_constants;
  a.err = (uint32_t *)P->wg_err.p;
  // workgroup size of the witness kernel (one workgroup per proof): 512 for
  // the aggregation circuits (their wide levels run many one-lane
  // permutations: 256-leaf subtree 0.422 -> 0.415 s, witness stage 87 -> 73
  // ms), 256 for the leaf circuits
  const unsigned wthreads = P->circuit->kind == qp_circuit::AGGREGATION ? 512u : 256u;
  // up to 4 Poseidon generators per wave per level run cooperatively (12 lanes
  // on one permutation) instead of one per lane
  a.coop_max = 4 * (wthreads / 64);
  // path hook wit_row=0: cooperative Poseidons one per wave instead of one per
  // 16-lane row
  a.row = qpk::path_opt("wit_row", 1) != 0;
  // a launch per dependency level over the whole batch (default for small
  // batches: one workgroup per proof leaves each level at a one-lane
  // permutation's latency) or one workgroup per proof (large batches, and the
  // voting circuit); path hook wit_mode=0|1 forces one
  const long wmode = qpk::path_opt("wit_mode", -1);
  // (measured: one aggregation proof 11.0 -> 9.4 ms, witness 2.9 -> 1.3 ms;
  // at 32 proofs per launch 3.78 vs 3.88 ms for one workgroup per proof,
  // profiles/r05_ab_witness_levels.log.  Wormhole: witness 3.2-3.6 -> 1.6-2.2
  // ms per call at 1-32 proofs, one proof 8.5 -> 6.8 ms; the 3-prover
  // headline neutral either way; voting at 171 proofs 4 % slower by level:
  // profiles/r06_wit_modes_by_batch.log, r06_ab_wit_levels.log)
  const auto kind = P->circuit->kind;
  const bool by_level = wmode >= 0 ? wmode == 1
                                   : (kind == qp_circuit::AGGREGATION && nb <= 24) ||
                                         (kind == qp_circuit::WORMHOLE && nb <= 32);
  if (by_level) {
    const auto &lo = P->circuit->cd.level_off;
    const auto &lp = P->circuit->cd.level_pos;
    for (uint32_t l = 0; l < P->wg_nlev; l++) {
      const uint32_t pcnt = lp[2 * l + 1], nother = lo[l + 1] - lo[l] - pcnt;
      const uint32_t na = cdiv(nother, 256), npb = cdiv(pcnt, a.row ? 16 : 4);
      if (na + npb) qpk::k_witness_level<<<dim3(na + npb, nb), 256, 0, s>>>(a, l, na);
    }
  } else {
    qpk::k_witness_gen<<<nb, wthreads, 0, s>>>(a);
  }
  qpk::k_witness_expand<<<dim3((unsigned)std::min<uint64_t>(cdiv(nw, 256), 1024), nb), 256, 0, s>>>(
      P->wg_vals.p, P->wg_nslots, (const uint32_t *)P->wg_wslot_cm.p, nw, P->wires.vals.p, P->wires.cbs(),
      (const uint32_t *)P->wg_pi_slots.p, P->npis, P->wg_pis.p);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(P->h_werr.data(), P->wg_err.p, (size_t)nb * 4, hipMemcpyDeviceToHost, s));
  if (P->npis)
    TRY(hipMemcpyAsync(P->h_wpis.data(), P->wg_pis.p, (size_t)nb * P->npis * 8, hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  for (uint32_t b = 0; b < nb; b++)
    if (P->h_werr[b]) {
      c->err = "proof " + std::to_string(b) +
               ": Partition containing a target was set twice with different values (device generator " +
               std::to_string(P->h_werr[b] - 1) + ")";
      return QP_ERR_WITNESS;
    }
  return QP_OK;
}

using FillFn = std::string (*)(const qp_circuit *, const void *, qc::Witness &, int *);

// WormholeProver::commit + prove (wormhole/prover/src/lib.rs:209-237) for a
// batch: commit() on the host pool, generation on the device, then prove
int prove_inputs(qp_prover *P, FillFn fill, const uint8_t *inputs, size_t in_size, uint32_t nproofs, uint8_t *out,
                 size_t stride, size_t *lens) {
  const qc::CircuitData &cd = P->circuit->cd;
  if (!cd.device_witness) {
    P->ctx->err = "this circuit's witness generators run on the host only: commit() and prove the witnesses";
    return QP_ERR_STATE;
  }
  for (uint32_t done = 0; done < nproofs;) {
    const uint32_t nb = std::min(P->max_batch, nproofs - done);
    std::atomic<uint32_t> first_bad{UINT32_MAX};
    std::vector<std::string> msgs(nb);
    std::vector<int> codes(nb, QP_OK);
    auto T0 = Clock::now();
    // commit() values (and the host chains' outputs) into the pinned input rows
    auto finish = [&](size_t b, const qc::Witness &w, std::string e, int code) {
      uint64_t *row = P->h_in + b * (size_t)P->wg_nin;
      if (e.empty())
        for (uint32_t i = 0; i < P->wg_nin; i++) {
          uint64_t v;
          if (!w.get_slot(cd.input_slots[i], v)) {
            e = "a circuit input target was not set by commit";
            code = QP_ERR_STATE;
            break;
          }
          row[i] = v;
        }
      if (!e.empty()) {
        msgs[b] = e;
        codes[b] = code ? code : QP_ERR_ARG;
        uint32_t cur = first_bad.load();
        while (b < cur && !first_bad.compare_exchange_weak(cur, (uint32_t)b)) {
        }
      }
    };
    // the long input-only Poseidon chains (CircuitData::host_gens) run on the
    // host after commit(); a batch smaller than the pool runs its proofs'
    // independent chains in parallel (a 32,768-input root: chains of 4,096
    // and twice ~2,150 permutations)
    const uint32_t nseg = cd.host_seg_off.empty() ? 0 : (uint32_t)cd.host_seg_off.size() - 1;
    if (nseg > 2 && nb <= P->pool->size()) {
      const uint32_t nch = nseg - 1;
      if (P->wscratch.size() < nb) P->wscratch.resize(nb);
      std::vector<std::unique_ptr<qc::Witness>> wv(nb);
      std::vector<std::string> em((size_t)nb * nch);
      P->pool->parallel_for(nb, [&](size_t b) {
        auto &sc = P->wscratch[b];
        if (sc.size() < cd.num_slots) sc.resize(cd.num_slots);
        wv[b].reset(new qc::Witness(cd, sc.data()));
        codes[b] = QP_OK;
        msgs[b] = fill(P->circuit, inputs + (done + b) * in_size, *wv[b], &codes[b]);
        if (msgs[b].empty() && !wv[b]->generate_host_chains(msgs[b], 0)) codes[b] = QP_ERR_WITNESS;
      });
      P->pool->parallel_for((size_t)nb * nch, [&](size_t k) {
        const size_t b = k / nch;
        if (msgs[b].empty()) wv[b]->generate_host_chains(em[k], 1 + (int)(k % nch));
      });
      P->pool->parallel_for(nb, [&](size_t b) {
        std::string e = msgs[b];
        int code = codes[b];
        for (uint32_t c = 0; c < nch && e.empty(); c++)
          if (!em[b * nch + c].empty()) {
            e = em[b * nch + c];
            code = QP_ERR_WITNESS;
          }
        msgs[b].clear();
        codes[b] = QP_OK;
        finish(b, *wv[b], e, code);
      });
    } else {
      P->pool->parallel_for(nb, [&](size_t b) {
        thread_local std::vector<uint64_t> scratch;
        if (scratch.size() < cd.num_slots) scratch.resize(cd.num_slots);
        qc::Witness w(cd, scratch.data());
        int code = QP_OK;
        std::string e = fill(P->circuit, inputs + (done + b) * in_size, w, &code);
        if (e.empty() && nseg && !w.generate_host_chains(e)) code = QP_ERR_WITNESS;
        finish(b, w, e, code);
      });
    }
    if (first_bad.load() != UINT32_MAX) {
      const uint32_t b = first_bad.load();
      P->ctx->err = "proof " + std::to_string(done + b) + ": " + msgs[b];
      return codes[b];
    }
    auto T1 = Clock::now();
    P->stage_ms[8] += std::chrono::duration<double, std::milli>(T1 - T0).count();
    int rc = gen_witness_batch(P, nb);
    P->stage_ms[9] += std::chrono::duration<double, std::milli>(Clock::now() - T1).count();
    if (rc) {
      P->ctx->err += " (batch offset " + std::to_string(done) + ")";
      return rc;
    }
    std::vector<const uint64_t *> pp(nb);
    for (uint32_t b = 0; b < nb; b++) pp[b] = P->h_wpis.data() + (size_t)b * P->npis;
    try {
      rc = prove_batch(P, P->wires.vals.p, nullptr, pp.data(), nb, out + (size_t)done * stride, stride,
                       lens ? lens + done : nullptr);
    } catch (const std::bad_alloc &) {
      rc = QP_ERR_OOM;
    }
    if (rc) return rc;
    done += nb;
  }
  return QP_OK;
}

}  // namespace

extern "C" {

int qp_prover_new(qp_ctx *c, const qp_circuit *circuit, uint32_t max_batch, qp_prover **out) {
  if (!c || !circuit || !out || !max_batch) return QP_ERR_ARG;
  *out = nullptr;
  qp_prover *P = new (std::nothrow) qp_prover();
  if (!P) return QP_ERR_OOM;
  P->ctx = c;
  P->circuit = circuit;
  P->max_batch = max_batch;
  int rc;
  try {
    rc = setup(P);
  } catch (const std::bad_alloc &) {
    rc = QP_ERR_OOM;
  }
  if (rc) {
    delete P;
    return rc;
  }
  *out = P;
  return QP_OK;
}

void qp_prover_free(qp_prover *P) {
  if (!P) return;
  (void)hipSetDevice(P->ctx->device);
  (void)hipStreamSynchronize(P->ctx->stream);
  delete P;
}

int qp_prover_proof_size(const qp_prover *P, size_t *len) {
  if (!P || !len) return QP_ERR_ARG;
  *len = P->proof_len;
  return QP_OK;
}

int qp_prover_verifier_data(const qp_prover *P, uint8_t *out, size_t cap, size_t *len) {
  if (!P) return QP_ERR_ARG;
  const size_t capw = 4u << P->cap_h;
  const size_t total = 8 + capw * 8 + 32 + P->common.size();
  if (len) *len = total;
  if (!out) return QP_OK;
  if (cap < total) return QP_ERR_ARG;
  qh::ByteWriter w(out);
  w.u64(P->cap_h);
  w.u64s(P->cs_cap, capw);
  w.u64s(P->digest, 4);
  memcpy(out + w.pos, P->common.data(), P->common.size());
  return QP_OK;
}

int qp_prover_prove_wires(qp_prover *P, const uint64_t *wires, const uint64_t *pis, uint32_t nproofs, uint8_t *out,
                          size_t stride, size_t *lens) {
  if (!P || !wires || !pis || !out || !nproofs) return QP_ERR_ARG;
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  const uint64_t wsz = (uint64_t)P->W << P->log_n;
  for (uint32_t done = 0; done < nproofs;) {
    const uint32_t nb = std::min(P->max_batch, nproofs - done);
    std::vector<const uint64_t *> wp(nb), pp(nb);
    for (uint32_t b = 0; b < nb; b++) {
      wp[b] = wires + (uint64_t)(done + b) * wsz;
      pp[b] = pis + (uint64_t)(done + b) * P->npis;
    }
    int rc;
    try {
      rc = prove_batch(P, nullptr, wp.data(), pp.data(), nb, out + (size_t)done * stride, stride,
                       lens ? lens + done : nullptr);
    } catch (const std::bad_alloc &) {
      rc = QP_ERR_OOM;
    }
    if (rc) return rc;
    done += nb;
  }
  return QP_OK;
}

// witnesses generated on the host (qp_wormhole_commit / qp_voting_commit):
// their partition values go up (num_slots words each, ~1/5 of the wire
// matrix) and are expanded into the wire matrices on the device
int qp_prover_prove(qp_prover *P, const qp_witness *const *w, uint32_t nproofs, uint8_t *out, size_t stride,
                    size_t *lens) {
  if (!P || !w || !out || !nproofs) return QP_ERR_ARG;
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  for (uint32_t i = 0; i < nproofs; i++)
    if (!w[i] || w[i]->circuit != P->circuit) {
      P->ctx->err = "witness belongs to a different circuit";
      return QP_ERR_ARG;
    }
  hipStream_t s = P->ctx->stream;
  const uint64_t nw = (uint64_t)P->W << P->log_n;
  for (const char *t : {"wg_vals", "wg_wslot_cm", "wg_pi_slots", "wg_pis", "wires.vals"}) {
    const void *p = !strcmp(t, "wg_vals") ? (const void *)P->wg_vals.p : !strcmp(t, "wg_wslot_cm") ? P->wg_wslot_cm.p
                  : !strcmp(t, "wg_pi_slots") ? P->wg_pi_slots.p : !strcmp(t, "wg_pis") ? P->wg_pis.p
                  : P->wires.vals.p;
    if (!p) {
      P->ctx->err = std::string("device table '") + t + "' is missing for this circuit (host-witness expansion)";
      return QP_ERR_STATE;
    }
  }
  for (uint32_t done = 0; done < nproofs;) {
    const uint32_t nb = std::min(P->max_batch, nproofs - done);
    std::vector<uint64_t> pis((size_t)nb * P->npis);
    std::vector<const uint64_t *> pp(nb);
    TRY(hipSetDevice(P->ctx->device));
    for (uint32_t b = 0; b < nb; b++) {
      const qc::Witness &wt = w[done + b]->w;
      TRY(hipMemcpyAsync(P->wg_vals.p + (size_t)b * P->wg_nslots, wt.slot_values(), (size_t)P->wg_nslots * 8,
                         hipMemcpyHostToDevice, s));
      auto pi = wt.public_inputs();
      memcpy(pis.data() + (size_t)b * P->npis, pi.data(), P->npis * 8);
      pp[b] = pis.data() + (size_t)b * P->npis;
    }
    qpk::k_witness_expand<<<dim3((unsigned)std::min<uint64_t>(cdiv(nw, 256), 1024), nb), 256, 0, s>>>(
        P->wg_vals.p, P->wg_nslots, (const uint32_t *)P->wg_wslot_cm.p, nw, P->wires.vals.p, P->wires.cbs(),
        (const uint32_t *)P->wg_pi_slots.p, P->npis, P->wg_pis.p);
    TRY(hipGetLastError());
    int rc;
    try {
      rc = prove_batch(P, P->wires.vals.p, nullptr, pp.data(), nb, out + (size_t)done * stride, stride,
                       lens ? lens + done : nullptr);
    } catch (const std::bad_alloc &) {
      rc = QP_ERR_OOM;
    }
    if (rc) return rc;
    done += nb;
  }
  return QP_OK;
}

int qp_prover_prove_wormhole_inputs(qp_prover *P, const qp_wormhole_inputs *in, uint32_t nproofs, uint8_t *out,
                                    size_t stride, size_t *lens) {
  if (!P || !in || !out || !nproofs) return QP_ERR_ARG;
  if (P->circuit->kind != qp_circuit::WORMHOLE) {
    P->ctx->err = "prover circuit is not the Wormhole circuit";
    return QP_ERR_ARG;
  }
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  TRY(hipSetDevice(P->ctx->device));
  try {
    return prove_inputs(P, wormhole_fill, (const uint8_t *)in, sizeof(qp_wormhole_inputs), nproofs, out, stride, lens);
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

int qp_prover_prove_voting_inputs(qp_prover *P, const qp_voting_inputs *in, uint32_t nproofs, uint8_t *out,
                                  size_t stride, size_t *lens) {
  if (!P || !in || !out || !nproofs) return QP_ERR_ARG;
  if (P->circuit->kind != qp_circuit::VOTING) {
    P->ctx->err = "prover circuit is not the voting circuit";
    return QP_ERR_ARG;
  }
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  TRY(hipSetDevice(P->ctx->device));
  try {
    return prove_inputs(P, voting_fill, (const uint8_t *)in, sizeof(qp_voting_inputs), nproofs, out, stride, lens);
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

int qp_prover_prove_aggregation(qp_prover *P, const qp_aggregation_chunk *chunks, uint32_t nchunks, uint8_t *out,
                                size_t stride, size_t *lens) {
  if (!P || !chunks || !out || !nchunks) return QP_ERR_ARG;
  if (P->circuit->kind != qp_circuit::AGGREGATION) {
    P->ctx->err = "prover circuit is not an aggregation circuit";
    return QP_ERR_ARG;
  }
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  TRY(hipSetDevice(P->ctx->device));
  try {
    return prove_inputs(P, aggregation_fill, (const uint8_t *)chunks, sizeof(qp_aggregation_chunk), nchunks, out,
                        stride, lens);
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

int qp_prover_debug_drop_table(qp_prover *P, const char *name) {
  if (!P || !name) return QP_ERR_ARG;
  (void)hipSetDevice(P->ctx->device);
  (void)hipStreamSynchronize(P->ctx->stream);
  DevBuf *d = !strcmp(name, "wg_wslot_cm") ? &P->wg_wslot_cm : !strcmp(name, "wg_gens") ? &P->wg_gens
            : !strcmp(name, "qtab") ? &P->qtab : nullptr;
  if (!d) return QP_ERR_ARG;
  if (d->p) (void)hipFree(d->p);
  d->p = nullptr;
  return QP_OK;
}

int qp_prover_debug_force_pow(qp_prover *P, uint64_t witness, int enable) {
  if (!P) return QP_ERR_ARG;
  P->pow_forced = enable != 0;
  P->pow_forced_witness = witness;
  return QP_OK;
}

int qp_prover_set_timing(qp_prover *P, int enable) {
  if (!P) return QP_ERR_ARG;
  P->timing = enable != 0;
  return QP_OK;
}

int qp_prover_kernel_stats(qp_prover *P, double *ms, double *units, uint64_t *launches, uint32_t n, int reset) {
  if (!P) return QP_ERR_ARG;
  for (uint32_t i = 0; i < n && i < 8; i++) {
    if (ms) ms[i] = P->kt[i].ms;
    if (units) units[i] = P->kt[i].units;
    if (launches) launches[i] = P->kt[i].launches;
    if (reset) {
      P->kt[i].ms = 0;
      P->kt[i].units = 0;
      P->kt[i].launches = 0;
    }
  }
  return QP_OK;
}

int qp_prover_prove_wires_dev(qp_prover *P, const uint64_t *d_wires, const uint64_t *pis, uint32_t nproofs,
                              uint8_t *out, size_t stride, size_t *lens) {
  if (!P || !d_wires || !pis || !out || !nproofs) return QP_ERR_ARG;
  if (stride < P->proof_len) {
    P->ctx->err = "output stride smaller than the proof size";
    return QP_ERR_ARG;
  }
  const uint64_t wsz = (uint64_t)P->W << P->log_n;
  for (uint32_t done = 0; done < nproofs;) {
    const uint32_t nb = std::min(P->max_batch, nproofs - done);
    std::vector<const uint64_t *> pp(nb);
    for (uint32_t b = 0; b < nb; b++) pp[b] = pis + (uint64_t)(done + b) * P->npis;
    int rc;
    try {
      rc = prove_batch(P, d_wires + (uint64_t)done * wsz, nullptr, pp.data(), nb, out + (size_t)done * stride, stride,
                       lens ? lens + done : nullptr);
    } catch (const std::bad_alloc &) {
      rc = QP_ERR_OOM;
    }
    if (rc) return rc;
    done += nb;
  }
  return QP_OK;
}

int qp_prover_stage_times(qp_prover *P, double *ms, uint32_t n, int reset) {
  if (!P) return QP_ERR_ARG;
  for (uint32_t i = 0; i < n && i < 16; i++) ms[i] = P->stage_ms[i];
  if (reset)
    for (double &x : P->stage_ms) x = 0;
  return QP_OK;
}

}  // extern "C"
