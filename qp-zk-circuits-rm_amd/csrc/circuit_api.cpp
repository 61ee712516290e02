// circuit_api.cpp — C ABI (include/qpgpu.h) for circuits and witnesses.
// Host only: builds the native circuit and generates witnesses; the device
// side of a circuit (constants/sigmas commitment) lives in prover.cpp.
#include <string.h>
#include <exception>
#include <random>
#include <memory>
#include <new>
#include "../../include/qpgpu.h"
#include "circuit_obj.h"
#include "host_util.h"

// The PublicInputGate row's unused wires (plonky2 randomize_unused_pi_wires ->
// RandomValueGenerator; qp-plonky2 fills them under both configs).  `given`
// holds num_wires - 4 canonical values (e.g. the reference's own, to reproduce
// one of its proofs byte for byte).  When it is null: zeros under the non-zk
// config (no hiding is claimed there); under the zk config
// hash_n_to_m_no_pad(domain tag || private felts), a deterministic nonce that
// hides like fresh randomness while the private inputs stay secret, so the
// proof remains a pure function of the inputs.
// os_random: under the zk config with no values given, draw them from the OS
// (the aggregation circuits: their only witness inputs are public proofs, so a
// nonce derived from them would not hide anything).
static std::string zk_fill(const qc::CircuitData &cd, const uint64_t *given, const std::vector<uint64_t> &priv,
                           qc::Witness &w, int *code, bool os_random = false) {
  *code = QP_ERR_ARG;
  const size_t m = cd.zk_slots.size();
  if (!m) return "";
  std::vector<uint64_t> v(m, 0);
  if (given) {
    for (size_t i = 0; i < m; i++) {
      if (given[i] >= gl::P) return "zk randomness value " + std::to_string(i) + " is not a canonical field element";
      v[i] = given[i];
    }
  } else if (cd.config.zero_knowledge && os_random) {
    // RandomValueGenerator: uniform field elements (rejection of the 2^32 - 1
    // values >= p), from the kernel's CSPRNG
    std::random_device rd("/dev/urandom");
    for (size_t i = 0; i < m; i++) {
      uint64_t x;
      do {
        x = (uint64_t)rd() << 32 | rd();
      } while (x >= gl::P);
      v[i] = x;
    }
  } else if (cd.config.zero_knowledge) {
    std::vector<uint64_t> in = {0x6b7a2d626c696e64ull % gl::P /* "zk-blind" */, (uint64_t)m};
    in.insert(in.end(), priv.begin(), priv.end());
    uint64_t st[12] = {0};
    for (size_t off = 0; off < in.size(); off += 8) {
      for (size_t i = 0; i < 8 && off + i < in.size(); i++) st[i] = gl::canon(in[off + i]);
      ps::permute(st);
    }
    for (size_t i = 0; i < m; i++) {
      if (i && i % 8 == 0) ps::permute(st);
      v[i] = st[i % 8];
    }
  }
  for (size_t i = 0; i < m; i++)
    if (!w.set_slot(cd.zk_slots[i], v[i])) {
      *code = QP_ERR_WITNESS;
      return "Partition containing a target was set twice with different values";
    }
  *code = QP_OK;
  return "";
}

static std::vector<uint64_t> bytes_as_u32_felts(const uint8_t *b, size_t n) {
  std::vector<uint64_t> v;
  for (size_t i = 0; i + 4 <= n; i += 4) v.push_back((uint64_t)b[i] | (uint64_t)b[i + 1] << 8 |
                                                     (uint64_t)b[i + 2] << 16 | (uint64_t)b[i + 3] << 24);
  return v;
}

std::string wormhole_fill(const qp_circuit *c, const void *vin, qc::Witness &w, int *code) {
  const qp_wormhole_inputs *in = (const qp_wormhole_inputs *)vin;
  *code = QP_ERR_ARG;
  if (!c || !in || c->kind != qp_circuit::WORMHOLE) return "not a Wormhole circuit / null inputs";
  if (in->num_nodes && (!in->nodes || !in->node_lens || !in->indices)) return "null storage-proof arrays";
  qw::CircuitInputs ci;
  memcpy(&ci.funding_amount_lo, in->funding_amount, 8);
  memcpy(&ci.funding_amount_hi, in->funding_amount + 8, 8);
  memcpy(ci.nullifier, in->nullifier, 32);
  memcpy(ci.root_hash, in->root_hash, 32);
  memcpy(ci.exit_account, in->exit_account, 32);
  memcpy(ci.secret, in->secret, 32);
  ci.transfer_count = in->transfer_count;
  memcpy(ci.funding_account, in->funding_account, 32);
  memcpy(ci.unspendable_account, in->unspendable_account, 32);
  for (uint32_t i = 0; i < in->num_nodes; i++) {
    ci.storage_proof.emplace_back(in->nodes[i], in->nodes[i] + in->node_lens[i]);
    ci.storage_indices.push_back(in->indices[i]);
  }
  std::string e = qw::commit(c->wormhole, ci, w);
  *code = e.empty() ? QP_OK : e.find("set twice") != std::string::npos ? QP_ERR_WITNESS : QP_ERR_ARG;
  if (!e.empty()) return e;
  std::vector<uint64_t> priv = bytes_as_u32_felts(in->secret, 32);
  for (const uint8_t *f : {in->funding_account, in->unspendable_account, in->nullifier, in->root_hash})
    for (uint64_t x : bytes_as_u32_felts(f, 32)) priv.push_back(x);
  priv.push_back(in->transfer_count & 0xFFFFFFFFu);
  priv.push_back(in->transfer_count >> 32);
  return zk_fill(c->cd, in->zk_randomness, priv, w, code);
}

std::string voting_fill(const qp_circuit *c, const void *vin, qc::Witness &w, int *code) {
  const qp_voting_inputs *in = (const qp_voting_inputs *)vin;
  *code = QP_ERR_ARG;
  if (!c || !in || c->kind != qp_circuit::VOTING) return "not a voting circuit / null inputs";
  if ((in->num_siblings && !in->siblings) || (in->num_path_indices && !in->path_indices)) return "null arrays";
  qv::VoteInputs vi;
  memcpy(vi.proposal_id, in->proposal_id, 32);
  memcpy(vi.merkle_root, in->merkle_root, 32);
  memcpy(vi.nullifier, in->nullifier, 32);
  vi.vote = in->vote != 0;
  memcpy(vi.private_key, in->private_key, 32);
  for (uint32_t i = 0; i < in->num_siblings; i++)
    vi.merkle_siblings.push_back({in->siblings[4 * i], in->siblings[4 * i + 1], in->siblings[4 * i + 2],
                                  in->siblings[4 * i + 3]});
  for (uint32_t i = 0; i < in->num_path_indices; i++) vi.path_indices.push_back(in->path_indices[i] != 0);
  vi.actual_merkle_depth = in->actual_merkle_depth;
  std::string e = qv::fill_targets(c->voting, vi, w);
  *code = e.empty() ? QP_OK : QP_ERR_ARG;
  if (!e.empty()) return e;
  std::vector<uint64_t> priv(in->private_key, in->private_key + 4);
  priv.insert(priv.end(), in->proposal_id, in->proposal_id + 4);
  priv.push_back(in->vote != 0);
  return zk_fill(c->cd, in->zk_randomness, priv, w, code);
}

// aggregate_chunk's set_verifier_data_target + set_proof_with_pis_target
// (tree.rs:129-134) and the PublicInputGate row's random cells (zk config:
// given, else OS randomness; the non-zk config: given, else zeros)
std::string aggregation_fill(const qp_circuit *c, const void *vin, qc::Witness &w, int *code) {
  const qp_aggregation_chunk *in = (const qp_aggregation_chunk *)vin;
  *code = QP_ERR_ARG;
  if (!c || !in || c->kind != qp_circuit::AGGREGATION) return "not an aggregation circuit / null chunk";
  if (!in->verifier_only || !in->proofs || !in->lens) return "null verifier data / proof arrays";
  std::string e = qr::fill_aggregation(c->aggregation, in->verifier_only, in->vlen, in->proofs, in->lens, in->nproofs, w);
  if (!e.empty()) {
    *code = e.find("set twice") != std::string::npos ? QP_ERR_WITNESS : QP_ERR_ARG;
    return e;
  }
  return zk_fill(c->cd, in->zk_randomness, {}, w, code, true);
}

extern "C" {

int qp_wormhole_circuit_new(int zk, qp_circuit **out) {
  if (!out) return QP_ERR_ARG;
  *out = nullptr;
  try {
    auto c = std::make_unique<qp_circuit>();
    c->kind = qp_circuit::WORMHOLE;
    qc::CircuitBuilder b(zk ? qc::CircuitConfig::standard_recursion_zk_config()
                            : qc::CircuitConfig::standard_recursion_config());
    c->wormhole = qw::build_wormhole(b);
    c->gates_used = (uint32_t)b.num_gates();
    c->cd = b.build();
    *out = c.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  } catch (const std::exception &) {
    return QP_ERR_STATE;
  }
}

int qp_voting_circuit_new(int zk, qp_circuit **out) {
  if (!out) return QP_ERR_ARG;
  *out = nullptr;
  try {
    auto c = std::make_unique<qp_circuit>();
    c->kind = qp_circuit::VOTING;
    qc::CircuitBuilder b(zk ? qc::CircuitConfig::standard_recursion_zk_config()
                            : qc::CircuitConfig::standard_recursion_config());
    c->voting = qv::build_voting(b);
    c->gates_used = (uint32_t)b.num_gates();
    c->cd = b.build();
    *out = c.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  } catch (const std::exception &) {
    return QP_ERR_STATE;
  }
}

// aggregate_chunk's circuit (wormhole/aggregator/src/circuits/tree.rs:106-127):
// CircuitBuilder::new(inner config) + add_virtual_verifier_data + nproofs x
// (add_virtual_proof_with_pis + verify_proof + register_public_inputs) + build
int qp_aggregation_circuit_new(const uint8_t *inner_common, size_t len, uint32_t nproofs, qp_circuit **out) {
  if (!out || !inner_common || !nproofs || nproofs > 64) return QP_ERR_ARG;
  *out = nullptr;
  try {
    qr::InnerCommon ic;
    if (!qr::parse_common(inner_common, len, ic).empty()) return QP_ERR_ARG;
    qc::CircuitConfig cfg = ic.zero_knowledge ? qc::CircuitConfig::standard_recursion_zk_config()
                                              : qc::CircuitConfig::standard_recursion_config();
    if (ic.num_wires != cfg.num_wires || ic.num_routed_wires != cfg.num_routed_wires ||
        ic.config_num_constants != cfg.num_constants || ic.rate_bits != cfg.rate_bits ||
        ic.cap_height != cfg.cap_height || ic.num_query_rounds != cfg.num_query_rounds || ic.pow_bits != cfg.pow_bits)
      return QP_ERR_ARG;
    auto c = std::make_unique<qp_circuit>();
    c->kind = qp_circuit::AGGREGATION;
    qc::CircuitBuilder b(cfg);
    c->aggregation = qr::build_aggregation(b, ic, nproofs);
    c->gates_used = (uint32_t)b.num_gates();
    c->cd = b.build();
    *out = c.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  } catch (const std::exception &) {
    return QP_ERR_STATE;
  }
}

void qp_circuit_free(qp_circuit *c) { delete c; }

int qp_circuit_info(const qp_circuit *c, uint32_t *info) {
  if (!c || !info) return QP_ERR_ARG;
  info[0] = c->cd.degree_bits;
  info[1] = c->cd.config.num_wires;
  info[2] = c->cd.config.num_routed_wires;
  info[3] = c->cd.num_constants;
  info[4] = c->cd.num_public_inputs;
  info[5] = c->gates_used;
  info[6] = c->cd.num_gate_constraints;
  info[7] = (uint32_t)c->cd.schedule.size();
  info[8] = c->cd.level_off.empty() ? 0 : (uint32_t)c->cd.level_off.size() - 1;
  return QP_OK;
}

int qp_circuit_census(const qp_circuit *c, uint32_t *gens, uint32_t *rows, uint32_t *level_gens) {
  if (!c || !gens || !rows) return QP_ERR_ARG;
  if (level_gens) {
    const auto &lo = c->cd.level_off;
    for (size_t l = 0; l + 1 < lo.size(); l++) {
      uint32_t *o = level_gens + 14 * l;
      memset(o, 0, 14 * sizeof(uint32_t));
      for (uint32_t i = lo[l]; i < lo[l + 1]; i++)
        if (c->cd.dev_gens[i].kind < 14) o[c->cd.dev_gens[i].kind]++;
    }
  }
  memset(gens, 0, 14 * sizeof(uint32_t));
  memset(rows, 0, qc::G_NKINDS * sizeof(uint32_t));
  for (const auto &g : c->cd.schedule)
    if (g.kind < 14) gens[g.kind]++;
  for (const auto &r : c->cd.rows) rows[r.kind]++;
  return QP_OK;
}

int qp_circuit_host_chains(const qp_circuit *c, uint32_t *gens, uint32_t *slots, uint32_t *chains) {
  if (!c || !gens || !slots) return QP_ERR_ARG;
  memset(gens, 0, 14 * sizeof(uint32_t));
  for (uint32_t i : c->cd.host_gens)
    if (c->cd.schedule[i].kind < 14) gens[c->cd.schedule[i].kind]++;
  *slots = (uint32_t)c->cd.input_slots.size();
  if (chains) *chains = c->cd.host_seg_off.size() > 1 ? (uint32_t)c->cd.host_seg_off.size() - 2 : 0;
  return QP_OK;
}

int qp_circuit_common_data(const qp_circuit *c, uint8_t *out, size_t cap, size_t *len) {
  if (!c) return QP_ERR_ARG;
  auto b = c->cd.common_bytes();
  if (len) *len = b.size();
  if (out) {
    if (cap < b.size()) return QP_ERR_ARG;
    memcpy(out, b.data(), b.size());
  }
  return QP_OK;
}

int qp_circuit_constants_sigmas(const qp_circuit *c, uint64_t *out) {
  if (!c || !out) return QP_ERR_ARG;
  memcpy(out, c->cd.constants_sigmas.data(), c->cd.constants_sigmas.size() * 8);
  return QP_OK;
}

// PolynomialValues::ifft of every constants||sigmas column on the host (the
// coefficients plonky2 keeps in ProverOnlyCircuitData.constants_sigmas_commitment):
// radix-2 DIT on bit-reversed input, scaled by 1/n
int qp_circuit_constants_sigmas_coeffs(const qp_circuit *c, uint64_t *out) {
  if (!c || !out) return QP_ERR_ARG;
  const uint32_t n = c->cd.n, lg = c->cd.degree_bits;
  const size_t ncols = c->cd.constants_sigmas.size() / n;
  std::vector<uint64_t> wi(n / 2);
  const uint64_t w = gl::inv(gl::root_of_unity(lg));
  for (uint32_t k = 0; k < n / 2; k++) wi[k] = k ? gl::mul(wi[k - 1], w) : 1;
  const uint64_t n_inv = gl::inv(n);
  for (size_t col = 0; col < ncols; col++) {
    const uint64_t *src = c->cd.constants_sigmas.data() + col * n;
    uint64_t *a = out + col * n;
    for (uint32_t i = 0; i < n; i++) a[gl::rev_bits(i, lg)] = src[i];
    for (uint32_t len = 2; len <= n; len <<= 1) {
      const uint32_t step = n / len;
      for (uint32_t i = 0; i < n; i += len)
        for (uint32_t j = 0; j < len / 2; j++) {
          const uint64_t u = a[i + j], v = gl::mul(a[i + j + len / 2], wi[j * step]);
          a[i + j] = gl::add(u, v);
          a[i + j + len / 2] = gl::sub(u, v);
        }
    }
    for (uint32_t i = 0; i < n; i++) a[i] = gl::mul(a[i], n_inv);
  }
  return QP_OK;
}

static void put_err(char *err, size_t cap, const std::string &m) {
  if (err && cap) {
    size_t k = m.size() < cap - 1 ? m.size() : cap - 1;
    memcpy(err, m.data(), k);
    err[k] = 0;
  }
}

int qp_wormhole_commit(const qp_circuit *c, const qp_wormhole_inputs *in, qp_witness **out, char *err, size_t errcap) {
  if (!c || !in || !out || c->kind != qp_circuit::WORMHOLE) return QP_ERR_ARG;
  *out = nullptr;
  try {
    auto w = std::make_unique<qp_witness>(c);
    int code = QP_OK;
    std::string e = wormhole_fill(c, in, w->w, &code);
    if (e.empty() && !w->w.generate(e)) code = QP_ERR_WITNESS;
    if (!e.empty()) {
      put_err(err, errcap, e);
      return code ? code : QP_ERR_ARG;
    }
    *out = w.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

int qp_voting_commit(const qp_circuit *c, const qp_voting_inputs *in, qp_witness **out, char *err, size_t errcap) {
  if (!c || !in || !out || c->kind != qp_circuit::VOTING) return QP_ERR_ARG;
  *out = nullptr;
  try {
    auto w = std::make_unique<qp_witness>(c);
    int code = QP_OK;
    std::string e = voting_fill(c, in, w->w, &code);
    if (e.empty() && !w->w.generate(e)) code = QP_ERR_WITNESS;
    if (!e.empty()) {
      put_err(err, errcap, e);
      return code ? code : QP_ERR_ARG;
    }
    *out = w.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

// aggregate_chunk's witness: set_verifier_data_target + set_proof_with_pis_target
// (tree.rs:129-134), then generation
int qp_aggregation_commit(const qp_circuit *c, const uint8_t *verifier_only, size_t vlen,
                          const uint8_t *const *proofs, const size_t *lens, uint32_t nproofs,
                          const uint64_t *zk_randomness, qp_witness **out, char *err, size_t errcap) {
  if (!c || !verifier_only || !proofs || !lens || !out || c->kind != qp_circuit::AGGREGATION) return QP_ERR_ARG;
  *out = nullptr;
  try {
    auto w = std::make_unique<qp_witness>(c);
    qp_aggregation_chunk ch{verifier_only, vlen, proofs, lens, nproofs, zk_randomness};
    int code = QP_OK;
    std::string e = aggregation_fill(c, &ch, w->w, &code);
    if (e.empty() && !w->w.generate(e)) code = QP_ERR_WITNESS;
    if (!e.empty()) {
      put_err(err, errcap, e);
      return code ? code : QP_ERR_ARG;
    }
    *out = w.release();
    return QP_OK;
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  }
}

int qp_witness_wires(const qp_witness *w, uint64_t *out) {
  if (!w || !out) return QP_ERR_ARG;
  w->w.wires_matrix(out);
  return QP_OK;
}

int qp_witness_public_inputs(const qp_witness *w, uint64_t *out, uint32_t cap, uint32_t *n) {
  if (!w) return QP_ERR_ARG;
  auto pi = w->w.public_inputs();
  if (n) *n = (uint32_t)pi.size();
  if (out) {
    if (cap < pi.size()) return QP_ERR_ARG;
    memcpy(out, pi.data(), pi.size() * 8);
  }
  return QP_OK;
}

void qp_witness_free(qp_witness *w) { delete w; }

int qp_hash_no_pad(const uint64_t *in, size_t n, uint64_t *out4) {
  if ((!in && n) || !out4) return QP_ERR_ARG;
  std::vector<uint64_t> v(in, in + n);
  for (auto &x : v) x = gl::canon(x);
  qh::hash_no_pad(v.data(), n, out4);
  return QP_OK;
}

}  // extern "C"
