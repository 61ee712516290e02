// prover_bin.cpp — upstream plonky2 ProverOnlyCircuitData::to_bytes of a leaf
// circuit: the prover.bin the reference's generate_circuit_binaries writes
// (wormhole/circuit-builder/src/lib.rs:53-59) and WormholeProver::new_from_bytes
// reads back (wormhole/prover/src/lib.rs:104-137), both through
// DefaultGeneratorSerializer.  The crate (qp-plonky2 1.1.1) is not vendored;
// restated from upstream plonky2:
//   util/serialization/mod.rs   write_prover_only_circuit_data, write_generator,
//                               write_polynomial_batch, write_merkle_tree,
//                               write_merkle_cap (u64 height + hashes),
//                               write_target (bool is_wire; row, column | index),
//                               every vector as u64 length + elements
//   util/serialization/generator_serialization.rs  DefaultGeneratorSerializer:
//                               u32 tag = the generator's index in its list, then
//                               the generator's own serialize()
//   plonk/circuit_builder.rs    build(): generator order (the gadgets' simple
//                               generators in call order, the PublicInputGate
//                               row's RandomValueGenerators, the ConstantGenerators
//                               in constants order, then every gate row's
//                               generators), generator_indices_by_watches (keyed by
//                               the watched target's representative), the
//                               sigmas' transpose, fft_root_table
//   plonk/permutation_argument.rs  Forest: merge(x, y) puts y's root under x's,
//                               representative_map = parents after compress_paths
//   hash/merkle_tree.rs         MerkleTree { leaves, digests (fill_subtree layout:
//                               left recursive || left child || right child ||
//                               right recursive, per cap subtree), cap }
// Parity unpinned: the reference commits no prover.bin (generated-bins/ is
// empty).  What a reference fixture does pin is the commitment inside it: the
// cap and circuit digest computed here equal the reference's own verifier data
// (tests/test_prover_bins_cpu.py).  Host-only (no device), so the file can be
// written and checked anywhere.
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <map>
#include <mutex>
#include <new>
#include <thread>
#include <vector>
#include "../../include/qpgpu.h"
#include "circuit_obj.h"
#include "field.h"
#include "host_util.h"

namespace {

using qc::Target;

// DefaultGeneratorSerializer tags (generator list index) of the leaf circuits' kinds
enum : uint32_t {
  TAG_ARITHMETIC_BASE = 0, TAG_BASE_SPLIT = 2, TAG_CONSTANT = 4, TAG_EQUALITY = 7, TAG_POSEIDON = 15,
  TAG_RANDOM_VALUE = 19, TAG_WIRE_SPLIT = 23
};

struct Buf {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void u32(uint32_t v) { b.insert(b.end(), (uint8_t *)&v, (uint8_t *)&v + 4); }
  void u64(uint64_t v) { b.insert(b.end(), (uint8_t *)&v, (uint8_t *)&v + 8); }
  void fields(const uint64_t *v, size_t n) {
    const size_t o = b.size();
    b.resize(o + 8 * n);
    memcpy(b.data() + o, v, 8 * n);
  }
  void field_vec(const uint64_t *v, size_t n) {  // write_usize(len) + write_field_vec
    u64(n);
    fields(v, n);
  }
  void target(Target t) {
    if (t.is_virtual()) {
      u8(0);
      u64(t.v & ~Target::VIRT);
    } else {
      u8(1);
      u64(t.row());
      u64(t.col());
    }
  }
};

// plonky2 Forest over wires (row * W + col) then virtual targets
struct Forest {
  std::vector<uint64_t> parents;
  uint64_t find(uint64_t x) {
    uint64_t r = x;
    while (parents[r] != r) r = parents[r];
    while (parents[x] != x) {
      const uint64_t up = parents[x];
      parents[x] = r;
      x = up;
    }
    return r;
  }
  void merge(uint64_t x, uint64_t y) {
    x = find(x);
    y = find(y);
    if (x != y) parents[y] = x;
  }
};

template <class F>
void parallel(size_t n, F f) {
  unsigned hw = std::thread::hardware_concurrency();
  const unsigned nt = (unsigned)std::min<size_t>(n, std::min(hw ? hw : 4, 16u));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      for (size_t i = t; i < n; i += nt) f(i);
    });
  for (auto &x : th) x.join();
}

// natural-order size-2^lg NTT in place (DIT on bit-reversed input)
void ntt(uint64_t *a, uint32_t lg, const std::vector<uint64_t> &w /* w_N^k, k < N/2 */) {
  const uint32_t n = 1u << lg;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t j = gl::rev_bits(i, lg);
    if (i < j) std::swap(a[i], a[j]);
  }
  for (uint32_t len = 2; len <= n; len <<= 1) {
    const uint32_t step = n / len;
    for (uint32_t i = 0; i < n; i += len)
      for (uint32_t j = 0; j < len / 2; j++) {
        const uint64_t u = a[i + j], v = gl::mul(a[i + j + len / 2], w[(size_t)j * step]);
        a[i + j] = gl::add(u, v);
        a[i + j + len / 2] = gl::sub(u, v);
      }
  }
}

// hash/merkle_tree.rs fill_subtree: digests of one cap subtree laid out as
// left recursive || left child || right child || right recursive
void fill_subtree(uint64_t *dig, size_t ndig, const uint64_t *leaf_hash, size_t nleaves, uint64_t out[4]) {
  if (ndig == 0) {
    memcpy(out, leaf_hash, 32);
    return;
  }
  const size_t half = ndig / 2;
  uint64_t l[4], r[4];
  fill_subtree(dig, half - 1, leaf_hash, nleaves / 2, l);
  fill_subtree(dig + 4 * (half + 1), half - 1, leaf_hash + 4 * (nleaves / 2), nleaves / 2, r);
  memcpy(dig + 4 * (half - 1), l, 32);
  memcpy(dig + 4 * half, r, 32);
  ps::two_to_one(l, r, out);
}

std::vector<uint8_t> prover_only_bytes(const qp_circuit *circ) {
  const qc::CircuitData &cd = circ->cd;
  const uint32_t n = cd.n, lg = cd.degree_bits, rb = cd.config.rate_bits, cap_h = cd.config.cap_height;
  const uint32_t W = cd.config.num_wires, R = cd.config.num_routed_wires;
  const uint64_t N = (uint64_t)n << rb, nwires = (uint64_t)n * W;
  const size_t ncols = cd.constants_sigmas.size() / n;
  uint32_t limbs = 0, arith_ops = 0;
  for (size_t i = 0; i < cd.gate_kinds.size(); i++) {
    if (cd.gate_kinds[i] == qc::G_BASE_SUM) limbs = cd.gate_params[i];
    if (cd.gate_kinds[i] == qc::G_ARITHMETIC) arith_ops = cd.gate_params[i];
  }
  auto tindex = [&](Target t) -> uint64_t {
    return t.is_virtual() ? nwires + (t.v & ~Target::VIRT) : (uint64_t)t.row() * W + t.col();
  };
  // ---- the Forest and its representative map
  Forest fo;
  fo.parents.resize(nwires + cd.num_virtual_targets);
  for (uint64_t i = 0; i < fo.parents.size(); i++) fo.parents[i] = i;
  for (const auto &cp : cd.copies) fo.merge(tindex(cp.first), tindex(cp.second));
  for (uint64_t i = 0; i < fo.parents.size(); i++) fo.find(i);
  // ---- generators in build() order, each with its watch list
  Buf g;
  std::map<uint64_t, std::vector<uint64_t>> watches;
  uint64_t ngen = 0;
  auto gen = [&](uint32_t tag, std::initializer_list<Target> watch) {
    for (Target t : watch) {
      auto &v = watches[fo.parents[tindex(t)]];
      if (v.empty() || v.back() != ngen) v.push_back(ngen);  // Vec::dedup of consecutive entries
    }
    g.u32(tag);
    ngen++;
  };
  for (const qc::Gen &s : cd.simple_gens) {
    if (s.kind == qc::GEN_EQUALITY) {
      gen(TAG_EQUALITY, {s.a, s.b});
      g.target(s.a);
      g.target(s.b);
      g.target(s.c);  // write_target_bool
      g.target(s.d);
    } else {  // GEN_WIRE_SPLIT
      gen(TAG_WIRE_SPLIT, {s.a});
      g.target(s.a);
      g.u64(s.op);
      for (uint32_t k = 0; k < s.op; k++) g.u64(s.row + k);
      g.u64(limbs);
    }
  }
  for (uint32_t j = 4; j < W; j++) {  // randomize_unused_pi_wires
    gen(TAG_RANDOM_VALUE, {});
    g.target(Target::wire(cd.pi_row, j));
  }
  for (uint32_t row = 0; row < n; row++)  // constants_to_targets (value order) zipped with the generators
    if (cd.rows[row].kind == qc::G_CONSTANT) {
      // the last ConstantGate of an odd count keeps its second generator unused;
      // 0 (the smallest constant) can only be the first gate's first constant
      const uint64_t c[2] = {cd.rows[row].c0, cd.rows[row].c1};
      for (uint32_t j = 0; j < 2 && j < cd.config.num_constants; j++) {
        if (j == 1 && c[1] == 0) break;
        gen(TAG_CONSTANT, {});
        g.u64(row);
        g.u64(j);
        g.u64(j);
        g.u64(c[j]);
      }
    }
  for (uint32_t row = 0; row < n; row++) {  // gate generators
    const qc::GateInst &gi = cd.rows[row];
    if (gi.kind == qc::G_ARITHMETIC) {
      for (uint32_t i = 0; i < arith_ops; i++) {
        gen(TAG_ARITHMETIC_BASE, {Target::wire(row, 4 * i), Target::wire(row, 4 * i + 1), Target::wire(row, 4 * i + 2)});
        g.u64(row);
        g.u64(gi.c0);
        g.u64(gi.c1);
        g.u64(i);
      }
    } else if (gi.kind == qc::G_POSEIDON) {
      gen(TAG_POSEIDON, {Target::wire(row, 0), Target::wire(row, 1), Target::wire(row, 2), Target::wire(row, 3),
                         Target::wire(row, 4), Target::wire(row, 5), Target::wire(row, 6), Target::wire(row, 7),
                         Target::wire(row, 8), Target::wire(row, 9), Target::wire(row, 10), Target::wire(row, 11),
                         Target::wire(row, 24)});
      g.u64(row);
    } else if (gi.kind == qc::G_BASE_SUM) {
      gen(TAG_BASE_SPLIT, {Target::wire(row, 0)});
      g.u64(row);
      g.u64(limbs);
    }
  }
  Buf o;
  o.u64(ngen);
  o.b.insert(o.b.end(), g.b.begin(), g.b.end());
  g.b.clear();
  g.b.shrink_to_fit();
  o.u64(watches.size());
  for (const auto &kv : watches) {
    o.u64(kv.first);
    o.u64(kv.second.size());
    for (uint64_t i : kv.second) o.u64(i);
  }
  // ---- constants_sigmas_commitment: coefficients, the Merkle tree over the
  // LDE rows in leaf (bit-reversed) order, degree_log, rate_bits, blinding
  std::vector<uint64_t> coeffs(ncols * (size_t)n);
  if (qp_circuit_constants_sigmas_coeffs(circ, coeffs.data()) != QP_OK) throw std::runtime_error("coefficients");
  o.u64(ncols);
  for (size_t c = 0; c < ncols; c++) o.field_vec(coeffs.data() + c * n, n);
  const uint32_t lgN = lg + rb;
  std::vector<uint64_t> wN(N / 2);
  const uint64_t w = gl::root_of_unity(lgN);
  for (uint64_t k = 0; k < N / 2; k++) wN[k] = k ? gl::mul(wN[k - 1], w) : 1;
  std::vector<uint64_t> leaves(N * ncols);  // [leaf][col]
  parallel(ncols, [&](size_t c) {
    std::vector<uint64_t> a(N, 0);
    uint64_t s = 1;
    for (uint32_t k = 0; k < n; k++) {
      a[k] = gl::mul(coeffs[c * n + k], s);
      s = gl::mul(s, gl::GEN);
    }
    ntt(a.data(), lgN, wN);
    for (uint64_t i = 0; i < N; i++) leaves[i * ncols + c] = a[gl::rev_bits((uint32_t)i, lgN)];
  });
  std::vector<uint64_t> lh(N * 4);
  parallel(N / 1024, [&](size_t blk) {
    for (uint64_t i = blk * 1024; i < (blk + 1) * 1024; i++) {
      if (ncols > 4) {
        qh::hash_no_pad(leaves.data() + i * ncols, ncols, lh.data() + i * 4);
      } else {
        for (size_t k = 0; k < 4; k++) lh[i * 4 + k] = k < ncols ? leaves[i * ncols + k] : 0;
      }
    }
  });
  const uint64_t ncap = 1ull << cap_h, ndig = 2 * (N - ncap);
  std::vector<uint64_t> dig(ndig * 4), cap(ncap * 4);
  const uint64_t sub_d = ndig / ncap, sub_l = N / ncap;
  parallel(ncap, [&](size_t k) { fill_subtree(dig.data() + 4 * k * sub_d, sub_d, lh.data() + 4 * k * sub_l, sub_l,
                                              cap.data() + 4 * k); });
  o.u64(N);
  for (uint64_t i = 0; i < N; i++) {
    o.u64(ncols);
    o.fields(leaves.data() + i * ncols, ncols);
  }
  leaves.clear();
  leaves.shrink_to_fit();
  o.u64(ndig);
  o.fields(dig.data(), dig.size());
  o.u64(cap_h);
  o.fields(cap.data(), cap.size());
  o.u64(lg);
  o.u64(rb);
  o.u8(0);  // blinding: CONSTANTS_SIGMAS is never blinded
  // ---- sigmas: the transpose of the sigma polynomials' values, [n][R]
  o.u64(n);
  for (uint32_t row = 0; row < n; row++) {
    o.u64(R);
    for (uint32_t j = 0; j < R; j++) o.u64(cd.constants_sigmas[(size_t)(cd.num_constants + j) * n + row]);
  }
  // ---- subgroup, public inputs, representative map
  o.u64(n);
  {
    const uint64_t wn = gl::root_of_unity(lg);
    uint64_t x = 1;
    for (uint32_t i = 0; i < n; i++, x = gl::mul(x, wn)) o.u64(x);
  }
  o.u64(cd.public_input_targets.size());
  for (Target t : cd.public_input_targets) o.target(t);
  o.u64(fo.parents.size());
  o.fields(fo.parents.data(), fo.parents.size());
  // ---- fft_root_table(max_fft_points): row lg_m - 1 = powers of w_{2^lg_m},
  // max(2^(lg_m - 1), 2) of them
  {
    uint32_t lq = 0;
    while ((1u << lq) < cd.quotient_degree_factor) lq++;
    const uint32_t lgn = lg + std::max(rb, lq);
    o.u8(1);
    o.u64(lgn);
    for (uint32_t lm = 1; lm <= lgn; lm++) {
      const uint64_t len = std::max<uint64_t>(1ull << (lm - 1), 2), b = gl::root_of_unity(lm);
      o.u64(len);
      uint64_t x = 1;
      for (uint64_t i = 0; i < len; i++, x = gl::mul(x, b)) o.u64(x);
    }
  }
  // ---- circuit digest: hash_no_pad(cap || hash_pad([]) || degree_bits)
  {
    std::vector<uint64_t> buf(cap);
    uint64_t dsep[4];
    qh::hash_pad(nullptr, 0, dsep);
    buf.insert(buf.end(), dsep, dsep + 4);
    buf.push_back(lg);
    uint64_t d[4];
    qh::hash_no_pad(buf.data(), buf.size(), d);
    o.fields(d, 4);
  }
  o.u64(0);  // lookup_rows
  o.u64(0);  // lut_to_lookups
  return std::move(o.b);
}

}  // namespace

extern "C" int qp_circuit_prover_only_bytes(const qp_circuit *c, uint8_t *out, size_t cap, size_t *len) {
  if (!c || (!out && !len)) return QP_ERR_ARG;
  for (qc::GateKind k : c->cd.gate_kinds)
    if (k > qc::G_POSEIDON) return QP_ERR_ARG;  // the leaf circuits' gate set only
  // the size query builds the file and keeps it for the copy call that follows;
  // concurrent calls on one shared circuit handle serialise here
  std::lock_guard<std::mutex> lk(c->prover_bin_mu);
  try {
    if (c->prover_bin.empty()) c->prover_bin = prover_only_bytes(c);
  } catch (const std::bad_alloc &) {
    return QP_ERR_OOM;
  } catch (const std::exception &) {
    return QP_ERR_STATE;
  }
  if (len) *len = c->prover_bin.size();
  if (out) {
    if (cap < c->prover_bin.size()) return QP_ERR_ARG;
    memcpy(out, c->prover_bin.data(), c->prover_bin.size());
    std::vector<uint8_t>().swap(c->prover_bin);  // written out: drop the cache
  }
  return QP_OK;
}
