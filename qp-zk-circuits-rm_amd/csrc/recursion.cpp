// recursion.cpp — see recursion.h.  Follows upstream plonky2 (qp-plonky2 1.1.1):
//   plonk/recursive_verifier.rs   verify_proof / verify_proof_with_challenges
//   plonk/get_challenges.rs       get_challenges (circuit version)
//   iop/challenger.rs             RecursiveChallenger (observe / absorb / get)
//   plonk/vanishing_poly.rs       eval_vanishing_poly_circuit, check_partial_products_circuit
//   gates/*::eval_unfiltered_circuit (values), gates/selectors.rs compute_filter
//   fri/recursive_verifier.rs     verify_fri_proof, fri_verifier_query_round,
//                                 fri_combine_initial, compute_evaluation
//   hash/merkle_proofs.rs         verify_merkle_proof_to_cap_with_cap_index
// Gate values are the ones SURVEY.md A.5 pins (the oracle verifier's).
#include "recursion.h"
#include <stdexcept>
#include <string.h>
#include "field.h"
#include "poseidon.h"

namespace qr {

using qc::CircuitBuilder;
static const F NEG_ONE = gl::P - 1;
static const uint64_t UNUSED_SELECTOR = 0xFFFFFFFFull;

// ------------------------------------------------------------------ common data

uint32_t InnerCommon::final_poly_len() const {
  uint32_t tot = 0;
  for (auto a : arity_bits) tot += a;
  return 1u << (degree_bits - tot);
}

uint32_t InnerCommon::width(int o) const {
  switch (o) {
    case 0: return num_constants + num_routed_wires;
    case 1: return num_wires;
    case 2: return num_challenges * (1 + num_partial_products);
    default: return num_challenges * quotient_degree_factor;
  }
}

namespace {
struct Reader {
  const uint8_t *b;
  size_t n, pos = 0;
  bool err = false;
  uint64_t u64() {
    if (pos + 8 > n) {
      err = true;
      return 0;
    }
    uint64_t v;
    memcpy(&v, b + pos, 8);
    pos += 8;
    return v;
  }
  uint32_t u32() {
    if (pos + 4 > n) {
      err = true;
      return 0;
    }
    uint32_t v;
    memcpy(&v, b + pos, 4);
    pos += 4;
    return v;
  }
  uint8_t u8() {
    if (pos + 1 > n) {
      err = true;
      return 0;
    }
    return b[pos++];
  }
};
}  // namespace

std::string parse_common(const uint8_t *b, size_t n, InnerCommon &c) {
  Reader r{b, n};
  c.bytes.assign(b, b + n);
  c.num_wires = (uint32_t)r.u64();
  c.num_routed_wires = (uint32_t)r.u64();
  c.config_num_constants = (uint32_t)r.u64();
  r.u64();  // security_bits
  c.num_challenges = (uint32_t)r.u64();
  r.u64();  // max_quotient_degree_factor
  r.u8();   // use_base_arithmetic_gate
  c.zero_knowledge = r.u8() != 0;
  auto fri_config = [&](bool keep) {
    uint64_t rate = r.u64(), cap = r.u64(), nq = r.u64();
    uint32_t pow = r.u32();
    uint8_t tag = r.u8();
    if (tag == 1) {
      r.u64();
      r.u64();
    } else {
      r.err = true;  // only ConstantArityBits
    }
    if (keep) {
      c.rate_bits = (uint32_t)rate;
      c.cap_height = (uint32_t)cap;
      c.num_query_rounds = (uint32_t)nq;
      c.pow_bits = pow;
    }
  };
  fri_config(true);
  fri_config(false);
  uint64_t na = r.u64();
  if (na > 16) return "bad FRI arity list";
  for (uint64_t i = 0; i < na; i++) c.arity_bits.push_back((uint32_t)r.u64());
  c.degree_bits = (uint32_t)r.u64();
  c.hiding = r.u8() != 0;
  uint64_t ns = r.u64();
  if (ns > 64) return "bad selector list";
  for (uint64_t i = 0; i < ns; i++) c.selector_indices.push_back((uint32_t)r.u64());
  uint64_t ng = r.u64();
  if (ng > 64) return "bad selector groups";
  for (uint64_t i = 0; i < ng; i++) {
    uint32_t lo = (uint32_t)r.u64(), hi = (uint32_t)r.u64();
    c.groups.push_back({lo, hi});
  }
  c.quotient_degree_factor = (uint32_t)r.u64();
  c.num_gate_constraints = (uint32_t)r.u64();
  c.num_constants = (uint32_t)r.u64();
  c.num_public_inputs = (uint32_t)r.u64();
  uint64_t nk = r.u64();
  if (nk > 256) return "bad k_is";
  for (uint64_t i = 0; i < nk; i++) c.k_is.push_back(r.u64());
  c.num_partial_products = (uint32_t)r.u64();
  if (r.u64() || r.u64() || r.u64()) return "lookups are not supported";
  uint64_t ngates = r.u64();
  if (ngates > 16) return "too many gates";
  for (uint64_t i = 0; i < ngates; i++) {
    InnerCommon::Gate g{};
    g.id = r.u32();
    switch (g.id) {
      case 9: case 12: case 11: break;                  // Noop, PublicInput, Poseidon
      case 3: case 2: case 0: g.p[0] = r.u64(); break;  // Constant, BaseSum<2>, Arithmetic
      case 13: g.p[0] = r.u64(); g.p[1] = r.u64(); g.p[2] = r.u64(); break;  // RandomAccess
      default: return "unsupported gate (DefaultGateSerializer id " + std::to_string(g.id) + ") in the inner circuit";
    }
    c.gates.push_back(g);
  }
  if (r.err || r.pos != n) return "malformed CommonCircuitData bytes";
  if (c.num_challenges != 2 || c.hiding) return "unsupported inner config";
  if (c.selector_indices.size() != c.gates.size() || c.k_is.size() != c.num_routed_wires)
    return "inconsistent CommonCircuitData";
  for (auto &g : c.gates)
    if (g.id == 13 && (g.p[0] != qc::RA_BITS || g.p[1] != qc::RA_COPIES || g.p[2] != qc::RA_EXTRA))
      return "unsupported RandomAccessGate shape";
  return "";
}

size_t proof_bytes(const InnerCommon &c, uint32_t npis) {
  const size_t cl = (size_t)1 << c.cap_height;
  const uint32_t logN = c.degree_bits + c.rate_bits;
  size_t s = 3 * cl * 32;
  s += (size_t)(c.width(0) + c.num_wires + 2 * c.num_challenges + c.num_challenges * c.num_partial_products +
                c.width(3)) * 16;
  s += c.arity_bits.size() * cl * 32;
  size_t q = 0;
  for (int o = 0; o < 4; o++) q += (size_t)c.width(o) * 8 + 1 + (size_t)(logN - c.cap_height) * 32;
  uint32_t lg = logN;
  for (auto a : c.arity_bits) {
    lg -= a;
    q += ((size_t)16 << a) + 1 + (size_t)(lg - c.cap_height) * 32;
  }
  s += q * c.num_query_rounds;
  s += (size_t)c.final_poly_len() * 16 + 8 + 8 + (size_t)npis * 8;
  return s;
}

// ------------------------------------------------------------------ gadgets

namespace {

struct G {
  CircuitBuilder &b;
  explicit G(CircuitBuilder &bb) : b(bb) {}

  Target zero() { return b.zero(); }
  Target one() { return b.one(); }
  ExtT ext(Target x) { return {x, b.zero()}; }
  ExtT ext_const(F c0, F c1 = 0) { return {b.constant(c0), b.constant(c1)}; }
  ExtT ext_zero() { return {b.zero(), b.zero()}; }
  ExtT add(ExtT a, ExtT c) { return {b.add(a.c0, c.c0), b.add(a.c1, c.c1)}; }
  ExtT sub(ExtT a, ExtT c) { return {b.sub(a.c0, c.c0), b.sub(a.c1, c.c1)}; }
  // (a0 + a1 X)(c0 + c1 X), X^2 = 7: (a0 c0 + 7 a1 c1) + (a0 c1 + a1 c0) X
  ExtT mul(ExtT a, ExtT c) {
    Target t = b.mul(a.c1, c.c1);
    Target r0 = b.arithmetic(1, gl::EXT_W, a.c0, c.c0, t);
    Target u = b.mul(a.c1, c.c0);
    Target r1 = b.mul_add(a.c0, c.c1, u);
    return {r0, r1};
  }
  // a * c + d
  ExtT mul_add(ExtT a, ExtT c, ExtT d) {
    Target t = b.mul(a.c1, c.c1);
    Target r0 = b.add(b.arithmetic(1, gl::EXT_W, a.c0, c.c0, t), d.c0);
    Target r1 = b.mul_add(a.c0, c.c1, b.mul_add(a.c1, c.c0, d.c1));
    return {r0, r1};
  }
  // a * c - d
  ExtT mul_sub(ExtT a, ExtT c, ExtT d) { return sub(mul(a, c), d); }
  ExtT mul_base(ExtT a, Target s) { return {b.mul(a.c0, s), b.mul(a.c1, s)}; }
  // a * s + d (s base)
  ExtT mul_base_add(ExtT a, Target s, ExtT d) { return {b.mul_add(a.c0, s, d.c0), b.mul_add(a.c1, s, d.c1)}; }
  ExtT scale(ExtT a, F c) { return {b.mul_const(c, a.c0), b.mul_const(c, a.c1)}; }
  ExtT add_const(ExtT a, F c) { return {b.add(a.c0, b.constant(c)), a.c1}; }
  ExtT sub_base(ExtT a, Target s) { return {b.sub(a.c0, s), a.c1}; }
  ExtT square(ExtT a) { return mul(a, a); }
  ExtT exp_pow2(ExtT a, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) a = square(a);
    return a;
  }
  // num / den: quotient from a host generator (QuotientGeneratorExtension),
  // checked as den * q == num
  ExtT div(ExtT num, ExtT den) {
    ExtT q{b.add_virtual_target(), b.add_virtual_target()};
    qc::Gen g{};
    g.kind = qc::GEN_EXT_DIV;
    g.a = num.c0;
    g.b = num.c1;
    g.c = den.c0;
    g.d = den.c1;
    g.e = q.c0;
    g.f = q.c1;
    b.add_generator(g);
    connect(mul(den, q), num);
    return q;
  }
  void connect(ExtT a, ExtT c) {
    b.connect(a.c0, c.c0);
    b.connect(a.c1, c.c1);
  }
  ExtT mul_many(const std::vector<ExtT> &v) {
    ExtT acc = v[0];
    for (size_t i = 1; i < v.size(); i++) acc = mul(acc, v[i]);
    return acc;
  }
  // sum_i c_i x_i with small constant c_i (MDS rows)
  Target lin_comb(const uint64_t *c, const Target *x, size_t n) {
    Target acc = b.mul_const(c[0], x[0]);
    for (size_t i = 1; i < n; i++) acc = b.mul_const_add(c[i], x[i], acc);
    return acc;
  }
  // ReducingFactorTarget::reduce: sum_k t_k alpha^k (Horner from the last term)
  ExtT reduce_base_alpha(const std::vector<ExtT> &t, Target alpha) {
    ExtT acc = ext_zero();
    for (size_t i = t.size(); i-- > 0;) acc = mul_base_add(acc, alpha, t[i]);
    return acc;
  }
  ExtT reduce_ext(const std::vector<ExtT> &t, ExtT alpha) {
    ExtT acc = ext_zero();
    for (size_t i = t.size(); i-- > 0;) acc = mul_add(acc, alpha, t[i]);
    return acc;
  }
  // exp_from_bits_const_base: prod (1 + bit_i (base^(2^i) - 1))
  Target exp_from_bits_const_base(F base, const std::vector<Target> &bits) {
    Target p = b.one();
    F bp = base;
    for (Target bit : bits) {
      p = b.arithmetic(gl::sub(bp, 1), 1, p, bit, p);
      bp = gl::mul(bp, bp);
    }
    return p;
  }
  Target le_sum(const std::vector<Target> &bits) {
    Target acc = bits.back();
    for (size_t i = bits.size() - 1; i-- > 0;) acc = b.mul_const_add(2, acc, bits[i]);
    return acc;
  }
  Target exp_pow2_base(Target x, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) x = b.mul(x, x);
    return x;
  }
};

// RecursiveChallenger (iop/challenger.rs)
struct Chal {
  CircuitBuilder &b;
  std::vector<Target> state, in, out;
  explicit Chal(CircuitBuilder &bb) : b(bb), state(12, bb.zero()) {}
  void observe(Target t) {
    out.clear();
    in.push_back(t);
  }
  void observe(const std::vector<Target> &v) {
    for (Target t : v) observe(t);
  }
  void observe(ExtT e) {
    observe(e.c0);
    observe(e.c1);
  }
  void absorb() {
    if (in.empty()) return;
    for (size_t off = 0; off < in.size(); off += 8) {
      for (size_t i = 0; i < 8 && off + i < in.size(); i++) state[i] = in[off + i];
      state = b.permute(state);
    }
    out.assign(state.begin(), state.begin() + 8);
    in.clear();
  }
  Target get() {
    absorb();
    if (out.empty()) {
      state = b.permute(state);
      out.assign(state.begin(), state.begin() + 8);
    }
    Target t = out.back();
    out.pop_back();
    return t;
  }
  ExtT get_ext() {
    Target a = get();
    Target c = get();
    return {a, c};
  }
};

constexpr uint64_t MDS_C[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};

// MDS layer on extension states (base constants act per component)
void mds_ext(G &g, ExtT s[12]) {
  ExtT o[12];
  for (int r = 0; r < 12; r++) {
    uint64_t c[13];
    Target x0[13], x1[13];
    for (int i = 0; i < 12; i++) {
      c[i] = MDS_C[i];
      x0[i] = s[(i + r) % 12].c0;
      x1[i] = s[(i + r) % 12].c1;
    }
    size_t n = 12;
    if (r == 0) {
      c[12] = 8;
      x0[12] = s[0].c0;
      x1[12] = s[0].c1;
      n = 13;
    }
    o[r] = {g.lin_comb(c, x0, n), g.lin_comb(c, x1, n)};
  }
  for (int r = 0; r < 12; r++) s[r] = o[r];
}

ExtT sbox_ext(G &g, ExtT x) {
  ExtT x2 = g.square(x);
  ExtT x4 = g.square(x2);
  ExtT x3 = g.mul(x2, x);
  return g.mul(x3, x4);
}

// gates/*::eval_unfiltered (values at zeta), SURVEY.md A.5
std::vector<ExtT> gate_constraints(G &g, const InnerCommon::Gate &gate, const std::vector<ExtT> &w,
                                   const ExtT *gc, const std::vector<Target> &pi_hash) {
  std::vector<ExtT> out;
  switch (gate.id) {
    case 9:  // Noop
      break;
    case 3:  // Constant
      for (uint32_t i = 0; i < gate.p[0]; i++) out.push_back(g.sub(gc[i], w[i]));
      break;
    case 12:  // PublicInput
      for (uint32_t i = 0; i < 4; i++) out.push_back(g.sub_base(w[i], pi_hash[i]));
      break;
    case 2: {  // BaseSum<2>
      const uint32_t L = (uint32_t)gate.p[0];
      ExtT acc = w[L];
      for (uint32_t i = L - 1; i-- > 0;) acc = g.add(g.scale(acc, 2), w[1 + i]);
      out.push_back(g.sub(acc, w[0]));
      for (uint32_t i = 0; i < L; i++) {
        ExtT l = w[1 + i];
        out.push_back(g.mul(l, g.add_const(l, NEG_ONE)));
      }
      break;
    }
    case 0: {  // Arithmetic: out - (c0 m0 m1 + c1 addend)
      for (uint32_t i = 0; i < gate.p[0]; i++) {
        ExtT prod = g.mul(g.mul(w[4 * i], w[4 * i + 1]), gc[0]);
        ExtT comp = g.mul_add(w[4 * i + 2], gc[1], prod);
        out.push_back(g.sub(w[4 * i + 3], comp));
      }
      break;
    }
    case 13: {  // RandomAccess{bits, copies, extra}
      const uint32_t bits = (uint32_t)gate.p[0], copies = (uint32_t)gate.p[1], extra = (uint32_t)gate.p[2];
      const uint32_t vec = 1u << bits, routed = (2 + vec) * copies + extra;
      for (uint32_t cp = 0; cp < copies; cp++) {
        const uint32_t base = (2 + vec) * cp;
        std::vector<ExtT> bw(bits);
        for (uint32_t i = 0; i < bits; i++) bw[i] = w[routed + cp * bits + i];
        for (uint32_t i = 0; i < bits; i++) out.push_back(g.mul(bw[i], g.add_const(bw[i], NEG_ONE)));
        ExtT idx = bw[bits - 1];
        for (uint32_t i = bits - 1; i-- > 0;) idx = g.add(g.scale(idx, 2), bw[i]);
        out.push_back(g.sub(idx, w[base]));
        std::vector<ExtT> list(w.begin() + base + 2, w.begin() + base + 2 + vec);
        for (uint32_t i = 0; i < bits; i++) {
          std::vector<ExtT> nx(list.size() / 2);
          for (size_t j = 0; j < nx.size(); j++) nx[j] = g.mul_add(bw[i], g.sub(list[2 * j + 1], list[2 * j]), list[2 * j]);
          list = nx;
        }
        out.push_back(g.sub(list[0], w[base + 1]));
      }
      for (uint32_t i = 0; i < extra; i++) out.push_back(g.sub(gc[i], w[(2 + vec) * copies + i]));
      break;
    }
    case 11: {  // Poseidon (naive rounds, wire substitution at every stored S-box input)
      ExtT swap = w[24];
      out.push_back(g.mul(swap, g.add_const(swap, NEG_ONE)));
      ExtT s[12];
      for (int i = 0; i < 4; i++) {
        ExtT delta = w[25 + i];
        out.push_back(g.sub(g.mul(swap, g.sub(w[i + 4], w[i])), delta));
        s[i] = g.add(w[i], delta);
        s[i + 4] = g.sub(w[i + 4], delta);
      }
      for (int i = 8; i < 12; i++) s[i] = w[i];
      int rc = 0;
      for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = g.add_const(s[i], ps::RC_HOST[rc * 12 + i]);
        if (r)
          for (int i = 0; i < 12; i++) {
            ExtT wi = w[29 + (r - 1) * 12 + i];
            out.push_back(g.sub(s[i], wi));
            s[i] = wi;
          }
        for (int i = 0; i < 12; i++) s[i] = sbox_ext(g, s[i]);
        mds_ext(g, s);
      }
      for (int r = 0; r < 22; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = g.add_const(s[i], ps::RC_HOST[rc * 12 + i]);
        ExtT wi = w[65 + r];
        out.push_back(g.sub(s[0], wi));
        s[0] = sbox_ext(g, wi);
        mds_ext(g, s);
      }
      for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = g.add_const(s[i], ps::RC_HOST[rc * 12 + i]);
        for (int i = 0; i < 12; i++) {
          ExtT wi = w[87 + r * 12 + i];
          out.push_back(g.sub(s[i], wi));
          s[i] = sbox_ext(g, wi);
        }
        mds_ext(g, s);
      }
      for (int i = 0; i < 12; i++) out.push_back(g.sub(s[i], w[12 + i]));
      break;
    }
    default:
      throw std::runtime_error("unsupported inner gate");
  }
  return out;
}

std::vector<Target> virt(CircuitBuilder &b, size_t n) {
  auto v = b.add_virtual_targets(n);
  b.mark_inputs(v);
  return v;
}
std::vector<ExtT> virt_ext(CircuitBuilder &b, size_t n) {
  std::vector<ExtT> v(n);
  for (auto &e : v) {
    e = {b.add_virtual_target(), b.add_virtual_target()};
    b.mark_input(e.c0);
    b.mark_input(e.c1);
  }
  return v;
}

// verify_merkle_proof_to_cap_with_cap_index
void verify_merkle(CircuitBuilder &b, const std::vector<Target> &leaf, const std::vector<Target> &bits,
                   Target cap_index, const std::vector<Target> &cap, const std::vector<Target> &sibs) {
  std::vector<Target> h = b.hash_or_noop(leaf);
  const size_t depth = sibs.size() / 4;
  for (size_t k = 0; k < depth; k++) {
    std::vector<Target> st(12, b.zero());
    for (int i = 0; i < 4; i++) {
      st[i] = h[i];
      st[4 + i] = sibs[4 * k + i];
    }
    auto o = b.permute_swapped(st, bits[k]);
    h.assign(o.begin(), o.begin() + 4);
  }
  const size_t cl = cap.size() / 4;
  for (int i = 0; i < 4; i++) {
    std::vector<Target> col(cl);
    for (size_t e = 0; e < cl; e++) col[e] = cap[4 * e + i];
    b.connect(b.random_access(cap_index, col), h[i]);
  }
}

// interpolate {(c g^i, e_i)} at beta (barycentric over the coset of size 2^ab):
// p(beta) = (beta^m - c^m) / (m c^m) * sum_i e_i y_i / (beta - y_i), y_i = c g^i
ExtT interpolate_coset(G &g, Target c, const std::vector<ExtT> &e, ExtT beta, uint32_t ab) {
  CircuitBuilder &b = g.b;
  const uint32_t m = 1u << ab;
  const F om = gl::root_of_unity(ab);
  ExtT sum = g.ext_zero();
  F gi = 1;
  for (uint32_t i = 0; i < m; i++) {
    Target y = i ? b.mul_const(gi, c) : c;
    ExtT num = g.mul_base(e[i], y);
    sum = g.add(sum, g.div(num, g.sub_base(beta, y)));
    gi = gl::mul(gi, om);
  }
  Target cm = g.exp_pow2_base(c, ab);
  ExtT zb = g.sub_base(g.exp_pow2(beta, ab), cm);
  Target mcm = b.mul_const(m, cm);
  return g.div(g.mul(zb, sum), g.ext(mcm));
}

}  // namespace

// ------------------------------------------------------------------ verify_proof

static ProofTargets add_virtual_proof(CircuitBuilder &b, const InnerCommon &c) {
  ProofTargets p;
  const size_t cl = (size_t)1 << c.cap_height;
  p.wires_cap = virt(b, cl * 4);
  p.zs_cap = virt(b, cl * 4);
  p.quot_cap = virt(b, cl * 4);
  p.constants_sigmas = virt_ext(b, c.width(0));
  p.wires = virt_ext(b, c.num_wires);
  p.zs = virt_ext(b, c.num_challenges);
  p.zs_next = virt_ext(b, c.num_challenges);
  p.pp = virt_ext(b, (size_t)c.num_challenges * c.num_partial_products);
  p.quotient = virt_ext(b, c.width(3));
  for (size_t l = 0; l < c.arity_bits.size(); l++) p.commit_caps.push_back(virt(b, cl * 4));
  const uint32_t logN = c.degree_bits + c.rate_bits;
  for (uint32_t q = 0; q < c.num_query_rounds; q++) {
    QueryTargets qt;
    for (int o = 0; o < 4; o++) {
      qt.leaf[o] = virt(b, c.width(o));
      qt.sib[o] = virt(b, (size_t)(logN - c.cap_height) * 4);
    }
    uint32_t lg = logN;
    for (auto a : c.arity_bits) {
      lg -= a;
      qt.evals.push_back(virt_ext(b, (size_t)1 << a));
      qt.lsib.push_back(virt(b, (size_t)(lg - c.cap_height) * 4));
    }
    p.queries.push_back(std::move(qt));
  }
  p.final_poly = virt_ext(b, c.final_poly_len());
  p.pow_witness = virt(b, 1)[0];
  p.pis = virt(b, c.num_public_inputs);
  return p;
}

static void verify_proof(CircuitBuilder &b, const InnerCommon &c, const ProofTargets &p,
                         const std::vector<Target> &vd_cap, const std::vector<Target> &vd_digest) {
  G g(b);
  const uint32_t nc = c.num_challenges, R = c.num_routed_wires, qdf = c.quotient_degree_factor;
  const uint32_t nsel = (uint32_t)c.groups.size(), npp = c.num_partial_products;
  const uint32_t log_n = c.degree_bits, logN = log_n + c.rate_bits;
  // ---- challenges (plonk/get_challenges.rs, circuit version)
  std::vector<Target> pi_hash = b.hash_n_to_hash_no_pad(p.pis);
  Chal ch(b);
  ch.observe(vd_digest);
  ch.observe(pi_hash);
  ch.observe(p.wires_cap);
  std::vector<Target> betas(nc), gammas(nc), alphas(nc);
  for (auto &t : betas) t = ch.get();
  for (auto &t : gammas) t = ch.get();
  ch.observe(p.zs_cap);
  for (auto &t : alphas) t = ch.get();
  ch.observe(p.quot_cap);
  ExtT zeta = ch.get_ext();
  // openings in FriOpenings order: zeta batch, then the g*zeta batch
  std::vector<ExtT> zbatch;
  for (auto *v : {&p.constants_sigmas, &p.wires, &p.zs, &p.pp, &p.quotient}) zbatch.insert(zbatch.end(), v->begin(), v->end());
  for (ExtT e : zbatch) ch.observe(e);
  for (ExtT e : p.zs_next) ch.observe(e);
  ExtT fri_alpha = ch.get_ext();
  std::vector<ExtT> fri_betas;
  for (auto &cap : p.commit_caps) {
    ch.observe(cap);
    fri_betas.push_back(ch.get_ext());
  }
  for (ExtT e : p.final_poly) ch.observe(e);
  ch.observe(p.pow_witness);
  Target pow_response = ch.get();
  std::vector<Target> qidx(c.num_query_rounds);
  for (auto &t : qidx) t = ch.get();
  // ---- proof of work: leading zeros (fri_verify_proof_of_work -> range_check)
  b.range_check(pow_response, 64 - c.pow_bits);

  // ---- vanishing polynomial at zeta (eval_vanishing_poly_circuit)
  ExtT zeta_n = g.exp_pow2(zeta, log_n);
  std::vector<ExtT> gate_terms(c.num_gate_constraints, g.ext_zero());
  for (size_t gi = 0; gi < c.gates.size(); gi++) {
    const uint32_t si = c.selector_indices[gi];
    const auto grp = c.groups[si];
    ExtT s = p.constants_sigmas[si];
    std::vector<ExtT> fac;
    for (uint32_t j = grp.first; j < grp.second; j++)
      if (j != gi) fac.push_back(g.sub(g.ext_const(j), s));
    if (nsel > 1) fac.push_back(g.sub(g.ext_const(UNUSED_SELECTOR), s));
    ExtT filter = fac.empty() ? g.ext_const(1) : g.mul_many(fac);
    auto cs = gate_constraints(g, c.gates[gi], p.wires, p.constants_sigmas.data() + nsel, pi_hash);
    if (cs.size() > gate_terms.size()) throw std::runtime_error("gate constraint count exceeds num_gate_constraints");
    for (size_t k = 0; k < cs.size(); k++) gate_terms[k] = g.mul_add(filter, cs[k], gate_terms[k]);
  }
  // L_0(zeta) = (zeta^n - 1) / (n (zeta - 1))
  ExtT zh = g.add_const(zeta_n, NEG_ONE);
  ExtT l0 = g.div(zh, g.scale(g.add_const(zeta, NEG_ONE), (F)1 << log_n));
  std::vector<ExtT> s_ids(R);
  for (uint32_t j = 0; j < R; j++) s_ids[j] = g.scale(zeta, c.k_is[j]);
  std::vector<ExtT> z1_terms, pp_terms;
  const ExtT *sig = p.constants_sigmas.data() + c.num_constants;
  for (uint32_t i = 0; i < nc; i++) {
    ExtT z = p.zs[i], zn = p.zs_next[i];
    z1_terms.push_back(g.mul_sub(l0, z, l0));
    std::vector<ExtT> num(R), den(R);
    for (uint32_t j = 0; j < R; j++) {
      ExtT wg = g.add(p.wires[j], g.ext(gammas[i]));
      num[j] = g.mul_base_add(s_ids[j], betas[i], wg);
      den[j] = g.mul_base_add(sig[j], betas[i], wg);
    }
    std::vector<ExtT> accs{z};
    for (uint32_t k = 0; k < npp; k++) accs.push_back(p.pp[i * npp + k]);
    accs.push_back(zn);
    for (uint32_t k = 0; k * qdf < R; k++) {
      const uint32_t lo = k * qdf, hi = std::min(R, lo + qdf);
      ExtT np = g.mul_many(std::vector<ExtT>(num.begin() + lo, num.begin() + hi));
      ExtT dp = g.mul_many(std::vector<ExtT>(den.begin() + lo, den.begin() + hi));
      pp_terms.push_back(g.sub(g.mul(accs[k], np), g.mul(accs[k + 1], dp)));
    }
  }
  std::vector<ExtT> terms = z1_terms;
  terms.insert(terms.end(), pp_terms.begin(), pp_terms.end());
  terms.insert(terms.end(), gate_terms.begin(), gate_terms.end());
  for (uint32_t i = 0; i < nc; i++) {
    ExtT van = g.reduce_base_alpha(terms, alphas[i]);
    std::vector<ExtT> chunk(p.quotient.begin() + i * qdf, p.quotient.begin() + (i + 1) * qdf);
    ExtT rec = g.reduce_ext(chunk, zeta_n);
    g.connect(van, g.mul(zh, rec));
  }

  // ---- FRI (verify_fri_proof)
  const F g_n = gl::root_of_unity(log_n);
  ExtT zeta_next = g.scale(zeta, g_n);
  // precomputed reduced openings (ReducingFactorTarget over each batch)
  ExtT red0 = g.reduce_ext(zbatch, fri_alpha);
  ExtT red1 = g.reduce_ext(p.zs_next, fri_alpha);
  // powers of alpha for the per-query base reductions (the same values as Horner)
  const size_t nb0 = zbatch.size();
  std::vector<ExtT> apow(nb0);
  apow[0] = g.ext_const(1);
  for (size_t k = 1; k < nb0; k++) apow[k] = g.mul(apow[k - 1], fri_alpha);
  ExtT alpha_sq = apow[nc];  // shift of the zeta-batch sum by alpha^(#g*zeta batch)
  const std::vector<Target> *caps[4] = {&vd_cap, &p.wires_cap, &p.zs_cap, &p.quot_cap};
  const F phi = gl::root_of_unity(logN);
  for (uint32_t q = 0; q < c.num_query_rounds; q++) {
    const QueryTargets &qt = p.queries[q];
    std::vector<Target> bits = b.split_le(qidx[q], 64);
    bits.resize(logN);
    Target cap_idx = g.le_sum(std::vector<Target>(bits.end() - c.cap_height, bits.end()));
    for (int o = 0; o < 4; o++) verify_merkle(b, qt.leaf[o], bits, cap_idx, *caps[o], qt.sib[o]);
    std::vector<Target> rbits(bits.rbegin(), bits.rend());
    Target x = b.mul(b.constant(gl::GEN), g.exp_from_bits_const_base(phi, rbits));
    // fri_combine_initial
    Target acc0 = b.zero(), acc1 = b.zero();
    size_t k = 0;
    for (int o = 0; o < 4; o++)
      for (Target v : qt.leaf[o]) {
        if (k == 0) {
          acc0 = v;
        } else {
          acc0 = b.mul_add(apow[k].c0, v, acc0);
          acc1 = b.mul_add(apow[k].c1, v, acc1);
        }
        k++;
      }
    ExtT rv0{acc0, acc1};
    // the g*zeta batch: the first nc polynomials of oracle 2 (the Z's)
    std::vector<ExtT> zl;
    for (uint32_t i = 0; i < nc; i++) zl.push_back(g.ext(qt.leaf[2][i]));
    ExtT rv1 = g.reduce_ext(zl, fri_alpha);
    ExtT t0 = g.div(g.sub(rv0, red0), g.sub(g.ext(x), zeta));
    ExtT t1 = g.div(g.sub(rv1, red1), g.sub(g.ext(x), zeta_next));
    ExtT old_eval = g.mul_add(t0, alpha_sq, t1);
    // folding layers
    Target sx = x;
    for (size_t l = 0; l < c.arity_bits.size(); l++) {
      const uint32_t ab = c.arity_bits[l];
      std::vector<Target> within(bits.begin(), bits.begin() + ab);
      std::vector<Target> coset(bits.begin() + ab, bits.end());
      Target within_idx = g.le_sum(within);
      const auto &ev = qt.evals[l];
      std::vector<Target> e0(ev.size()), e1(ev.size());
      for (size_t i = 0; i < ev.size(); i++) {
        e0[i] = ev[i].c0;
        e1[i] = ev[i].c1;
      }
      g.connect(ExtT{b.random_access(within_idx, e0), b.random_access(within_idx, e1)}, old_eval);
      // compute_evaluation: interpolate the bit-reversed evals over the coset
      // starting at x * g_inv^rev(within)
      const F gen = gl::root_of_unity(ab);
      const F g_inv = gl::pow(gen, (1ull << ab) - 1);
      std::vector<Target> rwithin(within.rbegin(), within.rend());
      Target start = b.mul(g.exp_from_bits_const_base(g_inv, rwithin), sx);
      std::vector<ExtT> erev(ev.size());
      for (uint32_t i = 0; i < ev.size(); i++) erev[gl::rev_bits(i, ab)] = ev[i];
      old_eval = interpolate_coset(g, start, erev, fri_betas[l], ab);
      std::vector<Target> flat;
      for (ExtT e : ev) {
        flat.push_back(e.c0);
        flat.push_back(e.c1);
      }
      verify_merkle(b, flat, coset, cap_idx, p.commit_caps[l], qt.lsib[l]);
      sx = g.exp_pow2_base(sx, ab);
      bits = coset;
    }
    // final polynomial at x (PolynomialCoeffsExtTarget::eval_scalar)
    ExtT fe = g.ext_zero();
    for (size_t i = p.final_poly.size(); i-- > 0;) fe = g.mul_base_add(fe, sx, p.final_poly[i]);
    g.connect(fe, old_eval);
  }
}

AggregationTargets build_aggregation(CircuitBuilder &b, const InnerCommon &inner, uint32_t nproofs) {
  AggregationTargets t;
  t.inner = inner;
  t.vd_cap = virt(b, ((size_t)1 << inner.cap_height) * 4);
  t.vd_digest = virt(b, 4);
  for (uint32_t i = 0; i < nproofs; i++) {
    ProofTargets p = add_virtual_proof(b, inner);
    verify_proof(b, inner, p, t.vd_cap, t.vd_digest);
    for (Target pi : p.pis) b.register_public_input(pi);
    t.proofs.push_back(std::move(p));
  }
  return t;
}

// ------------------------------------------------------------------ witness

namespace {
struct PR {  // proof reader
  const uint8_t *b;
  size_t n, pos = 0;
  bool err = false;
  F fe() {
    if (pos + 8 > n) {
      err = true;
      return 0;
    }
    F v;
    memcpy(&v, b + pos, 8);
    pos += 8;
    if (v >= gl::P) err = true;
    return v;
  }
  uint8_t u8() {
    if (pos >= n) {
      err = true;
      return 0;
    }
    return b[pos++];
  }
};
}  // namespace

std::string fill_aggregation(const AggregationTargets &t, const uint8_t *vo, size_t volen,
                             const uint8_t *const *proofs, const size_t *lens, uint32_t nproofs, qc::Witness &w) {
  const char *conflict = "Partition containing a target was set twice with different values";
  const InnerCommon &c = t.inner;
  if (nproofs != t.proofs.size())
    return "expected " + std::to_string(t.proofs.size()) + " proofs, got " + std::to_string(nproofs);
  const size_t cl = (size_t)1 << c.cap_height;
  if (volen != 8 + cl * 32 + 32) return "verifier-only data of " + std::to_string(volen) + " bytes";
  {
    uint64_t h;
    memcpy(&h, vo, 8);
    if (h != c.cap_height) return "verifier data cap height differs from the common data";
    PR r{vo + 8, volen - 8};
    for (Target x : t.vd_cap)
      if (!w.set(x, r.fe())) return conflict;
    for (Target x : t.vd_digest)
      if (!w.set(x, r.fe())) return conflict;
    if (r.err) return "non-canonical verifier data";
  }
  for (uint32_t pi = 0; pi < nproofs; pi++) {
    const ProofTargets &p = t.proofs[pi];
    if (!proofs[pi] || lens[pi] != proof_bytes(c, c.num_public_inputs))
      return "proof " + std::to_string(pi) + ": failed to deserialize (" + std::to_string(lens[pi]) + " bytes)";
    PR r{proofs[pi], lens[pi]};
    bool ok = true;
    auto set = [&](Target x) { ok = ok && w.set(x, r.fe()); };
    auto setx = [&](const ExtT &e) {
      set(e.c0);
      set(e.c1);
    };
    for (Target x : p.wires_cap) set(x);
    for (Target x : p.zs_cap) set(x);
    for (Target x : p.quot_cap) set(x);
    for (auto &e : p.constants_sigmas) setx(e);
    for (auto &e : p.wires) setx(e);
    for (auto &e : p.zs) setx(e);
    for (auto &e : p.zs_next) setx(e);
    for (auto &e : p.pp) setx(e);
    for (auto &e : p.quotient) setx(e);
    for (auto &cap : p.commit_caps)
      for (Target x : cap) set(x);
    for (auto &qt : p.queries) {
      for (int o = 0; o < 4; o++) {
        for (Target x : qt.leaf[o]) set(x);
        if (r.u8() != qt.sib[o].size() / 4) r.err = true;
        for (Target x : qt.sib[o]) set(x);
      }
      for (size_t l = 0; l < qt.evals.size(); l++) {
        for (auto &e : qt.evals[l]) setx(e);
        if (r.u8() != qt.lsib[l].size() / 4) r.err = true;
        for (Target x : qt.lsib[l]) set(x);
      }
    }
    for (auto &e : p.final_poly) setx(e);
    set(p.pow_witness);
    uint64_t npis = 0;
    if (r.pos + 8 <= r.n) memcpy(&npis, r.b + r.pos, 8);
    r.pos += 8;
    if (npis != p.pis.size()) return "proof " + std::to_string(pi) + ": public input count differs";
    for (Target x : p.pis) set(x);
    if (r.err || r.pos != r.n) return "proof " + std::to_string(pi) + ": failed to deserialize";
    if (!ok) return conflict;
  }
  return "";
}

}  // namespace qr
