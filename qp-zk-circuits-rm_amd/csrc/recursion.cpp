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
      case 9: case 12: case 11: case 10: break;         // Noop, PublicInput, Poseidon, PoseidonMds
      case 3: case 2: case 0:                           // Constant, BaseSum<2>, Arithmetic,
      case 1: case 8: case 15: case 14:                 // ArithmeticExtension, MulExtension, Reducing(Extension)
        g.p[0] = r.u64();
        break;
      case 13: g.p[0] = r.u64(); g.p[1] = r.u64(); g.p[2] = r.u64(); break;  // RandomAccess
      case 4: {  // CosetInterpolation: subgroup_bits, degree, barycentric_weights
        g.p[0] = r.u64();
        g.p[1] = r.u64();
        const uint64_t nw = r.u64();
        if (g.p[0] > 6 || nw != (1ull << g.p[0]) || g.p[1] < 2) return "bad CosetInterpolationGate";
        for (uint64_t i = 0; i < nw; i++) r.u64();
        break;
      }
      default: return "unsupported gate (DefaultGateSerializer id " + std::to_string(g.id) + ") in the inner circuit";
    }
    c.gates.push_back(g);
  }
  if (r.err || r.pos != n) return "malformed CommonCircuitData bytes";
  if (c.num_challenges != 2 || c.hiding) return "unsupported inner config";
  if (c.selector_indices.size() != c.gates.size() || c.k_is.size() != c.num_routed_wires)
    return "inconsistent CommonCircuitData";
  for (auto &g : c.gates) {
    if (g.id == 13 && (g.p[0] != qc::RA_BITS || g.p[1] != qc::RA_COPIES || g.p[2] != qc::RA_EXTRA))
      return "unsupported RandomAccessGate shape";
    if (g.id == 4 && (g.p[0] != qc::CI_BITS || g.p[1] != qc::CI_DEGREE)) return "unsupported CosetInterpolationGate shape";
  }
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

  // extension arithmetic on ArithmeticExtension / MulExtension gate ops
  // (gadgets/arithmetic_extension.rs), as upstream's recursive verifier builds it
  Target zero() { return b.zero(); }
  Target one() { return b.one(); }
  ExtT ext(Target x) { return b.convert_to_ext(x); }
  ExtT ext_const(F c0, F c1 = 0) { return b.constant_ext(c0, c1); }
  ExtT ext_zero() { return b.zero_ext(); }
  ExtT add(ExtT a, ExtT c) { return b.add_ext(a, c); }
  ExtT sub(ExtT a, ExtT c) { return b.sub_ext(a, c); }
  ExtT mul(ExtT a, ExtT c) { return b.mul_ext(a, c); }
  ExtT mul_add(ExtT a, ExtT c, ExtT d) { return b.mul_add_ext(a, c, d); }
  ExtT mul_sub(ExtT a, ExtT c, ExtT d) { return b.mul_sub_ext(a, c, d); }
  ExtT scale(ExtT a, F c) { return b.scalar_mul_ext(c, a); }
  ExtT add_const(ExtT a, F c) { return b.add_const_ext(a, c); }
  ExtT div(ExtT num, ExtT den) { return b.div_ext(num, den); }
  ExtT div_add(ExtT num, ExtT den, ExtT z) { return b.div_add_ext(num, den, z); }
  ExtT square(ExtT a) { return b.square_ext(a); }
  ExtT exp_pow2(ExtT a, uint32_t k) { return b.exp_power_of_2_ext(a, k); }
  void connect(ExtT a, ExtT c) { b.connect_ext(a, c); }
  ExtT mul_many(const std::vector<ExtT> &v) { return b.mul_many_ext(v); }
  // exp_from_bits_const_base: prod (1 + bit_i (base^(2^i) - 1)) (base arithmetic)
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
  // ExtensionAlgebraTarget<2> (the recursion gates' values at zeta: pairs of
  // extension targets a + b Y, Y^2 = 7; gadgets/arithmetic_extension.rs)
  struct Alg {
    ExtT a, b;
  };
  Alg alg(const std::vector<ExtT> &w, uint32_t i) { return {w[i], w[i + 1]}; }
  Alg alg_zero() { return {ext_zero(), ext_zero()}; }
  Alg alg_sub(Alg x, Alg y) { return {sub(x.a, y.a), sub(x.b, y.b)}; }
  // mul_add_ext_algebra: the W-weighted inner product first, then the plain one
  Alg alg_mul_add(Alg x, Alg y, Alg z) {
    ExtT r0 = b.arithmetic_extension(gl::EXT_W, 1, x.b, y.b, z.a);
    r0 = b.mul_add_ext(x.a, y.a, r0);
    ExtT r1 = b.mul_add_ext(x.a, y.b, z.b);
    r1 = b.mul_add_ext(x.b, y.a, r1);
    return {r0, r1};
  }
  Alg alg_mul(Alg x, Alg y) { return alg_mul_add(x, y, alg_zero()); }
  Alg alg_scalar_mul_add(ExtT c, Alg x, Alg z) { return {mul_add(c, x.a, z.a), mul_add(c, x.b, z.b)}; }
  Alg alg_scalar_mul(ExtT c, Alg x) { return alg_scalar_mul_add(c, x, alg_zero()); }
  void push(std::vector<ExtT> &out, Alg x) {
    out.push_back(x.a);
    out.push_back(x.b);
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

// MDS layer on ext states: one PoseidonMdsGate row (mds_layer_circuit with
// num_routed_wires >= 48)
void mds_ext(G &g, ExtT s[12]) {
  std::vector<ExtT> v(s, s + 12);
  v = g.b.poseidon_mds(v);
  for (int r = 0; r < 12; r++) s[r] = v[r];
}

// sbox_monomial_circuit: exp_u64_extension(x, 7)
ExtT sbox_ext(G &g, ExtT x) { return g.b.exp_u64_ext(x, 7); }

// gates/*::eval_unfiltered_circuit (values at zeta), in upstream plonky2's
// operation forms (values pinned by SURVEY.md A.5 for the leaf gates; the
// recursion gates' formulas restate upstream, parity unpinned)
std::vector<ExtT> gate_constraints(G &g, const InnerCommon::Gate &gate, const std::vector<ExtT> &w,
                                   const ExtT *gc, const std::vector<Target> &pi_hash) {
  std::vector<ExtT> out;
  CircuitBuilder &b = g.b;
  switch (gate.id) {
    case 9:  // Noop
      break;
    case 3:  // Constant
      for (uint32_t i = 0; i < gate.p[0]; i++) out.push_back(g.sub(gc[i], w[i]));
      break;
    case 12:  // PublicInput
      for (uint32_t i = 0; i < 4; i++) out.push_back(g.sub(w[i], g.ext(pi_hash[i])));
      break;
    case 2: {  // BaseSum<2>: the recomposed sum, then limb (limb - 1) per limb
      const uint32_t L = (uint32_t)gate.p[0];
      std::vector<ExtT> limbs(w.begin() + 1, w.begin() + 1 + L);
      out.push_back(g.sub(b.reduce_ext(g.ext_const(2), limbs), w[0]));
      for (ExtT l : limbs) out.push_back(g.mul_sub(l, l, l));
      break;
    }
    case 0: {  // Arithmetic: out - (c0 m0 m1 + c1 addend)
      for (uint32_t i = 0; i < gate.p[0]; i++) {
        ExtT scaled = g.mul_many({gc[0], w[4 * i], w[4 * i + 1]});
        ExtT comp = g.mul_add(gc[1], w[4 * i + 2], scaled);
        out.push_back(g.sub(w[4 * i + 3], comp));
      }
      break;
    }
    case 1:    // ArithmeticExtension{num_ops}: out - (c0 m0 m1 + c1 addend), algebra
    case 8: {  // MulExtension{num_ops}: out - c0 m0 m1
      const bool ae = gate.id == 1;
      for (uint32_t i = 0; i < gate.p[0]; i++) {
        const uint32_t o = ae ? 8 * i : 6 * i;
        G::Alg scaled = g.alg_scalar_mul(gc[0], g.alg_mul(g.alg(w, o), g.alg(w, o + 2)));
        if (ae) scaled = g.alg_scalar_mul_add(gc[1], g.alg(w, o + 4), scaled);
        g.push(out, g.alg_sub(g.alg(w, ae ? o + 6 : o + 4), scaled));
      }
      break;
    }
    case 15:    // Reducing{num_coeffs}: acc_i - (acc_{i-1} alpha + coeff_i), base coefficients
    case 14: {  // ReducingExtension{num_coeffs}: ext coefficients
      const uint32_t nc = (uint32_t)gate.p[0], cw = gate.id == 15 ? 1 : 2;
      const G::Alg alpha = g.alg(w, 2);
      G::Alg acc = g.alg(w, 4);
      for (uint32_t i = 0; i < nc; i++) {
        const G::Alg coeff = cw == 1 ? G::Alg{w[6 + i], g.ext_zero()} : g.alg(w, 6 + 2 * i);
        const G::Alg next = g.alg(w, i + 1 == nc ? 0 : 6 + cw * nc + 2 * i);
        g.push(out, g.alg_sub(g.alg_mul_add(acc, alpha, coeff), next));
        acc = next;
      }
      break;
    }
    case 10: {  // PoseidonMds: out_r - (sum_i CIRC[i] in_{i+r} + DIAG[r] in_r), algebra
      for (uint32_t r = 0; r < 12; r++) {
        G::Alg res = g.alg_zero();
        for (uint32_t i = 0; i < 12; i++)
          res = g.alg_scalar_mul_add(g.ext_const(ps::mds_circ(i)), g.alg(w, 2 * ((i + r) % 12)), res);
        res = g.alg_scalar_mul_add(g.ext_const(r == 0 ? 8 : 0), g.alg(w, 2 * r), res);
        g.push(out, g.alg_sub(g.alg(w, 24 + 2 * r), res));
      }
      break;
    }
    case 4: {  // CosetInterpolation{subgroup_bits, degree}
      const uint32_t nbits = (uint32_t)gate.p[0], deg = (uint32_t)gate.p[1], np = 1u << nbits;
      const uint32_t nint = (np - 2) / (deg - 1);
      const uint32_t sv = 1, sep = sv + 2 * np, sev = sep + 2, si = sev + 2, ssh = si + 4 * nint;
      const ExtT shift = w[0];
      const G::Alg ep = g.alg(w, sep), sp = g.alg(w, ssh);
      g.push(out, g.alg_scalar_mul_add(g.scale(shift, gl::P - 1), sp, ep));
      const F om = gl::root_of_unity(nbits), ninv = gl::inv(np);
      G::Alg ev = g.alg_zero(), pr{g.ext_const(1), g.ext_zero()};
      uint32_t lo = 0, hi = deg;
      for (uint32_t it = 0;; it++) {
        for (uint32_t i = lo; i < hi; i++) {
          const F x = gl::pow(om, i);
          const G::Alg term{g.sub(sp.a, g.ext_const(x)), sp.b};
          const G::Alg wv = g.alg_scalar_mul(g.ext_const(gl::mul(x, ninv)), g.alg(w, sv + 2 * i));
          ev = g.alg_mul_add(wv, pr, g.alg_mul(ev, term));
          pr = g.alg_mul(pr, term);
        }
        if (it == nint) break;
        const G::Alg ie = g.alg(w, si + 2 * it), ip = g.alg(w, si + 2 * (nint + it));
        g.push(out, g.alg_sub(ie, ev));
        g.push(out, g.alg_sub(ip, pr));
        ev = ie;
        pr = ip;
        lo = 1 + (deg - 1) * (it + 1);
        hi = std::min(lo + deg - 1, np);
      }
      g.push(out, g.alg_sub(g.alg(w, sev), ev));
      break;
    }
    case 13: {  // RandomAccess{bits, copies, extra}
      const uint32_t bits = (uint32_t)gate.p[0], copies = (uint32_t)gate.p[1], extra = (uint32_t)gate.p[2];
      const uint32_t vec = 1u << bits, routed = (2 + vec) * copies + extra;
      for (uint32_t cp = 0; cp < copies; cp++) {
        const uint32_t base = (2 + vec) * cp;
        std::vector<ExtT> bw(bits);
        for (uint32_t i = 0; i < bits; i++) bw[i] = w[routed + cp * bits + i];
        for (uint32_t i = 0; i < bits; i++) out.push_back(g.mul_sub(bw[i], bw[i], bw[i]));
        ExtT idx = g.ext_zero();
        for (uint32_t i = bits; i-- > 0;) idx = b.mul_const_add_ext(2, idx, bw[i]);
        out.push_back(g.sub(idx, w[base]));
        std::vector<ExtT> list(w.begin() + base + 2, w.begin() + base + 2 + vec);
        for (uint32_t i = 0; i < bits; i++) {
          std::vector<ExtT> nx(list.size() / 2);
          // select_ext_generalized(b, y, x) = b y - (b x - x)
          for (size_t j = 0; j < nx.size(); j++)
            nx[j] = g.mul_sub(bw[i], list[2 * j + 1], g.mul_sub(bw[i], list[2 * j], list[2 * j]));
          list = nx;
        }
        out.push_back(g.sub(list[0], w[base + 1]));
      }
      for (uint32_t i = 0; i < extra; i++) out.push_back(g.sub(gc[i], w[(2 + vec) * copies + i]));
      break;
    }
    case 11: {  // Poseidon: constant layers, x^7 S-boxes, PoseidonMdsGate layers, wire checks
      ExtT swap = w[24];
      out.push_back(g.mul_sub(swap, swap, swap));
      for (int i = 0; i < 4; i++) out.push_back(g.mul_sub(swap, g.sub(w[i + 4], w[i]), w[25 + i]));
      ExtT s[12];
      for (int i = 0; i < 4; i++) {
        ExtT delta = w[25 + i];
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
  // evaluate_gate_constraints_circuit: per gate its filter times each constraint
  std::vector<ExtT> gate_terms(c.num_gate_constraints, g.ext_zero());
  for (size_t gi = 0; gi < c.gates.size(); gi++) {
    const uint32_t si = c.selector_indices[gi];
    const auto grp = c.groups[si];
    ExtT s = p.constants_sigmas[si];
    std::vector<ExtT> fac;
    for (uint32_t j = grp.first; j < grp.second; j++)
      if (j != gi) fac.push_back(g.sub(g.ext_const(j), s));
    if (nsel > 1) fac.push_back(g.sub(g.ext_const(UNUSED_SELECTOR), s));
    ExtT filter = g.mul_many(fac);
    auto cs = gate_constraints(g, c.gates[gi], p.wires, p.constants_sigmas.data() + nsel, pi_hash);
    if (cs.size() > gate_terms.size()) throw std::runtime_error("gate constraint count exceeds num_gate_constraints");
    for (size_t k = 0; k < cs.size(); k++) gate_terms[k] = g.mul_add(filter, cs[k], gate_terms[k]);
  }
  // eval_l_0_circuit: L_0(zeta) = (zeta^n - 1) / (n (zeta - 1))
  ExtT zh = g.sub(zeta_n, g.ext_const(1));
  const F nn = (F)1 << log_n;
  ExtT l0 = g.div(zh, b.arithmetic_extension(nn, nn, zeta, g.ext_const(1), g.ext(b.constant(NEG_ONE))));
  std::vector<ExtT> s_ids(R);
  for (uint32_t j = 0; j < R; j++) s_ids[j] = b.mul_ext(b.convert_to_ext(b.constant(c.k_is[j])), zeta);
  std::vector<ExtT> z1_terms, pp_terms;
  const ExtT *sig = p.constants_sigmas.data() + c.num_constants;
  for (uint32_t i = 0; i < nc; i++) {
    ExtT z = p.zs[i], zn = p.zs_next[i];
    z1_terms.push_back(g.mul_sub(l0, z, l0));
    std::vector<ExtT> num(R), den(R);
    for (uint32_t j = 0; j < R; j++) {
      ExtT wg = g.add(p.wires[j], g.ext(gammas[i]));
      num[j] = g.mul_add(g.ext(betas[i]), s_ids[j], wg);
      den[j] = g.mul_add(g.ext(betas[i]), sig[j], wg);
    }
    // check_partial_products_circuit
    std::vector<ExtT> accs{z};
    for (uint32_t k = 0; k < npp; k++) accs.push_back(p.pp[i * npp + k]);
    accs.push_back(zn);
    for (uint32_t k = 0; k * qdf < R; k++) {
      const uint32_t lo = k * qdf, hi = std::min(R, lo + qdf);
      ExtT np = g.mul_many(std::vector<ExtT>(num.begin() + lo, num.begin() + hi));
      ExtT dp = g.mul_many(std::vector<ExtT>(den.begin() + lo, den.begin() + hi));
      pp_terms.push_back(g.mul_sub(accs[k], np, g.mul(accs[k + 1], dp)));
    }
  }
  std::vector<ExtT> terms = z1_terms;
  terms.insert(terms.end(), pp_terms.begin(), pp_terms.end());
  terms.insert(terms.end(), gate_terms.begin(), gate_terms.end());
  // verify_proof_with_challenges: vanishing(zeta) == Z_H(zeta) * sum_k q_k zeta^(n k)
  for (uint32_t i = 0; i < nc; i++) {
    ExtT van = b.reduce_ext(g.ext(alphas[i]), terms);
    std::vector<ExtT> chunk(p.quotient.begin() + i * qdf, p.quotient.begin() + (i + 1) * qdf);
    ExtT rec = b.reduce_ext(zeta_n, chunk);
    g.connect(van, g.mul(zh, rec));
  }

  // ---- FRI (verify_fri_proof)
  const F g_n = gl::root_of_unity(log_n);
  ExtT zeta_next = g.scale(zeta, g_n);
  // PrecomputedReducedOpeningsTarget::from_os_and_alpha
  ExtT red0 = b.reduce_ext(fri_alpha, zbatch);
  ExtT red1 = b.reduce_ext(fri_alpha, p.zs_next);
  const size_t nb0 = zbatch.size();
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
    // fri_combine_initial: per batch reduce_base of the opened leaf values,
    // shift the running sum by alpha^(batch length), div_add
    ExtT xe = g.ext(x);
    std::vector<Target> ev0;
    for (int o = 0; o < 4; o++) ev0.insert(ev0.end(), qt.leaf[o].begin(), qt.leaf[o].end());
    if (ev0.size() != nb0) throw std::runtime_error("opened leaf widths differ from the zeta batch");
    ExtT rv0 = b.reduce_base(fri_alpha, ev0);
    ExtT sum = g.div_add(g.sub(rv0, red0), g.sub(xe, zeta), g.ext_zero());
    std::vector<Target> ev1(qt.leaf[2].begin(), qt.leaf[2].begin() + nc);
    ExtT rv1 = b.reduce_base(fri_alpha, ev1);
    sum = g.mul(b.exp_u64_ext(fri_alpha, ev1.size()), sum);
    ExtT old_eval = g.div_add(g.sub(rv1, red1), g.sub(xe, zeta_next), sum);
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
      // random_access_extension
      g.connect(ExtT{b.random_access(within_idx, e0), b.random_access(within_idx, e1)}, old_eval);
      // compute_evaluation: interpolate the bit-reversed evals over the coset
      // starting at x * g_inv^rev(within) (CosetInterpolationGate)
      const F gen = gl::root_of_unity(ab);
      const F g_inv = gl::pow(gen, (1ull << ab) - 1);
      std::vector<Target> rwithin(within.rbegin(), within.rend());
      Target start = b.mul(g.exp_from_bits_const_base(g_inv, rwithin), sx);
      std::vector<ExtT> erev(ev.size());
      for (uint32_t i = 0; i < ev.size(); i++) erev[gl::rev_bits(i, ab)] = ev[i];
      if (ab != qc::CI_BITS) throw std::runtime_error("FRI arity other than 16 is not supported");
      old_eval = b.interpolate_coset(start, erev, fri_betas[l]);
      std::vector<Target> flat;
      for (ExtT e : ev) {
        flat.push_back(e.c0);
        flat.push_back(e.c1);
      }
      verify_merkle(b, flat, coset, cap_idx, p.commit_caps[l], qt.lsib[l]);
      sx = g.exp_pow2_base(sx, ab);
      bits = coset;
    }
    // final polynomial at x (PolynomialCoeffsExtTarget::eval_scalar: reduce by x)
    ExtT fe = b.reduce_ext(g.ext(sx), p.final_poly);
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
