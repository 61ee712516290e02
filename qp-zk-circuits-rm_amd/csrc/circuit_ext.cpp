// circuit_ext.cpp — the recursion gates on the native builder (see circuit.h):
// extension arithmetic (gadgets/arithmetic_extension.rs arithmetic_extension
// + special cases + operation dedup, find_slot over ArithmeticExtensionGate /
// MulExtensionGate ops), division through an inverse generator, PoseidonMdsGate
// rows, ReducingFactorTarget over ReducingGate / ReducingExtensionGate rows
// (gadgets/reducing.rs) and CosetInterpolationGate rows
// (gadgets/interpolation.rs), with their witness generators' wire sets.
// Restated from upstream plonky2 (qp-plonky2 1.1.1); parity unpinned: the
// reference commits no circuit with these gates.
#include <stdexcept>
#include "circuit.h"
#include "field.h"

namespace qc {

// ---- wire layouts (gates/*.rs), shared by the builder, the generators and
// the level schedule
namespace {
constexpr uint32_t ae_m0(uint32_t i) { return 8 * i; }
constexpr uint32_t ae_m1(uint32_t i) { return 8 * i + 2; }
constexpr uint32_t ae_add(uint32_t i) { return 8 * i + 4; }
constexpr uint32_t ae_out(uint32_t i) { return 8 * i + 6; }
constexpr uint32_t me_m0(uint32_t i) { return 6 * i; }
constexpr uint32_t me_m1(uint32_t i) { return 6 * i + 2; }
constexpr uint32_t me_out(uint32_t i) { return 6 * i + 4; }
// Reducing(Extension)Gate: output 0..2, alpha 2..4, old_acc 4..6, coefficients
// from 6 (cw wires each), accumulators (2 each, the last one is the output)
constexpr uint32_t RD_OUT = 0, RD_ALPHA = 2, RD_OLD = 4, RD_COEFFS = 6;
inline uint32_t rd_acc(uint32_t nc, uint32_t cw, uint32_t i) { return i + 1 == nc ? RD_OUT : RD_COEFFS + cw * nc + 2 * i; }
ExtT wext(uint32_t row, uint32_t col) { return {Target::wire(row, col), Target::wire(row, col + 1)}; }
}  // namespace

void gen_row_wires(GenKind k, uint32_t row, uint32_t op, std::vector<std::pair<uint32_t, uint32_t>> &rd,
                   std::vector<std::pair<uint32_t, uint32_t>> &wr) {
  auto r2 = [&](uint32_t c) { rd.push_back({row, c}); rd.push_back({row, c + 1}); };
  auto w2 = [&](uint32_t c) { wr.push_back({row, c}); wr.push_back({row, c + 1}); };
  switch (k) {
    case GEN_ARITH_EXT:
      r2(ae_m0(op)); r2(ae_m1(op)); r2(ae_add(op)); w2(ae_out(op));
      break;
    case GEN_MUL_EXT:
      r2(me_m0(op)); r2(me_m1(op)); w2(me_out(op));
      break;
    case GEN_REDUCING:
    case GEN_REDUCING_EXT: {
      const uint32_t nc = k == GEN_REDUCING ? RED_COEFFS : REDE_COEFFS, cw = k == GEN_REDUCING ? 1 : 2;
      r2(RD_ALPHA); r2(RD_OLD);
      for (uint32_t i = 0; i < nc * cw; i++) rd.push_back({row, RD_COEFFS + i});
      for (uint32_t i = 0; i < nc; i++) w2(rd_acc(nc, cw, i));
      break;
    }
    case GEN_POSEIDON_MDS:
      for (uint32_t i = 0; i < 24; i++) rd.push_back({row, i});
      for (uint32_t i = 24; i < 48; i++) wr.push_back({row, i});
      break;
    case GEN_COSET_INTERP:
      rd.push_back({row, 0});
      for (uint32_t i = 0; i < 2 * CI_POINTS; i++) rd.push_back({row, CI_VALUES + i});
      r2(CI_EVAL_POINT);
      w2(CI_EVAL_VALUE);
      for (uint32_t i = 0; i < 4 * CI_NINT; i++) wr.push_back({row, CI_INTER + i});
      w2(CI_SHIFTED);
      break;
    default:
      break;
  }
}

// ---- builder

ExtT CircuitBuilder::arithmetic_extension(F c0, F c1, ExtT m0, ExtT m1, ExtT addend) {
  c0 = gl::canon(c0);
  c1 = gl::canon(c1);
  // arithmetic_extension_special_cases (values in F_p2: (a0 + a1 X)(b0 + b1 X))
  const ExtT z = zero_ext();
  F m00, m01, m10, m11, a0, a1;
  const bool hm0 = as_const_ext(m0, m00, m01), hm1 = as_const_ext(m1, m10, m11), ha = as_const_ext(addend, a0, a1);
  const bool first_zero = c0 == 0 || m0 == z || m1 == z;
  const bool second_zero = c1 == 0 || addend == z;
  const gl::ext cc0{c0, 0};
  if ((first_zero || (hm0 && hm1)) && (second_zero || ha)) {
    gl::ext f{0, 0}, sd{0, 0};
    if (!first_zero) f = gl::ext_mul(gl::ext_mul(gl::ext{m00, m01}, gl::ext{m10, m11}), cc0);
    if (!second_zero) sd = gl::ext_scale(gl::ext{a0, a1}, c1);
    const gl::ext r = gl::ext_add(f, sd);
    return constant_ext(r.c0, r.c1);
  }
  if (first_zero && c1 == 1) return addend;
  if (second_zero) {
    if (hm0) {
      const gl::ext x = gl::ext_scale(gl::ext{m00, m01}, c0);
      if (x.c0 == 1 && x.c1 == 0) return m1;
    }
    if (hm1) {
      const gl::ext x = gl::ext_scale(gl::ext{m10, m11}, c0);
      if (x.c0 == 1 && x.c1 == 0) return m0;
    }
  }
  // the same operation computed before
  const auto key = std::make_tuple(c0, c1, m0.c0.v, m0.c1.v, m1.c0.v, m1.c1.v, addend.c0.v, addend.c1.v);
  auto it = ext_cache_.find(key);
  if (it != ext_cache_.end()) return it->second;
  ExtT out;
  Gen g{};
  g.k0 = c0;
  g.k1 = c1;
  if (addend == z) {
    // compute_mul_extension_operation: MulExtensionGate op keyed by const_0
    auto os = me_open_.find(c0);
    uint32_t row, op;
    if (os == me_open_.end() || os->second.second >= ME_OPS) {
      row = add_gate(G_MUL_EXT, c0, 0);
      op = 0;
    } else {
      row = os->second.first;
      op = os->second.second;
    }
    me_open_[c0] = {row, op + 1};
    connect_ext(m0, wext(row, me_m0(op)));
    connect_ext(m1, wext(row, me_m1(op)));
    out = wext(row, me_out(op));
    g.kind = GEN_MUL_EXT;
    g.row = row;
    g.op = op;
  } else {
    auto sk = std::make_pair(c0, c1);
    auto os = ae_open_.find(sk);
    uint32_t row, op;
    if (os == ae_open_.end() || os->second.second >= AE_OPS) {
      row = add_gate(G_ARITH_EXT, c0, c1);
      op = 0;
    } else {
      row = os->second.first;
      op = os->second.second;
    }
    ae_open_[sk] = {row, op + 1};
    connect_ext(m0, wext(row, ae_m0(op)));
    connect_ext(m1, wext(row, ae_m1(op)));
    connect_ext(addend, wext(row, ae_add(op)));
    out = wext(row, ae_out(op));
    g.kind = GEN_ARITH_EXT;
    g.row = row;
    g.op = op;
  }
  gens_.push_back(g);
  ext_cache_[key] = out;
  return out;
}

ExtT CircuitBuilder::mul_many_ext(const std::vector<ExtT> &v) {
  if (v.empty()) return one_ext();
  ExtT acc = v[0];
  for (size_t i = 1; i < v.size(); i++) acc = mul_ext(acc, v[i]);
  return acc;
}

ExtT CircuitBuilder::div_add_ext(ExtT x, ExtT y, ExtT z) {
  // div_add_extension: inv from QuotientGeneratorExtension(1 / y), y * inv == 1
  ExtT inv = add_virtual_ext();
  ExtT one = one_ext();
  Gen g{};
  g.kind = GEN_EXT_DIV;
  g.a = one.c0;
  g.b = one.c1;
  g.c = y.c0;
  g.d = y.c1;
  g.e = inv.c0;
  g.f = inv.c1;
  gens_.push_back(g);
  connect_ext(mul_ext(y, inv), one);
  return mul_add_ext(x, inv, z);
}

ExtT CircuitBuilder::exp_u64_ext(ExtT base, uint64_t e) {
  // exp_u64_extension: square and multiply, low bit first
  if (e == 0) return one_ext();
  if (e == 1) return base;
  if (e == 2) return square_ext(base);
  ExtT cur = base, prod = one_ext();
  for (uint32_t j = 0; (e >> j) != 0; j++) {
    if (j) cur = square_ext(cur);
    if ((e >> j) & 1) prod = mul_ext(prod, cur);
  }
  return prod;
}

ExtT CircuitBuilder::exp_power_of_2_ext(ExtT base, uint32_t k) {
  for (uint32_t i = 0; i < k; i++) base = square_ext(base);
  return base;
}

std::vector<ExtT> CircuitBuilder::poseidon_mds(const std::vector<ExtT> &s) {
  const uint32_t row = add_gate(G_POSEIDON_MDS);
  for (uint32_t i = 0; i < 12; i++) connect_ext(s[i], wext(row, 2 * i));
  Gen g{};
  g.kind = GEN_POSEIDON_MDS;
  g.row = row;
  gens_.push_back(g);
  std::vector<ExtT> out(12);
  for (uint32_t i = 0; i < 12; i++) out[i] = wext(row, 24 + 2 * i);
  return out;
}

ExtT CircuitBuilder::reduce_arithmetic(ExtT alpha, const std::vector<ExtT> &t) {
  // ReducingFactorTarget::reduce_arithmetic: Horner from the last term
  ExtT acc = zero_ext();
  for (size_t i = t.size(); i-- > 0;) acc = mul_add_ext(alpha, acc, t[i]);
  return acc;
}

ExtT CircuitBuilder::reduce_base(ExtT alpha, const std::vector<Target> &t) {
  if (t.size() <= AE_OPS + 1) {
    std::vector<ExtT> e;
    for (Target x : t) e.push_back(convert_to_ext(x));
    return reduce_arithmetic(alpha, e);
  }
  std::vector<Target> rev(t.rbegin(), t.rend());
  // pad to whole gates at the high end: the zeros go first after reversal
  std::vector<Target> padded(((t.size() + RED_COEFFS - 1) / RED_COEFFS) * RED_COEFFS - t.size(), zero());
  padded.insert(padded.end(), rev.begin(), rev.end());
  ExtT acc = zero_ext();
  for (size_t off = 0; off < padded.size(); off += RED_COEFFS) {
    const uint32_t row = add_gate(G_REDUCING);
    connect_ext(alpha, wext(row, RD_ALPHA));
    connect_ext(acc, wext(row, RD_OLD));
    for (uint32_t i = 0; i < RED_COEFFS; i++) connect(padded[off + i], Target::wire(row, RD_COEFFS + i));
    Gen g{};
    g.kind = GEN_REDUCING;
    g.row = row;
    gens_.push_back(g);
    acc = wext(row, RD_OUT);
  }
  return acc;
}

ExtT CircuitBuilder::reduce_ext(ExtT alpha, const std::vector<ExtT> &t) {
  if (t.size() <= AE_OPS + 1) return reduce_arithmetic(alpha, t);
  std::vector<ExtT> rev(t.rbegin(), t.rend());
  std::vector<ExtT> padded(((t.size() + REDE_COEFFS - 1) / REDE_COEFFS) * REDE_COEFFS - t.size(), zero_ext());
  padded.insert(padded.end(), rev.begin(), rev.end());
  ExtT acc = zero_ext();
  for (size_t off = 0; off < padded.size(); off += REDE_COEFFS) {
    const uint32_t row = add_gate(G_REDUCING_EXT);
    connect_ext(alpha, wext(row, RD_ALPHA));
    connect_ext(acc, wext(row, RD_OLD));
    for (uint32_t i = 0; i < REDE_COEFFS; i++) connect_ext(padded[off + i], wext(row, RD_COEFFS + 2 * i));
    Gen g{};
    g.kind = GEN_REDUCING_EXT;
    g.row = row;
    gens_.push_back(g);
    acc = wext(row, RD_OUT);
  }
  return acc;
}

ExtT CircuitBuilder::interpolate_coset(Target shift, const std::vector<ExtT> &values, ExtT point) {
  if (values.size() != CI_POINTS) throw std::runtime_error("interpolate_coset: 16 values");
  const uint32_t row = add_gate(G_COSET_INTERP);
  connect(shift, Target::wire(row, 0));
  for (uint32_t i = 0; i < CI_POINTS; i++) connect_ext(values[i], wext(row, CI_VALUES + 2 * i));
  connect_ext(point, wext(row, CI_EVAL_POINT));
  Gen g{};
  g.kind = GEN_COSET_INTERP;
  g.row = row;
  gens_.push_back(g);
  return wext(row, CI_EVAL_VALUE);
}

}  // namespace qc
