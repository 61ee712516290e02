// circuit.cpp — see circuit.h.  Follows upstream plonky2 (qp-plonky2 1.1.1):
//   gadgets/arithmetic.rs   arithmetic + special cases + operation dedup
//   gadgets/split_base.rs   split_le via BaseSumGate<2> (63 limbs)
//   gadgets/select.rs, gadgets/equality (is_equal + EqualityGenerator)
//   hash/hashing.rs         hash_n_to_m_no_pad (overwrite mode, PoseidonGate)
//   plonk/circuit_builder.rs build(): PI hash -> PublicInputGate, constant
//                           gates, padding to 2^k, selector_polynomials
//                           (greedy groups, max degree = qdf + 1), wire
//                           partition -> sigma polys (k_i * w^row)
//   gates/poseidon.rs       PoseidonGenerator wire layout
#include "circuit.h"
#include <algorithm>
#include <numeric>
#include <stdexcept>
#include "field.h"
#include "poseidon.h"

namespace qc {

static const F NEG_ONE = gl::P - 1;
static const uint64_t UNUSED_SELECTOR = 0xFFFFFFFFull;

static inline int gate_degree(GateKind k) {
  switch (k) {
    case G_NOOP: return 0;
    case G_CONSTANT: return 1;
    case G_PUBLIC_INPUT: return 1;
    case G_BASE_SUM: return 2;
    case G_ARITHMETIC: return 3;
    case G_POSEIDON: return 7;
    default: return 0;
  }
}

CircuitBuilder::CircuitBuilder(const CircuitConfig &cfg) : cfg_(cfg) {
  arith_ops_ = cfg.num_routed_wires / 4;
  base_sum_limbs_ = std::min<uint32_t>(63, cfg.num_routed_wires - 1);
}

Target CircuitBuilder::add_virtual_target() { return Target::virt(nvirt_++); }

std::vector<Target> CircuitBuilder::add_virtual_targets(size_t n) {
  std::vector<Target> v(n);
  for (auto &t : v) t = add_virtual_target();
  return v;
}

Target CircuitBuilder::add_virtual_public_input() {
  Target t = add_virtual_target();
  register_public_input(t);
  return t;
}

std::vector<Target> CircuitBuilder::add_virtual_hash_public_input() {
  auto v = add_virtual_hash();
  for (auto t : v) register_public_input(t);
  return v;
}

uint32_t CircuitBuilder::add_gate(GateKind k, F c0, F c1) {
  uint32_t row = (uint32_t)rows_.size();
  rows_.push_back(GateInst{k, c0, c1});
  Gen g{};
  g.row = row;
  if (k == G_CONSTANT) { g.kind = GEN_CONSTANT; gens_.push_back(g); }
  if (k == G_POSEIDON) { g.kind = GEN_POSEIDON; gens_.push_back(g); }
  if (k == G_BASE_SUM) { g.kind = GEN_BASE_SPLIT; gens_.push_back(g); }
  return row;
}

Target CircuitBuilder::constant(F c) {
  c = gl::canon(c);
  auto it = const_to_target_.find(c);
  if (it != const_to_target_.end()) return it->second;
  Target t = add_virtual_target();
  const_to_target_[c] = t;
  target_to_const_[t.v] = c;
  return t;
}

bool CircuitBuilder::as_const(Target t, F &v) const {
  auto it = target_to_const_.find(t.v);
  if (it == target_to_const_.end()) return false;
  v = it->second;
  return true;
}

void CircuitBuilder::connect(Target a, Target b) {
  if (!a.is_virtual() && a.col() >= cfg_.num_routed_wires) throw std::runtime_error("connect: unrouted wire");
  if (!b.is_virtual() && b.col() >= cfg_.num_routed_wires) throw std::runtime_error("connect: unrouted wire");
  copies_.push_back({a, b});
}

void CircuitBuilder::connect_hashes(const std::vector<Target> &a, const std::vector<Target> &b) {
  for (size_t i = 0; i < 4; i++) connect(a[i], b[i]);
}

Target CircuitBuilder::arithmetic(F c0, F c1, Target m0, Target m1, Target addend) {
  // arithmetic_special_cases
  Target z = zero();
  F m0c, m1c, ac;
  bool hm0 = as_const(m0, m0c), hm1 = as_const(m1, m1c), ha = as_const(addend, ac);
  bool first_zero = c0 == 0 || m0 == z || m1 == z;
  bool second_zero = c1 == 0 || addend == z;
  bool first_const = first_zero || (hm0 && hm1);
  F first_val = first_zero ? 0 : (first_const ? gl::mul(gl::mul(m0c, m1c), c0) : 0);
  bool second_const = second_zero || ha;
  F second_val = second_zero ? 0 : (ha ? gl::mul(ac, c1) : 0);
  if (first_const && second_const) return constant(gl::add(first_val, second_val));
  if (first_zero && c1 == 1) return addend;
  if (second_zero) {
    if (hm0 && gl::mul(m0c, c0) == 1) return m1;
    if (hm1 && gl::mul(m1c, c0) == 1) return m0;
  }
  auto key = std::make_tuple(c0, c1, m0.v, m1.v, addend.v);
  auto it = arith_cache_.find(key);
  if (it != arith_cache_.end()) return it->second;
  // find_slot for ArithmeticGate with constants (c0, c1)
  auto sk = std::make_pair(c0, c1);
  auto os = arith_open_.find(sk);
  uint32_t row, op;
  if (os == arith_open_.end() || os->second.second >= arith_ops_) {
    row = add_gate(G_ARITHMETIC, c0, c1);
    op = 0;
  } else {
    row = os->second.first;
    op = os->second.second;
  }
  arith_open_[sk] = {row, op + 1};
  connect(m0, Target::wire(row, 4 * op));
  connect(m1, Target::wire(row, 4 * op + 1));
  connect(addend, Target::wire(row, 4 * op + 2));
  Gen g{};
  g.kind = GEN_ARITH;
  g.row = row;
  g.op = op;
  gens_.push_back(g);
  Target out = Target::wire(row, 4 * op + 3);
  arith_cache_[key] = out;
  return out;
}

Target CircuitBuilder::add(Target x, Target y) { return arithmetic(1, 1, x, one(), y); }
Target CircuitBuilder::sub(Target x, Target y) { return arithmetic(1, NEG_ONE, x, one(), y); }
Target CircuitBuilder::mul(Target x, Target y) { return arithmetic(1, 0, x, y, x); }
Target CircuitBuilder::mul_add(Target x, Target y, Target z) { return arithmetic(1, 1, x, y, z); }
Target CircuitBuilder::mul_sub(Target x, Target y, Target z) { return arithmetic(1, NEG_ONE, x, y, z); }
Target CircuitBuilder::mul_const(F c, Target x) {
  Target ct = constant(c);
  return mul(ct, x);
}
Target CircuitBuilder::mul_const_add(F c, Target x, Target y) {
  Target ct = constant(c);
  return mul_add(ct, x, y);
}
Target CircuitBuilder::add_virtual_bool_target_safe() {
  Target t = add_virtual_target();
  connect(mul_sub(t, t, t), zero());
  return t;
}

// common/src/gadgets.rs:53-65: a + b - 2ab
Target xor_gadget(CircuitBuilder &b, Target a, Target c) {
  Target ab = b.mul(a, c);
  Target two_ab = b.mul_const(2, ab);
  Target a_plus_b = b.add(a, c);
  return b.sub(a_plus_b, two_ab);
}

// common/src/gadgets.rs:14-41: left < right for a constant left
Target is_const_less_than(CircuitBuilder &b, uint32_t left, Target right, uint32_t n_log) {
  auto right_bits = b.split_le(right, n_log);
  Target lt = b._false();
  Target eq = b._true();
  for (uint32_t i = n_log; i-- > 0;) {
    Target a = b.constant_bool((left >> i) & 1);
    Target bb = right_bits[i];
    Target not_a = b._not(a);
    Target not_a_and_b = b._and(not_a, bb);
    Target this_lt = b._and(not_a_and_b, eq);
    lt = b._or(lt, this_lt);
    Target a_xor_b = xor_gadget(b, a, bb);
    Target not_xor = b._not(a_xor_b);
    eq = b._and(eq, not_xor);
  }
  return lt;
}

Target CircuitBuilder::_not(Target b) {
  Target o = one();
  return sub(o, b);
}
Target CircuitBuilder::_or(Target a, Target b) {
  Target t = arithmetic(NEG_ONE, 1, a, b, a);
  return add(t, b);
}
Target CircuitBuilder::select(Target b, Target x, Target y) {
  Target tmp = mul_sub(b, y, y);
  return mul_sub(b, x, tmp);
}

Target CircuitBuilder::is_equal(Target x, Target y) {
  Target z = zero();
  Target equal = add_virtual_target();
  Target not_equal = _not(equal);
  Target inv = add_virtual_target();
  Gen g{};
  g.kind = GEN_EQUALITY;
  g.a = x; g.b = y; g.c = equal; g.d = inv;
  gens_.push_back(g);
  Target diff = sub(x, y);
  Target not_equal_check = mul(equal, diff);
  Target eq_check = mul(diff, inv);
  connect(not_equal_check, z);
  connect(eq_check, not_equal);
  return equal;
}

std::vector<Target> CircuitBuilder::split_le(Target x, uint32_t num_bits) {
  std::vector<Target> bits;
  if (num_bits == 0) {
    assert_zero(x);
    return bits;
  }
  uint32_t L = base_sum_limbs_;
  uint32_t k = (num_bits + L - 1) / L;
  std::vector<uint32_t> gates;
  for (uint32_t i = 0; i < k; i++) gates.push_back(add_gate(G_BASE_SUM));
  for (uint32_t g : gates)
    for (uint32_t l = 0; l < L; l++) bits.push_back(Target::wire(g, 1 + l));
  for (size_t i = num_bits; i < bits.size(); i++) assert_zero(bits[i]);
  bits.resize(num_bits);
  Target acc = zero();
  F base = gl::pow(2, L);
  for (size_t i = gates.size(); i-- > 0;) acc = mul_const_add(base, acc, Target::wire(gates[i], 0));
  connect(acc, x);
  if (k > 1) throw std::runtime_error("split_le: more than one BaseSum gate is not supported");
  return bits;
}

std::vector<Target> CircuitBuilder::permute(const std::vector<Target> &state) {
  uint32_t row = add_gate(G_POSEIDON);
  connect(_false(), Target::wire(row, 24));
  for (uint32_t i = 0; i < 12; i++) connect(state[i], Target::wire(row, i));
  std::vector<Target> out(12);
  for (uint32_t i = 0; i < 12; i++) out[i] = Target::wire(row, 12 + i);
  return out;
}

std::vector<Target> CircuitBuilder::hash_n_to_hash_no_pad(const std::vector<Target> &inputs) {
  Target z = zero();
  std::vector<Target> state(12, z);
  for (size_t off = 0; off < inputs.size(); off += 8) {
    for (size_t i = 0; i < 8 && off + i < inputs.size(); i++) state[i] = inputs[off + i];
    state = permute(state);
  }
  return std::vector<Target>(state.begin(), state.begin() + 4);
}

// ---------------------------------------------------------------- build

namespace {
struct UF {
  std::vector<uint32_t> p;
  explicit UF(size_t n) : p(n) { std::iota(p.begin(), p.end(), 0); }
  uint32_t find(uint32_t x) {
    while (p[x] != x) {
      p[x] = p[p[x]];
      x = p[x];
    }
    return x;
  }
  void unite(uint32_t a, uint32_t b) {
    a = find(a);
    b = find(b);
    if (a != b) p[std::max(a, b)] = std::min(a, b);
  }
};
}  // namespace

CircuitData CircuitBuilder::build() {
  // public-input hash routed to a PublicInputGate
  auto pih = hash_n_to_hash_no_pad(public_inputs_);
  uint32_t pi_row = add_gate(G_PUBLIC_INPUT);
  for (uint32_t i = 0; i < 4; i++) connect(pih[i], Target::wire(pi_row, i));
  // constant gates: cfg.num_constants constants per ConstantGate row, in
  // ascending canonical value (plonky2 build(): constants_to_targets
  // .sorted_by_key(|(c, _)| c.to_canonical_u64()) zipped with the generators)
  std::vector<std::pair<F, Target>> consts;
  for (auto &kv : const_to_target_) consts.push_back({kv.first, kv.second});
  std::sort(consts.begin(), consts.end(), [](const std::pair<F, Target> &a, const std::pair<F, Target> &b) {
    return a.first < b.first;
  });
  const uint32_t ncg = cfg_.num_constants;
  for (size_t i = 0; i < consts.size(); i += ncg) {
    F c0 = consts[i].first, c1 = i + 1 < consts.size() ? consts[i + 1].first : 0;
    uint32_t row = add_gate(G_CONSTANT, c0, c1);
    for (uint32_t j = 0; j < ncg && i + j < consts.size(); j++) connect(consts[i + j].second, Target::wire(row, j));
  }
  // pad to a power of two with NoopGate
  size_t nrows = rows_.size();
  size_t n = 1;
  while (n < nrows) n <<= 1;
  if (n < 8) n = 8;
  while (rows_.size() < n) add_gate(G_NOOP);

  CircuitData cd;
  cd.config = cfg_;
  cd.n = (uint32_t)n;
  cd.degree_bits = 0;
  while ((1u << cd.degree_bits) < n) cd.degree_bits++;
  cd.rows = rows_;
  cd.quotient_degree_factor = cfg_.max_quotient_degree_factor;
  cd.num_public_inputs = (uint32_t)public_inputs_.size();
  // gate set in common-data order (degree, id string)
  bool present[G_NKINDS] = {false};
  for (auto &r : rows_) present[r.kind] = true;
  const GateKind order[] = {G_NOOP, G_CONSTANT, G_PUBLIC_INPUT, G_BASE_SUM, G_ARITHMETIC, G_POSEIDON};
  for (GateKind k : order)
    if (present[k]) {
      cd.gate_kinds.push_back(k);
      cd.gate_params.push_back(k == G_CONSTANT ? ncg : k == G_BASE_SUM ? base_sum_limbs_ : k == G_ARITHMETIC ? arith_ops_ : 0);
    }
  const uint32_t num_gates = (uint32_t)cd.gate_kinds.size();
  uint32_t gate_index[G_NKINDS];
  for (uint32_t i = 0; i < num_gates; i++) gate_index[cd.gate_kinds[i]] = i;
  // selector_polynomials
  const uint32_t max_degree = cd.quotient_degree_factor + 1;
  const int max_gate_degree = gate_degree(cd.gate_kinds.back());
  if ((uint32_t)max_gate_degree + num_gates - 1 <= max_degree) {
    cd.groups.push_back({0, num_gates});
    cd.selector_indices.assign(num_gates, 0);
  } else {
    uint32_t start = 0;
    while (start < num_gates) {
      uint32_t size = 0;
      while (start + size < num_gates && size + gate_degree(cd.gate_kinds[start + size]) < max_degree) size++;
      if (!size) throw std::runtime_error("gate degree too high for the quotient degree factor");
      cd.groups.push_back({start, start + size});
      start += size;
    }
    for (uint32_t i = 0; i < num_gates; i++)
      for (uint32_t g = 0; g < cd.groups.size(); g++)
        if (i >= cd.groups[g].first && i < cd.groups[g].second) cd.selector_indices.push_back(g);
  }
  const uint32_t nsel = (uint32_t)cd.groups.size();
  uint32_t max_gate_consts = 0;
  for (GateKind k : cd.gate_kinds)
    max_gate_consts = std::max<uint32_t>(max_gate_consts, k == G_CONSTANT ? ncg : k == G_ARITHMETIC ? 2 : 0);
  cd.num_constants = nsel + max_gate_consts;
  // constraint count = max over gates
  cd.num_gate_constraints = 0;
  for (uint32_t i = 0; i < num_gates; i++) {
    GateKind k = cd.gate_kinds[i];
    uint32_t c = k == G_CONSTANT ? ncg : k == G_PUBLIC_INPUT ? 4 : k == G_BASE_SUM ? base_sum_limbs_ + 1
               : k == G_ARITHMETIC ? arith_ops_ : k == G_POSEIDON ? 123 : 0;
    cd.num_gate_constraints = std::max(cd.num_gate_constraints, c);
  }
  // num_partial_products: routed wires in chunks of qdf, minus one
  cd.num_partial_products = (cfg_.num_routed_wires + cd.quotient_degree_factor - 1) / cd.quotient_degree_factor - 1;
  cd.k_is.resize(cfg_.num_routed_wires);
  for (uint32_t i = 0; i < cfg_.num_routed_wires; i++) cd.k_is[i] = gl::pow(gl::GEN, i);
  {
    uint32_t db = cd.degree_bits;
    while (db > cfg_.final_poly_bits && db + cfg_.rate_bits - cfg_.arity_bits >= cfg_.cap_height) {
      cd.fri_arity_bits.push_back(cfg_.arity_bits);
      db -= cfg_.arity_bits;
    }
  }
  // ---- partition of targets
  const uint32_t W = cfg_.num_wires, R = cfg_.num_routed_wires;
  const size_t nwires = n * (size_t)W;
  auto tindex = [&](Target t) -> uint32_t { return t.is_virtual() ? (uint32_t)(nwires + (t.v & ~Target::VIRT)) : t.row() * W + t.col(); };
  UF uf(nwires + nvirt_);
  for (auto &cp : copies_) uf.unite(tindex(cp.first), tindex(cp.second));
  std::vector<uint32_t> slot_of_rep(nwires + nvirt_, 0xFFFFFFFFu);
  uint32_t nslots = 0;
  std::vector<uint32_t> slot(nwires + nvirt_);
  for (size_t i = 0; i < nwires + nvirt_; i++) {
    uint32_t r = uf.find((uint32_t)i);
    if (slot_of_rep[r] == 0xFFFFFFFFu) slot_of_rep[r] = nslots++;
    slot[i] = slot_of_rep[r];
  }
  cd.num_slots = nslots;
  cd.wire_slot.assign(slot.begin(), slot.begin() + nwires);
  for (uint32_t v = 0; v < nvirt_; v++) cd.target_slot_virtual[v] = slot[nwires + v];
  // ---- sigma polynomials: each partition's routed wires form a cycle
  {
    std::vector<std::vector<uint32_t>> members(nslots);
    for (uint32_t row = 0; row < n; row++)
      for (uint32_t col = 0; col < R; col++) members[slot[row * W + col]].push_back(row * W + col);
    const uint64_t w = gl::root_of_unity(cd.degree_bits);
    std::vector<F> wpow(n);
    wpow[0] = 1;
    for (uint32_t i = 1; i < n; i++) wpow[i] = gl::mul(wpow[i - 1], w);
    cd.constants_sigmas.assign((size_t)(cd.num_constants + R) * n, 0);
    F *sig = cd.constants_sigmas.data() + (size_t)cd.num_constants * n;
    for (auto &m : members) {
      for (size_t i = 0; i < m.size(); i++) {
        uint32_t src = m[i], dst = m[(i + 1) % m.size()];
        uint32_t srow = src / W, scol = src % W, drow = dst / W, dcol = dst % W;
        sig[(size_t)scol * n + srow] = gl::mul(cd.k_is[dcol], wpow[drow]);
      }
    }
    // selectors + gate constants
    for (uint32_t row = 0; row < n; row++) {
      const GateInst &gi = rows_[row];
      uint32_t gidx = gate_index[gi.kind];
      uint32_t grp = cd.selector_indices[gidx];
      for (uint32_t s = 0; s < nsel; s++)
        cd.constants_sigmas[(size_t)s * n + row] = s == grp ? (F)gidx : (nsel > 1 ? UNUSED_SELECTOR : (F)gidx);
      if (max_gate_consts >= 1) cd.constants_sigmas[(size_t)nsel * n + row] = gi.c0;
      if (max_gate_consts >= 2) cd.constants_sigmas[(size_t)(nsel + 1) * n + row] = gi.c1;
    }
  }
  // ---- generator schedule (worklist over partition slots)
  {
    auto sl = [&](Target t) { return slot[tindex(t)]; };
    auto wsl = [&](uint32_t row, uint32_t col) { return slot[row * W + col]; };
    std::vector<std::vector<uint32_t>> gin(gens_.size()), gout(gens_.size());
    for (size_t gi = 0; gi < gens_.size(); gi++) {
      const Gen &g = gens_[gi];
      switch (g.kind) {
        case GEN_CONSTANT:
          for (uint32_t j = 0; j < ncg; j++) gout[gi].push_back(wsl(g.row, j));
          break;
        case GEN_ARITH:
          for (uint32_t j = 0; j < 3; j++) gin[gi].push_back(wsl(g.row, 4 * g.op + j));
          gout[gi].push_back(wsl(g.row, 4 * g.op + 3));
          break;
        case GEN_POSEIDON:
          for (uint32_t j = 0; j < 12; j++) gin[gi].push_back(wsl(g.row, j));
          gin[gi].push_back(wsl(g.row, 24));
          for (uint32_t j = 12; j < W; j++)
            if (j != 24) gout[gi].push_back(wsl(g.row, j));
          break;
        case GEN_BASE_SPLIT:
          gin[gi].push_back(wsl(g.row, 0));
          for (uint32_t j = 1; j <= base_sum_limbs_; j++) gout[gi].push_back(wsl(g.row, j));
          break;
        case GEN_EQUALITY:
          gin[gi].push_back(sl(g.a));
          gin[gi].push_back(sl(g.b));
          gout[gi].push_back(sl(g.c));
          gout[gi].push_back(sl(g.d));
          break;
      }
      std::sort(gin[gi].begin(), gin[gi].end());
      gin[gi].erase(std::unique(gin[gi].begin(), gin[gi].end()), gin[gi].end());
    }
    std::vector<std::vector<uint32_t>> watchers(nslots);
    std::vector<uint32_t> remaining(gens_.size());
    for (size_t gi = 0; gi < gens_.size(); gi++) {
      remaining[gi] = (uint32_t)gin[gi].size();
      for (uint32_t s : gin[gi]) watchers[s].push_back((uint32_t)gi);
    }
    std::vector<uint8_t> known(nslots, 0);
    std::vector<uint32_t> queue;
    auto mark = [&](uint32_t s) {
      if (!known[s]) {
        known[s] = 1;
        queue.push_back(s);
      }
    };
    for (Target t : inputs_) mark(sl(t));
    std::vector<uint32_t> ready;
    for (size_t gi = 0; gi < gens_.size(); gi++)
      if (!remaining[gi]) ready.push_back((uint32_t)gi);
    size_t qh = 0;
    while (true) {
      while (!ready.empty()) {
        uint32_t gi = ready.back();
        ready.pop_back();
        cd.schedule.push_back(gens_[gi]);
        for (uint32_t s : gout[gi]) mark(s);
      }
      if (qh == queue.size()) break;
      uint32_t s = queue[qh++];
      for (uint32_t gi : watchers[s])
        if (--remaining[gi] == 0) ready.push_back(gi);
    }
    if (cd.schedule.size() != gens_.size())
      throw std::runtime_error("witness generation cannot be scheduled: " +
                               std::to_string(gens_.size() - cd.schedule.size()) + " generators never become ready");
    for (Target t : public_inputs_) cd.pi_slots.push_back(sl(t));
  }
  return cd;
}

uint32_t CircuitData::slot_of(Target t) const {
  if (t.is_virtual()) {
    auto it = target_slot_virtual.find(t.v & ~Target::VIRT);
    return it == target_slot_virtual.end() ? 0xFFFFFFFFu : it->second;
  }
  return wire_slot[(size_t)t.row() * config.num_wires + t.col()];
}

// ---------------------------------------------------------------- serialization

namespace {
struct ByteWriter {
  std::vector<uint8_t> b;
  void u64(uint64_t v) {
    for (int i = 0; i < 8; i++) b.push_back((uint8_t)(v >> (8 * i)));
  }
  void u32(uint32_t v) {
    for (int i = 0; i < 4; i++) b.push_back((uint8_t)(v >> (8 * i)));
  }
  void u8(uint8_t v) { b.push_back(v); }
};
void write_fri_config(ByteWriter &w, const CircuitConfig &c) {
  w.u64(c.rate_bits);
  w.u64(c.cap_height);
  w.u64(c.num_query_rounds);
  w.u32(c.pow_bits);
  w.u8(1);  // FriReductionStrategy::ConstantArityBits
  w.u64(c.arity_bits);
  w.u64(c.final_poly_bits);
}
}  // namespace

std::vector<uint8_t> CircuitData::common_bytes() const {
  ByteWriter w;
  const CircuitConfig &c = config;
  w.u64(c.num_wires);
  w.u64(c.num_routed_wires);
  w.u64(c.num_constants);
  w.u64(c.security_bits);
  w.u64(c.num_challenges);
  w.u64(c.max_quotient_degree_factor);
  w.u8(c.use_base_arithmetic_gate);
  w.u8(c.zero_knowledge);
  write_fri_config(w, c);
  write_fri_config(w, c);
  w.u64(fri_arity_bits.size());
  for (auto a : fri_arity_bits) w.u64(a);
  w.u64(degree_bits);
  w.u8(c.zero_knowledge);  // FriParams.hiding
  w.u64(selector_indices.size());
  for (auto s : selector_indices) w.u64(s);
  w.u64(groups.size());
  for (auto &g : groups) {
    w.u64(g.first);
    w.u64(g.second);
  }
  w.u64(quotient_degree_factor);
  w.u64(num_gate_constraints);
  w.u64(num_constants);
  w.u64(num_public_inputs);
  w.u64(k_is.size());
  for (auto k : k_is) w.u64(k);
  w.u64(num_partial_products);
  w.u64(0);  // num_lookup_polys
  w.u64(0);  // num_lookup_selectors
  w.u64(0);  // luts
  w.u64(gate_kinds.size());
  for (size_t i = 0; i < gate_kinds.size(); i++) {
    w.u32(gate_serial_id(gate_kinds[i]));
    GateKind k = gate_kinds[i];
    if (k == G_CONSTANT || k == G_BASE_SUM || k == G_ARITHMETIC) w.u64(gate_params[i]);
  }
  return w.b;
}

// ---------------------------------------------------------------- witness

Witness::Witness(const CircuitData &cd) : cd_(cd), val_(cd.num_slots, 0), known_(cd.num_slots, 0) {}

bool Witness::set_slot(uint32_t s, F v) {
  v = gl::canon(v);
  if (known_[s]) {
    if (val_[s] != v) {
      conflict_ = true;
      return false;
    }
    return true;
  }
  known_[s] = 1;
  val_[s] = v;
  return true;
}

bool Witness::set(Target t, F v) {
  uint32_t s = cd_.slot_of(t);
  if (s == 0xFFFFFFFFu) return false;
  return set_slot(s, v);
}

bool Witness::set_wire(uint32_t row, uint32_t col, F v) {
  return set_slot(cd_.wire_slot[(size_t)row * cd_.config.num_wires + col], v);
}

F Witness::wire(uint32_t row, uint32_t col) const {
  return val_[cd_.wire_slot[(size_t)row * cd_.config.num_wires + col]];
}

bool Witness::generate(std::string &err) {
  const uint32_t ncg = cd_.config.num_constants;
  for (const Gen &g : cd_.schedule) {
    bool ok = true;
    switch (g.kind) {
      case GEN_CONSTANT: {
        const GateInst &gi = cd_.rows[g.row];
        ok = set_wire(g.row, 0, gi.c0) && (ncg < 2 || set_wire(g.row, 1, gi.c1));
        break;
      }
      case GEN_ARITH: {
        const GateInst &gi = cd_.rows[g.row];
        F m0 = wire(g.row, 4 * g.op), m1 = wire(g.row, 4 * g.op + 1), a = wire(g.row, 4 * g.op + 2);
        ok = set_wire(g.row, 4 * g.op + 3, gl::add(gl::mul(gl::mul(m0, m1), gi.c0), gl::mul(a, gi.c1)));
        break;
      }
      case GEN_BASE_SPLIT: {
        F sum = wire(g.row, 0);
        const uint32_t L = cd_.config.num_routed_wires - 1 < 63 ? cd_.config.num_routed_wires - 1 : 63;
        for (uint32_t l = 0; l < L && ok; l++) ok = set_wire(g.row, 1 + l, (sum >> l) & 1);
        break;
      }
      case GEN_EQUALITY: {
        F x = val_[cd_.slot_of(g.a)], y = val_[cd_.slot_of(g.b)];
        ok = set(g.c, x == y ? 1 : 0) && set(g.d, x == y ? 0 : gl::inv(gl::sub(x, y)));
        break;
      }
      case GEN_POSEIDON: {
        F s[12];
        for (int i = 0; i < 12; i++) s[i] = wire(g.row, i);
        F swap = wire(g.row, 24);
        for (int i = 0; i < 4 && ok; i++) ok = set_wire(g.row, 25 + i, gl::mul(swap, gl::sub(s[i + 4], s[i])));
        if (swap == 1)
          for (int i = 0; i < 4; i++) std::swap(s[i], s[i + 4]);
        int rc = 0;
        for (int r = 0; r < 4; r++, rc++) {
          for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
          if (r)
            for (int i = 0; i < 12 && ok; i++) ok = set_wire(g.row, 29 + (r - 1) * 12 + i, s[i]);
          for (int i = 0; i < 12; i++) s[i] = ps::sbox(s[i]);
          ps::mds(s);
        }
        for (int r = 0; r < 22; r++, rc++) {
          for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
          if (ok) ok = set_wire(g.row, 65 + r, s[0]);
          s[0] = ps::sbox(s[0]);
          ps::mds(s);
        }
        for (int r = 0; r < 4; r++, rc++) {
          for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
          for (int i = 0; i < 12 && ok; i++) ok = set_wire(g.row, 87 + r * 12 + i, s[i]);
          for (int i = 0; i < 12; i++) s[i] = ps::sbox(s[i]);
          ps::mds(s);
        }
        for (int i = 0; i < 12 && ok; i++) ok = set_wire(g.row, 12 + i, s[i]);
        break;
      }
    }
    if (!ok) {
      err = "Partition containing a target was set twice with different values (generator kind " +
            std::to_string(g.kind) + " at row " + std::to_string(g.row) + ")";
      return false;
    }
  }
  return true;
}

void Witness::wires_matrix(F *out) const {
  const uint32_t n = cd_.n, W = cd_.config.num_wires;
  for (uint32_t row = 0; row < n; row++) {
    const uint32_t *ws = cd_.wire_slot.data() + (size_t)row * W;
    for (uint32_t col = 0; col < W; col++) {
      uint32_t s = ws[col];
      out[(size_t)col * n + row] = known_[s] ? val_[s] : 0;
    }
  }
}

std::vector<F> Witness::public_inputs() const {
  std::vector<F> v;
  for (uint32_t s : cd_.pi_slots) v.push_back(val_[s]);
  return v;
}

}  // namespace qc
