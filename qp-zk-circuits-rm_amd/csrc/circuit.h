// circuit.h — native Plonky2-compatible circuit builder, preprocessing and
// witness generation (host side of the prover).
//
// Replaces qp-plonky2 1.1.1 plonk/circuit_builder.rs (CircuitBuilder::build,
// SURVEY.md a0/a1), iop/generator.rs (generate_partial_witness, a3) and the
// gadgets the reference circuits use (arithmetic.rs, split_base.rs,
// hash/hashing.rs hash_n_to_m_no_pad, select, is_equal).  Gate set: Noop,
// Constant, PublicInput, BaseSum<2>, Arithmetic, Poseidon — exactly the
// Wormhole circuit's ([FIX] common.bin).
//
// Witness generation is schedule-driven: build() resolves the generator
// dependency order once (generators are structural, values are not), so a
// proof's witness is one linear pass over the schedule — cheap enough to run
// 256 proofs per batch on the host threads.
#pragma once
#include <stdint.h>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace qc {

using F = uint64_t;

struct Target {
  uint32_t v = 0xFFFFFFFFu;
  static constexpr uint32_t VIRT = 0x80000000u;
  static Target wire(uint32_t row, uint32_t col) { return Target{(row << 8) | col}; }
  static Target virt(uint32_t idx) { return Target{VIRT | idx}; }
  bool is_virtual() const { return v & VIRT; }
  uint32_t row() const { return v >> 8; }
  uint32_t col() const { return v & 0xFF; }
  bool operator==(const Target &o) const { return v == o.v; }
  bool operator!=(const Target &o) const { return v != o.v; }
  bool operator<(const Target &o) const { return v < o.v; }
};

enum GateKind : uint8_t {
  G_NOOP = 0, G_CONSTANT, G_PUBLIC_INPUT, G_BASE_SUM, G_ARITHMETIC, G_POSEIDON,
  // the recursive verifier's gates (plonky2 verify_proof; aggregation circuits)
  G_RANDOM_ACCESS,   // RandomAccessGate{bits 4, copies 4, extra constants 2}
  G_ARITH_EXT,       // ArithmeticExtensionGate{num_ops 10}: out = c0 m0 m1 + c1 addend (ext)
  G_MUL_EXT,         // MulExtensionGate{num_ops 13}: out = c0 m0 m1 (ext)
  G_REDUCING,        // ReducingGate{num_coeffs 43}: Horner of base coefficients by an ext alpha
  G_REDUCING_EXT,    // ReducingExtensionGate{num_coeffs 32}: the same over ext coefficients
  G_POSEIDON_MDS,    // PoseidonMdsGate: the 12x12 MDS layer on ext values
  G_COSET_INTERP,    // CosetInterpolationGate{subgroup_bits 4, degree 6}
  G_NKINDS
};

// extension-field target (a, b) = a + b X, X^2 = 7 (plonky2 ExtensionTarget<2>)
struct ExtT {
  Target c0, c1;
  bool operator==(const ExtT &o) const { return c0 == o.c0 && c1 == o.c1; }
};

// new_from_config shapes of the standard config (80 routed of 135 wires, D = 2)
constexpr uint32_t AE_OPS = 10;       // ArithmeticExtensionGate: routed / (4 D)
constexpr uint32_t ME_OPS = 13;       // MulExtensionGate: routed / (3 D)
constexpr uint32_t RED_COEFFS = 43;   // ReducingGate::max_coeffs_len: min(routed - 3D, (wires - 2D) / (D + 1))
constexpr uint32_t REDE_COEFFS = 32;  // ReducingExtensionGate::max_coeffs_len: min((routed - 3D) / D, (wires - 2D) / 2D)
// CosetInterpolationGate::with_max_degree(4, 8): degree (14 / 3) + 2 = 6, 2 intermediates;
// wires: shift 0, values 1.., evaluation point, evaluation value, intermediate
// evals, intermediate products, shifted evaluation point
constexpr uint32_t CI_BITS = 4, CI_POINTS = 16, CI_DEGREE = 6, CI_NINT = (CI_POINTS - 2) / (CI_DEGREE - 1);
constexpr uint32_t CI_VALUES = 1, CI_EVAL_POINT = CI_VALUES + 2 * CI_POINTS, CI_EVAL_VALUE = CI_EVAL_POINT + 2,
                   CI_INTER = CI_EVAL_VALUE + 2, CI_SHIFTED = CI_INTER + 4 * CI_NINT;

// RandomAccessGate::new_from_config(standard config, bits = 4) (gates/random_access.rs):
// per copy c: access index at 18c, claimed element at 18c + 1, list items at
// 18c + 2 + i; extra-constant wires 72..73; bit i of copy c at 74 + 4c + i
constexpr uint32_t RA_BITS = 4, RA_VEC = 1u << RA_BITS, RA_COPIES = 4, RA_EXTRA = 2;
constexpr uint32_t ra_wire_index(uint32_t c) { return (2 + RA_VEC) * c; }
constexpr uint32_t ra_wire_claimed(uint32_t c) { return (2 + RA_VEC) * c + 1; }
constexpr uint32_t ra_wire_item(uint32_t i, uint32_t c) { return (2 + RA_VEC) * c + 2 + i; }
constexpr uint32_t ra_wire_bit(uint32_t i, uint32_t c) { return (2 + RA_VEC) * RA_COPIES + RA_EXTRA + RA_BITS * c + i; }

// plonky2 DefaultGateSerializer ids
inline uint32_t gate_serial_id(GateKind k) {
  switch (k) {
    case G_NOOP: return 9;
    case G_CONSTANT: return 3;
    case G_PUBLIC_INPUT: return 12;
    case G_BASE_SUM: return 2;
    case G_ARITHMETIC: return 0;
    case G_POSEIDON: return 11;
    case G_RANDOM_ACCESS: return 13;
    case G_ARITH_EXT: return 1;
    case G_MUL_EXT: return 8;
    case G_REDUCING: return 15;
    case G_REDUCING_EXT: return 14;
    case G_POSEIDON_MDS: return 10;
    case G_COSET_INTERP: return 4;
    default: return 0xFFFFFFFF;
  }
}

struct CircuitConfig {
  uint32_t num_wires = 135, num_routed_wires = 80, num_constants = 2;
  bool use_base_arithmetic_gate = true;
  uint32_t security_bits = 100, num_challenges = 2;
  bool zero_knowledge = false;
  uint32_t max_quotient_degree_factor = 8;
  uint32_t rate_bits = 3, cap_height = 4, pow_bits = 16, num_query_rounds = 28;
  uint32_t arity_bits = 4, final_poly_bits = 5;  // ConstantArityBits(4, 5)
  static CircuitConfig standard_recursion_config() { return CircuitConfig(); }
  static CircuitConfig standard_recursion_zk_config() {
    CircuitConfig c;
    c.zero_knowledge = true;
    return c;
  }
};

struct GateInst {
  GateKind kind;
  F c0 = 0, c1 = 0;
};

// generator record: run by witness generation in schedule order (host) or
// level by level (device, witness.hip); the last three are the recursive
// verifier's (aggregation circuits)
enum GenKind : uint8_t {
  GEN_CONSTANT = 0, GEN_ARITH, GEN_POSEIDON, GEN_BASE_SPLIT, GEN_EQUALITY,
  GEN_WIRE_SPLIT,     // WireSplitGenerator: integer -> the sums of `op` consecutive BaseSum gates from `row`
  GEN_EXT_DIV,        // QuotientGeneratorExtension: (e, f) = (a + bX) / (c + dX)
  GEN_RANDOM_ACCESS,  // RandomAccessGenerator of copy `op` of the RandomAccessGate at `row`
  GEN_ARITH_EXT,      // ArithmeticExtensionGenerator of op `op` at `row` (constants k0, k1)
  GEN_MUL_EXT,        // MulExtensionGenerator of op `op` at `row` (constant k0)
  GEN_REDUCING,       // ReducingGenerator of the ReducingGate at `row`
  GEN_REDUCING_EXT,   // ReducingExtensionGenerator of the ReducingExtensionGate at `row`
  GEN_POSEIDON_MDS,   // PoseidonMdsGenerator of the gate at `row`
  GEN_COSET_INTERP,   // InterpolationGenerator of the CosetInterpolationGate at `row`
};
// (row, column) wires a row generator reads and writes (schedule + device levels)
void gen_row_wires(GenKind k, uint32_t row, uint32_t op, std::vector<std::pair<uint32_t, uint32_t>> &rd,
                   std::vector<std::pair<uint32_t, uint32_t>> &wr);
struct Gen {
  GenKind kind;
  uint32_t row = 0, op = 0;             // gate row / arithmetic op index
  Target a, b, c, d, e, f;              // EQUALITY: x, y, equal, inv; EXT_DIV: num, den, quotient
  // resolved at build(): value slots the generator reads/writes
  //   ARITH: m0, m1, addend, output   EQUALITY: x, y, equal, inv
  //   CONSTANT: wire 0, wire 1         BASE_SPLIT: sum
  uint32_t s[6] = {0, 0, 0, 0, 0, 0};
  F k0 = 0, k1 = 0;                     // ARITH / CONSTANT gate constants
};

// Device witness generation (plonky2 iop/generator.rs generate_partial_witness
// on the GPU): one record per generator, grouped into dependency levels so a
// workgroup can run one proof's generators level by level (same layout as the
// device struct in witness.hip).  Kind-specific packing: WIRE_SPLIT s[1] = gate
// count; EXT_DIV k0 = the two quotient slots (lo | hi << 32); RANDOM_ACCESS
// s[0] = copy.  Slot fields carry DEV_MULTI (below).
// slot ids in DevGen and CircuitData::dev_wslot carry DEV_MULTI when the slot
// has more than one writer (or is the shared zero slot)
constexpr uint32_t DEV_MULTI = 0x80000000u;
// device witness: Poseidon chains over inputs alone at least this many
// permutations deep run on the host (CircuitData::host_gens; the environment
// variable QPGPU_HOST_CHAIN overrides, 0 = none)
constexpr uint32_t HOST_CHAIN_MIN = 64;
struct DevGen {
  uint32_t kind, row;
  uint32_t s[4];
  uint64_t k0, k1;
};
static_assert(sizeof(DevGen) == 40, "DevGen layout");

// everything the prover needs about a built circuit (plonky2 ProverCircuitData
// + CommonCircuitData), kept in host memory
struct CircuitData {
  CircuitConfig config;
  uint32_t degree_bits = 0, n = 0;
  uint32_t num_constants = 0;           // selectors + gate constants
  uint32_t num_gate_constraints = 0, quotient_degree_factor = 0, num_partial_products = 0;
  uint32_t num_public_inputs = 0;
  std::vector<GateKind> gate_kinds;     // common-data gate order
  std::vector<uint32_t> gate_params;    // parameter per gate kind (num_ops / num_limbs / num_consts / RA bits)
  std::vector<uint32_t> gate_params2, gate_params3;  // RandomAccess copies, extra constants
  std::vector<uint32_t> selector_indices;
  std::vector<std::pair<uint32_t, uint32_t>> groups;
  std::vector<F> k_is;
  std::vector<uint32_t> fri_arity_bits;
  // preprocessed polynomials, column-major values over H (natural row order)
  std::vector<F> constants_sigmas;      // [num_constants + num_routed][n]
  std::vector<GateInst> rows;
  // witness layout: one value slot per copy-constraint partition that some
  // generator or input sets; slot 0 is the shared never-set (zero) slot of
  // every other wire (padding rows, unused gate slots, unrouted leftovers)
  uint32_t num_slots = 0;
  std::vector<uint32_t> wire_slot;      // [n * num_wires] row-major: slot of wire (row, col)
  std::vector<uint32_t> wire_slot_cm;   // [num_wires * n] column-major (wire-matrix expansion)
  std::vector<Gen> schedule;            // generators in dependency order
  std::vector<uint32_t> pi_slots;       // public input slots (in order)
  std::vector<uint32_t> virt_slot;      // virtual target index -> slot
  uint32_t zero_const_slot = 0;         // slot of builder.zero() (0 if the circuit has none)
  // distinct slots set on the host before the device schedule runs: the
  // targets commit() sets, then the outputs of host_gens
  std::vector<uint32_t> input_slots;
  // generators the host runs for the device witness (schedule indices, in
  // schedule order): Poseidon chains over inputs alone (with the constants they
  // read) at least HOST_CHAIN_MIN permutations deep, and what leads into them
  // -- the public-input hashes and the transcript sponges behind them.  A
  // one-lane permutation chain is ~10x slower on one GPU wave than on a host
  // core, and these chains set the device schedule's depth (a 32,768-input
  // aggregation root: 4,097 levels without them)
  std::vector<uint32_t> host_gens;
  // host_gens segments [host_seg_off[k], host_seg_off[k + 1]): segment 0 the
  // constants the chains read, then each independent chain (they can run in
  // parallel once segment 0 has); empty if host_gens is
  std::vector<uint32_t> host_seg_off;
  // zk config: the PublicInputGate row's unused wires 4..num_wires-1, which
  // plonky2's build() hands to RandomValueGenerators (randomize_unused_pi_wires,
  // plonk/circuit_builder.rs).  Here they are commit() inputs (zk randomness is an
  // ABI input, so a proof is a pure function of its inputs); empty if not zk
  std::vector<uint32_t> zk_slots;
  uint32_t pi_row = 0;
  bool device_witness = true;           // every generator kind has a device form (witness.hip)
  std::vector<DevGen> dev_gens;         // generators ordered by dependency level, then kind
  std::vector<uint32_t> dev_wslot;      // wire_slot with DEV_MULTI flags (device witness)
  std::vector<uint32_t> level_off;      // [levels + 1] offsets into dev_gens
  std::vector<uint32_t> level_pos;      // [levels][2]: first Poseidon generator of the level, count
  // what upstream's ProverOnlyCircuitData records beyond the above (prover.bin,
  // prover_bin.cpp): the simple generators the gadgets added, in call order
  // (EqualityGenerator, WireSplitGenerator -- every split_le, also of one gate),
  // the copy constraints in connect() order, the virtual target count and the
  // public-input targets
  std::vector<Gen> simple_gens;
  std::vector<std::pair<Target, Target>> copies;
  uint32_t num_virtual_targets = 0;
  std::vector<Target> public_input_targets;
  // commitments (filled by the prover backend at setup)
  F constants_sigmas_cap[64 * 4] = {0};
  F circuit_digest[4] = {0};
  bool digest_ready = false;

  uint32_t slot_of(Target t) const;
  // plonky2 CommonCircuitData::to_bytes (util/serialization.rs)
  std::vector<uint8_t> common_bytes() const;
};

class Witness;

class CircuitBuilder {
 public:
  explicit CircuitBuilder(const CircuitConfig &cfg);

  Target add_virtual_target();
  std::vector<Target> add_virtual_targets(size_t n);
  std::vector<Target> add_virtual_hash() { return add_virtual_targets(4); }
  Target add_virtual_public_input();
  std::vector<Target> add_virtual_hash_public_input();
  void register_public_input(Target t) { public_inputs_.push_back(t); }
  // virtual target + assert_bool (b*b - b == 0)
  Target add_virtual_bool_target_safe();

  Target constant(F c);
  Target zero() { return constant(0); }
  Target one() { return constant(1); }
  Target _false() { return zero(); }
  Target _true() { return one(); }
  Target constant_bool(bool b) { return constant(b ? 1 : 0); }

  void connect(Target a, Target b);
  void connect_hashes(const std::vector<Target> &a, const std::vector<Target> &b);
  void assert_zero(Target t) { connect(t, zero()); }
  // gadgets/range_check.rs assert_bool: b*b - b == 0
  void assert_bool(Target b) { connect(mul_sub(b, b, b), zero()); }

  // plonky2 gadgets/arithmetic.rs
  Target arithmetic(F c0, F c1, Target m0, Target m1, Target addend);
  Target add(Target x, Target y);
  Target sub(Target x, Target y);
  Target mul(Target x, Target y);
  Target mul_add(Target x, Target y, Target z);
  Target mul_sub(Target x, Target y, Target z);
  Target mul_const(F c, Target x);
  Target mul_const_add(F c, Target x, Target y);
  Target _not(Target b);
  Target _and(Target a, Target b) { return mul(a, b); }
  Target _or(Target a, Target b);
  Target select(Target b, Target x, Target y);
  Target is_equal(Target x, Target y);

  // gadgets/split_base.rs / range_check.rs
  std::vector<Target> split_le(Target x, uint32_t num_bits);
  void range_check(Target x, uint32_t n_log) { split_le(x, n_log); }

  // hash/hashing.rs hash_n_to_m_no_pad (Poseidon, overwrite mode)
  std::vector<Target> hash_n_to_hash_no_pad(const std::vector<Target> &inputs);
  std::vector<Target> hash_or_noop(const std::vector<Target> &inputs);
  // PoseidonHash::permute_swapped (hash/poseidon.rs): one PoseidonGate row;
  // swap = 1 exchanges input lanes 0..3 with 4..7
  std::vector<Target> permute(const std::vector<Target> &state) { return permute_swapped(state, _false()); }
  std::vector<Target> permute_swapped(const std::vector<Target> &state, Target swap);
  // gadgets/random_access.rs: v[index] for |v| = 16 through a RandomAccessGate copy
  Target random_access(Target index, const std::vector<Target> &v);
  // a generator the gadget layer creates (GEN_EXT_DIV ...); inputs must be targets
  void add_generator(const Gen &g) { gens_.push_back(g); }

  // ---- extension arithmetic on the recursion gates (gadgets/arithmetic_extension.rs)
  ExtT zero_ext() { return {zero(), zero()}; }
  ExtT one_ext() { return {one(), zero()}; }
  ExtT constant_ext(F c0, F c1 = 0) { return {constant(c0), constant(c1)}; }
  ExtT convert_to_ext(Target t) { return {t, zero()}; }
  ExtT add_virtual_ext() { return {add_virtual_target(), add_virtual_target()}; }
  void connect_ext(ExtT a, ExtT b) { connect(a.c0, b.c0); connect(a.c1, b.c1); }
  // c0 m0 m1 + c1 addend: special cases, operation dedup, then an
  // ArithmeticExtensionGate op (MulExtensionGate op when the addend is zero)
  ExtT arithmetic_extension(F c0, F c1, ExtT m0, ExtT m1, ExtT addend);
  ExtT add_ext(ExtT a, ExtT b) { return arithmetic_extension(1, 1, one_ext(), a, b); }
  ExtT sub_ext(ExtT a, ExtT b) { return arithmetic_extension(1, gl_neg_one(), one_ext(), a, b); }
  ExtT mul_ext(ExtT a, ExtT b) { return arithmetic_extension(1, 0, a, b, zero_ext()); }
  ExtT mul_add_ext(ExtT a, ExtT b, ExtT c) { return arithmetic_extension(1, 1, a, b, c); }
  ExtT mul_sub_ext(ExtT a, ExtT b, ExtT c) { return arithmetic_extension(1, gl_neg_one(), a, b, c); }
  ExtT scalar_mul_ext(F c, ExtT x) { return arithmetic_extension(c, 0, one_ext(), x, zero_ext()); }
  ExtT mul_const_add_ext(F c, ExtT x, ExtT y) { return arithmetic_extension(c, 1, one_ext(), x, y); }
  ExtT add_const_ext(ExtT x, F c) { return add_ext(x, constant_ext(c)); }
  ExtT square_ext(ExtT x) { return mul_ext(x, x); }
  ExtT mul_many_ext(const std::vector<ExtT> &v);
  // x / y: the inverse from a generator checked as y * inv == 1, then x * inv + z
  ExtT div_add_ext(ExtT x, ExtT y, ExtT z);
  ExtT div_ext(ExtT x, ExtT y) { return div_add_ext(x, y, zero_ext()); }
  ExtT exp_u64_ext(ExtT base, uint64_t e);
  ExtT exp_power_of_2_ext(ExtT base, uint32_t k);
  // PoseidonMdsGate row: the MDS layer of 12 ext values
  std::vector<ExtT> poseidon_mds(const std::vector<ExtT> &s);
  // ReducingFactorTarget::reduce_base / reduce: sum_i t_i alpha^i through
  // ReducingGate / ReducingExtensionGate rows (short inputs: arithmetic ops)
  ExtT reduce_base(ExtT alpha, const std::vector<Target> &t);
  ExtT reduce_ext(ExtT alpha, const std::vector<ExtT> &t);
  ExtT reduce_arithmetic(ExtT alpha, const std::vector<ExtT> &t);
  // CosetInterpolationGate row: the value at `point` of the polynomial through
  // (shift w^i, values[i]), i < 16 (w = the 16th root of unity)
  ExtT interpolate_coset(Target shift, const std::vector<ExtT> &values, ExtT point);

  // targets whose values the caller sets before witness generation (fill_targets)
  void mark_input(Target t) { inputs_.push_back(t); }
  void mark_inputs(const std::vector<Target> &ts) { inputs_.insert(inputs_.end(), ts.begin(), ts.end()); }

  size_t num_gates() const { return rows_.size(); }
  // CircuitBuilder::build: PI hash + PublicInputGate, constant gates, padding,
  // selectors, sigmas, generator schedule.  Throws std::runtime_error on failure.
  CircuitData build();

 private:
  uint32_t add_gate(GateKind k, F c0 = 0, F c1 = 0);
 public:
  bool as_const(Target t, F &v) const;

 private:

  CircuitConfig cfg_;
  std::vector<GateInst> rows_;
  uint32_t nvirt_ = 0;
  std::vector<std::pair<Target, Target>> copies_;
  std::vector<Gen> gens_;
  std::vector<Gen> simple_gens_;  // CircuitData::simple_gens
  std::vector<Target> public_inputs_;
  std::vector<Target> inputs_;
  std::unordered_map<F, Target> const_to_target_;
  std::unordered_map<uint32_t, F> target_to_const_;
  std::map<std::pair<F, F>, std::pair<uint32_t, uint32_t>> arith_open_;  // (c0,c1) -> (row, next op)
  using ArithKey = std::tuple<F, F, uint32_t, uint32_t, uint32_t>;
  struct ArithKeyHash {
    size_t operator()(const ArithKey &k) const {
      uint64_t h = std::get<0>(k) * 0x9E3779B97F4A7C15ull ^ std::get<1>(k);
      h = (h ^ (h >> 29)) * 0xBF58476D1CE4E5B9ull ^ std::get<2>(k);
      h = (h ^ (h >> 31)) * 0x94D049BB133111EBull ^ ((uint64_t)std::get<3>(k) << 32 | std::get<4>(k));
      return (size_t)(h ^ (h >> 32));
    }
  };
  std::unordered_map<ArithKey, Target, ArithKeyHash> arith_cache_;  // find/insert only (no iteration)
  std::map<std::pair<F, F>, std::pair<uint32_t, uint32_t>> ae_open_;  // ArithmeticExtensionGate slots
  std::map<F, std::pair<uint32_t, uint32_t>> me_open_;                 // MulExtensionGate slots
  std::map<std::tuple<F, F, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, ExtT> ext_cache_;
  static F gl_neg_one() { return 0xFFFFFFFF00000000ull; }
  bool as_const_ext(ExtT t, F &c0, F &c1) const { return as_const(t.c0, c0) && as_const(t.c1, c1); }
  std::pair<uint32_t, uint32_t> ra_open_{0, RA_COPIES};                  // (row, next copy) of the open RandomAccessGate
  uint32_t arith_ops_, base_sum_limbs_;
};

// common/src/gadgets.rs:14-65 (shared by the Wormhole and voting circuits)
Target xor_gadget(CircuitBuilder &b, Target a, Target c);
Target is_const_less_than(CircuitBuilder &b, uint32_t left, Target right, uint32_t n_log);

// Per-proof witness: values per partition slot.
class Witness {
 public:
  // vals: optional caller-owned storage of cd.num_slots words (e.g. a pinned
  // staging buffer the prover uploads directly); zeroed here
  explicit Witness(const CircuitData &cd, F *vals = nullptr);
  Witness(const Witness &) = delete;
  Witness &operator=(const Witness &) = delete;
  // PartialWitness::set_target; returns false on "set twice with different values"
  bool set(Target t, F v);
  bool set_slot(uint32_t s, F v);
  bool get_slot(uint32_t s, F &v) const {
    v = vals_[s];
    return known_[s];
  }
  // slot values [num_slots] (slot 0 = 0): wire (r, c) = slot_values()[wire_slot[r * W + c]]
  const F *slot_values() const { return vals_; }
  // run the generator schedule; returns false (and a message) on conflict / missing input
  bool generate(std::string &err);
  // run CircuitData::host_gens (the device witness's host part): segment seg
  // (0 = the constants, then one per independent chain), or all if seg < 0
  bool generate_host_chains(std::string &err, int seg = -1);
  // one generator of the schedule
  bool run(const Gen &g, std::string &err);
  // full wire matrix, column-major [num_wires][n]
  void wires_matrix(F *out) const;
  std::vector<F> public_inputs() const;

 private:
  bool set_wire(uint32_t row, uint32_t col, F v);
  F wire(uint32_t row, uint32_t col) const;
  const CircuitData &cd_;
  std::vector<F> own_;
  F *vals_;
  std::vector<uint8_t> known_;
};

}  // namespace qc
