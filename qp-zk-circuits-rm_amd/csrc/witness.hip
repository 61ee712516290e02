// witness.hip — witness generation on the device (plonky2 iop/generator.rs
// generate_partial_witness), for the circuits of the
// native builder (circuit.cpp).
//
// The host only runs commit() (the fragments' fill_targets: a few thousand
// input values per proof, uploaded as one compact row); every generator —
// Poseidon gates, BaseSum limbs, arithmetic, equality (inverse), constants —
// runs here.  build() groups the generators into dependency levels; one
// workgroup owns one proof and walks the levels with a barrier between them,
// so B proofs occupy B CUs with no grid-wide synchronisation.
//
// Partition values live in HBM, one u64 per value slot, UNSET = 2^64 - 1 (not
// a canonical field element) until written.  A write is a compare-and-swap
// from UNSET: writing a different value to a written slot is the reference's
// "Partition containing ... was set twice with different values" failure and
// flags the proof.  Slot 0 is the shared never-set slot (value 0).
#include <hip/hip_runtime.h>
#include "field.h"
#include "poseidon.h"
#include "poseidon_dev.h"
#include "poseidon_coop.h"
#include "witness_kernels.h"

namespace qpk {

constexpr uint64_t UNSET = ~0ull;

struct DevGenD {  // == qc::DevGen
  uint32_t kind, row;
  uint32_t s[4];
  uint64_t k0, k1;
};
enum : uint32_t { WG_CONSTANT = 0, WG_ARITH, WG_POSEIDON, WG_BASE_SPLIT, WG_EQUALITY,
                  WG_WIRE_SPLIT, WG_EXT_DIV, WG_RANDOM_ACCESS, WG_ARITH_EXT, WG_MUL_EXT, WG_REDUCING,
                  WG_REDUCING_EXT, WG_POSEIDON_MDS, WG_COSET_INTERP };
// recursion-gate shapes (circuit.h): ReducingGate / ReducingExtensionGate
// coefficients, CosetInterpolationGate{4, 6} wires
constexpr uint32_t RED_COEFFS = 43, REDE_COEFFS = 32;
constexpr uint32_t CI_BITS = 4, CI_POINTS = 16, CI_DEGREE = 6, CI_NINT = (CI_POINTS - 2) / (CI_DEGREE - 1);
constexpr uint32_t CI_VALUES = 1, CI_EVAL_POINT = CI_VALUES + 2 * CI_POINTS, CI_EVAL_VALUE = CI_EVAL_POINT + 2,
                   CI_INTER = CI_EVAL_VALUE + 2, CI_SHIFTED = CI_INTER + 4 * CI_NINT;
// RandomAccessGate{bits 4, copies 4, extra constants 2} wire layout (circuit.h ra_wire_*)
constexpr uint32_t RA_BITS = 4, RA_VEC = 16, RA_COPIES = 4, RA_EXTRA = 2;

// both writes always happen (a && b would skip the second after a failure)
__device__ __forceinline__ bool both(bool a, bool b) { return a && b; }

// slot ids of the generator records and the wire-slot table carry MULTI when
// the slot has several writers (circuit.cpp, qc::DEV_MULTI): only those take
// the compare-and-swap; a single writer stores (a write needs no round trip)
constexpr uint32_t MULTI = 0x80000000u;
__device__ __forceinline__ bool wset(uint64_t *v, uint32_t s, uint64_t x) {
  if (!(s & MULTI)) {
    v[s] = x;
    return true;
  }
  const unsigned long long old = atomicCAS((unsigned long long *)(v + (s & ~MULTI)), (unsigned long long)UNSET,
                                           (unsigned long long)x);
  return old == UNSET || old == x;
}

__global__ void k_witness_init(uint64_t *vals, uint64_t v_bstride, uint32_t nslots, const uint32_t *in_slots,
                               const uint64_t *in_vals, uint32_t nin) {
  const uint32_t b = blockIdx.y;
  uint64_t *v = vals + (uint64_t)b * v_bstride;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += gridDim.x * blockDim.x)
    v[s] = s ? UNSET : 0;
}

__global__ void k_witness_inputs(uint64_t *vals, uint64_t v_bstride, const uint32_t *in_slots,
                                 const uint64_t *in_vals, uint32_t nin) {
  const uint32_t b = blockIdx.y;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nin) vals[(uint64_t)b * v_bstride + in_slots[i]] = in_vals[(uint64_t)b * nin + i];
}

// a generator input still UNSET means a scheduling bug or a missing input: the
// generator fails (reported like a conflict) instead of computing on 2^64-1
__device__ __forceinline__ uint64_t rd(const uint64_t *v, uint32_t s, bool &ok) {
  const uint64_t x = v[s & ~MULTI];
  ok &= x != UNSET;
  return x;
}

// PoseidonGenerator on the throughput permutation (poseidon_fast.h: round
// constants as literal operands, sparse partial rounds whose lane 0 before
// each S-box is the plain form's S-box input): the gate's wires are written
// as the rounds reach them.  State values are non-canonical in [0, 2^64)
// between rounds; every written value is canonicalised.  The slot ids of a
// phase's writes are loaded one phase ahead, so their latency hides behind
// the rounds (a lookup per write would stall the lane on every store).
__device__ __noinline__ bool wset_multi(uint64_t *v, uint32_t s, uint64_t x) { return wset(v, s, x); }
__device__ __forceinline__ void wput(uint64_t *v, uint32_t s, uint64_t x, bool &ok) {
  x = psd::canon(x);
  if (!(s & MULTI)) v[s] = x;
  else ok &= wset_multi(v, s, x);
}
template <int N>
__device__ __forceinline__ void slots_load(uint32_t (&sl)[N], const uint32_t *ws, uint32_t j0) {
#pragma unroll
  for (int i = 0; i < N; i++) sl[i] = ws[j0 + i];
}
// Every round a loop iteration with the round constants from memory, plain
// partial rounds (full MDS): a few thousand instructions of code.  Measured
// against the unrolled sparse-round form (~280 KB of code) and a first form
// with a slot lookup per write (tools/gpu_session.sh wit_ab, 256-leaf subtree,
// profiles/r04_wit_ab.log): rolled 0.566 s, unrolled 0.607 s, plain 0.668 s
__device__ __noinline__ bool poseidon_witness_rolled(uint64_t *v, const uint32_t *__restrict__ ws) {
  bool in_ok = true, ok = true;
  uint64_t s[12];
  for (int i = 0; i < 12; i++) s[i] = rd(v, ws[i], in_ok);
  const uint64_t swap = rd(v, ws[24], in_ok);
  if (!in_ok) return false;
  for (int i = 0; i < 4; i++) wput(v, ws[25 + i], gl::mul(swap, gl::sub(s[i + 4], s[i])), ok);
  if (swap == 1)
    for (int i = 0; i < 4; i++) {
      const uint64_t t = s[i];
      s[i] = s[i + 4];
      s[i + 4] = t;
    }
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = pf::add_c(s[i], ps::rc_cx(i));
  uint32_t sl[12];
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
    if (r) {
#pragma unroll
      for (int i = 0; i < 12; i++) wput(v, sl[i], s[i], ok);
    }
    slots_load(sl, ws, r < 3 ? 29 + 12 * r : 65);
    pf::full_round_dyn(s, ps::RC_DEV + (r + 1) * 12);
  }
#pragma unroll 1
  for (int r = 0; r < 22; r++) {
    const uint32_t nx = ws[r < 21 ? 66 + r : 87];
    wput(v, sl[0], s[0], ok);
    sl[0] = nx;
    s[0] = pf::sbox(s[0]);
    uint32_t lo[12], hi[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
      lo[i] = pf::lo32(s[i]);
      hi[i] = pf::hi32(s[i]);
    }
    pf::mds_rows_block_dyn<0>(s, lo, hi, ps::RC_DEV + (r + 5) * 12);
  }
  slots_load(sl, ws, 87);
#pragma unroll 1
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) wput(v, sl[i], s[i], ok);
    slots_load(sl, ws, 99 + 12 * r);
    pf::full_round_dyn(s, ps::RC_DEV + (r + 27) * 12);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) wput(v, sl[i], s[i], ok);
  slots_load(sl, ws, 12);
  pf::sbox12(s);
  pf::mds<3, -1>(s);
#pragma unroll
  for (int i = 0; i < 12; i++) wput(v, sl[i], s[i], ok);
  return ok;
}

// Cooperative PoseidonGenerator: one wave, lane i < 12 holding state element
// i, for the narrow levels of the schedule (the transcript sponges and the
// public-input hash are chains of single permutations, one level each).  Per
// round: constant add and S-box lane-parallel, then the MDS row of lane r from
// the 12 S-box outputs broadcast through v_readlane (24 SGPR values) times
// the lane's own circulant coefficients, four accumulators of 6 products.
// The dependent chain of a round is one S-box plus six products (the
// one-lane form runs all 12 S-boxes and 12 MDS rows in sequence).  All 64
// lanes must be active; lanes >= 12 compute and never write.
// ROW: one generator per 16-lane row (pc::row_mds, four per wave; a row is
// wholly active or inactive); else one per wave (pc::wave_mds_row, all 64
// lanes active)
template <bool ROW>
__device__ __forceinline__ uint64_t coop_mds(uint64_t y, const uint32_t (&coef)[12]) {
  if constexpr (ROW) return pc::row_mds(y, coef);
  else return pc::wave_mds_row(y, coef);
}
template <bool ROW>
__device__ __noinline__ bool poseidon_coop(uint64_t *v, const uint32_t *__restrict__ ws) {
  const uint32_t lane = threadIdx.x & (ROW ? 15 : 63);
  const bool act = lane < 12;
  const uint32_t i = act ? lane : 0;
  // MDS row i: coefficient of element j = CIRC[(j - i) mod 12] (+ 8 on the diagonal of row 0)
  uint32_t coef[12];
#pragma unroll
  for (int j = 0; j < 12; j++) coef[j] = ps::mds_circ((j - (int)i + 12) % 12) + (i == 0 && j == 0 ? 8u : 0u);
  bool in_ok = true, ok = true;
  const uint32_t partner = i < 4 ? i + 4 : i < 8 ? i - 4 : i;
  const uint64_t a = rd(v, ws[i], in_ok), b = rd(v, ws[partner], in_ok);
  const uint64_t swap = rd(v, ws[24], in_ok);
  uint32_t sl = ws[act ? 29 + i : 29];
  if constexpr (ROW) {
    if ((__ballot(!in_ok) >> (threadIdx.x & 48)) & 0xffffull) return false;  // this row's lanes
  } else {
    if (!__all(in_ok)) return false;
  }
  if (act && i < 4) wput(v, ws[25 + i], gl::mul(swap, gl::sub(b, a)), ok);
  uint64_t x = swap == 1 && i < 8 ? b : a;
  x = pf::add_c(x, ps::RC_DEV[i]);
  // rounds 0..3: the state entering rounds 1..3 (after their constants) is written
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
    if (r && act) wput(v, sl, x, ok);
    sl = ws[act ? (r < 3 ? 29 + 12 * r + i : 65) : 29];
    const uint64_t rc = ps::RC_DEV[(r + 1) * 12 + i];
    x = pf::add_c(coop_mds<ROW>(pf::sbox(x), coef), rc);
  }
  // partial rounds 4..25: lane 0's S-box input is the wire
#pragma unroll 1
  for (int r = 4; r < 26; r++) {
    if (lane == 0) wput(v, sl, x, ok);
    sl = ws[lane == 0 ? (r < 25 ? 66 + (r - 4) : 87) : (act ? 87 + i : 87)];
    const uint64_t rc = ps::RC_DEV[(r + 1) * 12 + i];
    const uint64_t y = pf::sbox(x);
    x = pf::add_c(coop_mds<ROW>(lane == 0 ? y : x, coef), rc);
  }
  if (act) sl = ws[87 + i];
  // rounds 26..29: the state entering each is written, then the output
#pragma unroll 1
  for (int r = 26; r < 30; r++) {
    if (act) wput(v, sl, x, ok);
    sl = ws[act ? (r < 29 ? 87 + 12 * (r - 25) + i : 12 + i) : 12];
    x = coop_mds<ROW>(pf::sbox(x), coef);
    if (r < 29) x = pf::add_c(x, ps::RC_DEV[(r + 1) * 12 + i]);
  }
  if (act) wput(v, sl, x, ok);
  return ok;
}


__device__ bool run_gen(const DevGenD &g, uint64_t *__restrict__ v, const uint32_t *__restrict__ wslot, uint32_t W, uint32_t limbs,
                        uint32_t zslot, uint32_t num_consts) {
  bool in_ok = true;
  switch (g.kind) {
    case WG_CONSTANT:
      return wset(v, g.s[0], g.k0) && (num_consts < 2 || wset(v, g.s[1], g.k1));
    case WG_ARITH: {
      const uint64_t m = gl::mul(gl::mul(rd(v, g.s[0], in_ok), rd(v, g.s[1], in_ok)), g.k0);
      const uint64_t a = rd(v, g.s[2], in_ok);
      return in_ok && wset(v, g.s[3], gl::add(m, gl::mul(a, g.k1)));
    }
    case WG_BASE_SPLIT: {
      const uint64_t sum = rd(v, g.s[0], in_ok);
      if (!in_ok) return false;
      const uint32_t *ws = wslot + (uint64_t)g.row * W + 1;
      bool ok = true;
      for (uint32_t l = 0; l < limbs; l++) {
        const uint64_t bit = (sum >> l) & 1;
        if (zslot && (ws[l] & ~MULTI) == zslot) ok &= bit == 0;
        else ok &= wset(v, ws[l], bit);
      }
      return ok;
    }
    case WG_EQUALITY: {
      const uint64_t x = rd(v, g.s[0], in_ok), y = rd(v, g.s[1], in_ok);
      if (!in_ok) return false;
      const bool eq = x == y;
      return wset(v, g.s[2], eq ? 1 : 0) && wset(v, g.s[3], eq ? 0 : gl::inv(gl::sub(x, y)));
    }
    case WG_WIRE_SPLIT: {
      // WireSplitGenerator (gadgets/split_base.rs): the integer's `limbs`-bit
      // chunks into the sum wires of s[1] consecutive BaseSum gates
      uint64_t x = rd(v, g.s[0], in_ok);
      if (!in_ok) return false;
      bool ok = true;
      for (uint32_t j = 0; j < g.s[1]; j++) {
        const uint64_t sum = limbs < 64 ? (x & ((1ull << limbs) - 1)) : x;
        x = limbs < 64 ? x >> limbs : 0;
        ok &= wset(v, wslot[(uint64_t)(g.row + j) * W], sum);
      }
      return ok;
    }
    case WG_EXT_DIV: {
      // QuotientGeneratorExtension (gadgets/arithmetic_extension.rs): (a + bX) / (c + dX)
      const gl::ext num{rd(v, g.s[0], in_ok), rd(v, g.s[1], in_ok)};
      const gl::ext den{rd(v, g.s[2], in_ok), rd(v, g.s[3], in_ok)};
      if (!in_ok || (den.c0 == 0 && den.c1 == 0)) return false;
      const gl::ext q = gl::ext_mul(num, gl::ext_inv(den));
      return wset(v, (uint32_t)g.k0, q.c0) && wset(v, (uint32_t)(g.k0 >> 32), q.c1);
    }
    case WG_RANDOM_ACCESS: {
      // RandomAccessGenerator (gates/random_access.rs) of copy s[0]
      const uint32_t c = g.s[0];
      const uint32_t *ws = wslot + (uint64_t)g.row * W + (2 + RA_VEC) * c;
      const uint64_t idx = rd(v, ws[0], in_ok);
      if (!in_ok || idx >= RA_VEC) return false;
      const uint64_t item = rd(v, ws[2 + idx], in_ok);
      if (!in_ok) return false;
      bool ok = wset(v, ws[1], item);
      const uint32_t *wb = wslot + (uint64_t)g.row * W + (2 + RA_VEC) * RA_COPIES + RA_EXTRA + RA_BITS * c;
      for (uint32_t i = 0; i < RA_BITS; i++) ok &= wset(v, wb[i], (idx >> i) & 1);
      return ok;
    }
    case WG_ARITH_EXT:
    case WG_MUL_EXT: {
      // ArithmeticExtensionGenerator / MulExtensionGenerator of op s[0]
      const uint32_t *ws = wslot + (uint64_t)g.row * W;
      const bool ae = g.kind == WG_ARITH_EXT;
      const uint32_t o = ae ? 8 * g.s[0] : 6 * g.s[0];
      const gl::ext m0{rd(v, ws[o], in_ok), rd(v, ws[o + 1], in_ok)};
      const gl::ext m1{rd(v, ws[o + 2], in_ok), rd(v, ws[o + 3], in_ok)};
      gl::ext r = gl::ext_scale(gl::ext_mul(m0, m1), g.k0);
      if (ae) r = gl::ext_add(r, gl::ext_scale(gl::ext{rd(v, ws[o + 4], in_ok), rd(v, ws[o + 5], in_ok)}, g.k1));
      if (!in_ok) return false;
      const uint32_t oo = ae ? o + 6 : o + 4;
      return both(wset(v, ws[oo], r.c0), wset(v, ws[oo + 1], r.c1));
    }
    case WG_REDUCING:
    case WG_REDUCING_EXT: {
      // ReducingGenerator: acc <- acc alpha + coeff_i, every accumulator
      // written.  Chunks of 8 coefficients: the chunk's slot ids, then its
      // values, are loaded together (two memory latencies per chunk instead
      // of two per coefficient)
      const uint32_t *__restrict__ ws = wslot + (uint64_t)g.row * W;
      const bool base = g.kind == WG_REDUCING;
      const uint32_t nc = base ? RED_COEFFS : REDE_COEFFS, cw = base ? 1 : 2;
      const gl::ext alpha{rd(v, ws[2], in_ok), rd(v, ws[3], in_ok)};
      gl::ext acc{rd(v, ws[4], in_ok), rd(v, ws[5], in_ok)};
      bool ok = true;
      constexpr uint32_t CH = 8;
      for (uint32_t c0 = 0; c0 < nc; c0 += CH) {
        uint32_t cs[2 * CH], as[2 * CH];
        uint64_t cv[2 * CH];
#pragma unroll
        for (uint32_t k = 0; k < CH; k++) {
          const uint32_t i = c0 + k < nc ? c0 + k : nc - 1;
          cs[2 * k] = ws[6 + cw * i];
          cs[2 * k + 1] = base ? 0 : ws[7 + 2 * i];
          const uint32_t aw = i + 1 == nc ? 0 : 6 + cw * nc + 2 * i;
          as[2 * k] = ws[aw];
          as[2 * k + 1] = ws[aw + 1];
        }
#pragma unroll
        for (uint32_t k = 0; k < 2 * CH; k++) cv[k] = (k & 1) && base ? 0 : rd(v, cs[k], in_ok);
#pragma unroll
        for (uint32_t k = 0; k < CH; k++) {
          if (c0 + k >= nc) break;
          acc = gl::ext_add(gl::ext_mul(acc, alpha), gl::ext{cv[2 * k], cv[2 * k + 1]});
          ok &= both(wset(v, as[2 * k], acc.c0), wset(v, as[2 * k + 1], acc.c1));
        }
      }
      return ok && in_ok;
    }
    case WG_POSEIDON_MDS: {
      // PoseidonMdsGenerator: the MDS layer of each component
      const uint32_t *ws = wslot + (uint64_t)g.row * W;
      uint64_t a[12], b[12];
      for (int i = 0; i < 12; i++) {
        a[i] = rd(v, ws[2 * i], in_ok);
        b[i] = rd(v, ws[2 * i + 1], in_ok);
      }
      if (!in_ok) return false;
      ps::mds(a);
      ps::mds(b);
      bool ok = true;
      for (int i = 0; i < 12; i++) ok &= both(wset(v, ws[24 + 2 * i], a[i]), wset(v, ws[25 + 2 * i], b[i]));
      return ok;
    }
    case WG_COSET_INTERP: {
      // InterpolationGenerator: shifted point, partial barycentric sums per
      // chunk of the subgroup (intermediate wires), the value
      const uint32_t *ws = wslot + (uint64_t)g.row * W;
      const uint64_t shift = rd(v, ws[0], in_ok);
      gl::ext pt{rd(v, ws[CI_EVAL_POINT], in_ok), rd(v, ws[CI_EVAL_POINT + 1], in_ok)};
      // the 16 values, loaded together before any write
      uint64_t vals[2 * CI_POINTS];
#pragma unroll
      for (uint32_t k = 0; k < 2 * CI_POINTS; k++) vals[k] = rd(v, ws[CI_VALUES + k], in_ok);
      if (!in_ok || shift == 0) return false;
      pt = gl::ext_scale(pt, gl::inv(shift));
      bool ok = both(wset(v, ws[CI_SHIFTED], pt.c0), wset(v, ws[CI_SHIFTED + 1], pt.c1));
      const uint64_t om = gl::root_of_unity(CI_BITS), ninv = gl::inv(CI_POINTS);
      gl::ext ev{0, 0}, pr{1, 0};
      uint64_t x = 1;
      // points [0, 6), then [6, 11), [11, 16): the partial sums after the first
      // two chunks are the intermediate wires (compile-time indices: vals stays
      // in registers)
#pragma clang loop unroll(full)
      for (uint32_t i = 0; i < CI_POINTS; i++) {
        if (i >= CI_DEGREE && (i - 1) % (CI_DEGREE - 1) == 0) {
          const uint32_t it = (i - 1) / (CI_DEGREE - 1) - 1;
          ok &= both(wset(v, ws[CI_INTER + 2 * it], ev.c0), wset(v, ws[CI_INTER + 2 * it + 1], ev.c1));
          ok &= both(wset(v, ws[CI_INTER + 2 * (CI_NINT + it)], pr.c0),
                     wset(v, ws[CI_INTER + 2 * (CI_NINT + it) + 1], pr.c1));
        }
        const gl::ext term = gl::ext_sub(pt, gl::ext{x, 0});
        const gl::ext val = gl::ext_scale(gl::ext{vals[2 * i], vals[2 * i + 1]}, gl::mul(x, ninv));
        ev = gl::ext_add(gl::ext_mul(ev, term), gl::ext_mul(val, pr));
        pr = gl::ext_mul(pr, term);
        x = gl::mul(x, om);
      }
      ok &= both(wset(v, ws[CI_EVAL_VALUE], ev.c0), wset(v, ws[CI_EVAL_VALUE + 1], ev.c1));
      return ok && in_ok;
    }
    case WG_POSEIDON:
      // PoseidonGenerator (gates/poseidon.rs), wire layout SURVEY.md A.5
      return poseidon_witness_rolled(v, wslot + (uint64_t)g.row * W);
    default:
      return false;
  }
}

// one workgroup per proof; levels separated by workgroup barriers.  Every
// wave reaches every barrier (no early exit), so the grid always drains.
__global__ void __launch_bounds__(512) k_witness_gen(const WitnessGenArgs a) {
  const uint32_t b = blockIdx.x;
  uint64_t *v = a.vals + (uint64_t)b * a.v_bstride;
  const DevGenD *gens = (const DevGenD *)a.gens;
  const uint32_t nwaves = blockDim.x >> 6, wave = threadIdx.x >> 6;
  bool ok = true;
  uint32_t bad = 0;
  for (uint32_t l = 0; l < a.nlevels; l++) {
    const uint32_t lo = a.level_off[l], hi = a.level_off[l + 1];
    const uint32_t plo = a.level_pos[2 * l], pcnt = a.level_pos[2 * l + 1];
    // narrow levels: their Poseidon generators one per wave (poseidon_coop),
    // the level's other generators one per lane as usual
    const bool coop = pcnt && pcnt <= a.coop_max;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      if (coop && i >= plo && i < plo + pcnt) continue;
      if (!run_gen(gens[i], v, a.wslot, a.W, a.limbs, a.zero_slot, a.num_consts) && ok) {
        ok = false;
        bad = i + 1;
      }
    }
    if (coop && a.row) {
      for (uint32_t p = plo + (threadIdx.x >> 4); p < plo + pcnt; p += blockDim.x >> 4)  // row-uniform
        if (!poseidon_coop<true>(v, a.wslot + (uint64_t)gens[p].row * a.W) && ok) {
          ok = false;
          bad = p + 1;
        }
    } else if (coop) {
      for (uint32_t p = plo + wave; p < plo + pcnt; p += nwaves)  // wave-uniform: every lane active
        if (!poseidon_coop<false>(v, a.wslot + (uint64_t)gens[p].row * a.W) && ok) {
          ok = false;
          bad = p + 1;
        }
    }
    __syncthreads();
  }
  if (!ok) atomicCAS(a.err + b, 0u, bad);
}

// one dependency level over the whole batch (the level-launch mode for small
// batches: a launch per level instead of one workgroup per proof walking every
// level): blocks [0, na) run the level's non-Poseidon generators one per lane,
// blocks [na, ..) its Poseidon generators one per row (poseidon_coop; one
// per wave under QPGPU_WIT_ROW=0), so a
// level costs one cooperative permutation's latency (≈25 us) rather than a
// one-lane permutation's (≈65 us) or several cooperative ones in sequence.
// Stream order separates the levels; the first failure per proof wins the CAS.
__global__ void __launch_bounds__(256) k_witness_level(const WitnessGenArgs a, uint32_t l, uint32_t na) {
  const uint32_t b = blockIdx.y;
  uint64_t *v = a.vals + (uint64_t)b * a.v_bstride;
  const DevGenD *gens = (const DevGenD *)a.gens;
  const uint32_t lo = a.level_off[l], hi = a.level_off[l + 1];
  const uint32_t plo = a.level_pos[2 * l], pcnt = a.level_pos[2 * l + 1];
  uint32_t bad = 0;
  if (blockIdx.x < na) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < hi - lo - pcnt) {
      const uint32_t i = k < plo - lo ? lo + k : lo + k + pcnt;  // skip the Poseidon run [plo, plo + pcnt)
      if (!run_gen(gens[i], v, a.wslot, a.W, a.limbs, a.zero_slot, a.num_consts)) bad = i + 1;
    }
  } else {
    if (a.row) {
      const uint32_t p = (blockIdx.x - na) * (blockDim.x >> 4) + (threadIdx.x >> 4);  // row-uniform
      if (p < pcnt && !poseidon_coop<true>(v, a.wslot + (uint64_t)gens[plo + p].row * a.W)) bad = plo + p + 1;
    } else {
      const uint32_t p = (blockIdx.x - na) * (blockDim.x >> 6) + (threadIdx.x >> 6);  // wave-uniform
      if (p < pcnt && !poseidon_coop<false>(v, a.wslot + (uint64_t)gens[plo + p].row * a.W)) bad = plo + p + 1;
    }
  }
  if (bad) atomicCAS(a.err + b, 0u, bad);
}

// wires [b][col][row] = slot values through the column-major slot map;
// public inputs gathered alongside
__global__ void k_witness_expand(const uint64_t *vals, uint64_t v_bstride, const uint32_t *wslot_cm, uint64_t nwires,
                                 uint64_t *wires, uint64_t w_bstride, const uint32_t *pi_slots, uint32_t npis,
                                 uint64_t *pis) {
  const uint32_t b = blockIdx.y;
  const uint64_t *v = vals + (uint64_t)b * v_bstride;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwires; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = v[wslot_cm[i]];
    wires[(uint64_t)b * w_bstride + i] = x == UNSET ? 0 : x;
  }
  if (blockIdx.x == 0) {
    // any number of public inputs (an aggregation root registers 16 per leaf)
    for (uint32_t k = threadIdx.x; k < npis; k += blockDim.x) {
      const uint64_t x = v[pi_slots[k]];
      pis[(uint64_t)b * npis + k] = x == UNSET ? 0 : x;
    }
  }
}

}  // namespace qpk
