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

__device__ bool run_gen(const DevGenD &g, uint64_t *v, const uint32_t *wslot, uint32_t W, uint32_t limbs,
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
      // ReducingGenerator: acc <- acc alpha + coeff_i, every accumulator written
      const uint32_t *ws = wslot + (uint64_t)g.row * W;
      const bool base = g.kind == WG_REDUCING;
      const uint32_t nc = base ? RED_COEFFS : REDE_COEFFS, cw = base ? 1 : 2;
      const gl::ext alpha{rd(v, ws[2], in_ok), rd(v, ws[3], in_ok)};
      gl::ext acc{rd(v, ws[4], in_ok), rd(v, ws[5], in_ok)};
      bool ok = true;
      for (uint32_t i = 0; i < nc; i++) {
        const gl::ext c{rd(v, ws[6 + cw * i], in_ok), base ? 0 : rd(v, ws[7 + 2 * i], in_ok)};
        acc = gl::ext_add(gl::ext_mul(acc, alpha), c);
        const uint32_t aw = i + 1 == nc ? 0 : 6 + cw * nc + 2 * i;
        ok &= both(wset(v, ws[aw], acc.c0), wset(v, ws[aw + 1], acc.c1));
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
      if (!in_ok || shift == 0) return false;
      pt = gl::ext_scale(pt, gl::inv(shift));
      bool ok = both(wset(v, ws[CI_SHIFTED], pt.c0), wset(v, ws[CI_SHIFTED + 1], pt.c1));
      const uint64_t om = gl::root_of_unity(CI_BITS), ninv = gl::inv(CI_POINTS);
      gl::ext ev{0, 0}, pr{1, 0};
      uint32_t lo = 0, hi = CI_DEGREE;
      uint64_t x = 1;
      for (uint32_t it = 0;; it++) {
        for (uint32_t i = lo; i < hi; i++) {
          const gl::ext term = gl::ext_sub(pt, gl::ext{x, 0});
          const gl::ext val = gl::ext_scale(gl::ext{rd(v, ws[CI_VALUES + 2 * i], in_ok),
                                                    rd(v, ws[CI_VALUES + 2 * i + 1], in_ok)}, gl::mul(x, ninv));
          ev = gl::ext_add(gl::ext_mul(ev, term), gl::ext_mul(val, pr));
          pr = gl::ext_mul(pr, term);
          x = gl::mul(x, om);
        }
        if (it == CI_NINT) break;
        ok &= both(wset(v, ws[CI_INTER + 2 * it], ev.c0), wset(v, ws[CI_INTER + 2 * it + 1], ev.c1));
        ok &= both(wset(v, ws[CI_INTER + 2 * (CI_NINT + it)], pr.c0), wset(v, ws[CI_INTER + 2 * (CI_NINT + it) + 1], pr.c1));
        lo = 1 + (CI_DEGREE - 1) * (it + 1);
        hi = lo + CI_DEGREE - 1 < CI_POINTS ? lo + CI_DEGREE - 1 : CI_POINTS;
      }
      ok &= both(wset(v, ws[CI_EVAL_VALUE], ev.c0), wset(v, ws[CI_EVAL_VALUE + 1], ev.c1));
      return ok && in_ok;
    }
    case WG_POSEIDON: {
      // PoseidonGenerator (gates/poseidon.rs), wire layout SURVEY.md A.5
      const uint32_t *ws = wslot + (uint64_t)g.row * W;
      uint64_t s[12];
      for (int i = 0; i < 12; i++) s[i] = rd(v, ws[i], in_ok);
      const uint64_t swap = rd(v, ws[24], in_ok);
      if (!in_ok) return false;
      bool ok = true;
      for (int i = 0; i < 4; i++) ok &= wset(v, ws[25 + i], gl::mul(swap, gl::sub(s[i + 4], s[i])));
      if (swap == 1)
        for (int i = 0; i < 4; i++) {
          const uint64_t t = s[i];
          s[i] = s[i + 4];
          s[i + 4] = t;
        }
      int rc = 0;
      for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
        if (r)
          for (int i = 0; i < 12; i++) ok &= wset(v, ws[29 + (r - 1) * 12 + i], s[i]);
        for (int i = 0; i < 12; i++) s[i] = ps::sbox(s[i]);
        ps::mds(s);
      }
      for (int r = 0; r < 22; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
        ok &= wset(v, ws[65 + r], s[0]);
        s[0] = ps::sbox(s[0]);
        ps::mds(s);
      }
      for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = gl::add(s[i], ps::rc(rc * 12 + i));
        for (int i = 0; i < 12; i++) ok &= wset(v, ws[87 + r * 12 + i], s[i]);
        for (int i = 0; i < 12; i++) s[i] = ps::sbox(s[i]);
        ps::mds(s);
      }
      for (int i = 0; i < 12; i++) ok &= wset(v, ws[12 + i], s[i]);
      return ok;
    }
    default:
      return false;
  }
}

// one workgroup per proof; levels separated by workgroup barriers.  Every
// wave reaches every barrier (no early exit), so the grid always drains.
__global__ void __launch_bounds__(256) k_witness_gen(const WitnessGenArgs a) {
  const uint32_t b = blockIdx.x;
  uint64_t *v = a.vals + (uint64_t)b * a.v_bstride;
  const DevGenD *gens = (const DevGenD *)a.gens;
  bool ok = true;
  uint32_t bad = 0;
  for (uint32_t l = 0; l < a.nlevels; l++) {
    const uint32_t lo = a.level_off[l], hi = a.level_off[l + 1];
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      if (!run_gen(gens[i], v, a.wslot, a.W, a.limbs, a.zero_slot, a.num_consts) && ok) {
        ok = false;
        bad = i + 1;
      }
    }
    __syncthreads();
  }
  if (!ok) atomicCAS(a.err + b, 0u, bad);
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
