"""Device prover and the WormholeProver mirror.

`Prover` wraps qp_prover (include/qpgpu.h): B proofs of one circuit per call on
one MI355X.  `WormholeProver` mirrors qp-wormhole-prover's API
(wormhole/prover/src/lib.rs:74-237): new(config) -> commit(inputs) -> prove(),
single use, commit twice is an error, prove before commit is an error;
new_from_bytes / new_from_files / default() load the circuit binaries that
`generate_circuit_binaries` writes (wormhole/circuit-builder/src/lib.rs:11-66).
"""
import ctypes
import hashlib
import os
import struct
import threading
import warnings

import numpy as np

from ._native import Context, QpError, lib
from .circuits import Circuit, CircuitInputs

STAGES = ["commit_wires", "zs_pp", "quotient", "openings", "fri", "pow", "queries", "serialize", "commit_inputs",
          "witness_gen"]


class ProofWithPublicInputs:
    """Serialized plonky2 ProofWithPublicInputs (ProofWithPublicInputs::to_bytes)."""

    def __init__(self, data: bytes, public_inputs):
        self.data = data
        self.public_inputs = [int(x) for x in public_inputs]

    def to_bytes(self):
        return self.data


class Prover:
    def __init__(self, ctx: Context, circuit: Circuit, max_batch=1):
        self.ctx, self.circuit, self.max_batch = ctx, circuit, max_batch
        h = ctypes.c_void_p()
        ctx.check(lib().qp_prover_new(ctx.h, circuit.h, max_batch, ctypes.byref(h)), "qp_prover_new")
        self.h = h
        ln = ctypes.c_size_t()
        lib().qp_prover_proof_size(self.h, ctypes.byref(ln))
        self.proof_size = ln.value
        self._out = self._mv = self._lens = None
        self._lock = threading.Lock()  # one prove call at a time (the device buffers and the output rows)

    def _out_buffers(self, nb):
        """The output rows ([nb][proof_size]) and lengths the prove calls write:
        kept across calls (a prover proves one batch at a time), so a call neither
        zero-fills a fresh buffer nor copies it whole before splitting it."""
        need = self.proof_size * nb
        if self._out is None or len(self._out) < need:
            self._out = (ctypes.c_char * need)()
            self._mv = memoryview(self._out).cast("B")
        if self._lens is None or len(self._lens) < nb:
            self._lens = (ctypes.c_size_t * nb)()
        return self._out, self._lens

    def _proofs(self, nb):
        """The nb serialized proofs of the last call, one copy each."""
        mv, ps, lens = self._mv, self.proof_size, self._lens
        return [mv[i * ps:i * ps + lens[i]].tobytes() for i in range(nb)]

    def _prove(self, nb, what, call):
        """call(out, lens) -> status for nb proofs, under the prover's lock."""
        with self._lock:
            out, lens = self._out_buffers(nb)
            self.ctx.check(call(out, lens), what)
            return self._proofs(nb)

    def verifier_data(self):
        ln = ctypes.c_size_t()
        lib().qp_prover_verifier_data(self.h, None, 0, ctypes.byref(ln))
        buf = ctypes.create_string_buffer(ln.value)
        self.ctx.check(lib().qp_prover_verifier_data(self.h, buf, ln.value, ctypes.byref(ln)), "verifier_data")
        return buf.raw[:ln.value]

    def prove_witnesses(self, witnesses):
        nb = len(witnesses)
        arr = (ctypes.c_void_p * nb)(*[w.h.value for w in witnesses])
        return self._prove(nb, "qp_prover_prove",
                           lambda out, lens: lib().qp_prover_prove(self.h, arr, nb, out, self.proof_size, lens))

    def inputs_array(self, inputs):
        """CircuitInputs / VoteCircuitData list -> contiguous C-ABI struct array."""
        structs = [x.to_c() for x in inputs]
        arr = (type(structs[0]) * len(structs))(*structs)
        arr._keep = structs  # node byte strings referenced by the structs
        return arr

    def prove_inputs_array(self, arr, nb):
        fn = lib().qp_prover_prove_voting_inputs if self.circuit.kind == "voting" else \
            lib().qp_prover_prove_wormhole_inputs
        return self._prove(nb, "qp_prover_prove_inputs",
                           lambda out, lens: fn(self.h, ctypes.cast(arr, ctypes.c_void_p), nb, out, self.proof_size,
                                                lens))

    def prove_inputs(self, inputs):
        """End to end: commit(inputs) + prove() for a list of CircuitInputs (Wormhole)
        or VoteCircuitData (voting) -- commit on the host pool, witness generation on
        the device (qp_prover_prove_{wormhole,voting}_inputs)."""
        if not inputs:
            return []
        return self.prove_inputs_array(self.inputs_array(inputs), len(inputs))

    def prove_aggregation(self, verifier_only: bytes, chunks, zk_randomness=None):
        """aggregate_chunk (tree.rs:106-143) for every chunk of inner proofs as one
        batch: the proof bytes are deserialized into the circuit's targets on the
        host pool, the recursive verifier's witness is generated on the device
        (qp_prover_prove_aggregation).  zk_randomness: per chunk a list of
        num_wires - 4 felts, or None (OS randomness under zk, zeros otherwise)."""
        from .circuits import _zk_ptr
        nb = len(chunks)
        if not nb:
            return []

        class _Chunk(ctypes.Structure):
            _fields_ = [("verifier_only", ctypes.c_char_p), ("vlen", ctypes.c_size_t),
                        ("proofs", ctypes.c_void_p), ("lens", ctypes.c_void_p), ("nproofs", ctypes.c_uint32),
                        ("zk_randomness", ctypes.c_void_p)]

        vo = bytes(verifier_only)
        arr = (_Chunk * nb)()
        keep = [vo]
        for i, ch in enumerate(chunks):
            ps = [bytes(p) for p in ch]
            pa = (ctypes.c_char_p * len(ps))(*ps)
            la = (ctypes.c_size_t * len(ps))(*[len(p) for p in ps])
            zp, zk = _zk_ptr(zk_randomness[i] if zk_randomness is not None else None)
            keep += [ps, pa, la, zk]
            arr[i].verifier_only, arr[i].vlen = vo, len(vo)
            arr[i].proofs, arr[i].lens, arr[i].nproofs = ctypes.cast(pa, ctypes.c_void_p), \
                ctypes.cast(la, ctypes.c_void_p), len(ps)
            arr[i].zk_randomness = ctypes.cast(zp, ctypes.c_void_p) if zp else None
        return self._prove(nb, "qp_prover_prove_aggregation",
                           lambda out, lens: lib().qp_prover_prove_aggregation(
                               self.h, ctypes.cast(arr, ctypes.c_void_p), nb, out, self.proof_size, lens))

    def prove_wires(self, wires, pis):
        wires = np.ascontiguousarray(wires, dtype=np.uint64)
        pis = np.ascontiguousarray(pis, dtype=np.uint64)
        nb = wires.shape[0]
        return self._prove(nb, "qp_prover_prove_wires",
                           lambda out, lens: lib().qp_prover_prove_wires(self.h, wires, pis, nb, out,
                                                                          self.proof_size, lens))

    def prove_wires_dev(self, d_wires_ptr, pis, nproofs):
        """wires already resident on the device (device pointer [nproofs][W][n])."""
        pis = np.ascontiguousarray(pis, dtype=np.uint64)
        return self._prove(nproofs, "qp_prover_prove_wires_dev",
                           lambda out, lens: lib().qp_prover_prove_wires_dev(self.h, d_wires_ptr, pis, nproofs, out,
                                                                              self.proof_size, lens))

    def set_timing(self, enable=True):
        lib().qp_prover_set_timing(self.h, int(enable))

    def debug_force_pow(self, witness, enable=True):
        """TEST-ONLY (qp_prover_debug_force_pow): every proof's PoW witness is
        `witness` instead of the minimal one -- how a reference proof, whose
        find_any witness is nondeterministic, is reproduced byte for byte."""
        self.ctx.check(lib().qp_prover_debug_force_pow(self.h, int(witness), int(enable)), "qp_prover_debug_force_pow")

    def set_host_threads(self, nthreads):
        """Host threads (caller included) of this prover's pool: several provers in
        one process split the host cores instead of each taking min(cores, 16)."""
        self.ctx.check(lib().qp_prover_set_host_threads(self.h, int(nthreads)), "qp_prover_set_host_threads")

    def kernel_stats(self, reset=False):
        ms = (ctypes.c_double * 8)()
        units = (ctypes.c_double * 8)()
        cnt = (ctypes.c_uint64 * 8)()
        lib().qp_prover_kernel_stats(self.h, ms, units, cnt, 8, int(reset))
        names = ["lde_wires", "leaf_hash_wires", "merkle_wires", "quotient"]
        return {nm: {"ms": ms[i], "units": units[i], "launches": cnt[i]} for i, nm in enumerate(names)}

    def stage_times(self, reset=False):
        ms = (ctypes.c_double * 16)()
        lib().qp_prover_stage_times(self.h, ms, 16, int(reset))
        return dict(zip(STAGES, list(ms)[:len(STAGES)]))

    def free(self):
        if self.h:
            lib().qp_prover_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_cache = {}
_lock = threading.Lock()


def _shared(config, device):
    """Circuit + device prover per (config, device): the reference rebuilds in
    WormholeProver::new; here the built circuit and its device preprocessing are
    cached (the role of generated-bins/ in WormholeProver::default, lib.rs:81-101)."""
    key = (config, device)
    with _lock:
        if key not in _cache:
            ctx = Context(device)
            circ = Circuit.wormhole(zero_knowledge=(config == "standard_recursion_zk_config"))
            # one lock per shared prover: its device buffers, host staging and
            # stream serve one prove() at a time (ctypes releases the GIL)
            _cache[key] = (ctx, circ, Prover(ctx, circ, 1), threading.Lock())
        return _cache[key]


CONFIGS = ("standard_recursion_config", "standard_recursion_zk_config")

# prover.bin.  By default generate_circuit_binaries writes upstream plonky2's
# ProverOnlyCircuitData::to_bytes through DefaultGeneratorSerializer, as the
# reference's circuit-builder does (circuit-builder/src/lib.rs:53-59; read back
# by WormholeProver::new_from_bytes, prover/src/lib.rs:104-137): the native
# writer qp_circuit_prover_only_bytes (csrc/prover_bin.cpp, host only) emits the
# generators with their tags and bodies, the watch index, the constants||sigmas
# PolynomialBatch with its Merkle tree, the sigmas' transpose, the subgroup,
# the public-input targets, the representative map, the fft root table and the
# circuit digest.  read_upstream_prover_only walks that layout field by field
# (restated from upstream plonky2's util/serialization; parity unpinned: the
# reference commits no prover.bin -- what IS pinned is the commitment, equal to
# the reference's verifier data), and upstream_prover_layout checks a walked
# file against a circuit.
#
# This backend's own, smaller prover.bin (prover_format="backend") records the
# circuit identity and its preprocessed commitment: magic, version, circuit
# kind, zk flag, degree bits, SHA-256 of common.bin, then the
# VerifierOnlyCircuitData bytes (constants||sigmas cap + circuit digest).
# Loading either rebuilds the native circuit and refuses data whose
# preprocessing differs from it.
PROVER_MAGIC = b"QPGPU-PROVER-ONLY\0"
PROVER_VERSION = 1
_KINDS = {"wormhole": 0, "voting": 1}


_common_memo = {}


def _common_of(cfg):
    """CommonCircuitData bytes of the native Wormhole circuit for a config (memoised:
    building the degree-13 circuit takes ~0.3 s)."""
    with _lock:
        if cfg not in _common_memo:
            _common_memo[cfg] = Circuit.wormhole(zero_knowledge=(cfg == CONFIGS[1])).common_data()
        return _common_memo[cfg]


def _config_of_common(common_bytes):
    """The Wormhole circuit config whose CommonCircuitData::to_bytes equals common_bytes."""
    for cfg in CONFIGS:
        if _common_of(cfg) == bytes(common_bytes):
            return cfg
    return None


def _verifier_only(circuit, prover):
    """VerifierOnlyCircuitData::to_bytes (constants||sigmas cap + circuit digest):
    qp_prover_verifier_data returns it followed by the common data."""
    full = prover.verifier_data()
    common = circuit.common_data()
    assert full.endswith(common)
    return full[:len(full) - len(common)]


def prover_only_bytes(circuit, prover=None, prover_format="upstream"):
    """prover.bin of a built leaf circuit: upstream ProverOnlyCircuitData::to_bytes
    (default; host only) or, with prover_format="backend", this backend's
    identity + commitment blob (needs the circuit's device prover)."""
    if prover_format == "upstream":
        return circuit.prover_only_bytes()
    if prover_format != "backend":
        raise ValueError(f"unknown prover.bin format {prover_format!r}")
    common = circuit.common_data()
    head = PROVER_MAGIC + struct.pack("<IBBI", PROVER_VERSION, _KINDS[circuit.kind], int(circuit.zk),
                                      circuit.degree_bits)
    return head + hashlib.sha256(common).digest() + _verifier_only(circuit, prover)


# plonky2 Goldilocks POWER_OF_TWO_GENERATOR: w_{2^k} = TWO_ADIC_GEN^(2^(32-k))
TWO_ADIC_GEN = 7277203076849721926
_P = 0xFFFFFFFF00000001


def _goldilocks_powers(w, n):
    out = np.empty(n, np.uint64)
    x = 1
    for i in range(n):
        out[i] = x
        x = x * w % _P
    return out


# DefaultGeneratorSerializer (plonky2 util/serialization/generator_serialization.rs):
# tag = index in its generator list; the leaf circuits' kinds and the fields of
# their serialize() bodies (u: usize, f: field, t: target, U: usize vec)
UPSTREAM_GENERATORS = {
    0: ("ArithmeticBaseGenerator", "uffu"),   # row, const_0, const_1, i
    2: ("BaseSplitGenerator", "uu"),          # row, num_limbs
    4: ("ConstantGenerator", "uuuf"),         # row, constant_index, wire_index, constant
    7: ("EqualityGenerator", "tttt"),         # x, y, equal, inv
    15: ("PoseidonGenerator", "u"),           # row
    19: ("RandomValueGenerator", "t"),        # target
    23: ("WireSplitGenerator", "tUu"),        # integer, gates, num_limbs
}


class _Walk:
    """Cursor over upstream plonky2 serialization (little-endian; usize = u64;
    every vector = u64 length + elements)."""

    def __init__(self, data):
        self.d = data
        self.p = 0

    def need(self, k, what):
        if k < 0 or self.p + k > len(self.d):
            raise ValueError(f"truncated in {what} at offset {self.p}")

    def u8(self, what="u8"):
        self.need(1, what)
        self.p += 1
        return self.d[self.p - 1]

    def u32(self, what="u32"):
        self.need(4, what)
        (v,) = struct.unpack_from("<I", self.d, self.p)
        self.p += 4
        return v

    def u64(self, what="usize"):
        self.need(8, what)
        (v,) = struct.unpack_from("<Q", self.d, self.p)
        self.p += 8
        return v

    def u64s(self, n, what):
        if n > (len(self.d) - self.p) // 8:
            raise ValueError(f"truncated in {what} at offset {self.p} ({n} words announced)")
        a = np.frombuffer(self.d, np.uint64, n, self.p)
        self.p += 8 * n
        return a

    def vec(self, what):
        return self.u64s(self.u64(what), what)

    def fields(self, n, what):
        a = self.u64s(n, what)
        if (a >= _P).any():
            raise ValueError(f"non-canonical field element in {what}")
        return a

    def field_vec(self, what):
        return self.fields(self.u64(what), what)

    def target(self, what="target"):
        b = self.u8(what)
        if b == 1:
            return ("wire", self.u64(what), self.u64(what))
        if b == 0:
            return ("virtual", self.u64(what))
        raise ValueError(f"malformed target in {what} at offset {self.p - 1}")


def read_upstream_prover_only(data):
    """Walk an upstream ProverOnlyCircuitData::to_bytes file (plonky2
    write_prover_only_circuit_data, restated; parity unpinned) of a lookup-free
    leaf circuit and return its fields, or raise ValueError naming the first
    thing that does not parse: a truncation, a foreign generator tag, a
    non-canonical element, a malformed section, bytes past the end."""
    data = bytes(data)
    if data[:len(PROVER_MAGIC)] == PROVER_MAGIC:
        raise ValueError("this backend's prover.bin, not an upstream one")
    w = _Walk(data)
    out = {}
    ngen = w.u64("generators")
    if not 0 < ngen <= len(data) // 8:
        raise ValueError(f"implausible generator count {ngen}")
    gens = []
    for i in range(ngen):
        tag = w.u32("generator tag")
        if tag not in UPSTREAM_GENERATORS:
            raise ValueError(f"generator {i}: tag {tag} is not one of the leaf circuits' generator kinds "
                             f"(foreign generator)")
        name, body = UPSTREAM_GENERATORS[tag]
        fields = []
        for k in body:
            if k == "u":
                fields.append(w.u64(name))
            elif k == "f":
                f = w.u64(name)
                if f >= _P:
                    raise ValueError(f"generator {i} ({name}): non-canonical field element")
                fields.append(f)
            elif k == "t":
                fields.append(w.target(name))
            else:
                fields.append([int(x) for x in w.vec(name)])
        gens.append((name, fields))
    out["generators"] = gens
    nw = w.u64("generator_indices_by_watches")
    watches, last = {}, -1
    for _ in range(nw):
        key = w.u64("watch key")
        if key <= last:
            raise ValueError("generator_indices_by_watches keys out of order")
        idx = w.vec("watch indices")
        if len(idx) == 0 or (idx >= ngen).any():
            raise ValueError("generator_indices_by_watches names no or unknown generators")
        watches[key] = idx
        last = key
    out["watches"] = watches
    # constants_sigmas_commitment: PolynomialBatch
    npoly = w.u64("polynomials")
    if not 0 < npoly <= 1024:
        raise ValueError(f"implausible polynomial count {npoly}")
    polys = [w.field_vec(f"polynomial {c}") for c in range(npoly)]
    if len({len(p) for p in polys}) != 1:
        raise ValueError("constants||sigmas polynomials of different lengths")
    out["coeffs"] = np.stack(polys)
    nleaves = w.u64("merkle leaves")
    width = w.u64("merkle leaf") if nleaves else 0
    w.p -= 8 if nleaves else 0
    rows = w.u64s(nleaves * (1 + width), "merkle leaves").reshape(nleaves, 1 + width) if nleaves else None
    if nleaves and ((rows[:, 0] != width).any() or width != npoly):
        raise ValueError("merkle leaves of the wrong width")
    if nleaves and (rows[:, 1:] >= _P).any():
        raise ValueError("non-canonical field element in merkle leaves")
    out["leaves"] = rows[:, 1:] if nleaves else np.zeros((0, 0), np.uint64)
    nd = w.u64("merkle digests")
    out["digests"] = w.fields(4 * nd, "merkle digests").reshape(nd, 4)
    cap_h = w.u64("merkle cap height")
    if cap_h > 20:
        raise ValueError(f"implausible cap height {cap_h}")
    out["cap"] = w.fields(4 << cap_h, "merkle cap")
    if nd != 2 * (nleaves - (1 << cap_h)) if nleaves >= (1 << cap_h) else nd != 0:
        raise ValueError(f"{nd} digests for {nleaves} leaves under a height-{cap_h} cap")
    out["degree_log"] = w.u64("degree_log")
    out["rate_bits"] = w.u64("rate_bits")
    out["blinding"] = w.u8("blinding")
    if out["blinding"] > 1:
        raise ValueError("malformed blinding flag")
    n = 1 << out["degree_log"] if out["degree_log"] < 32 else 0
    if out["coeffs"].shape[1] != n or nleaves != n << out["rate_bits"]:
        raise ValueError("polynomial / leaf counts disagree with degree_log and rate_bits")
    # sigmas: the transpose of the sigma polynomials, n rows
    nrows = w.u64("sigmas")
    if nrows != n:
        raise ValueError(f"{nrows} sigma rows for degree {n}")
    r0 = w.u64("sigma row")
    w.p -= 8
    sg = w.u64s(nrows * (1 + r0), "sigmas").reshape(nrows, 1 + r0)
    if (sg[:, 0] != r0).any() or (sg[:, 1:] >= _P).any():
        raise ValueError("malformed sigma rows")
    out["sigmas"] = sg[:, 1:]
    out["subgroup"] = w.field_vec("subgroup")
    npi = w.u64("public inputs")
    if npi > len(data):
        raise ValueError("implausible public-input count")
    out["public_inputs"] = [w.target("public inputs") for _ in range(npi)]
    rep = w.vec("representative_map")
    if len(rep) < n * 1 or (rep >= len(rep)).any() or (rep[rep] != rep).any():
        raise ValueError("representative_map is not a compressed forest")
    out["representative_map"] = rep
    has = w.u8("fft_root_table")
    table = None
    if has == 1:
        table = [w.field_vec("fft_root_table row") for _ in range(w.u64("fft_root_table"))]
    elif has != 0:
        raise ValueError("malformed fft_root_table flag")
    out["fft_root_table"] = table
    out["circuit_digest"] = tuple(int(x) for x in w.fields(4, "circuit digest"))
    if w.u64("lookup_rows") != 0 or w.u64("lut_to_lookups") != 0:
        raise ValueError("lookup tables present (the leaf circuits have none)")
    if w.p != len(data):
        raise ValueError(f"{len(data) - w.p} bytes past lut_to_lookups")
    return out


def _hash(v):
    from ._native import hash_no_pad
    return hash_no_pad(np.asarray(v, np.uint64))


def _merkle_subtree_ok(leaves, digests, cap, k, ncap):
    """hash/merkle_tree.rs fill_subtree layout of cap subtree k: rebuild its
    digests from its leaves and compare them and the cap entry."""
    nl = len(leaves) // ncap
    nd = len(digests) // ncap
    L = leaves[k * nl:(k + 1) * nl]
    D = digests[k * nd:(k + 1) * nd]

    def fill(lo, nleaves, dlo, nd_):
        if nd_ == 0:
            row = L[lo]
            return _hash(row) if len(row) > 4 else [int(x) for x in row] + [0] * (4 - len(row))
        half = nd_ // 2
        left = fill(lo, nleaves // 2, dlo, half - 1)
        right = fill(lo + nleaves // 2, nleaves // 2, dlo + half + 1, half - 1)
        if [int(x) for x in D[dlo + half - 1]] != left or [int(x) for x in D[dlo + half]] != right:
            raise ValueError(f"merkle digests of cap subtree {k} do not hash up from its leaves")
        return _hash(left + right)
    if fill(0, nl, 0, nd) != [int(x) for x in cap[4 * k:4 * k + 4]]:
        raise ValueError(f"cap entry {k} is not the root of its subtree")


def upstream_prover_layout(data, circuit, cap=None, check_subtrees=1):
    """Walk an upstream prover.bin (read_upstream_prover_only) and check it
    against `circuit`; return its circuit digest (4 ints), or raise ValueError.
    Checked: the generators are the circuit's kinds and counts (one
    PoseidonGenerator per Poseidon row, num_ops ArithmeticBaseGenerators per
    arithmetic row, one BaseSplitGenerator per BaseSum row, the PublicInputGate
    row's RandomValueGenerators), the constants||sigmas coefficients, degree,
    rate and blinding, the sigmas, the subgroup, the public-input count, the
    fft root table; the Merkle cap (against `cap` when given: the caller's
    device-computed or reference one), the first `check_subtrees` cap subtrees
    rebuilt from their leaves, the leaves' first row against the coefficients'
    value at g (the coset LDE's first leaf), and the digest as
    hash_no_pad(cap || hash_pad([]) || degree_bits)."""
    f = read_upstream_prover_only(data)
    n = circuit.n
    if f["degree_log"] != circuit.degree_bits or f["rate_bits"] != 3 or f["blinding"]:
        raise ValueError("degree, rate or blinding differ from this circuit's")
    co = circuit.constants_sigmas_coeffs()
    if f["coeffs"].shape != co.shape:
        raise ValueError("constants||sigmas polynomial count differs from this circuit's")
    for c in range(co.shape[0]):
        if not np.array_equal(f["coeffs"][c], co[c]):
            raise ValueError(f"constants||sigmas coefficient column {c} differs from this circuit's")
    vals = circuit.constants_sigmas()
    sig = vals[circuit.num_constants:]
    if f["sigmas"].shape != (n, sig.shape[0]) or not np.array_equal(f["sigmas"], sig.T):
        raise ValueError("sigma rows differ from this circuit's sigma columns")
    wn = pow(TWO_ADIC_GEN, 1 << (32 - circuit.degree_bits), _P)
    if not np.array_equal(f["subgroup"], _goldilocks_powers(wn, n)):
        raise ValueError("subgroup is not the powers of w_n")
    if len(f["public_inputs"]) != circuit.num_public_inputs:
        raise ValueError(f"{len(f['public_inputs'])} public-input targets, the circuit has "
                         f"{circuit.num_public_inputs}")
    gk, rows = circuit.census()
    count = {}
    for name, _ in f["generators"]:
        count[name] = count.get(name, 0) + 1
    want = {"PoseidonGenerator": rows["poseidon"], "BaseSplitGenerator": rows["base_sum"],
            "ArithmeticBaseGenerator": rows["arithmetic"] * (circuit.num_routed_wires // 4),
            "RandomValueGenerator": circuit.num_wires - 4}
    for name, k in want.items():
        if count.get(name, 0) != k:
            raise ValueError(f"{count.get(name, 0)} {name}s, the circuit needs {k}")
    tab = f["fft_root_table"]
    if tab is None or [len(r) for r in tab] != [max(1 << (m - 1), 2) for m in range(1, len(tab) + 1)]:
        raise ValueError("fft_root_table missing or of the wrong shape")
    fcap = f["cap"]
    if cap is not None and not np.array_equal(fcap, np.asarray(cap, np.uint64)):
        raise ValueError("constants||sigmas Merkle cap differs from this circuit's")
    # leaf 0 is the LDE at g (rev(0) = 0): each column's polynomial at the shift
    g0 = [0] * co.shape[0]
    for c in range(co.shape[0]):
        acc = 0
        for x in reversed([int(v) for v in co[c]]):
            acc = (acc * 0xC65C18B67785D900 + x) % _P
        g0[c] = acc
    if [int(x) for x in f["leaves"][0]] != g0:
        raise ValueError("merkle leaf 0 is not the constants||sigmas LDE at the coset shift")
    ncap = len(fcap) // 4
    for k in range(min(check_subtrees, ncap)):
        _merkle_subtree_ok(f["leaves"], f["digests"], fcap, k, ncap)
    dsep = _hash([1, 0, 0, 0, 0, 0, 0, 1])
    if tuple(_hash(list(fcap) + dsep + [circuit.degree_bits])) != f["circuit_digest"]:
        raise ValueError("circuit digest is not the hash of the cap and degree")
    return f["circuit_digest"]


def _parse_prover_only(data, common_bytes, circuit=None, vo=None):
    """-> (zk, degree_bits, VerifierOnlyCircuitData bytes) for this backend's
    prover.bin, or (None, None, circuit digest) for an upstream one, which is
    walked (upstream_prover_layout) against `circuit` and the constants||sigmas
    cap of its VerifierOnlyCircuitData bytes `vo`."""
    data = bytes(data)
    n = len(PROVER_MAGIC)
    if data[:n] != PROVER_MAGIC:
        if len(data) < 8 + 48 or data[-16:] != bytes(16):
            raise ValueError("neither this backend's prover.bin (bad magic) nor an upstream plonky2 "
                             "ProverOnlyCircuitData::to_bytes file of a lookup-free circuit")
        if circuit is None:
            raise ValueError("an upstream prover.bin needs the circuit to be checked against")
        cap = None
        if vo is not None:
            (h,) = struct.unpack_from("<Q", vo, 0)
            cap = np.frombuffer(vo, np.uint64, 4 << h, 8)
        return None, None, upstream_prover_layout(data, circuit, cap)
    if len(data) < n + 10 + 32:
        raise ValueError("truncated prover.bin header")
    version, kind, zk, degree_bits = struct.unpack_from("<IBBI", data, n)
    if version != PROVER_VERSION:
        raise ValueError(f"unsupported version {version}")
    if kind != _KINDS["wormhole"]:
        raise ValueError("not a Wormhole circuit")
    off = n + 10
    if data[off:off + 32] != hashlib.sha256(bytes(common_bytes)).digest():
        raise ValueError("prover data was written for different common data")
    # the header's config must agree with the common data it was written for
    # (CommonCircuitData: config.zero_knowledge at byte 49; FriParams.degree_bits
    # follows the two FriConfigs and the reduction arity list)
    cb = bytes(common_bytes)
    if len(cb) > 49 and bool(cb[49]) != bool(zk):
        raise ValueError("prover data header zk flag disagrees with the common data")
    c_db = _common_degree_bits(cb)
    if c_db is not None and c_db != degree_bits:
        raise ValueError(f"prover data header degree_bits {degree_bits} disagrees with the common data ({c_db})")
    return bool(zk), degree_bits, data[off + 32:]


def _same_preprocessing(mine, parsed):
    """This circuit's VerifierOnlyCircuitData bytes vs what a prover.bin holds:
    the whole VerifierOnlyCircuitData (this backend's file) or the circuit
    digest (an upstream file; the last 32 bytes of VerifierOnlyCircuitData)."""
    if isinstance(parsed, tuple):
        return struct.unpack_from("<4Q", mine, len(mine) - 32) == parsed
    return mine == parsed


def _common_degree_bits(cb):
    """FriParams.degree_bits of CommonCircuitData bytes, or None."""
    try:
        off = 6 * 8 + 2                      # six u64 config fields, two u8 flags
        fri = 8 * 3 + 4 + 1 + 16             # FriConfig: rate, cap, queries, pow u32, strategy tag + 2 u64
        off += fri + fri                     # CircuitConfig.fri_config, FriParams.config
        (na,) = struct.unpack_from("<Q", cb, off)
        off += 8 + 8 * na
        (db,) = struct.unpack_from("<Q", cb, off)
        return int(db)
    except struct.error:
        return None


def generate_circuit_binaries(output_dir, include_prover=True, config="standard_recursion_config", device=0,
                              prover_format="upstream"):
    """wormhole/circuit-builder/src/lib.rs:11-66: build the circuit and write
    common.bin (CommonCircuitData::to_bytes), verifier.bin
    (VerifierOnlyCircuitData::to_bytes) and, if asked, prover.bin: upstream
    ProverOnlyCircuitData::to_bytes (default) or this backend's identity +
    commitment blob (prover_format="backend", see PROVER_MAGIC)."""
    ctx, circ, prover, lock = _shared(config, device)
    os.makedirs(output_dir, exist_ok=True)
    with open(os.path.join(output_dir, "common.bin"), "wb") as f:
        f.write(circ.common_data())
    with lock:
        vd = _verifier_only(circ, prover)
        pb = prover_only_bytes(circ, prover, prover_format) if include_prover else None
    with open(os.path.join(output_dir, "verifier.bin"), "wb") as f:
        f.write(vd)
    if include_prover:
        with open(os.path.join(output_dir, "prover.bin"), "wb") as f:
            f.write(pb)


class WormholeProver:
    def __init__(self, config="standard_recursion_config", device=0):
        if config not in CONFIGS:
            raise ValueError(f"unknown circuit config {config!r}")
        self.config = config
        self.ctx, self.circuit, self.prover, self._prove_lock = _shared(config, device)
        self._witness = None
        self._committed = False

    @classmethod
    def new_from_bytes(cls, prover_only_bytes, common_bytes, device=0):
        """WormholeProver::new_from_bytes (lib.rs:105-138): the config comes from
        the common data; errors carry the reference's messages."""
        cfg = _config_of_common(common_bytes)
        if cfg is None:
            raise ValueError("Failed to deserialize common circuit data")
        self = cls(cfg, device)
        with self._prove_lock:
            mine = _verifier_only(self.circuit, self.prover)
        try:
            _, _, vd = _parse_prover_only(prover_only_bytes, common_bytes, self.circuit, mine)
        except ValueError as e:
            raise ValueError(f"Failed to deserialize prover only data: {e}") from None
        if not _same_preprocessing(mine, vd):
            raise ValueError("Failed to deserialize prover only data: preprocessed commitment differs")
        return self

    @classmethod
    def new_from_files(cls, prover_data_path, common_data_path, device=0):
        """WormholeProver::new_from_files (lib.rs:141-187)."""
        with open(common_data_path, "rb") as f:
            common = f.read()
        cfg = _config_of_common(common)
        if cfg is None:
            raise ValueError(f"Failed to deserialize common circuit data from {str(common_data_path)!r}")
        with open(prover_data_path, "rb") as f:
            pb = f.read()
        self = cls(cfg, device)
        with self._prove_lock:
            mine = _verifier_only(self.circuit, self.prover)
        try:
            _, _, vd = _parse_prover_only(pb, common, self.circuit, mine)
        except ValueError as e:
            raise ValueError(f"Failed to deserialize prover only data from {str(prover_data_path)!r}: {e}") from None
        if not _same_preprocessing(mine, vd):
            raise ValueError(f"Failed to deserialize prover only data from {str(prover_data_path)!r}: "
                             "preprocessed commitment differs")
        return self

    @classmethod
    def default(cls, device=0):
        """WormholeProver::default (lib.rs:81-101): generated-bins/ if loadable, else build."""
        pb, cb = os.path.join("generated-bins", "prover.bin"), os.path.join("generated-bins", "common.bin")
        if not (os.path.exists(pb) and os.path.exists(cb)):
            return cls("standard_recursion_config", device)
        try:
            return cls.new_from_files(pb, cb, device)
        except (OSError, ValueError) as e:
            warnings.warn(f"WormholeProver::default: ignoring generated-bins ({e}); building the circuit")
            return cls("standard_recursion_config", device)

    def commit(self, inputs: CircuitInputs):
        if self._committed:
            raise QpError(4, "prover has already commited to inputs")
        self._witness = self.circuit.commit(inputs)
        self._committed = True
        return self

    def prove(self) -> ProofWithPublicInputs:
        if self._witness is None:
            raise QpError(4, "prover has not commited to any inputs")
        w = self._witness
        self._witness = None
        with self._prove_lock:
            data = self.prover.prove_witnesses([w])[0]
        return ProofWithPublicInputs(data, w.public_inputs())
