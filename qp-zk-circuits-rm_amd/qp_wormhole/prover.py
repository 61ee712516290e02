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

    def verifier_data(self):
        ln = ctypes.c_size_t()
        lib().qp_prover_verifier_data(self.h, None, 0, ctypes.byref(ln))
        buf = ctypes.create_string_buffer(ln.value)
        self.ctx.check(lib().qp_prover_verifier_data(self.h, buf, ln.value, ctypes.byref(ln)), "verifier_data")
        return buf.raw[:ln.value]

    def prove_witnesses(self, witnesses):
        nb = len(witnesses)
        arr = (ctypes.c_void_p * nb)(*[w.h.value for w in witnesses])
        out = ctypes.create_string_buffer(self.proof_size * nb)
        lens = (ctypes.c_size_t * nb)()
        self.ctx.check(lib().qp_prover_prove(self.h, arr, nb, out, self.proof_size, lens), "qp_prover_prove")
        raw = out.raw
        return [raw[i * self.proof_size:i * self.proof_size + lens[i]] for i in range(nb)]

    def inputs_array(self, inputs):
        """CircuitInputs / VoteCircuitData list -> contiguous C-ABI struct array."""
        structs = [x.to_c() for x in inputs]
        arr = (type(structs[0]) * len(structs))(*structs)
        arr._keep = structs  # node byte strings referenced by the structs
        return arr

    def prove_inputs_array(self, arr, nb):
        out = ctypes.create_string_buffer(self.proof_size * nb)
        lens = (ctypes.c_size_t * nb)()
        fn = lib().qp_prover_prove_voting_inputs if self.circuit.kind == "voting" else \
            lib().qp_prover_prove_wormhole_inputs
        self.ctx.check(fn(self.h, ctypes.cast(arr, ctypes.c_void_p), nb, out, self.proof_size, lens),
                       "qp_prover_prove_inputs")
        raw = out.raw
        return [raw[i * self.proof_size:i * self.proof_size + lens[i]] for i in range(nb)]

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
        out = ctypes.create_string_buffer(self.proof_size * nb)
        lens = (ctypes.c_size_t * nb)()
        self.ctx.check(lib().qp_prover_prove_aggregation(self.h, ctypes.cast(arr, ctypes.c_void_p), nb, out,
                                                         self.proof_size, lens), "qp_prover_prove_aggregation")
        raw = out.raw
        return [raw[i * self.proof_size:i * self.proof_size + lens[i]] for i in range(nb)]

    def prove_wires(self, wires, pis):
        wires = np.ascontiguousarray(wires, dtype=np.uint64)
        pis = np.ascontiguousarray(pis, dtype=np.uint64)
        nb = wires.shape[0]
        out = ctypes.create_string_buffer(self.proof_size * nb)
        lens = (ctypes.c_size_t * nb)()
        self.ctx.check(lib().qp_prover_prove_wires(self.h, wires, pis, nb, out, self.proof_size, lens),
                       "qp_prover_prove_wires")
        raw = out.raw
        return [raw[i * self.proof_size:i * self.proof_size + lens[i]] for i in range(nb)]

    def prove_wires_dev(self, d_wires_ptr, pis, nproofs):
        """wires already resident on the device (device pointer [nproofs][W][n])."""
        pis = np.ascontiguousarray(pis, dtype=np.uint64)
        out = ctypes.create_string_buffer(self.proof_size * nproofs)
        lens = (ctypes.c_size_t * nproofs)()
        self.ctx.check(lib().qp_prover_prove_wires_dev(self.h, d_wires_ptr, pis, nproofs, out, self.proof_size, lens),
                       "qp_prover_prove_wires_dev")
        raw = out.raw
        return [raw[i * self.proof_size:i * self.proof_size + lens[i]] for i in range(nproofs)]

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

# prover.bin of this backend.  plonky2's ProverOnlyCircuitData::to_bytes
# (generators through DefaultGeneratorSerializer, the constants||sigmas
# PolynomialBatch, fft root table, ...) has no fixture in the reference
# (generated-bins/ is empty) and would be rebuilt by the device preprocessing
# anyway, so the file records the circuit identity and its preprocessed
# commitment: magic, version, circuit kind, zk flag, degree bits, SHA-256 of
# common.bin, then the VerifierOnlyCircuitData bytes (constants||sigmas cap +
# circuit digest).  Loading rebuilds the native circuit for that identity and
# refuses data whose commitment differs.
#
# An upstream prover.bin (ProverOnlyCircuitData::to_bytes of the reference's
# generate_circuit_binaries, circuit-builder/src/lib.rs:54-60; read back by
# WormholeProver::new_from_bytes, prover/src/lib.rs:105-137) is walked by
# upstream_prover_layout: the framing is restated from upstream plonky2's
# write_prover_only_circuit_data (parity unpinned: the reference commits no
# such file) and the walk checks the CONTENT the preprocessing fixes, so a
# truncated or foreign blob is refused even if it ends like one.  The native
# circuit IS the reference's (same constants||sigmas columns, cap and circuit
# digest: tests/test_reference_layout.py), so a file of the reference's circuit
# passes; its generators are not needed (witness generation is native).
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


def prover_only_bytes(circuit, prover):
    """This backend's prover.bin for a built circuit and its device prover."""
    common = circuit.common_data()
    head = PROVER_MAGIC + struct.pack("<IBBI", PROVER_VERSION, _KINDS[circuit.kind], int(circuit.zk),
                                      circuit.degree_bits)
    return head + hashlib.sha256(common).digest() + _verifier_only(circuit, prover)


# plonky2 Goldilocks POWER_OF_TWO_GENERATOR: w_{2^k} = TWO_ADIC_GEN^(2^(32-k))
TWO_ADIC_GEN = 7277203076849721926


def _goldilocks_powers(w, n):
    out = np.empty(n, np.uint64)
    x = 1
    for i in range(n):
        out[i] = x
        x = x * w % 0xFFFFFFFF00000001
    return out


def upstream_prover_layout(data, circuit, cap=None):
    """Walk an upstream ProverOnlyCircuitData::to_bytes file of `circuit` and
    return its circuit digest (4 ints), or raise ValueError naming what is
    missing.  Restated framing (plonky2 util/serialization write_prover_only_
    circuit_data), in file order:
      generators.len() u64, the generators (tag u32 + body each),
      generator_indices_by_watches, then the constants||sigmas PolynomialBatch:
      polynomials.len() u64 and per polynomial its coefficients as a field vec
      (u64 length + values), the MerkleTree (leaves, digests, cap: u64 length +
      16 hashes), degree_log, rate_bits, blinding; sigmas.len() u64 and the
      sigma value vectors; the subgroup (powers of w_n); public-input targets;
      representative_map; the fft root table (optional); circuit_digest
      (4 u64); lookup_rows and lut_to_lookups (empty: two u64 zeros).
    What is checked is what the preprocessing fixes: this circuit's
    constants||sigmas coefficients (every column, consecutive), the cap
    (when given: the caller's device-computed one), the 80 sigma value
    columns, the subgroup, and the empty lookup tail.  The generator bodies and
    the Merkle leaves/digests are skipped by search, so only their presence is
    restated, not their layout."""
    data = bytes(data)
    if data[:len(PROVER_MAGIC)] == PROVER_MAGIC:
        raise ValueError("this backend's prover.bin, not an upstream one")
    if len(data) < 8 + 48 or data[-16:] != bytes(16):
        raise ValueError("does not end with the circuit digest and empty lookup tables")
    (ngen,) = struct.unpack_from("<Q", data, 0)
    dig = struct.unpack_from("<4Q", data, len(data) - 48)
    if not 0 < ngen < len(data) // 8 or any(x >= 0xFFFFFFFF00000001 for x in dig):
        raise ValueError("implausible generator count or non-canonical digest")
    n = circuit.n
    N = struct.pack("<Q", n)
    coeffs = circuit.constants_sigmas_coeffs()
    vals = circuit.constants_sigmas()
    ncs = coeffs.shape[0]

    def column(pos, arr, what):
        blob = N + arr.tobytes()
        if data[pos:pos + len(blob)] != blob:
            raise ValueError(f"{what} does not follow at offset {pos}")
        return pos + len(blob)

    # the PolynomialBatch's coefficient columns: located by column 0, then every
    # column must follow at the same gap (0 or 8 extra bytes per polynomial)
    p0 = data.find(N + coeffs[0].tobytes(), 8 + 8 * ngen)
    if p0 < 0:
        raise ValueError("constants||sigmas coefficients of this circuit not found")
    if struct.pack("<Q", ncs) not in data[max(0, p0 - 16):p0]:
        raise ValueError("polynomial count missing before the coefficients")
    e = p0 + 8 + 8 * n
    gap = None
    for g in (0, 8):
        if data[e + g:e + g + 8 + 8 * n] == N + coeffs[1].tobytes():
            gap = g
            break
    if gap is None:
        raise ValueError("constants||sigmas coefficient column 1 does not follow column 0")
    for c in range(1, ncs):
        e = column(e + gap, coeffs[c], f"coefficient column {c}")
    # the Merkle tree's cap (the leaves and digests precede it)
    pos = e
    if cap is not None:
        cb = struct.pack("<Q", len(cap) // 4) + np.ascontiguousarray(cap, dtype=np.uint64).tobytes()
        pc = data.find(cb, e)
        if pc < 0:
            raise ValueError("constants||sigmas Merkle cap differs from this circuit's")
        pos = pc + len(cb)
    # sigmas: count, then the value vectors
    nsig = ncs - circuit.num_constants
    ps = data.find(struct.pack("<Q", nsig) + N + vals[circuit.num_constants].tobytes(), pos)
    if ps < 0:
        raise ValueError("sigma columns of this circuit not found")
    e = ps + 8
    for j in range(nsig):
        e = column(e, vals[circuit.num_constants + j], f"sigma column {j}")
    # subgroup: powers of w_n
    w = pow(TWO_ADIC_GEN, 1 << (32 - circuit.degree_bits), 0xFFFFFFFF00000001)
    e = column(e, _goldilocks_powers(w, n), "subgroup")
    # public_inputs: target vec (write_target: bool Wire? + row, column | index)
    end = len(data) - 48
    try:
        (npi,) = struct.unpack_from("<Q", data, e)
        if npi != circuit.num_public_inputs:
            raise ValueError(f"{npi} public-input targets, the circuit has {circuit.num_public_inputs}")
        e += 8
        for _ in range(npi):
            e += 17 if data[e] == 1 else 9 if data[e] == 0 else 1 << 62
        # representative_map: one entry per wire target and virtual target
        (nrep,) = struct.unpack_from("<Q", data, e)
        if nrep < n * circuit.num_wires:
            raise ValueError(f"representative_map of {nrep} entries for {n} x {circuit.num_wires} wires")
        e += 8 + 8 * nrep
        # fft_root_table: Option<Vec<Vec<F>>>
        if data[e] == 1:
            (k,) = struct.unpack_from("<Q", data, e + 1)
            e += 9
            for _ in range(k):
                (m,) = struct.unpack_from("<Q", data, e)
                e += 8 + 8 * m
        elif data[e] == 0:
            e += 1
        else:
            raise ValueError("malformed fft_root_table")
    except (struct.error, IndexError):
        raise ValueError("truncated after the subgroup") from None
    if e != end:
        raise ValueError(f"{end - e} bytes between the fft root table and the circuit digest")
    return dig


def upstream_prover_digest(data):
    """Circuit digest of a blob that ENDS like an upstream prover.bin (no
    structural walk; upstream_prover_layout does that), or None."""
    data = bytes(data)
    if data[:len(PROVER_MAGIC)] == PROVER_MAGIC or len(data) < 8 + 48 or data[-16:] != bytes(16):
        return None
    (ngen,) = struct.unpack_from("<Q", data, 0)
    dig = struct.unpack_from("<4Q", data, len(data) - 48)
    if not 0 < ngen < len(data) or any(x >= 0xFFFFFFFF00000001 for x in dig):
        return None
    return dig


def _parse_prover_only(data, common_bytes, circuit=None, vo=None):
    """-> (zk, degree_bits, VerifierOnlyCircuitData bytes) for this backend's
    prover.bin, or (None, None, circuit digest) for an upstream one, which is
    walked (upstream_prover_layout) against `circuit` and the constants||sigmas
    cap of its VerifierOnlyCircuitData bytes `vo`."""
    data = bytes(data)
    n = len(PROVER_MAGIC)
    if data[:n] != PROVER_MAGIC and upstream_prover_digest(data) is not None:
        if circuit is None:
            raise ValueError("an upstream prover.bin needs the circuit to be checked against")
        cap = None
        if vo is not None:
            (h,) = struct.unpack_from("<Q", vo, 0)
            cap = np.frombuffer(vo, np.uint64, 4 << h, 8)
        return None, None, upstream_prover_layout(data, circuit, cap)
    if len(data) < n + 10 + 32 or data[:n] != PROVER_MAGIC:
        raise ValueError("neither this backend's prover.bin (bad magic) nor an upstream plonky2 "
                         "ProverOnlyCircuitData::to_bytes file of a lookup-free circuit")
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


def generate_circuit_binaries(output_dir, include_prover=True, config="standard_recursion_config", device=0):
    """wormhole/circuit-builder/src/lib.rs:11-66: build the circuit and write
    common.bin (CommonCircuitData::to_bytes), verifier.bin
    (VerifierOnlyCircuitData::to_bytes) and, if asked, prover.bin (this
    backend's format, see PROVER_MAGIC)."""
    ctx, circ, prover, lock = _shared(config, device)
    os.makedirs(output_dir, exist_ok=True)
    with open(os.path.join(output_dir, "common.bin"), "wb") as f:
        f.write(circ.common_data())
    with lock:
        vd = _verifier_only(circ, prover)
        pb = prover_only_bytes(circ, prover) if include_prover else None
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
