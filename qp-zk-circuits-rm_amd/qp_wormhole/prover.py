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
# generate_circuit_binaries, circuit-builder/src/lib.rs:54-60) is accepted by
# its circuit digest: plonky2 writes the digest (HashOut, 4 u64) right before
# the lookup tables, which are two empty vectors (u64 length 0 each) for a
# lookup-free circuit such as Wormhole, so the file ends with digest || 0u64 ||
# 0u64.  The native circuit IS the reference's (same constants||sigmas cap and
# circuit digest: tests/test_reference_layout.py), so an equal digest means the
# file describes this circuit's preprocessing; its generators are not needed
# (witness generation is native).
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


def upstream_prover_digest(data):
    """Circuit digest (4 u64) of an upstream ProverOnlyCircuitData::to_bytes file of a
    lookup-free circuit, or None when `data` does not end like one."""
    data = bytes(data)
    if data[:len(PROVER_MAGIC)] == PROVER_MAGIC or len(data) < 8 + 48 or data[-16:] != bytes(16):
        return None
    (ngen,) = struct.unpack_from("<Q", data, 0)   # generators.len() opens the file
    dig = struct.unpack_from("<4Q", data, len(data) - 48)
    if not 0 < ngen < len(data) or any(x >= 0xFFFFFFFF00000001 for x in dig):
        return None
    return dig


def _parse_prover_only(data, common_bytes):
    """-> (zk, degree_bits, VerifierOnlyCircuitData bytes) for this backend's
    prover.bin, or (None, None, circuit digest) for an upstream one."""
    data = bytes(data)
    n = len(PROVER_MAGIC)
    if data[:n] != PROVER_MAGIC:
        dig = upstream_prover_digest(data)
        if dig is not None:
            return None, None, dig
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
        try:
            _, _, vd = _parse_prover_only(prover_only_bytes, common_bytes)
        except ValueError as e:
            raise ValueError(f"Failed to deserialize prover only data: {e}") from None
        self = cls(cfg, device)
        with self._prove_lock:
            mine = _verifier_only(self.circuit, self.prover)
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
        try:
            _, _, vd = _parse_prover_only(pb, common)
        except ValueError as e:
            raise ValueError(f"Failed to deserialize prover only data from {str(prover_data_path)!r}: {e}") from None
        self = cls(cfg, device)
        with self._prove_lock:
            if not _same_preprocessing(_verifier_only(self.circuit, self.prover), vd):
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
