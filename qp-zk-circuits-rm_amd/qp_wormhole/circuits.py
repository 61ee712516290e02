"""Host-side mirror of the reference's circuit / prover input types.

VoteCircuitData mirrors voting/src/lib.rs:26-52, :113-121 (VotePublicInputs +
VotePrivateInputs); Circuit.voting() builds the native voting circuit
(VoteTargets::new + VoteCircuitData::circuit, voting/src/lib.rs:71-197).

CircuitInputs mirrors wormhole/circuit/src/inputs.rs:21-52 (public +
private inputs); WormholeCircuit builds the native circuit
(wormhole/circuit/src/circuit.rs:63-109) through the C ABI; Witness is the
result of WormholeProver::commit (wormhole/prover/src/lib.rs:209-225).
"""
import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from ._native import QpError, lib

U8_32 = ctypes.c_uint8 * 32


class _Inputs(ctypes.Structure):
    _fields_ = [("funding_amount", ctypes.c_uint8 * 16), ("nullifier", U8_32), ("root_hash", U8_32),
                ("exit_account", U8_32), ("secret", U8_32), ("transfer_count", ctypes.c_uint64),
                ("funding_account", U8_32), ("unspendable_account", U8_32), ("num_nodes", ctypes.c_uint32),
                ("nodes", ctypes.POINTER(ctypes.c_char_p)), ("node_lens", ctypes.POINTER(ctypes.c_uint32)),
                ("indices", ctypes.POINTER(ctypes.c_uint64)), ("zk_randomness", ctypes.POINTER(ctypes.c_uint64))]


@dataclass
class ProcessedStorageProof:
    """storage_proof/mod.rs:58-76: node byte strings + hex-char child-hash indices."""
    proof: List[bytes] = field(default_factory=list)
    indices: List[int] = field(default_factory=list)

    def validate(self):
        if len(self.proof) != len(self.indices):
            raise ValueError("indices length must be equal to proof length, actual lengths: "
                             f"{len(self.proof)}, {len(self.indices)}")


@dataclass
class PublicCircuitInputs:
    funding_amount: int
    nullifier: bytes
    root_hash: bytes
    exit_account: bytes


@dataclass
class PrivateCircuitInputs:
    secret: bytes
    storage_proof: ProcessedStorageProof
    transfer_count: int
    funding_account: bytes
    unspendable_account: bytes


@dataclass
class CircuitInputs:
    public: PublicCircuitInputs
    private: PrivateCircuitInputs
    # zk config only: the random cells of the PublicInputGate row (see _zk_ptr)
    zk_randomness: Optional[List[int]] = None

    def to_c(self):
        s = _Inputs()
        s.funding_amount[:] = list(int(self.public.funding_amount).to_bytes(16, "little"))
        s.nullifier[:] = list(self.public.nullifier)
        s.root_hash[:] = list(self.public.root_hash)
        s.exit_account[:] = list(self.public.exit_account)
        s.secret[:] = list(self.private.secret)
        s.transfer_count = self.private.transfer_count
        s.funding_account[:] = list(self.private.funding_account)
        s.unspendable_account[:] = list(self.private.unspendable_account)
        sp = self.private.storage_proof
        sp.validate()
        n = len(sp.proof)
        s.num_nodes = n
        keep = [bytes(p) for p in sp.proof]
        s.nodes = (ctypes.c_char_p * max(n, 1))(*keep) if n else None
        s.node_lens = (ctypes.c_uint32 * max(n, 1))(*[len(p) for p in keep]) if n else None
        s.indices = (ctypes.c_uint64 * max(len(sp.indices), 1))(*sp.indices) if n else None
        s.zk_randomness, zk_keep = _zk_ptr(self.zk_randomness)
        s._keep = (keep, zk_keep)
        return s


U64_4 = ctypes.c_uint64 * 4


class _VoteInputs(ctypes.Structure):
    _fields_ = [("proposal_id", U64_4), ("merkle_root", U64_4), ("nullifier", U64_4), ("vote", ctypes.c_uint8),
                ("private_key", U64_4), ("num_siblings", ctypes.c_uint32),
                ("siblings", ctypes.POINTER(ctypes.c_uint64)), ("num_path_indices", ctypes.c_uint32),
                ("path_indices", ctypes.POINTER(ctypes.c_uint8)), ("actual_merkle_depth", ctypes.c_uint64),
                ("zk_randomness", ctypes.POINTER(ctypes.c_uint64))]


def _zk_ptr(values):
    """zk config: values of the PublicInputGate row's unused wires (num_wires - 4
    felts; plonky2 randomize_unused_pi_wires).  None = derived from the private
    inputs by the library (deterministic Poseidon nonce)."""
    if values is None:
        return None, None
    keep = (ctypes.c_uint64 * len(values))(*[int(v) for v in values])
    return ctypes.cast(keep, ctypes.POINTER(ctypes.c_uint64)), keep


@dataclass
class VotePublicInputs:
    """voting/src/lib.rs:26-36 (digests are 4 field elements)."""
    proposal_id: List[int]
    merkle_root: List[int]
    vote: bool
    nullifier: List[int]


@dataclass
class VotePrivateInputs:
    """voting/src/lib.rs:42-52."""
    private_key: List[int]
    merkle_siblings: List[List[int]]
    path_indices: List[bool]
    actual_merkle_depth: int


@dataclass
class VoteCircuitData:
    """voting/src/lib.rs:113-121: the witness data fill_targets consumes."""
    public_inputs: VotePublicInputs
    private_inputs: VotePrivateInputs
    zk_randomness: Optional[List[int]] = None

    def to_c(self):
        s = _VoteInputs()
        pub, prv = self.public_inputs, self.private_inputs
        s.proposal_id[:] = list(pub.proposal_id)
        s.merkle_root[:] = list(pub.merkle_root)
        s.nullifier[:] = list(pub.nullifier)
        s.vote = 1 if pub.vote else 0
        s.private_key[:] = list(prv.private_key)
        sibs = [int(x) for d in prv.merkle_siblings for x in d]
        s.num_siblings = len(prv.merkle_siblings)
        keep_s = (ctypes.c_uint64 * max(len(sibs), 1))(*sibs)
        s.siblings = ctypes.cast(keep_s, ctypes.POINTER(ctypes.c_uint64))
        s.num_path_indices = len(prv.path_indices)
        keep_p = (ctypes.c_uint8 * max(len(prv.path_indices), 1))(*[1 if b else 0 for b in prv.path_indices])
        s.path_indices = ctypes.cast(keep_p, ctypes.POINTER(ctypes.c_uint8))
        s.actual_merkle_depth = prv.actual_merkle_depth
        s.zk_randomness, zk_keep = _zk_ptr(self.zk_randomness)
        s._keep = (keep_s, keep_p, zk_keep)
        return s


class Witness:
    def __init__(self, circuit, handle):
        self.circuit, self.h = circuit, handle

    def wires(self):
        out = np.zeros((self.circuit.num_wires, self.circuit.n), np.uint64)
        rc = lib().qp_witness_wires(self.h, out)
        if rc:
            raise QpError(rc, "qp_witness_wires")
        return out

    def public_inputs(self):
        n = ctypes.c_uint32()
        rc = lib().qp_witness_public_inputs(self.h, None, 0, ctypes.byref(n))
        if rc:
            raise QpError(rc, "qp_witness_public_inputs")
        out = np.zeros(max(n.value, 1), np.uint64)
        rc = lib().qp_witness_public_inputs(self.h, out.ctypes.data, len(out), ctypes.byref(n))
        if rc:
            raise QpError(rc, "qp_witness_public_inputs")
        return out[:n.value].copy()

    def free(self):
        if self.h:
            lib().qp_witness_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Circuit:
    """A built circuit (plonky2 ProverCircuitData + CommonCircuitData)."""

    def __init__(self, handle, kind):
        self.h, self.kind = handle, kind
        self.zk = False
        info = (ctypes.c_uint32 * 9)()
        lib().qp_circuit_info(self.h, info)
        (self.degree_bits, self.num_wires, self.num_routed_wires, self.num_constants, self.num_public_inputs,
         self.gates_used, self.num_gate_constraints, self.num_generators, self.witness_levels) = list(info)
        self.n = 1 << self.degree_bits

    GEN_KINDS = ("constant", "arithmetic", "poseidon", "base_split", "equality", "wire_split", "ext_div",
                 "random_access", "arith_ext", "mul_ext", "reducing", "reducing_ext", "poseidon_mds", "coset_interp")
    GATE_KINDS = ("noop", "constant", "public_input", "base_sum", "arithmetic", "poseidon", "random_access",
                  "arith_ext", "mul_ext", "reducing", "reducing_ext", "poseidon_mds", "coset_interp")

    def census(self, levels=False):
        """({generator kind: count}, {gate kind: rows}) of the built circuit
        (qp_circuit_census; all n rows, padding counted as noop); levels=True
        adds the device witness schedule: per dependency level {kind: count}."""
        g, r = (ctypes.c_uint32 * 14)(), (ctypes.c_uint32 * 13)()
        lv = (ctypes.c_uint32 * (14 * max(self.witness_levels, 1)))() if levels else None
        rc = lib().qp_circuit_census(self.h, g, r, lv)
        if rc:
            raise QpError(rc, "qp_circuit_census")
        out = (dict(zip(self.GEN_KINDS, g)), dict(zip(self.GATE_KINDS, r)))
        if levels:
            out += ([{k: v for k, v in zip(self.GEN_KINDS, lv[14 * l:14 * l + 14]) if v}
                     for l in range(self.witness_levels)],)
        return out

    def host_chains(self):
        """({generator kind: count} the host runs before the device schedule,
        value slots set on the host, independent chains among those
        generators) -- qp_circuit_host_chains."""
        g, n, ch = (ctypes.c_uint32 * 14)(), ctypes.c_uint32(), ctypes.c_uint32()
        rc = lib().qp_circuit_host_chains(self.h, g, ctypes.byref(n), ctypes.byref(ch))
        if rc:
            raise QpError(rc, "qp_circuit_host_chains")
        return {k: v for k, v in zip(self.GEN_KINDS, g) if v}, n.value, ch.value

    @classmethod
    def wormhole(cls, zero_knowledge=False):
        h = ctypes.c_void_p()
        rc = lib().qp_wormhole_circuit_new(int(zero_knowledge), ctypes.byref(h))
        if rc:
            raise QpError(rc, "qp_wormhole_circuit_new")
        c = cls(h, "wormhole")
        c.zk = bool(zero_knowledge)
        return c

    @classmethod
    def voting(cls, zero_knowledge=False):
        """VoteTargets::new + VoteCircuitData::circuit + builder.build() (voting/src/lib.rs:346-357)."""
        h = ctypes.c_void_p()
        rc = lib().qp_voting_circuit_new(int(zero_knowledge), ctypes.byref(h))
        if rc:
            raise QpError(rc, "qp_voting_circuit_new")
        c = cls(h, "voting")
        c.zk = bool(zero_knowledge)
        return c

    @classmethod
    def aggregation(cls, inner_common: bytes, num_proofs: int):
        """aggregate_chunk's circuit (wormhole/aggregator/src/circuits/tree.rs:106-127):
        a recursive verifier of `num_proofs` proofs of the circuit with CommonCircuitData
        `inner_common`, their public inputs registered in order."""
        h = ctypes.c_void_p()
        rc = lib().qp_aggregation_circuit_new(bytes(inner_common), len(inner_common), int(num_proofs),
                                              ctypes.byref(h))
        if rc:
            raise QpError(rc, "qp_aggregation_circuit_new (unsupported inner common data?)")
        c = cls(h, "aggregation")
        c.zk = bool(inner_common[49])
        c.num_proofs = int(num_proofs)
        return c

    def commit_proofs(self, verifier_only: bytes, proofs, zk_randomness=None) -> "Witness":
        """aggregate_chunk's witness (tree.rs:129-134): the inner verifier-only data
        (cap height, constants/sigmas cap, circuit digest) and the proofs to verify."""
        proofs = [bytes(p) for p in proofs]
        arr = (ctypes.c_char_p * len(proofs))(*proofs)
        lens = (ctypes.c_size_t * len(proofs))(*[len(p) for p in proofs])
        zk_ptr, zk_keep = _zk_ptr(zk_randomness)
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = lib().qp_aggregation_commit(self.h, bytes(verifier_only), len(verifier_only),
                                         ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p),
                                         len(proofs), ctypes.cast(zk_ptr, ctypes.c_void_p) if zk_ptr else None,
                                         ctypes.byref(h), err, 512)
        if rc:
            raise QpError(rc, err.value.decode())
        return Witness(self, h)

    def common_data(self):
        ln = ctypes.c_size_t()
        lib().qp_circuit_common_data(self.h, None, 0, ctypes.byref(ln))
        buf = ctypes.create_string_buffer(ln.value)
        rc = lib().qp_circuit_common_data(self.h, buf, ln.value, ctypes.byref(ln))
        if rc:
            raise QpError(rc, "qp_circuit_common_data")
        return buf.raw[:ln.value]

    def constants_sigmas(self):
        out = np.zeros((self.num_constants + self.num_routed_wires, self.n), np.uint64)
        rc = lib().qp_circuit_constants_sigmas(self.h, out)
        if rc:
            raise QpError(rc, "qp_circuit_constants_sigmas")
        return out

    def constants_sigmas_coeffs(self):
        """Coefficients of the constants||sigmas columns (PolynomialValues::ifft, host)."""
        out = np.zeros((self.num_constants + self.num_routed_wires, self.n), np.uint64)
        rc = lib().qp_circuit_constants_sigmas_coeffs(self.h, out)
        if rc:
            raise QpError(rc, "qp_circuit_constants_sigmas_coeffs")
        return out

    def prover_only_bytes(self):
        """Upstream ProverOnlyCircuitData::to_bytes of this leaf circuit
        (DefaultGeneratorSerializer; csrc/prover_bin.cpp, host only)."""
        ln = ctypes.c_size_t()
        rc = lib().qp_circuit_prover_only_bytes(self.h, None, 0, ctypes.byref(ln))
        if rc:
            raise QpError(rc, "qp_circuit_prover_only_bytes")
        buf = ctypes.create_string_buffer(ln.value)
        rc = lib().qp_circuit_prover_only_bytes(self.h, buf, ln.value, ctypes.byref(ln))
        if rc:
            raise QpError(rc, "qp_circuit_prover_only_bytes")
        return buf.raw[:ln.value]

    def commit(self, inputs) -> Witness:
        """WormholeProver::commit (CircuitInputs) or VoteCircuitData::fill_targets
        (VoteCircuitData) followed by witness generation."""
        s = inputs.to_c()
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        fn = lib().qp_voting_commit if self.kind == "voting" else lib().qp_wormhole_commit
        rc = fn(self.h, ctypes.byref(s), ctypes.byref(h), err, 512)
        if rc:
            raise QpError(rc, err.value.decode())
        return Witness(self, h)

    def free(self):
        if self.h:
            lib().qp_circuit_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
