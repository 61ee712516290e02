"""ctypes binding of libqpgpu.so (include/qpgpu.h).

The product path is the HIP library only: if libqpgpu.so is missing or cannot
be loaded this module raises, there is no CPU fallback.
"""
import ctypes
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QPGPU_LIB") or os.path.join(HERE, "libqpgpu.so")  # QPGPU_LIB: A/B tuning builds
HEADER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "qpgpu.h")

U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
U32P = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
VP = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)

STATUS = {0: "QP_OK", 1: "QP_ERR_ARG", 2: "QP_ERR_HIP", 3: "QP_ERR_OOM", 4: "QP_ERR_STATE",
          5: "QP_ERR_WITNESS", 6: "QP_ERR_FORMAT"}


MAX_GATES = 16
GATE_KINDS = ["noop", "constant", "public_input", "base_sum", "arithmetic", "poseidon", "arithmetic_extension",
              "mul_extension", "random_access", "exponentiation", "reducing", "reducing_extension", "poseidon_mds",
              "coset_interpolation"]  # QP_GATE_* order


class GateDesc(ctypes.Structure):
    """qp_gate_desc: the parts of CommonCircuitData the vanishing polynomial reads."""
    _fields_ = [("num_gates", ctypes.c_uint32), ("kind", ctypes.c_uint32 * MAX_GATES),
                ("param", ctypes.c_uint32 * MAX_GATES), ("param2", ctypes.c_uint32 * MAX_GATES),
                ("param3", ctypes.c_uint32 * MAX_GATES), ("selector_index", ctypes.c_uint32 * MAX_GATES),
                ("num_selectors", ctypes.c_uint32), ("group_lo", ctypes.c_uint32 * MAX_GATES),
                ("group_hi", ctypes.c_uint32 * MAX_GATES), ("num_constants", ctypes.c_uint32),
                ("num_routed_wires", ctypes.c_uint32), ("num_wires", ctypes.c_uint32),
                ("quotient_degree_factor", ctypes.c_uint32), ("num_challenges", ctypes.c_uint32),
                ("num_gate_constraints", ctypes.c_uint32)]

    @classmethod
    def build(cls, gates, groups, num_wires=135, num_routed_wires=80, num_gate_constants=2, rate_bits=3,
              num_gate_constraints=None):
        """gates: [(kind name, params tuple, selector index)], groups: [(lo, hi)]"""
        g = cls()
        g.num_gates = len(gates)
        for i, (kind, params, sel) in enumerate(gates):
            g.kind[i] = GATE_KINDS.index(kind)
            params = tuple(params) + (0, 0, 0)
            g.param[i], g.param2[i], g.param3[i] = params[:3]
            g.selector_index[i] = sel
        g.num_selectors = len(groups)
        for i, (lo, hi) in enumerate(groups):
            g.group_lo[i], g.group_hi[i] = lo, hi
        g.num_constants = len(groups) + num_gate_constants
        g.num_routed_wires, g.num_wires = num_routed_wires, num_wires
        g.quotient_degree_factor, g.num_challenges = 1 << rate_bits, 2
        g.num_gate_constraints = num_gate_constraints or 0
        return g


class QpError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"{STATUS.get(code, code)}: {msg}")


_lib = None


def header_symbols():
    """Function names declared in include/qpgpu.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s+\*?\s*(qp_\w+)\s*\(", txt, re.M)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "qp_version": (ctypes.c_char_p, []),
        "qp_ctx_create": (ctypes.c_int, [ctypes.c_int, PP]),
        "qp_ctx_destroy": (None, [VP]),
        "qp_ctx_last_error": (ctypes.c_char_p, [VP]),
        "qp_ctx_set_stream": (ctypes.c_int, [VP, VP]),
        "qp_ctx_set_priority": (ctypes.c_int, [VP, ctypes.c_int]),
        "qp_ctx_synchronize": (ctypes.c_int, [VP]),
        "qp_commit_values": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, VP, ctypes.c_uint32, VP, U64P, PP]),
        "qp_commit_coeffs": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, VP, ctypes.c_uint32, U64P, PP]),
        "qp_commit_values_dev": (ctypes.c_int, [VP, VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.c_uint32, VP, PP]),
        "qp_batch_open": (ctypes.c_int, [VP, U32P, ctypes.c_uint32, U64P, U64P]),
        "qp_batch_lde": (ctypes.c_int, [VP, U64P]),
        "qp_batch_coeffs": (ctypes.c_int, [VP, U64P]),
        "qp_batch_free": (None, [VP]),
        "qp_ifft": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32]),
        "qp_lde": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                  U64P]),
        "qp_poseidon_permute": (ctypes.c_int, [VP, U64P, ctypes.c_uint64]),
        "qp_wormhole_circuit_new": (ctypes.c_int, [ctypes.c_int, PP]),
        "qp_circuit_free": (None, [VP]),
        "qp_circuit_info": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_uint32)]),
        "qp_circuit_host_chains": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                                   ctypes.POINTER(ctypes.c_uint32)]),
        "qp_circuit_census": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                              ctypes.POINTER(ctypes.c_uint32)]),
        "qp_circuit_common_data": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_size_t,
                                                  ctypes.POINTER(ctypes.c_size_t)]),
        "qp_circuit_constants_sigmas": (ctypes.c_int, [VP, U64P]),
        "qp_circuit_constants_sigmas_coeffs": (ctypes.c_int, [VP, U64P]),
        "qp_circuit_prover_only_bytes": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_size_t,
                                                        ctypes.POINTER(ctypes.c_size_t)]),
        "qp_wormhole_commit": (ctypes.c_int, [VP, VP, PP, ctypes.c_char_p, ctypes.c_size_t]),
        "qp_voting_circuit_new": (ctypes.c_int, [ctypes.c_int, PP]),
        "qp_voting_commit": (ctypes.c_int, [VP, VP, PP, ctypes.c_char_p, ctypes.c_size_t]),
        "qp_aggregation_circuit_new": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, PP]),
        "qp_aggregation_commit": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_size_t, VP, VP, ctypes.c_uint32,
                                                 VP, PP, ctypes.c_char_p, ctypes.c_size_t]),
        "qp_witness_wires": (ctypes.c_int, [VP, U64P]),
        "qp_witness_public_inputs": (ctypes.c_int, [VP, VP, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
        "qp_witness_free": (None, [VP]),
        "qp_hash_no_pad": (ctypes.c_int, [U64P, ctypes.c_size_t, U64P]),
        "qp_prover_new": (ctypes.c_int, [VP, VP, ctypes.c_uint32, PP]),
        "qp_prover_free": (None, [VP]),
        "qp_prover_proof_size": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_verifier_data": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_size_t,
                                                   ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_char_p,
                                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove_wires": (ctypes.c_int, [VP, U64P, U64P, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove_wires_dev": (ctypes.c_int, [VP, VP, U64P, ctypes.c_uint32, ctypes.c_char_p,
                                                     ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove_wormhole_inputs": (ctypes.c_int, [VP, VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                                           ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove_voting_inputs": (ctypes.c_int, [VP, VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                                         ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_prove_aggregation": (ctypes.c_int, [VP, VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                                       ctypes.POINTER(ctypes.c_size_t)]),
        "qp_prover_set_timing": (ctypes.c_int, [VP, ctypes.c_int]),
        "qp_prover_debug_force_pow": (ctypes.c_int, [VP, ctypes.c_uint64, ctypes.c_int]),
        "qp_prover_debug_drop_table": (ctypes.c_int, [VP, ctypes.c_char_p]),
        "qp_prover_set_host_threads": (ctypes.c_int, [VP, ctypes.c_uint32]),
        "qp_prover_kernel_stats": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                                  ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_int]),
        "qp_prover_stage_times": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_double), ctypes.c_uint32, ctypes.c_int]),
        "qp_circuit_gate_desc": (ctypes.c_int, [VP, ctypes.POINTER(GateDesc)]),
        "qp_quotient": (ctypes.c_int, [VP, VP, VP, VP, ctypes.POINTER(GateDesc), U64P, U64P, U64P, U64P, U64P]),
        "qp_fri_layer_commit": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                               ctypes.c_uint32, ctypes.c_uint32, U64P, PP]),
        "qp_fri_layer_open": (ctypes.c_int, [VP, U32P, ctypes.c_uint32, U64P, U64P]),
        "qp_fri_layer_free": (None, [VP]),
        "qp_fri_fold": (ctypes.c_int, [VP, U64P, ctypes.c_uint32, ctypes.c_uint32, U64P, U64P]),
        "qp_pow_grind": (ctypes.c_int, [VP, U64P, U32P, ctypes.c_uint32, ctypes.c_uint32, U64P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class Context:
    """One HIP stream on one device (qp_ctx)."""

    def __init__(self, device=0):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.qp_ctx_create(device, ctypes.byref(h))
        if rc:
            raise QpError(rc, f"qp_ctx_create(device={device})")
        self.h = h

    def check(self, rc, what=""):
        if rc:
            raise QpError(rc, f"{what}: {lib().qp_ctx_last_error(self.h).decode()}")

    def set_priority(self, high=True):
        """Own stream at the device's greatest (or the default) priority."""
        self.check(lib().qp_ctx_set_priority(self.h, int(bool(high))), "set_priority")

    def close(self):
        if self.h:
            lib().qp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        self.check(lib().qp_ctx_set_stream(self.h, stream_ptr), "set_stream")

    def synchronize(self):
        self.check(lib().qp_ctx_synchronize(self.h), "synchronize")


class PolynomialBatch:
    """Device-resident committed polynomial batch (plonky2 PolynomialBatch)."""

    def __init__(self, ctx, handle, npolys, nsalt, log_n, rate_bits, cap_height, cap, coeffs=None):
        self.ctx, self.h = ctx, handle
        self.npolys, self.nsalt, self.log_n, self.rate_bits, self.cap_height = npolys, nsalt, log_n, rate_bits, cap_height
        self.cap, self.coeffs = cap, coeffs

    @classmethod
    def from_values(cls, ctx, values, rate_bits, cap_height, salt=None, keep=True):
        values = np.ascontiguousarray(values, dtype=np.uint64)
        npolys, n = values.shape
        log_n = n.bit_length() - 1
        nsalt = 0 if salt is None else salt.shape[1]
        salt_c = None if salt is None else np.ascontiguousarray(salt, dtype=np.uint64)
        coeffs = np.zeros_like(values)
        cap = np.zeros(((1 << cap_height), 4), np.uint64)
        h = ctypes.c_void_p()
        rc = lib().qp_commit_values(ctx.h, values, npolys, log_n, rate_bits, cap_height,
                                    None if salt_c is None else salt_c.ctypes.data, nsalt, coeffs.ctypes.data, cap,
                                    ctypes.byref(h) if keep else None)
        ctx.check(rc, "qp_commit_values")
        return cls(ctx, h if keep else None, npolys, nsalt, log_n, rate_bits, cap_height, cap, coeffs)

    @classmethod
    def from_coeffs(cls, ctx, coeffs, rate_bits, cap_height, salt=None, keep=True):
        coeffs = np.ascontiguousarray(coeffs, dtype=np.uint64)
        npolys, n = coeffs.shape
        log_n = n.bit_length() - 1
        nsalt = 0 if salt is None else salt.shape[1]
        salt_c = None if salt is None else np.ascontiguousarray(salt, dtype=np.uint64)
        cap = np.zeros(((1 << cap_height), 4), np.uint64)
        h = ctypes.c_void_p()
        rc = lib().qp_commit_coeffs(ctx.h, coeffs, npolys, log_n, rate_bits, cap_height,
                                    None if salt_c is None else salt_c.ctypes.data, nsalt, cap,
                                    ctypes.byref(h) if keep else None)
        ctx.check(rc, "qp_commit_coeffs")
        return cls(ctx, h if keep else None, npolys, nsalt, log_n, rate_bits, cap_height, cap, coeffs)

    def open(self, indices):
        idx = np.ascontiguousarray(indices, dtype=np.uint32)
        W = self.npolys + self.nsalt
        depth = self.log_n + self.rate_bits - self.cap_height
        leaves = np.zeros((len(idx), W), np.uint64)
        sibs = np.zeros((len(idx), depth, 4), np.uint64)
        self.ctx.check(lib().qp_batch_open(self.h, idx, len(idx), leaves, sibs), "qp_batch_open")
        return leaves, sibs

    def lde(self):
        out = np.zeros((self.npolys, 1 << (self.log_n + self.rate_bits)), np.uint64)
        self.ctx.check(lib().qp_batch_lde(self.h, out), "qp_batch_lde")
        return out

    def free(self):
        if self.h:
            lib().qp_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def ifft(ctx, data):
    a = np.ascontiguousarray(data, dtype=np.uint64).copy()
    ncols, n = a.shape
    ctx.check(lib().qp_ifft(ctx.h, a, ncols, n.bit_length() - 1), "qp_ifft")
    return a


def lde(ctx, coeffs, rate_bits, shift=0xC65C18B67785D900):
    c = np.ascontiguousarray(coeffs, dtype=np.uint64)
    ncols, n = c.shape
    out = np.zeros((ncols, n << rate_bits), np.uint64)
    ctx.check(lib().qp_lde(ctx.h, c, ncols, n.bit_length() - 1, rate_bits, shift, out), "qp_lde")
    return out


def poseidon_permute(ctx, states):
    s = np.ascontiguousarray(states, dtype=np.uint64).copy()
    ctx.check(lib().qp_poseidon_permute(ctx.h, s, s.shape[0]), "qp_poseidon_permute")
    return s


def hash_no_pad(values):
    """PoseidonHash::hash_no_pad on the host (libqpgpu host code)."""
    a = np.ascontiguousarray(values, dtype=np.uint64)
    out = np.zeros(4, np.uint64)
    rc = lib().qp_hash_no_pad(a, len(a), out)
    if rc:
        raise QpError(rc, "qp_hash_no_pad")
    return [int(x) for x in out]


# ---- routine-level seams (include/qpgpu.h "routine-level seams") ----------

def gate_desc(circuit):
    """qp_circuit_gate_desc for a built Circuit."""
    g = GateDesc()
    rc = lib().qp_circuit_gate_desc(circuit.h, ctypes.byref(g))
    if rc:
        raise QpError(rc, "qp_circuit_gate_desc")
    return g


def _u64(v, n=None):
    a = np.ascontiguousarray([int(x) for x in v] if not isinstance(v, np.ndarray) else v, dtype=np.uint64)
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} values, got {a.size}")
    return a


def quotient(ctx, cs, wires, zs_pp, gd, betas, gammas, alphas, pi_hash):
    """compute_quotient_polys: returns quotient coefficients [nc * qdf][n]."""
    nc, qdf = gd.num_challenges, gd.quotient_degree_factor
    out = np.zeros((nc * qdf, 1 << cs.log_n), np.uint64)
    ctx.check(lib().qp_quotient(ctx.h, cs.h, wires.h, zs_pp.h, ctypes.byref(gd), _u64(betas, nc), _u64(gammas, nc),
                                _u64(alphas, nc), _u64(pi_hash, 4), out), "qp_quotient")
    return out


class FriLayer:
    """One committed FRI reduction layer (fri_committed_trees)."""

    def __init__(self, ctx, coeffs, log_values, shift, arity_bits, cap_height):
        c = np.ascontiguousarray(coeffs, dtype=np.uint64)
        if c.ndim != 2 or c.shape[0] != 2:
            raise ValueError("coeffs must be [2][2^k] (ext c0 row, c1 row)")
        self.ctx, self.log_values, self.arity_bits, self.cap_height = ctx, log_values, arity_bits, cap_height
        self.cap = np.zeros((1 << cap_height, 4), np.uint64)
        h = ctypes.c_void_p()
        ctx.check(lib().qp_fri_layer_commit(ctx.h, c, c.shape[1].bit_length() - 1, log_values, shift, arity_bits,
                                            cap_height, self.cap, ctypes.byref(h)), "qp_fri_layer_commit")
        self.h = h

    def open(self, indices):
        idx = np.ascontiguousarray(indices, dtype=np.uint32)
        depth = self.log_values - self.arity_bits - self.cap_height
        evals = np.zeros((len(idx), 1 << self.arity_bits, 2), np.uint64)
        sibs = np.zeros((len(idx), depth, 4), np.uint64)
        self.ctx.check(lib().qp_fri_layer_open(self.h, idx, len(idx), evals, sibs), "qp_fri_layer_open")
        return evals, sibs

    def free(self):
        if self.h:
            lib().qp_fri_layer_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def fri_fold(ctx, coeffs, arity_bits, beta):
    c = np.ascontiguousarray(coeffs, dtype=np.uint64)
    out = np.zeros((2, c.shape[1] >> arity_bits), np.uint64)
    ctx.check(lib().qp_fri_fold(ctx.h, c, c.shape[1].bit_length() - 1, arity_bits, _u64(beta, 2), out), "qp_fri_fold")
    return out


def pow_grind(ctx, states, pos, pow_bits):
    """fri_proof_of_work for n duplex states [n][12] with pending-input counts pos[n]."""
    st = np.ascontiguousarray(states, dtype=np.uint64).reshape(-1, 12)
    p = np.ascontiguousarray(pos, dtype=np.uint32)
    out = np.zeros(st.shape[0], np.uint64)
    ctx.check(lib().qp_pow_grind(ctx.h, st, p, st.shape[0], pow_bits, out), "qp_pow_grind")
    return out
