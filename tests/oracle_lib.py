"""ctypes loader for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the thing measured
or shipped.  Built from oracle/ sources with `make -C oracle` if missing.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
P = 0xFFFFFFFF00000001

_lib = None


def lib():
    global _lib
    if _lib is None:
        so = os.path.join(ORACLE_DIR, "liboracle.so")
        srcs = [f for f in os.listdir(ORACLE_DIR) if f.endswith((".c", ".h", "Makefile"))]
        stale = not os.path.exists(so) or any(
            os.path.getmtime(os.path.join(ORACLE_DIR, f)) > os.path.getmtime(so) for f in srcs)
        if stale:
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(so)
        L.ora_permute.argtypes = [U64P]
        L.ora_hash_no_pad.argtypes = [U64P, ctypes.c_size_t, U64P]
        L.ora_hash_or_noop.argtypes = [U64P, ctypes.c_size_t, U64P]
        L.ora_two_to_one.argtypes = [U64P, U64P, U64P]
        L.ora_mul_many.argtypes = [U64P, U64P, U64P, ctypes.c_size_t]
        for f in ("ora_fft", "ora_ifft"):
            getattr(L, f).argtypes = [U64P, ctypes.c_uint]
        for f in ("ora_coset_fft", "ora_coset_ifft"):
            getattr(L, f).argtypes = [U64P, ctypes.c_uint, ctypes.c_uint64]
        L.ora_lde.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64, U64P]
        L.ora_root_of_unity.restype = ctypes.c_uint64
        L.ora_root_of_unity.argtypes = [ctypes.c_uint]
        L.ora_commit_values.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                        ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, U64P]
        L.ora_merkle.argtypes = [U64P, ctypes.c_uint, ctypes.c_size_t, ctypes.c_uint, U64P, U64P,
                                 ctypes.c_size_t, U64P]
        L.ora_verify.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.ora_proof_roundtrip.restype = ctypes.c_long
        L.ora_proof_roundtrip.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.c_char_p]
        L.ora_common_roundtrip.restype = ctypes.c_long
        L.ora_common_roundtrip.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.ora_challenges.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, U64P]
        L.ora_circuit_digest.argtypes = [U64P, ctypes.c_size_t, ctypes.c_uint64, U64P]
        L.ora_quotient.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, U64P, U64P, U64P, U64P, U64P]
        L.ora_fri_layer.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint,
                                    U64P, np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS"), ctypes.c_uint,
                                    U64P, U64P]
        L.ora_fri_fold.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, U64P, U64P]
        L.ora_quotient_desc.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, U64P, U64P, U64P, U64P, U64P,
                                        U64P, U64P, U64P]
        L.ora_gate_eval.restype = ctypes.c_long
        L.ora_gate_eval.argtypes = [ctypes.c_void_p, ctypes.c_uint, U64P, U64P, U64P, U64P]
        L.ora_eval_values.argtypes = [U64P, ctypes.c_size_t, ctypes.c_uint, U64P, ctypes.c_size_t, U64P]
        L.ora_force_pow_witness.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.ora_pow_grind.restype = ctypes.c_uint64
        L.ora_pow_grind.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint]
        _lib = L
    return _lib


def golden(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


def hash_no_pad(v):
    a = np.ascontiguousarray(v, dtype=np.uint64)
    o = np.zeros(4, np.uint64)
    lib().ora_hash_no_pad(a, len(a), o)
    return [int(x) for x in o]


def permute(state):
    s = np.ascontiguousarray(state, dtype=np.uint64).copy()
    lib().ora_permute(s)
    return s


def commit_values(vals, log_n, rate_bits, cap_h, salt=None, from_coeffs=False, want_leaves=False):
    """PolynomialBatch::from_values/from_coeffs: returns (coeffs, leaves, cap)."""
    npolys = vals.shape[0]
    n = 1 << log_n
    N = n << rate_bits
    nsalt = 0 if salt is None else salt.shape[1]
    coeffs = np.zeros((npolys, n), np.uint64)
    leaves = np.zeros((N, npolys + nsalt), np.uint64) if want_leaves else None
    cap = np.zeros(((1 << cap_h), 4), np.uint64)
    v = np.ascontiguousarray(vals, dtype=np.uint64)
    rc = lib().ora_commit_values(v, npolys, log_n, rate_bits, cap_h,
                                 None if salt is None else np.ascontiguousarray(salt).ctypes.data,
                                 nsalt, int(from_coeffs), coeffs.ctypes.data,
                                 None if leaves is None else leaves.ctypes.data, cap)
    assert rc == 0
    return coeffs, leaves, cap
