"""Sparse-difference probes of the native circuit's constants||sigmas columns
against the reference's current-circuit proofs (development tool).

Each of tests/golden/dummy_proof{,_zk}.bin opens the constants||sigmas leaf at
28 LDE points (leaf i = g * w_{2^16}^{rev16(i)}), 56 points in all: for every
column that is 56 linear measurements of the reference's 8192 row values.  A
difference confined to at most ~27 rows is located exactly
(layout_sparse.c ls_rational_fit); so is one between the reference and a
rotated copy of ours.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "qp-zk-circuits-rm_amd")]

P = 0xFFFFFFFF00000001
LOG_N = 13
N = 1 << LOG_N
GEN = 0xc65c18b67785d900  # coset shift (qp-plonky2-field multiplicative generator, oracle/gl.h GL_GEN)
SO = "/tmp/liblsparse.so"
U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def lib():
    if not os.path.exists(SO):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", SO, os.path.join(ROOT, "tools/layout_sparse.c"),
                               os.path.join(ROOT, "tools/layout_probe.c")])
    L = ctypes.CDLL(SO)
    L.lp_eval.argtypes = [U64P, ctypes.c_size_t, ctypes.c_uint, U64P, ctypes.c_size_t, U64P]
    L.ls_coeffs.argtypes = [U64P, ctypes.c_uint, U64P]
    L.ls_shift_evals.argtypes = [U64P, ctypes.c_uint, U64P, ctypes.c_size_t, U64P]
    L.ls_rational_fit.argtypes = [U64P, U64P, ctypes.c_size_t, ctypes.c_uint, U64P]
    L.ls_rational_fit.restype = ctypes.c_int
    L.ls_roots.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, np.ctypeslib.ndpointer(np.uint32), ctypes.c_size_t]
    L.ls_roots.restype = ctypes.c_long
    return L


def rev(i, bits):
    return int(format(i, f"0{bits}b")[::-1], 2)


def root(k):
    from oracle_lib import lib as olib
    f = olib().ora_root_of_unity
    f.restype = ctypes.c_uint64
    return int(f(k))


def fixture_points():
    """(xs, ref constants||sigmas leaves [m][84]) over both dummy proofs."""
    from current_circuit_vd import parse_queries, query_indices
    from oracle_lib import golden
    w16 = root(16)
    xs, leaves, seen = [], [], set()
    for name in ("dummy_proof.bin", "dummy_proof_zk.bin"):
        pf = golden(name)
        for q, i in zip(parse_queries(pf), query_indices(name)):
            if i in seen:
                continue
            seen.add(i)
            xs.append(GEN * pow(w16, rev(i, 16), P) % P)
            leaves.append(q[0][0])
    return np.array(xs, np.uint64), np.stack(leaves)


def evals(L, vals, xs):
    vals = np.ascontiguousarray(vals, np.uint64)
    out = np.zeros(vals.shape[0] * len(xs), np.uint64)
    L.lp_eval(vals.reshape(-1), vals.shape[0], LOG_N, xs, len(xs), out)
    return out.reshape(vals.shape[0], len(xs))


def residual_R(D, xs):
    """R = D * n / (x^n - 1)"""
    out = np.zeros_like(D)
    for k, (d, x) in enumerate(zip(D, xs)):
        out[k] = int(d) * N % P * pow((pow(int(x), N, P) - 1) % P, P - 2, P) % P
    return out


def sparse_rows(L, D, xs, s_max=27):
    R = residual_R(D, xs)
    q = np.zeros(s_max + 1, np.uint64)
    s = L.ls_rational_fit(xs, R, len(xs), s_max, q)
    if s <= 0:
        return s, []
    rows = np.zeros(s + 4, np.uint32)
    nr = L.ls_roots(q, s, LOG_N, rows, len(rows))
    return s, list(rows[:nr])


def sub(a, b):
    return ((a.astype(object) - b.astype(object)) % P).astype(np.uint64)


def main():
    from qp_wormhole import Circuit
    L = lib()
    xs, ref = fixture_points()
    print("points:", len(xs))
    c = Circuit.wormhole(zero_knowledge=False)
    cs = np.ascontiguousarray(c.constants_sigmas())
    ours = evals(L, cs, xs)                       # [84][m]
    # self-check: plant 5 differences in column 0
    planted = cs[0].copy()
    for r in (3, 100, 4000, 6855, 8191):
        planted[r] = (int(planted[r]) + 12345) % P
    d = sub(evals(L, planted[None], xs)[0], ours[0])
    print("planted:", sparse_rows(L, d, xs))
    for col in range(84):
        s, rows = sparse_rows(L, sub(ref[:, col], ours[col]), xs)
        if s != -1:
            print("col", col, "sparse diff", s, rows)
    # rotations of ours
    coeffs = np.zeros(N, np.uint64)
    sh = np.zeros(len(xs) * N, np.uint64)
    for col in range(4):
        L.ls_coeffs(cs[col], LOG_N, coeffs)
        L.ls_shift_evals(coeffs, LOG_N, xs, len(xs), sh)
        shm = sh.reshape(len(xs), N)
        exact = [d for d in range(N) if np.array_equal(shm[:, d], ref[:, col])]
        print("col", col, "exact rotations:", exact[:10])
        hits = []
        for d in range(N):
            s, rows = sparse_rows(L, sub(ref[:, col], shm[:, d]), xs, 12)
            if s != -1:
                hits.append((d, s, rows))
        print("col", col, "rotation+sparse hits:", hits[:10])


if __name__ == "__main__":
    main()
