"""Block-position scans of the reference's constants columns (development tool).

The reference's current-circuit proofs open the 4 constants columns (S0, S1
selectors, C0, C1 gate constants) at 56 LDE points.  Over the gate kinds of
the circuit (Noop 0, Constant 1, PublicInput 2, BaseSum 3, Arithmetic 4 in
selector group 0; Poseidon 5 in group 1):

    P   = (S1 - U) / (5 - U)                 (Poseidon-row indicator)
    M   = S0 - U*P - C0 + 3*P

M is 3 on every BaseSum / Arithmetic(c0 = 1) / Poseidon row, 5 on an
Arithmetic row with c0 = -1, 2 on the PublicInput row, 1 - c on a ConstantGate
row whose first constant is c, and 0 on Noop rows.  Under plonky2's build()
the rows are [user gadgets + PI hash] [PublicInputGate] [ConstantGates]
[Noop padding], so M is a head of 3s, a known tail, and zeros, up to a few
c0 = -1 rows: one unknown (the PI row) scanned with a sparse residual test.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "qp-zk-circuits-rm_amd")]
import layout_sparse as lsp  # noqa: E402

P = lsp.P
N = lsp.N
U = 0xFFFFFFFF
SO = "/tmp/liblscan.so"
U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def lib():
    if not os.path.exists(SO):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", SO] +
                              [os.path.join(ROOT, "tools", f) for f in ("layout_scan.c", "layout_sparse.c", "layout_probe.c")])
    L = ctypes.CDLL(SO)
    L.ls_block_scan.argtypes = [U64P, U64P, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint64, U64P, ctypes.c_size_t,
                                ctypes.c_uint, ctypes.c_uint32, ctypes.c_uint32,
                                np.ctypeslib.ndpointer(np.uint32), np.ctypeslib.ndpointer(np.int32),
                                np.ctypeslib.ndpointer(np.uint32), ctypes.c_size_t]
    L.ls_block_scan.restype = ctypes.c_long
    L.lp_eval.argtypes = [U64P, ctypes.c_size_t, ctypes.c_uint, U64P, ctypes.c_size_t, U64P]
    return L


def inv(a):
    return pow(int(a) % P, P - 2, P)


def combo(S0, S1, C0):
    out = []
    k = inv(5 - U)
    for s0, s1, c0 in zip(S0, S1, C0):
        p_ = (int(s1) - U) * k % P
        out.append((int(s0) - U * p_ - int(c0) + 3 * p_) % P)
    return np.array(out, np.uint64)


def scan(L, xs, meas, head, tail, s_max=12, lo=0, hi=N):
    mh = 64
    hits = np.zeros(mh, np.uint32)
    hs = np.zeros(mh, np.int32)
    hr = np.zeros(mh * 16, np.uint32)
    tail = np.ascontiguousarray(np.array([t % P for t in tail], np.uint64))
    nh = L.ls_block_scan(xs, meas, len(xs), 13, head % P, tail, len(tail), s_max, lo, hi, hits, hs, hr, mh)
    return [(int(hits[i]), int(hs[i]), [int(r) for r in hr[i * 16:(i + 1) * 16] if r != 0xFFFFFFFF])
            for i in range(min(nh, mh))]


def constant_tail(consts):
    """M values from the PI row on: 2, then 1 - c for each ConstantGate's first constant."""
    cs = sorted(consts)
    return [2] + [(1 - c) % P for c in cs[0::2]]


def main():
    from qp_wormhole import Circuit
    L = lib()
    xs, ref = lsp.fixture_points()
    ours_cols = np.ascontiguousarray(Circuit.wormhole(zero_knowledge=False).constants_sigmas()[:4])
    ours = np.zeros(4 * len(xs), np.uint64)
    L.lp_eval(ours_cols.reshape(-1), 4, 13, xs, len(xs), ours)
    ours = ours.reshape(4, len(xs))
    # our circuit's constants: ConstantGate rows' (C0, C1) after the PI row
    S0 = ours_cols[0]
    pi_row = int(np.nonzero(S0 == 2)[0][0])
    consts = []
    r = pi_row + 1
    while S0[r] == 1:
        consts += [int(ours_cols[2][r]), int(ours_cols[3][r])]
        r += 1
    print("ours: pi_row", pi_row, "constant rows", r - pi_row - 1)
    tail = [2] + [(1 - consts[i]) % P for i in range(0, len(consts), 2)]
    m_ours = combo(ours[0], ours[1], ours[2])
    print("self-check (ours):", scan(L, xs, m_ours, 3, tail, lo=pi_row - 3, hi=pi_row + 4))
    m_ref = combo(ref[:, 0], ref[:, 1], ref[:, 2])
    print("reference, our constant set:", scan(L, xs, m_ref, 3, tail))
    print("reference, PI row + no constants:", scan(L, xs, m_ref, 3, [2], s_max=20))


if __name__ == "__main__":
    main()
