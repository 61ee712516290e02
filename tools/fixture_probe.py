"""Compare the native circuit's preprocessed / witness LDE rows with the leaves
opened by the reference's own current-circuit proofs (tests/golden/dummy_proof*.bin).

Per query the fixture opens the full constants||sigmas (84), wires (135), zs_pp
(20) and quotient (16) leaves; the leaf index is recovered from the wires Merkle
path.  Prints, per column, how many of the 28 query rows agree.  Development
tool (uses the oracle as the checker); the pinned assertions live in
tests/test_plonky2_layout.py.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "qp-zk-circuits-rm_amd")]

from oracle_lib import U64P, commit_values, golden, lib  # noqa: E402


def parse_queries(pf, widths=(84, 135, 20, 16), nq=28, layer_sibs=(8, 4)):
    off = 3 * 512 + 257 * 16 + len(layer_sibs) * 512
    qs = []
    for _ in range(nq):
        q = []
        for w in widths:
            leaf = np.frombuffer(pf[off:off + 8 * w], np.uint64).copy()
            off += 8 * w
            ns = pf[off]
            off += 1
            sibs = np.frombuffer(pf[off:off + 32 * ns], np.uint64).copy()
            off += 32 * ns
            q.append((leaf, sibs))
        for s in layer_sibs:
            off += 256 + 1 + 32 * s
        qs.append(q)
    return qs


def query_indices(pf, qs):
    L = lib()
    L.ora_merkle_find_index.restype = ctypes.c_long
    L.ora_merkle_find_index.argtypes = [U64P, ctypes.c_size_t, U64P, ctypes.c_uint, U64P, ctypes.c_uint]
    caps = np.frombuffer(pf[:3 * 512], np.uint64).reshape(3, 16, 4)
    out = []
    for q in qs:
        leaf, sibs = q[1]
        out.append(int(L.ora_merkle_find_index(leaf, 135, sibs, len(sibs) // 4, caps[0].copy(), 4)))
    return out


def lde_rows(vals, idx):
    log_n = int(np.log2(vals.shape[1]))
    _, leaves, _ = commit_values(vals, log_n, 3, 4, want_leaves=True)
    return leaves[idx]


def main(name="dummy_proof.bin", zk=False):
    import wormhole_inputs as WI
    from qp_wormhole import Circuit
    pf = golden(name)
    qs = parse_queries(pf)
    idx = query_indices(pf, qs)
    print("query leaf indices:", idx)
    c = Circuit.wormhole(zero_knowledge=zk)
    print("gates used:", c.gates_used, "degree_bits:", c.degree_bits)
    cs = lde_rows(c.constants_sigmas(), idx)
    ref_cs = np.stack([q[0][0] for q in qs])
    ok = (cs == ref_cs).sum(axis=0)
    print("constants||sigmas columns matching (of 28 rows):", list(ok))
    w = c.commit(WI.test_inputs())
    wl = lde_rows(w.wires(), idx)
    ref_w = np.stack([q[1][0] for q in qs])
    ok = (wl == ref_w).sum(axis=0)
    print("wire columns matching:", list(ok))
    return qs, idx, c, w


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["dummy_proof.bin"]))
