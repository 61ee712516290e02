"""Verifier data of the reference's CURRENT (degree-13) Wormhole circuit,
reconstructed from the reference's own proofs of it.

The reference commits no verifier data for the current circuit
(wormhole/circuit-builder writes generated-bins/, which is empty), only two
proofs of it: wormhole/aggregator/data/dummy_proof.bin (standard_recursion_config)
and dummy_proof_zk.bin (standard_recursion_zk_config), both on the default test
inputs (prover_tests.rs:56-82).  Every query opens the full constants||sigmas
leaf with its 12-sibling Merkle path, so each query fixes one entry of the
constants||sigmas cap.  The two proofs' queries together reach all 16 cap
entries (and agree wherever they overlap), which gives the whole
VerifierOnlyCircuitData: the cap and the circuit digest
hash_no_pad(cap || hash_pad([]) || degree_bits) (plonk/circuit_builder.rs build).

Test infrastructure: uses the oracle as the checker.
"""
import functools
import json
import os
import struct

import numpy as np

from oracle_lib import golden, lib

WIDTHS = (84, 135, 20, 16)          # constants||sigmas, wires, zs||pp, quotient
LAYER_SIBS = (8, 4)                 # FRI arity bits [4,4]: 4096- and 256-leaf layer trees


def parse_queries(pf, nq=28):
    """Query rounds of a degree-13 Wormhole proof: per query the
    4 initial-tree (leaf, siblings) pairs."""
    off = 3 * 512 + 257 * 16 + len(LAYER_SIBS) * 512
    qs = []
    for _ in range(nq):
        q = []
        for w in WIDTHS:
            leaf = np.frombuffer(pf[off:off + 8 * w], np.uint64).copy()
            off += 8 * w
            ns = pf[off]
            off += 1
            q.append((leaf, np.frombuffer(pf[off:off + 32 * ns], np.uint64).copy()))
            off += 32 * ns
        for s in LAYER_SIBS:
            off += 256 + 1 + 32 * s
        qs.append(q)
    return qs


def _hash_or_noop(v):
    v = np.ascontiguousarray(v, np.uint64)
    o = np.zeros(4, np.uint64)
    lib().ora_hash_or_noop(v, len(v), o)
    return o


def _two_to_one(a, b):
    o = np.zeros(4, np.uint64)
    lib().ora_two_to_one(np.ascontiguousarray(a), np.ascontiguousarray(b), o)
    return o


def cap_entry(leaf, sibs, idx):
    """MerkleProof::verify's climb: returns (cap index, root)."""
    h = _hash_or_noop(leaf)
    s = sibs.reshape(-1, 4)
    for k in range(len(s)):
        h = _two_to_one(h, s[k]) if ((idx >> k) & 1) == 0 else _two_to_one(s[k], h)
    return idx >> len(s), tuple(int(x) for x in h)


def query_leaf_index(pf, q):
    """Leaf index of a query, from its wires Merkle path against the wires cap."""
    import ctypes
    from oracle_lib import U64P
    L = lib()
    L.ora_merkle_find_index.restype = ctypes.c_long
    L.ora_merkle_find_index.argtypes = [U64P, ctypes.c_size_t, U64P, ctypes.c_uint, U64P, ctypes.c_uint]
    caps = np.frombuffer(pf[:512], np.uint64).reshape(16, 4).copy()
    leaf, sibs = q[1]
    return int(L.ora_merkle_find_index(leaf, 135, sibs, len(sibs) // 4, caps, 4))


INDEX_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dummy_query_indices.json")


def brute_force_query_indices(name, count=None):
    """Leaf indices of the fixture's queries by searching the wires Merkle paths (slow: ~25 s)."""
    pf = golden(name)
    return tuple(query_leaf_index(pf, q) for q in parse_queries(pf)[:count])


@functools.lru_cache(maxsize=None)
def query_indices(name):
    """The query leaf indices, from tests/golden/dummy_query_indices.json (written by
    `python tests/current_circuit_vd.py` with brute_force_query_indices; the fixture
    tests re-derive them from the transcript and spot-check the search)."""
    if os.path.exists(INDEX_FILE):
        with open(INDEX_FILE) as f:
            idx = json.load(f)
        if name in idx:
            return tuple(idx[name])
    return brute_force_query_indices(name)


@functools.lru_cache(maxsize=None)
def constants_sigmas_cap_entries(name):
    pf = golden(name)
    out = {}
    for q, idx in zip(parse_queries(pf), query_indices(name)):
        c, h = cap_entry(q[0][0], q[0][1], idx)
        out.setdefault(c, set()).add(h)
    return out


def current_circuit_verifier_data(common_bytes):
    """cap_height || constants_sigmas_cap || circuit_digest || common (verifier.bin layout)."""
    a = constants_sigmas_cap_entries("dummy_proof.bin")
    b = constants_sigmas_cap_entries("dummy_proof_zk.bin")
    cap = np.zeros((16, 4), np.uint64)
    for c in range(16):
        s = a.get(c, set()) | b.get(c, set())
        assert len(s) == 1, f"cap entry {c}: {len(s)} candidates"
        cap[c] = list(s)[0]
    dig = np.zeros(4, np.uint64)
    lib().ora_circuit_digest(cap.reshape(-1).copy(), 16, 13, dig)
    return struct.pack("<Q", 4) + cap.tobytes() + dig.tobytes() + common_bytes, cap, dig


if __name__ == "__main__":
    data = {n: list(brute_force_query_indices(n)) for n in ("dummy_proof.bin", "dummy_proof_zk.bin")}
    data["source"] = "leaf indices of the 28 queries of wormhole/aggregator/data/dummy_proof{,_zk}.bin (Merkle search)"
    with open(INDEX_FILE, "w") as f:
        json.dump(data, f, indent=1)
