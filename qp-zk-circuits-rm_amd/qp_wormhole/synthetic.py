"""Seeded synthetic Wormhole circuit inputs.

Mirrors the reference's input construction:
  unspendable account = H(H("wormhole" || secret))        unspendable_account.rs:38-63
  nullifier           = H(H("~nullif~" || secret || tc))  nullifier.rs:53-73
  storage proof, variant A: empty proof, root = H(leaf inputs)
      (wormhole/example/src/main.rs:24-31, circuit_data_tests.rs:141-172)
  storage proof, variant B: a synthetic trie of depth d <= 20: node i holds the
      8 LE u32 limbs of H(node i+1) at felt offset j_i; the last node holds the
      leaf-input hash; root = H(node 0 padded to 188 felts)
The circuit cost does not depend on the witness (all 20 node hashes are always
computed, storage_proof/mod.rs:169-243).
"""
import struct

import numpy as np

from ._native import hash_no_pad
from .circuits import CircuitInputs, PrivateCircuitInputs, ProcessedStorageProof, PublicCircuitInputs

P = 0xFFFFFFFF00000001
MASK64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def injective_bytes_to_felts(b):
    out = []
    for i in range(0, len(b), 4):
        c = b[i:i + 4]
        out.append(struct.unpack("<I", c + b"\0" * (4 - len(c)))[0])
    return out


def digest_to_bytes(d):
    return b"".join(struct.pack("<Q", x) for x in d)


def bytes_to_digest(b):
    return [struct.unpack("<Q", b[8 * i:8 * i + 8])[0] for i in range(4)]


def u64_to_felts(x):
    return [(x >> 32) & 0xFFFFFFFF, x & 0xFFFFFFFF]


def u128_to_felts(x):
    return [(x >> (96 - 32 * i)) & 0xFFFFFFFF for i in range(4)]


def unspendable_account(secret: bytes) -> bytes:
    pre = injective_bytes_to_felts(b"wormhole") + injective_bytes_to_felts(secret)
    return digest_to_bytes(hash_no_pad(hash_no_pad(pre)))


def nullifier(secret: bytes, transfer_count: int) -> bytes:
    pre = injective_bytes_to_felts(b"~nullif~") + injective_bytes_to_felts(secret) + u64_to_felts(transfer_count)
    return digest_to_bytes(hash_no_pad(hash_no_pad(pre)))


def leaf_hash(transfer_count, funding_account, to_account, funding_amount):
    leaf = (u64_to_felts(transfer_count) + bytes_to_digest(funding_account) + bytes_to_digest(to_account) +
            u128_to_felts(funding_amount))
    return hash_no_pad(leaf)


class _Rng:
    def __init__(self, seed):
        self.s = splitmix64(0x5EED0000 + seed)

    def u64(self):
        self.s = splitmix64(self.s)
        return self.s

    def bytes32_u32limbs(self):
        return b"".join(struct.pack("<Q", self.u64()) for _ in range(4))

    def felt_bytes(self):
        return b"".join(struct.pack("<Q", self.u64() % P) for _ in range(4))


def synthetic_inputs(k: int, depth: int = -1) -> CircuitInputs:
    """Inputs of proof k.  depth = 0: empty storage proof (variant A);
    depth in [1, 20]: synthetic trie (variant B); -1: depth drawn from the seed."""
    r = _Rng(k)
    secret = r.bytes32_u32limbs()
    transfer_count = r.u64()
    funding_amount = r.u64()
    funding_account = r.felt_bytes()
    exit_account = r.felt_bytes()
    unspendable = unspendable_account(secret)
    null = nullifier(secret, transfer_count)
    lh = leaf_hash(transfer_count, funding_account, unspendable, funding_amount)
    if depth < 0:
        depth = int(r.u64() % 21)
    nodes, indices = [], []
    if depth == 0:
        root = digest_to_bytes(lh)
    else:
        child = lh
        for i in reversed(range(depth)):
            nfelts = 60 + int(r.u64() % 120)            # node length in u32 limbs (<= 180)
            felts = [r.u64() & 0xFFFFFFFF for _ in range(nfelts)]
            j = int(r.u64() % (nfelts - 7))
            limbs = []
            for h in child:
                limbs += [h & 0xFFFFFFFF, h >> 32]
            felts[j:j + 8] = limbs
            node = b"".join(struct.pack("<I", f) for f in felts)
            nodes.insert(0, node)
            indices.insert(0, 8 * j)
            padded = felts + [0] * (188 - len(felts))
            child = hash_no_pad(padded)
        root = digest_to_bytes(child)
    return CircuitInputs(
        PublicCircuitInputs(funding_amount, null, root, exit_account),
        PrivateCircuitInputs(secret, ProcessedStorageProof(nodes, indices), transfer_count, funding_account,
                             unspendable))


# ---------------------------------------------------------------- voting circuit

def vote_nullifier(private_key, proposal_id):
    """voting/src/lib.rs:277-283: H(H(private_key) || proposal_id)."""
    return hash_no_pad(list(hash_no_pad(list(private_key))) + list(proposal_id))


def vote_test_inputs():
    """create_test_inputs (voting/src/lib.rs:285-337): 4-leaf tree of H([k;32] as
    felts), voter = key 1 at depth 2, proposal id = [42;32], vote = yes."""
    from .circuits import VoteCircuitData, VotePrivateInputs, VotePublicInputs
    keys = [bytes_to_digest(bytes([k] * 32)) for k in (1, 2, 3, 4)]
    leaves = [hash_no_pad(k) for k in keys]
    level1 = [hash_no_pad(leaves[0] + leaves[1]), hash_no_pad(leaves[2] + leaves[3])]
    root = hash_no_pad(level1[0] + level1[1])
    proposal = bytes_to_digest(bytes([42] * 32))
    return VoteCircuitData(
        VotePublicInputs(proposal_id=proposal, merkle_root=root, vote=True,
                         nullifier=vote_nullifier(keys[0], proposal)),
        VotePrivateInputs(private_key=keys[0], merkle_siblings=[leaves[1], level1[1]], path_indices=[False, False],
                          actual_merkle_depth=2))


def synthetic_vote_inputs(k: int, depth: int = -1):
    """Seeded voter k: random key, a random Merkle path of `depth` levels
    (default: seeded in [0, 31]; 32 does not fit the circuit's 5-bit depth
    split, see tests/test_voting.py) with random siblings and sides, the root it
    implies, a random proposal id and vote, and the matching nullifier."""
    from .circuits import VoteCircuitData, VotePrivateInputs, VotePublicInputs
    r = _Rng(0x10000 + k)
    key = [r.u64() % P for _ in range(4)]
    if depth < 0:
        depth = r.u64() % 32
    cur = hash_no_pad(key)
    sibs, path = [], []
    for _ in range(depth):
        s = [r.u64() % P for _ in range(4)]
        right = bool(r.u64() & 1)
        cur = hash_no_pad(s + cur if right else cur + s)
        sibs.append(s)
        path.append(right)
    proposal = [r.u64() % P for _ in range(4)]
    return VoteCircuitData(
        VotePublicInputs(proposal_id=proposal, merkle_root=cur, vote=bool(r.u64() & 1),
                         nullifier=vote_nullifier(key, proposal)),
        VotePrivateInputs(private_key=key, merkle_siblings=sibs, path_indices=path, actual_merkle_depth=depth))
