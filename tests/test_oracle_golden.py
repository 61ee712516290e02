"""Pin the CPU oracle against the reference's own golden data.

* Poseidon KATs from the reference tests:
  wormhole/tests/src/prover/prover_tests.rs:21-45 (nullifier bytes),
  wormhole/tests/src/circuit/unspendable_account_tests.rs:12-28 (secret->address),
  wormhole/tests/test-helpers/src/lib.rs:60-80 + storage_proof_tests.rs:25-28
  (7-node storage proof chaining to DEFAULT_ROOT_HASH, leaf-input hash).
* Committed fixtures (tests/golden/ = copies of wormhole/bench-data/*.bin and
  wormhole/aggregator/data/dummy_proof*.bin): full verification of proof.bin,
  byte-exact re-serialisation, circuit digest, transcript, Merkle
  self-consistency of the dummy proofs, negative controls (verifier_tests.rs:25-66).
"""
import ctypes
import hashlib
import struct

import numpy as np
import pytest

from oracle_lib import P, U64P, golden, hash_no_pad, lib
from wormhole_codec import (digest_bytes_to_felts, digest_felts_to_bytes, injective_bytes_to_felts,
                            injective_string_to_felt, u128_to_felts, u64_to_felts)

DEFAULT_SECRET = "4c8587bd422e01d961acdc75e7d66f6761b7af7c9b1864a492f369c9d6724f05"
NULLIFIER_BYTES = bytes([169, 76, 150, 35, 66, 248, 76, 193, 57, 204, 106, 33, 169, 160, 248, 113, 235, 144,
                         212, 48, 9, 232, 146, 7, 105, 125, 170, 24, 33, 54, 135, 28])
SECRETS = [
    "cd94df2e3c38a87f3e429b62af022dbe4363143811219d80037e8798b2ec9229",
    "8b680b2421968a0c1d3cff6f3408e9d780157ae725724a78c3bc0998d1ac8194",
    "87f5fc11df0d12f332ccfeb92ddd8995e6c11709501a8b59c2aaf9eefee63ec1",
    "ef69da4e3aa2a6f15b3a9eec5e481f17260ac812faf1e685e450713327c3ab1c",
    "9aa84f99ef2de22e3070394176868df41d6a148117a36132d010529e19b018b7",
]
ADDRESSES = [
    "582d3b97e9b09c7776921d3ead2d8186e3aa199cf8d63f5d014e65d04ac80f26",
    "b0807446c24263def407aa8328400fef981ec30fc8453d7adbcc57bcf8af3bbf",
    "ac081f035cc995574fef749f33b455c31cb02759932d01b6367ab852bb5599ac",
    "a5073c13573f10552c37f35080dc0118bda22f1217381611cf4644909377ce05",
    "73378f4b54f48a38b17073e08440531594f2b771ceefc5c3cd621e1309fbe927",
]
DEFAULT_ROOT_HASH = "5ffa2ab5b0db9883b22b1e5810932ea9d9eab1840730fd39ace71c26bb8d082d"
DEFAULT_FUNDING_ACCOUNT = bytes([226, 124, 203, 9, 80, 60, 124, 205, 165, 5, 178, 216, 195, 15, 149, 38, 116, 1,
                                 238, 133, 181, 154, 106, 17, 41, 228, 118, 179, 82, 141, 225, 76])
DEFAULT_TO_ACCOUNT = bytes([162, 77, 187, 9, 249, 178, 185, 87, 194, 50, 198, 98, 179, 134, 179, 126, 123, 21,
                            247, 44, 50, 216, 140, 243, 97, 177, 13, 94, 26, 255, 19, 170])
DEFAULT_FUNDING_AMOUNT = 1_000_000_000_000


def storage_proof_nodes():
    from golden_storage_proof import DEFAULT_STORAGE_PROOF, DEFAULT_STORAGE_PROOF_INDICES
    return [bytes.fromhex(h) for h in DEFAULT_STORAGE_PROOF], DEFAULT_STORAGE_PROOF_INDICES


def test_nullifier_kat():
    # nullifier.rs:53-73: H(H(salt || secret || transfer_count))
    secret = bytes.fromhex(DEFAULT_SECRET)
    pre = injective_string_to_felt("~nullif~") + injective_bytes_to_felts(secret) + u64_to_felts(4)
    h = hash_no_pad(hash_no_pad(pre))
    assert digest_felts_to_bytes(h) == NULLIFIER_BYTES


@pytest.mark.parametrize("secret,address", list(zip(SECRETS, ADDRESSES)))
def test_unspendable_account_kat(secret, address):
    # unspendable_account.rs:38-63
    pre = injective_string_to_felt("wormhole") + injective_bytes_to_felts(bytes.fromhex(secret))
    assert digest_felts_to_bytes(hash_no_pad(hash_no_pad(pre))).hex() == address


def test_default_to_account_is_unspendable_of_default_secret():
    pre = injective_string_to_felt("wormhole") + injective_bytes_to_felts(bytes.fromhex(DEFAULT_SECRET))
    assert digest_felts_to_bytes(hash_no_pad(hash_no_pad(pre))) == DEFAULT_TO_ACCOUNT


def test_storage_proof_chain_kat():
    # storage_proof/mod.rs:163-243 evaluated natively on the default test inputs
    nodes, indices = storage_proof_nodes()
    prev = digest_bytes_to_felts(bytes.fromhex(DEFAULT_ROOT_HASH))
    for node, idx in zip(nodes, indices):
        felts = injective_bytes_to_felts(node)
        felts = felts + [0] * (188 - len(felts))
        assert hash_no_pad(felts) == prev
        j = idx // 8
        prev = [felts[j + 2 * k] + (felts[j + 2 * k + 1] << 32) for k in range(4)]
    leaf = (u64_to_felts(4) + digest_bytes_to_felts(DEFAULT_FUNDING_ACCOUNT) +
            digest_bytes_to_felts(DEFAULT_TO_ACCOUNT) + u128_to_felts(DEFAULT_FUNDING_AMOUNT))
    assert hash_no_pad(leaf)[1:] == prev[1:]


def test_bench_proof_verifies():
    vd, pf = golden("verifier.bin"), golden("proof.bin")
    assert lib().ora_verify(vd, len(vd), pf, len(pf)) == 0


def test_bench_proof_transcript():
    vd, pf = golden("verifier.bin"), golden("proof.bin")
    out = np.zeros(256, np.uint64)
    k = lib().ora_challenges(vd, len(vd), pf, len(pf), out)
    q = [int(x) for x in out[k - 28:k]]
    assert q[:4] == [34707, 64718, 9922, 116687]
    pow_resp = int(out[k - 29])
    assert 64 - pow_resp.bit_length() == 19


def test_circuit_digest_matches_verifier_bin():
    vd = golden("verifier.bin")
    cap = np.frombuffer(vd[8:8 + 512], np.uint64).copy()
    digest = np.frombuffer(vd[520:552], np.uint64)
    out = np.zeros(4, np.uint64)
    lib().ora_circuit_digest(cap, 16, 14, out)
    assert (out == digest).all()


@pytest.mark.parametrize("name", ["proof.bin", "dummy_proof.bin", "dummy_proof_zk.bin"])
def test_proof_bytes_roundtrip(name):
    # dummy proofs are the current (deg 13) circuit; their common data matches
    # bench-data's except degree_bits/hiding/arity, so rebuild it from the fixture
    pf = golden(name)
    cm = golden("common.bin") if name == "proof.bin" else current_common_bytes()
    out = ctypes.create_string_buffer(len(pf) + 64)
    n = lib().ora_proof_roundtrip(cm, len(cm), pf, len(pf), out)
    assert n == len(pf)
    assert out.raw[:n] == pf


def current_common_bytes():
    """common.bin with the current circuit's FRI shape: degree_bits 13, no hiding,
    arity [4,4] ([FIX] from the dummy proofs)."""
    cm = bytearray(golden("common.bin"))
    # FriParams.reduction_arity_bits: u64 len at 140 then 3 x u64; degree_bits at 172; hiding at 180
    assert struct.unpack_from("<Q", cm, 140)[0] == 3
    body = cm[:140] + struct.pack("<QQQ", 2, 4, 4) + struct.pack("<Q", 13) + bytes([0]) + cm[181:]
    # config.zero_knowledge (byte 49) off for the non-zk export
    body[49] = 0
    return bytes(body)


def test_common_roundtrip():
    cm = golden("common.bin")
    out = ctypes.create_string_buffer(len(cm) + 64)
    assert lib().ora_common_roundtrip(cm, len(cm), out) == len(cm)
    assert out.raw[:len(cm)] == cm


@pytest.mark.parametrize("name", ["dummy_proof.bin", "dummy_proof_zk.bin"])
def test_dummy_proof_merkle_self_consistency(name):
    """Every query's wires / zs_pp / quotient leaves hash up to their caps at one
    common leaf index (no verifier data is committed for the current circuit)."""
    pf = golden(name)
    L = lib()
    L.ora_merkle_find_index.restype = ctypes.c_long
    L.ora_merkle_find_index.argtypes = [U64P, ctypes.c_size_t, U64P, ctypes.c_uint, U64P, ctypes.c_uint]
    words = np.frombuffer(pf[:-(8 + 8 + 16 * 8)], np.uint8)
    caps = np.frombuffer(pf[:3 * 512], np.uint64).reshape(3, 16, 4)
    off = 3 * 512 + 257 * 16 + 2 * 512
    widths = [84, 135, 20, 16]
    for q in range(3):
        idx = []
        for o, w in enumerate(widths):
            leaf = np.frombuffer(pf[off:off + 8 * w], np.uint64).copy()
            off += 8 * w
            ns = pf[off]
            off += 1
            sibs = np.frombuffer(pf[off:off + 32 * ns], np.uint64).copy()
            off += 32 * ns
            assert ns == 12
            if o >= 1:
                cap = caps[o - 1].copy()
                idx.append(L.ora_merkle_find_index(leaf, w, sibs, ns, cap, 4))
        assert idx[0] >= 0 and idx[0] == idx[1] == idx[2]
        off += 256 + 1 + 8 * 32 + 256 + 1 + 4 * 32
    del words


def _flip(buf, pos):
    b = bytearray(buf)
    b[pos] ^= 1
    return bytes(b)


def test_negative_controls():
    vd, pf = golden("verifier.bin"), golden("proof.bin")
    L = lib()
    # corrupt an opening (first wire opening)
    assert L.ora_verify(vd, len(vd), _flip(pf, 3 * 512 + 84 * 16 + 3), len(pf)) != 0
    # corrupt a public input (verifier_tests.rs:25-66)
    assert L.ora_verify(vd, len(vd), _flip(pf, len(pf) - 8), len(pf)) != 0
    # corrupt the PoW witness
    assert L.ora_verify(vd, len(vd), _flip(pf, len(pf) - 136 - 8), len(pf)) != 0
    # corrupt a query leaf
    off = 3 * 512 + 257 * 16 + 3 * 512 + 8
    assert L.ora_verify(vd, len(vd), _flip(pf, off), len(pf)) != 0


def test_field_mul_against_python_bigint():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 2**63, 4096, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, 4096, dtype=np.uint64)
    b = rng.integers(0, 2**63, 4096, dtype=np.uint64) * np.uint64(2)
    a %= np.uint64(P)
    b %= np.uint64(P)
    edge = np.array([0, 1, P - 1, P - 2, 2**32, 2**32 - 1, 2**63, P - 2**32], np.uint64)
    a = np.concatenate([a, edge, edge])
    b = np.concatenate([b, edge, edge[::-1]])
    o = np.zeros_like(a)
    lib().ora_mul_many(a, b, o, len(a))
    for x, y, z in zip(a, b, o):
        assert int(z) == (int(x) * int(y)) % P


def test_ntt_conventions():
    rng = np.random.default_rng(2)
    log_n = 6
    n = 1 << log_n
    c = rng.integers(0, P, n, dtype=np.uint64)
    v = c.copy()
    lib().ora_fft(v, log_n)
    w = int(lib().ora_root_of_unity(log_n))
    for i in (0, 1, 5, 63):
        x = pow(w, i, P)
        assert int(v[i]) == sum(int(ck) * pow(x, k, P) for k, ck in enumerate(c)) % P
    back = v.copy()
    lib().ora_ifft(back, log_n)
    assert (back == c).all()
    g = 0xC65C18B67785D900
    lde = np.zeros(n * 8, np.uint64)
    lib().ora_lde(c, log_n, 3, g, lde)
    wN = int(lib().ora_root_of_unity(log_n + 3))
    for j in (0, 7, 100, 511):
        x = g * pow(wN, j, P) % P
        assert int(lde[j]) == sum(int(ck) * pow(x, k, P) for k, ck in enumerate(c)) % P
