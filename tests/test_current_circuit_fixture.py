"""The reference's current-circuit proofs (tests/golden/dummy_proof{,_zk}.bin)
verify in full under verifier data reconstructed from their own Merkle paths.

This pins, by a reference-held fixture rather than by synthesis:
* the degree-13 CommonCircuitData the native circuit emits (gate list,
  selector groups, constants count, k_is, FRI shape): the oracle verifier's
  zeta-identity over all 6 gates and the permutation argument holds for both
  proofs, as do all 28 queries x (4 initial trees + 2 FRI layer trees), the
  folds, the final polynomial and the PoW;
* that standard_recursion_zk_config under the workspace's `no_random` feature
  (Cargo.toml:20-22) changes neither the preprocessing (identical
  constants||sigmas cap) nor the proof shape (no salt columns);
* the transcript (the query indices derived from it equal the leaf indices the
  Merkle paths prove).
"""
import numpy as np
import pytest

from current_circuit_vd import (brute_force_query_indices, constants_sigmas_cap_entries,
                                current_circuit_verifier_data, query_indices)
from oracle_lib import golden, lib
from test_oracle_golden import current_common_bytes


@pytest.fixture(scope="module")
def vd():
    return current_circuit_verifier_data(current_common_bytes())[0]


def test_zk_and_non_zk_share_the_constants_sigmas_commitment():
    a = constants_sigmas_cap_entries("dummy_proof.bin")
    b = constants_sigmas_cap_entries("dummy_proof_zk.bin")
    common = set(a) & set(b)
    assert len(common) >= 8
    for c in common:
        assert a[c] == b[c]
    assert set(a) | set(b) == set(range(16))


@pytest.mark.parametrize("name", ["dummy_proof.bin", "dummy_proof_zk.bin"])
def test_dummy_proof_verifies_under_reconstructed_verifier_data(vd, name):
    pf = golden(name)
    assert lib().ora_verify(vd, len(vd), pf, len(pf)) == 0


@pytest.mark.parametrize("name", ["dummy_proof.bin", "dummy_proof_zk.bin"])
def test_transcript_query_indices_match_merkle_paths(vd, name):
    pf = golden(name)
    out = np.zeros(256, np.uint64)
    k = lib().ora_challenges(vd, len(vd), pf, len(pf), out)
    q = [int(x) for x in out[k - 28:k]]
    assert q == list(query_indices(name))
    assert 64 - int(out[k - 29]).bit_length() >= 16  # PoW response


def test_negative_controls(vd):
    pf = golden("dummy_proof.bin")
    L = lib()
    bad = bytearray(vd)
    bad[8 + 5 * 32] ^= 1  # one constants||sigmas cap entry
    assert L.ora_verify(bytes(bad), len(bad), pf, len(pf)) != 0
    bad = bytearray(vd)
    bad[8 + 512] ^= 1  # circuit digest
    assert L.ora_verify(bytes(bad), len(bad), pf, len(pf)) != 0
    p2 = bytearray(pf)
    p2[3 * 512 + 84 * 16 + 5] ^= 1  # a wire opening at zeta
    assert L.ora_verify(vd, len(vd), bytes(p2), len(p2)) != 0
    # k_is[1] of the common data (the coset shift g) replaced by 7
    cb = bytearray(current_common_bytes())
    k1 = cb.index((0xc65c18b67785d900).to_bytes(8, "little"))
    cb[k1:k1 + 8] = (7).to_bytes(8, "little")
    bad = vd[:len(vd) - len(cb)] + bytes(cb)
    assert L.ora_verify(bad, len(bad), pf, len(pf)) != 0


def test_native_circuit_common_data_is_the_verified_one():
    from qp_wormhole import Circuit
    c = Circuit.wormhole()
    assert c.common_data() == current_common_bytes()


@pytest.mark.parametrize("name", ["dummy_proof.bin", "dummy_proof_zk.bin"])
def test_committed_query_indices_match_the_merkle_search(name):
    """tests/golden/dummy_query_indices.json against a fresh Merkle-path search
    (first 3 queries; the transcript test above covers all 28)."""
    assert brute_force_query_indices(name, 3) == query_indices(name)[:3]
