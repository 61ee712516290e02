"""Default Wormhole test inputs, mirroring wormhole/tests/test-helpers/src/lib.rs:10-59
(TestInputs for CircuitInputs) with the storage-proof nodes loaded from the
committed fixture tests/golden/storage_proof.json."""
from golden_storage_proof import DEFAULT_STORAGE_PROOF, DEFAULT_STORAGE_PROOF_INDICES
from qp_wormhole import CircuitInputs, PrivateCircuitInputs, ProcessedStorageProof, PublicCircuitInputs
from qp_wormhole.synthetic import nullifier, unspendable_account

DEFAULT_SECRET = bytes.fromhex("4c8587bd422e01d961acdc75e7d66f6761b7af7c9b1864a492f369c9d6724f05")
DEFAULT_TRANSFER_COUNT = 4
DEFAULT_FUNDING_ACCOUNT = bytes([226, 124, 203, 9, 80, 60, 124, 205, 165, 5, 178, 216, 195, 15, 149, 38, 116, 1,
                                 238, 133, 181, 154, 106, 17, 41, 228, 118, 179, 82, 141, 225, 76])
DEFAULT_FUNDING_AMOUNT = int.from_bytes(bytes([0, 16, 165, 212, 232] + [0] * 11), "little")
DEFAULT_EXIT_ACCOUNT = bytes([4] * 32)
DEFAULT_ROOT_HASH = bytes.fromhex("5ffa2ab5b0db9883b22b1e5810932ea9d9eab1840730fd39ace71c26bb8d082d")
EXPECTED_NULLIFIER = bytes([169, 76, 150, 35, 66, 248, 76, 193, 57, 204, 106, 33, 169, 160, 248, 113, 235, 144,
                            212, 48, 9, 232, 146, 7, 105, 125, 170, 24, 33, 54, 135, 28])


def storage_proof():
    return ProcessedStorageProof([bytes.fromhex(h) for h in DEFAULT_STORAGE_PROOF],
                                 list(DEFAULT_STORAGE_PROOF_INDICES))


def test_inputs():
    return CircuitInputs(
        PublicCircuitInputs(DEFAULT_FUNDING_AMOUNT, nullifier(DEFAULT_SECRET, DEFAULT_TRANSFER_COUNT),
                            DEFAULT_ROOT_HASH, DEFAULT_EXIT_ACCOUNT),
        PrivateCircuitInputs(DEFAULT_SECRET, storage_proof(), DEFAULT_TRANSFER_COUNT, DEFAULT_FUNDING_ACCOUNT,
                             unspendable_account(DEFAULT_SECRET)))


def public_inputs_to_fields(pis):
    """PublicCircuitInputs::try_from_slice (wormhole/circuit/src/inputs.rs:91-124)."""
    import struct
    assert len(pis) == 16
    d2b = lambda d: b"".join(struct.pack("<Q", int(x)) for x in d)  # noqa: E731
    amount = 0
    for i, limb in enumerate(pis[8:12]):
        assert int(limb) < 2**32
        amount |= int(limb) << (96 - 32 * i)
    return {"nullifier": d2b(pis[0:4]), "root_hash": d2b(pis[4:8]), "funding_amount": amount,
            "exit_account": d2b(pis[12:16])}
