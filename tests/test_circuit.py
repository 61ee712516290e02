"""Native Wormhole circuit (host side, CPU): shape, witness generation and the
reference's negative tests.

* CommonCircuitData bytes equal the reference's current-circuit common data
  (tests/golden/common.bin with the degree-13 non-zk FRI shape: SURVEY.md 0.4).
* Witnesses for the default test inputs and synthetic inputs satisfy every gate
  and copy constraint (oracle check on H).
* Public inputs decode as in prover_tests.rs:21-45.
* Witness conflicts raise "set twice with different values" like
  storage_proof_tests.rs:30-100; bad lengths raise like mod.rs:254-290.
"""
import ctypes

import numpy as np
import pytest

import wormhole_inputs as WI
from oracle_lib import U64P, lib as olib
from test_oracle_golden import current_common_bytes


@pytest.fixture(scope="module")
def circuit():
    from qp_wormhole import Circuit
    return Circuit.wormhole()


def check(circuit, w):
    L = olib()
    L.ora_check_witness.restype = ctypes.c_long
    L.ora_check_witness.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t]
    cb = circuit.common_data()
    pis = w.public_inputs()
    return L.ora_check_witness(cb, len(cb), circuit.constants_sigmas(), w.wires(), pis, len(pis))


def test_shape_matches_reference_common_data(circuit):
    assert circuit.degree_bits == 13
    assert circuit.num_wires == 135 and circuit.num_routed_wires == 80
    assert 4096 < circuit.gates_used <= 8192
    assert circuit.common_data() == current_common_bytes()


def test_zk_config_common_data():
    from qp_wormhole import Circuit
    c = Circuit.wormhole(zero_knowledge=True)
    cb = c.common_data()
    assert cb[49] == 1  # config.zero_knowledge


def test_default_inputs_witness(circuit):
    w = circuit.commit(WI.test_inputs())
    assert check(circuit, w) == -1
    f = WI.public_inputs_to_fields(w.public_inputs())
    assert f["nullifier"] == WI.EXPECTED_NULLIFIER
    assert f["root_hash"] == WI.DEFAULT_ROOT_HASH
    assert f["funding_amount"] == 1_000_000_000_000
    assert f["exit_account"] == bytes([4] * 32)


@pytest.mark.parametrize("k,depth", [(0, 0), (1, 1), (2, 7), (3, 20), (4, -1)])
def test_synthetic_witness(circuit, k, depth):
    from qp_wormhole.synthetic import synthetic_inputs
    w = circuit.commit(synthetic_inputs(k, depth))
    assert check(circuit, w) == -1


def test_wrong_witness_violates_constraints(circuit):
    w = circuit.commit(WI.test_inputs())
    wires = w.wires()
    wires[3, 10] ^= 1
    L = olib()
    cb = circuit.common_data()
    pis = w.public_inputs()
    assert L.ora_check_witness(cb, len(cb), circuit.constants_sigmas(), wires, pis, len(pis)) != -1


def _expect_conflict(circuit, inputs):
    from qp_wormhole import QpError
    with pytest.raises(QpError, match="set twice with different values"):
        circuit.commit(inputs)


def test_invalid_root_hash_fails(circuit):
    i = WI.test_inputs()
    i.public.root_hash = bytes(32)
    _expect_conflict(circuit, i)


def test_tampered_proof_fails(circuit):
    i = WI.test_inputs()
    node = bytearray(i.private.storage_proof.proof[0])
    node[i.private.storage_proof.indices[0] // 2] ^= 0xFF
    i.private.storage_proof.proof[0] = bytes(node)
    _expect_conflict(circuit, i)


def test_invalid_nonce_fails(circuit):
    i = WI.test_inputs()
    i.private.transfer_count = 5
    _expect_conflict(circuit, i)


def test_invalid_unspendable_account_fails(circuit):
    i = WI.test_inputs()
    i.private.unspendable_account = bytes(32)
    _expect_conflict(circuit, i)


def test_wrong_nullifier_fails(circuit):
    i = WI.test_inputs()
    i.public.nullifier = bytes(32)
    _expect_conflict(circuit, i)


def test_proof_too_long(circuit):
    from qp_wormhole import QpError
    i = WI.test_inputs()
    i.private.storage_proof.proof = i.private.storage_proof.proof * 3
    i.private.storage_proof.indices = i.private.storage_proof.indices * 3
    with pytest.raises(QpError, match="exceeds maximum allowed length"):
        circuit.commit(i)


def test_mismatched_indices(circuit):
    i = WI.test_inputs()
    i.private.storage_proof.indices = i.private.storage_proof.indices[:-1]
    with pytest.raises(ValueError, match="indices length"):
        circuit.commit(i)


def test_digest_out_of_field_range(circuit):
    from qp_wormhole import QpError
    i = WI.test_inputs()
    i.public.exit_account = bytes([0xFF] * 32)
    with pytest.raises(QpError, match="out of field range"):
        circuit.commit(i)


def test_oracle_prove_and_verify_default(circuit):
    """CPU oracle proof of the native circuit verifies and has the reference's
    current-circuit proof size (132,712 B)."""
    import struct
    w = circuit.commit(WI.test_inputs())
    cb = circuit.common_data()
    cs = circuit.constants_sigmas()
    pis = w.public_inputs()
    L = olib()
    L.ora_prove.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t, ctypes.c_char_p,
                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), U64P, U64P]
    out = ctypes.create_string_buffer(400000)
    ln = ctypes.c_size_t()
    cap = np.zeros(64, np.uint64)
    dig = np.zeros(4, np.uint64)
    assert L.ora_prove(cb, len(cb), cs, w.wires(), pis, len(pis), out, 400000, ctypes.byref(ln), cap, dig) == 0
    assert ln.value == 132712
    vd = struct.pack("<Q", 4) + cap.tobytes() + dig.tobytes() + cb
    pf = out.raw[:ln.value]
    assert L.ora_verify(vd, len(vd), pf, len(pf)) == 0
