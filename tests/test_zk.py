"""The zk config (standard_recursion_zk_config, the reference prover's default:
wormhole/circuit/src/circuit.rs:68-73) and the PublicInputGate row's random
witness cells.

What the reference's own fixtures say (wormhole/aggregator/data/dummy_proof{,_zk}.bin,
proofs of the same test_inputs() under the two configs, prover_tests.rs:56-82):
* the constants||sigmas commitment is shared (test_current_circuit_fixture.py), and
  neither proof has salt columns -- the preprocessing and proof shape are the same;
* the witnesses are equal except for the PublicInputGate row's unused wires
  4..num_wires-1, which the reference fills from RandomValueGenerators
  (randomize_unused_pi_wires) under BOTH configs, with different values in the
  two proofs (tests/test_reference_layout.py reads them out of the fixtures'
  openings and reproduces both proofs byte for byte with them).

So here those cells are an input of commit() (CircuitInputs.zk_randomness) in
both configs, and a proof stays a pure function of its inputs.  Left out they
are zeros under the non-zk config and a Poseidon nonce of the private inputs
under the zk config (the reference's RNG output is not reproducible by
construction).
"""
import ctypes

import numpy as np
import pytest

import wormhole_inputs as WI
from current_circuit_vd import parse_queries
from oracle_lib import P, U64P, golden, lib as olib


def test_reference_zk_and_non_zk_wires_caps_differ_under_one_constants_sigmas_cap():
    """The fixture pair: same public inputs, same constants||sigmas leaves where the
    two proofs open the same constants||sigmas cap entry, different wires caps."""
    a, b = golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")
    assert a[:512] != b[:512]                      # wires caps
    assert a[-8 * 17:] == b[-8 * 17:]              # PI length + 16 public inputs
    from current_circuit_vd import constants_sigmas_cap_entries
    ca, cb = constants_sigmas_cap_entries("dummy_proof.bin"), constants_sigmas_cap_entries("dummy_proof_zk.bin")
    shared = set(ca) & set(cb)
    assert shared and all(ca[c] == cb[c] for c in shared)
    # no salt columns in either: every query's wires leaf is exactly 135 felts
    for pf in (a, b):
        for q in parse_queries(pf)[:4]:
            assert len(q[1][0]) == 135


@pytest.fixture(scope="module")
def circuits():
    from qp_wormhole import Circuit
    return Circuit.wormhole(), Circuit.wormhole(zero_knowledge=True)


def _check(circ, w):
    L = olib()
    L.ora_check_witness.restype = ctypes.c_long
    L.ora_check_witness.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t]
    cb = circ.common_data()
    pis = w.public_inputs()
    return L.ora_check_witness(cb, len(cb), circ.constants_sigmas(), w.wires(), pis, len(pis))


def _pi_row(circ):
    sel0 = circ.constants_sigmas()[0]
    rows = np.nonzero(sel0 == 2)[0]     # PublicInputGate: gate index 2 in common-data order
    assert len(rows) == 1
    return int(rows[0])


def test_zk_preprocessing_equals_non_zk(circuits):
    nz, zk = circuits
    assert np.array_equal(nz.constants_sigmas(), zk.constants_sigmas())
    a, b = bytearray(nz.common_data()), bytearray(zk.common_data())
    assert a[49] == 0 and b[49] == 1            # config.zero_knowledge
    b[49] = 0
    assert a == b


def test_zk_cells_are_the_public_input_row_and_take_given_values(circuits):
    nz, zk = circuits
    import dataclasses
    r = [(0x1234_5678_9abc_def0 * (i + 1)) % P for i in range(zk.num_wires - 4)]
    inp = dataclasses.replace(WI.test_inputs(), zk_randomness=r)
    wz = zk.commit(inp).wires()
    wn = nz.commit(WI.test_inputs()).wires()
    row = _pi_row(zk)
    assert [int(x) for x in wz[4:, row]] == r
    diff = np.argwhere(wz != wn)
    assert all(int(c) >= 4 and int(rr) == row for c, rr in diff)
    assert _check(zk, zk.commit(inp)) == -1


def test_zk_default_randomness_is_deterministic_and_input_dependent(circuits):
    from qp_wormhole.synthetic import synthetic_inputs
    _, zk = circuits
    row = _pi_row(zk)
    w1 = zk.commit(WI.test_inputs()).wires()[4:, row]
    w2 = zk.commit(WI.test_inputs()).wires()[4:, row]
    w3 = zk.commit(synthetic_inputs(5, 3)).wires()[4:, row]
    assert np.array_equal(w1, w2)
    assert not np.array_equal(w1, w3)
    assert len(set(int(x) for x in w1)) == len(w1)   # no repeated / zero cells
    assert _check(zk, zk.commit(WI.test_inputs())) == -1


def test_zk_randomness_rejected_when_invalid(circuits):
    import dataclasses
    from qp_wormhole import QpError
    nz, zk = circuits
    for c in (nz, zk):
        with pytest.raises(QpError, match="canonical"):
            c.commit(dataclasses.replace(WI.test_inputs(), zk_randomness=[P] * (c.num_wires - 4)))


def test_non_zk_config_takes_given_pi_row_cells(circuits):
    """The reference's non-zk proofs carry random PI-row cells too."""
    import dataclasses
    nz, _ = circuits
    r = [(0x0fed_cba9_8765_4321 * (i + 3)) % P for i in range(nz.num_wires - 4)]
    w = nz.commit(dataclasses.replace(WI.test_inputs(), zk_randomness=r))
    row = _pi_row(nz)
    assert [int(x) for x in w.wires()[4:, row]] == r
    assert not nz.commit(WI.test_inputs()).wires()[4:, row].any()   # default: zeros
    assert _check(nz, w) == -1


def test_voting_zk_cells(circuits):
    import dataclasses
    from qp_wormhole import Circuit
    from qp_wormhole.synthetic import vote_test_inputs
    zk = Circuit.voting(zero_knowledge=True)
    nz = Circuit.voting()
    r = list(range(7, 7 + zk.num_wires - 4))
    wz = zk.commit(dataclasses.replace(vote_test_inputs(), zk_randomness=r)).wires()
    wn = nz.commit(vote_test_inputs()).wires()
    row = _pi_row(zk)
    assert [int(x) for x in wz[4:, row]] == r
    assert all(int(c) >= 4 and int(rr) == row for c, rr in np.argwhere(wz != wn))
