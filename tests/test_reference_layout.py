"""The native Wormhole circuit's preprocessing and witness against the
reference's own current-circuit proofs (tests/golden/dummy_proof{,_zk}.bin,
written by the Rust prover: wormhole/tests/src/prover/prover_tests.rs:56-82).

Each proof opens every constants||sigmas and wire column at its 28 query
points g * w_{2^16}^rev16(i) (g = 0xc65c18b67785d900, the qp-plonky2-field
coset shift) and at zeta: 29 evaluations of a degree < 2^13 polynomial per
column and proof, so equality at all of them is equality of the columns
(a wrong column matches one random point with probability 2^13 / p).

Pinned here:
* the 4 constants columns (2 selectors, 2 gate constants) and the 80 sigma
  columns equal the reference's: the gate kind and gate constants of every one
  of the 8192 rows -- plonky2's build order (user gadgets, PI hash,
  PublicInputGate at row 7039, ConstantGates in canonical constant order, Noop
  padding) -- and the copy-constraint routing, including qp-plonky2's is_equal
  (diff * inv == not_equal checked by a sub op connected to zero instead of
  upstream's copy constraint: csrc/circuit.cpp is_equal); so the
  constants||sigmas Merkle cap and the circuit digest are the reference's own,
  and the reference's proofs verify under the library's verifier data;
* the witness of CircuitInputs::test_inputs() (test-helpers/src/lib.rs:10-59)
  equals the reference's in all 135 columns at every row but the
  PublicInputGate row, whose spare wires the reference fills with
  RandomValueGenerator values in both configs (different in the two proofs);
* with those cells taken from a reference proof and its PoW witness forced
  (find_any's witness is nondeterministic), the CPU oracle prover's bytes ARE
  the reference's proof, for both fixtures (the GPU prover is held to the
  fixtures themselves by tests/test_gpu_reference_proof.py);
* the aggregator pads with the reference's own dummy proof (util.rs:6-9).
"""
import numpy as np
import pytest

from current_circuit_vd import current_circuit_verifier_data, parse_queries, query_indices
from oracle_lib import P, golden, lib
from test_oracle_golden import current_common_bytes
from wormhole_inputs import test_inputs as reference_test_inputs

GEN = 0xc65c18b67785d900
LOG_N = 13
N = 1 << LOG_N
PI_ROW = 7039
OPEN_OFF = 3 * 512          # openings follow the wires / zs / quotient caps
NUM_CS = 84
MATCHING_WIRE_COLS = list(range(135))
PROOFS = ["dummy_proof.bin", "dummy_proof_zk.bin"]


def _rev(i, bits):
    return int(format(i, f"0{bits}b")[::-1], 2)


@pytest.fixture(scope="module")
def points():
    return fixture_points()


def fixture_points():
    """per proof: (xs [m][2] ext points: 28 query points then zeta,
    constants||sigmas values [m][84], wire values [m][135][2])"""
    vd = current_circuit_verifier_data(current_common_bytes())[0]
    L = lib()
    w16 = int(L.ora_root_of_unity(16))
    out = {}
    for name in PROOFS:
        pf = golden(name)
        qs = parse_queries(pf)
        xs = [(GEN * pow(w16, _rev(i, 16), P) % P, 0) for i in query_indices(name)]
        ch = np.zeros(256, np.uint64)
        L.ora_challenges(vd, len(vd), pf, len(pf), ch)
        xs.append((int(ch[6]), int(ch[7])))
        op = np.frombuffer(pf[OPEN_OFF:OPEN_OFF + 16 * (NUM_CS + 135)], np.uint64).reshape(-1, 2)
        cs = [np.stack([q[0][0], np.zeros(NUM_CS, np.uint64)], 1) for q in qs] + [op[:NUM_CS]]
        wires = [np.stack([q[1][0], np.zeros(135, np.uint64)], 1) for q in qs] + [op[NUM_CS:]]
        out[name] = (np.array(xs, np.uint64), np.stack(cs), np.stack(wires))
    return out


def evaluate(cols, xs):
    """[ncols][n] values -> [ncols][m][2] evaluations at ext points xs [m][2]"""
    cols = np.ascontiguousarray(cols, np.uint64)
    out = np.zeros(cols.shape[0] * len(xs) * 2, np.uint64)
    lib().ora_eval_values(cols.reshape(-1), cols.shape[0], LOG_N, np.ascontiguousarray(xs).reshape(-1), len(xs), out)
    return out.reshape(cols.shape[0], len(xs), 2)


def _ext_mul(a, b):
    return ((a[0] * b[0] + 7 * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _ext_inv(a):
    d = (a[0] * a[0] - 7 * a[1] * a[1]) % P
    di = pow(d, P - 2, P)
    return (a[0] * di % P, (P - a[1]) * di % P)


@pytest.fixture(scope="module")
def circuit():
    from qp_wormhole import Circuit
    return Circuit.wormhole(zero_knowledge=False)


@pytest.mark.parametrize("name", PROOFS)
def test_constants_columns_equal_the_reference(points, circuit, name):
    xs, ref_cs, _ = points[name]
    ours = evaluate(circuit.constants_sigmas()[:4], xs)
    for c in range(4):
        assert np.array_equal(ours[c], ref_cs[:, c]), f"constants column {c}"


def test_public_input_gate_row(circuit):
    sel0 = circuit.constants_sigmas()[0]
    assert int(np.nonzero(sel0 == 2)[0][0]) == PI_ROW
    # ConstantGates (selector value 1) right after it, Noop (0) padding after those
    r = PI_ROW + 1
    while sel0[r] == 1:
        r += 1
    assert r == PI_ROW + 1 + 93 and not sel0[r:].any()


@pytest.mark.parametrize("name", PROOFS)
def test_witness_equals_the_reference_outside_the_pi_row(points, circuit, name):
    """ref - ours = delta_c * L_PI_ROW(x) at all 29 points, one delta per column."""
    xs, _, ref_w = points[name]
    inp = reference_test_inputs()
    inp.zk_randomness = [0] * 131
    wv = circuit.commit(inp).wires()
    ours = evaluate(wv[MATCHING_WIRE_COLS], xs)
    unit = np.zeros((1, N), np.uint64)
    unit[0, PI_ROW] = 1
    lpi = evaluate(unit, xs)[0]
    deltas = []
    for k, col in enumerate(MATCHING_WIRE_COLS):
        diff = [((int(ref_w[j, col, 0]) - int(ours[k, j, 0])) % P, (int(ref_w[j, col, 1]) - int(ours[k, j, 1])) % P)
                for j in range(len(xs))]
        delta = _ext_mul(diff[0], _ext_inv((int(lpi[0, 0]), int(lpi[0, 1]))))
        assert delta[1] == 0, f"column {col}: PI-row value not in the base field"
        for j in range(1, len(xs)):
            assert diff[j] == _ext_mul(delta, (int(lpi[j, 0]), int(lpi[j, 1]))), f"column {col}, point {j}"
        deltas.append(delta[0])
    assert not any(deltas[:4])  # the PI row's public-input-hash wires
    assert all(deltas[4:])  # the reference's random PI-row cells (ours: zero)


def test_pi_row_cells_differ_between_the_two_proofs(points, circuit):
    """The PI row's random cells are fresh per proof (zk and non-zk alike)."""
    inp = reference_test_inputs()
    inp.zk_randomness = [0] * 131
    wv = circuit.commit(inp).wires()
    col = 80
    vals = []
    for name in PROOFS:
        xs, _, ref_w = points[name]
        unit = np.zeros((1, N), np.uint64)
        unit[0, PI_ROW] = 1
        lpi = evaluate(unit, xs[:1])[0, 0]
        ours = evaluate(wv[col:col + 1], xs[:1])[0, 0]
        d = ((int(ref_w[0, col, 0]) - int(ours[0])) % P, 0)
        vals.append(_ext_mul(d, _ext_inv((int(lpi[0]), int(lpi[1]))))[0])
    assert vals[0] != vals[1]


def reference_pi_cells(points, circuit, name):
    """The 131 random PublicInputGate-row cells of a reference proof: the
    one-row residual of each wire column (proven one-row by the test above)."""
    xs, _, ref_w = points[name]
    inp = reference_test_inputs()
    inp.zk_randomness = [0] * 131
    wv = circuit.commit(inp).wires()
    ours = evaluate(wv[4:], xs[:1])
    unit = np.zeros((1, N), np.uint64)
    unit[0, PI_ROW] = 1
    li = _ext_inv(tuple(int(v) for v in evaluate(unit, xs[:1])[0, 0]))
    return [_ext_mul(((int(ref_w[0, 4 + k, 0]) - int(ours[k, 0, 0])) % P, 0), li)[0] for k in range(131)]


def test_preprocessing_commitment_is_the_reference_one(circuit):
    """constants||sigmas LDE + Merkle cap (oracle commit) == the cap the
    fixtures' query paths climb to; circuit digest with it."""
    vd, cap, dig = current_circuit_verifier_data(current_common_bytes())
    cs = np.ascontiguousarray(circuit.constants_sigmas(), np.uint64)
    out = np.zeros(64, np.uint64)
    rc = lib().ora_commit_values(cs.reshape(-1), NUM_CS, LOG_N, 3, 4, None, 0, 0, None, None, out)
    assert rc == 0
    assert np.array_equal(out.reshape(16, 4), cap)


def reference_proof_via_oracle(points, name):
    import ctypes
    import struct
    from oracle_lib import U64P
    from qp_wormhole import Circuit
    zk = name.endswith("_zk.bin")
    circ = Circuit.wormhole(zero_knowledge=zk)
    inp = reference_test_inputs()
    inp.zk_randomness = reference_pi_cells(points, circ, name)
    w = circ.commit(inp)
    pf = golden(name)
    npis = 16
    pow_w = struct.unpack_from("<Q", pf, len(pf) - 8 * (2 + npis))[0]
    L = lib()
    L.ora_prove.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t, ctypes.c_char_p,
                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), U64P, U64P]
    L.ora_force_pow_witness.argtypes = [ctypes.c_uint64, ctypes.c_int]
    cb = circ.common_data()
    out = ctypes.create_string_buffer(400000)
    ln = ctypes.c_size_t()
    cap = np.zeros(64, np.uint64)
    dig = np.zeros(4, np.uint64)
    pis = np.ascontiguousarray(w.public_inputs(), np.uint64)
    L.ora_force_pow_witness(pow_w, 1)
    try:
        rc = L.ora_prove(cb, len(cb), circ.constants_sigmas(), np.ascontiguousarray(w.wires(), np.uint64), pis,
                         len(pis), out, 400000, ctypes.byref(ln), cap, dig)
    finally:
        L.ora_force_pow_witness(0, 0)
    assert rc == 0
    return out.raw[:ln.value], cap, dig


@pytest.mark.parametrize("name", PROOFS)
def test_oracle_prover_reproduces_the_reference_proof(points, name):
    proof, cap, dig = reference_proof_via_oracle(points, name)
    vd, ref_cap, ref_dig = current_circuit_verifier_data(current_common_bytes())
    assert np.array_equal(cap.reshape(16, 4), ref_cap)
    assert np.array_equal(dig, ref_dig)
    assert proof == golden(name)


@pytest.mark.parametrize("name", PROOFS)
def test_reference_proofs_verify_under_the_library_verifier_data(name):
    """VerifierOnlyCircuitData assembled from the native circuit alone (oracle
    commit of its constants||sigmas, circuit digest) accepts the reference's
    proofs -- what the aggregator's padding with them relies on."""
    import struct
    from qp_wormhole import Circuit
    circ = Circuit.wormhole(zero_knowledge=name.endswith("_zk.bin"))
    cs = np.ascontiguousarray(circ.constants_sigmas(), np.uint64)
    cap = np.zeros(64, np.uint64)
    assert lib().ora_commit_values(cs.reshape(-1), NUM_CS, LOG_N, 3, 4, None, 0, 0, None, None, cap) == 0
    dig = np.zeros(4, np.uint64)
    lib().ora_circuit_digest(cap, 16, LOG_N, dig)
    vd = struct.pack("<Q", 4) + cap.tobytes() + dig.tobytes() + circ.common_data()
    pf = golden(name)
    assert lib().ora_verify(vd, len(vd), pf, len(pf)) == 0


def test_aggregator_pads_with_the_reference_dummy_proof():
    """util.rs:6-9: the padding proof is the reference's own (zk unless no_zk)."""
    from qp_wormhole.aggregator import CircuitData, WormholeProofAggregator
    from qp_wormhole import Circuit
    for zk, name in ((True, "dummy_proof_zk.bin"), (False, "dummy_proof.bin")):
        agg = WormholeProofAggregator(CircuitData(Circuit.wormhole(zero_knowledge=zk).common_data(), b""))
        d = agg.dummy_proof()
        assert d.to_bytes() == golden(name)
        assert len(d.public_inputs) == 16


def test_committed_pi_cells_fixture_is_current():
    """tests/golden/reference_pi_cells.json (what bench.py's parity check and the
    GPU test read) equals a fresh derivation from the fixtures."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_pi_cells import cells
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_pi_cells.json")) as f:
        assert json.load(f) == json.loads(json.dumps(cells()))
