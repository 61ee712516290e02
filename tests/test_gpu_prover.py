"""GPU prover parity: proof bytes from the HIP prover (via the C ABI) are
bit-identical to the CPU oracle prover's on the same witness, verify under the
oracle verifier (which accepts the reference's own wormhole/bench-data proof),
and are independent of batch composition.  SURVEY.md 8 rows a2-a14."""
import ctypes
import struct

import numpy as np
import pytest

import wormhole_inputs as WI
from oracle_lib import U64P, lib as olib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import qp_wormhole
    ctx = qp_wormhole.Context(0)
    circ = qp_wormhole.Circuit.wormhole()
    prover = qp_wormhole.Prover(ctx, circ, max_batch=4)
    yield ctx, circ, prover
    prover.free()
    ctx.close()


def oracle_prove(circ, wires, pis):
    L = olib()
    L.ora_prove.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t, ctypes.c_char_p,
                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), U64P, U64P]
    cb = circ.common_data()
    out = ctypes.create_string_buffer(400000)
    ln = ctypes.c_size_t()
    cap = np.zeros(64, np.uint64)
    dig = np.zeros(4, np.uint64)
    pis = np.ascontiguousarray(pis, np.uint64)
    rc = L.ora_prove(cb, len(cb), circ.constants_sigmas(), np.ascontiguousarray(wires, np.uint64), pis, len(pis),
                     out, 400000, ctypes.byref(ln), cap, dig)
    assert rc == 0
    vd = struct.pack("<Q", 4) + cap.tobytes() + dig.tobytes() + cb
    return out.raw[:ln.value], vd


def verify(vd, pf):
    return olib().ora_verify(vd, len(vd), pf, len(pf))


def test_verifier_data_matches_oracle(env):
    ctx, circ, prover = env
    w = circ.commit(WI.test_inputs())
    _, vd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert prover.verifier_data() == vd


def test_default_proof_bit_exact(env):
    ctx, circ, prover = env
    w = circ.commit(WI.test_inputs())
    gpu = prover.prove_witnesses([w])[0]
    cpu, vd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert len(gpu) == 132712
    assert gpu == cpu
    assert verify(prover.verifier_data(), gpu) == 0


def test_synthetic_batch_bit_exact_and_batch_independent(env):
    from qp_wormhole.synthetic import synthetic_inputs
    ctx, circ, prover = env
    ws = [circ.commit(synthetic_inputs(k, d)) for k, d in ((11, 0), (12, 3), (13, 20))]
    batch = prover.prove_witnesses(ws)
    vd = prover.verifier_data()
    for i, w in enumerate(ws):
        assert verify(vd, batch[i]) == 0, i
    cpu, _ = oracle_prove(circ, ws[1].wires(), ws[1].public_inputs())
    assert batch[1] == cpu
    single = prover.prove_witnesses([ws[2]])[0]
    assert single == batch[2]
    # more proofs than max_batch: split into batches transparently
    many = prover.prove_witnesses(ws + ws[:2])
    assert many[3] == batch[0] and many[4] == batch[1]


def test_prove_wires_matches_witness_path(env):
    ctx, circ, prover = env
    w = circ.commit(WI.test_inputs())
    a = prover.prove_witnesses([w])[0]
    b = prover.prove_wires(w.wires()[None], w.public_inputs()[None])[0]
    assert a == b


def test_unsatisfied_witness_does_not_verify(env):
    ctx, circ, prover = env
    w = circ.commit(WI.test_inputs())
    wires = w.wires()
    wires[3, 10] ^= 1
    pf = prover.prove_wires(wires[None], w.public_inputs()[None])[0]
    assert verify(prover.verifier_data(), pf) != 0


def test_wormhole_prover_api():
    """prover_tests.rs:14-56: commit_and_prove, proof_can_be_deserialized; commit
    is single-use (lib.rs:209-212)."""
    import qp_wormhole
    p = qp_wormhole.WormholeProver("standard_recursion_config")
    proof = p.commit(WI.test_inputs()).prove()
    f = WI.public_inputs_to_fields(proof.public_inputs)
    assert f["nullifier"] == WI.EXPECTED_NULLIFIER
    assert f["root_hash"] == WI.DEFAULT_ROOT_HASH
    assert f["funding_amount"] == 1_000_000_000_000
    assert f["exit_account"] == bytes([4] * 32)
    assert len(proof.to_bytes()) == 132712
    p2 = qp_wormhole.WormholeProver()
    p2.commit(WI.test_inputs())
    with pytest.raises(qp_wormhole.QpError):
        p2.commit(WI.test_inputs())
    with pytest.raises(qp_wormhole.QpError):
        qp_wormhole.WormholeProver().prove()


def test_per_gate_quotient_launches_bit_exact(env, monkeypatch):
    """The per-gate quotient launches (k_quotient_prefix + k_quotient_part, the
    aggregation circuits' path; path hook quotient_parts=1 forces them) on the
    leaf circuit: the same proofs as the single-read kernel, for a satisfied
    witness and one with a corrupted routed wire (nonzero gate and permutation
    terms everywhere)."""
    import qp_wormhole
    ctx, circ, prover = env
    w = circ.commit(WI.test_inputs())
    wires = np.stack([w.wires(), w.wires()])
    wires[1, 41, 5] ^= 1
    pis = np.stack([w.public_inputs(), w.public_inputs()])
    ref = prover.prove_wires(wires, pis)
    monkeypatch.setenv("QPGPU_PATHS", "quotient_parts=1")
    parts = qp_wormhole.Prover(ctx, circ, max_batch=4)
    try:
        assert parts.prove_wires(wires, pis) == ref
    finally:
        parts.free()