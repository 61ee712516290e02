"""INTEGRATION.md binding A end to end: plonky2's prove() composed from the
routine-level seams (tests/seam_prover.py; the oracle plays the host code a
patched qp-plonky2 keeps) produces byte for byte the proof of the oracle's
monolithic CPU prover and of the GPU whole-circuit prover, and it verifies."""
import numpy as np
import pytest

import wormhole_inputs as WI
from seam_prover import prove
from test_gpu_prover import oracle_prove, verify

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import qp_wormhole
    c = qp_wormhole.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("zk", [False, True])
def test_seam_composed_wormhole_proof(ctx, zk):
    import qp_wormhole
    circ = qp_wormhole.Circuit.wormhole(zero_knowledge=zk)
    w = circ.commit(WI.test_inputs())
    wires, pis = w.wires(), w.public_inputs()
    seam = prove(ctx, circ, wires, pis)
    whole = qp_wormhole.Prover(ctx, circ, 1)
    gpu = whole.prove_witnesses([w])[0]
    assert seam == gpu
    if not zk:
        cpu, vd = oracle_prove(circ, wires, pis)
        assert seam == cpu
    assert verify(whole.verifier_data(), seam) == 0


def test_seam_composed_voting_proof(ctx):
    """A second shape: degree 8, one FRI layer, 13 public inputs."""
    import qp_wormhole
    from qp_wormhole.synthetic import synthetic_vote_inputs
    circ = qp_wormhole.Circuit.voting()
    w = circ.commit(synthetic_vote_inputs(3))
    seam = prove(ctx, circ, w.wires(), w.public_inputs())
    whole = qp_wormhole.Prover(ctx, circ, 1)
    assert seam == whole.prove_witnesses([w])[0]
    assert verify(whole.verifier_data(), seam) == 0


def test_seam_composed_degree15_aggregation_proof(ctx):
    """tree.rs:136's CircuitData::prove at degree 2^15 through the seams: the
    aggregation circuit of five of the reference's own leaf proofs (level 1 of a
    5-ary tree, benches/aggregator.rs:119-123; a 2048-leaf root has this degree
    too).  qp_quotient's coset iNTT and the commitments take their large-n forms;
    bytes == the GPU whole-circuit prover's == the oracle's, and it verifies."""
    import qp_wormhole
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    vo = vd[:len(vd) - len(cb)]
    leaves = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    chunk = [leaves[i % 2] for i in range(5)]
    circ = qp_wormhole.Circuit.aggregation(cb, 5)
    assert circ.degree_bits == 15
    w = circ.commit_proofs(vo, chunk)
    wires, pis = w.wires(), w.public_inputs()
    seam = prove(ctx, circ, wires, pis)
    whole = qp_wormhole.Prover(ctx, circ, 1)
    assert seam == whole.prove_witnesses([w])[0]
    cpu, ovd = oracle_prove(circ, wires, pis)
    assert seam == cpu
    assert verify(ovd, seam) == 0
    whole.free()
