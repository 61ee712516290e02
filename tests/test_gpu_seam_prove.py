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
