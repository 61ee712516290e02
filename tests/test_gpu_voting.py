"""GPU prover on the voting circuit (BASELINE config 5: "Voting circuit proof
on 1xMI355X", voting/src/lib.rs): degree 2^8, one FRI layer (arity 16), final
polynomial of 16 coefficients — the small-circuit shape of the same prove()
path.  Proof bytes are bit-identical to the CPU oracle prover's and verify
under the oracle verifier; batches are independent of composition."""
import pytest

from test_voting import oracle_prove
from oracle_lib import lib as olib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import qp_wormhole
    ctx = qp_wormhole.Context(0)
    circ = qp_wormhole.Circuit.voting()
    prover = qp_wormhole.Prover(ctx, circ, max_batch=8)
    yield ctx, circ, prover
    prover.free()
    ctx.close()


def verify(vd, pf):
    return olib().ora_verify(vd, len(vd), pf, len(pf))


def test_vote_end_to_end_bit_exact(env):
    """test_vote_circuit_end_to_end (voting/src/lib.rs:339-357) on the GPU."""
    from qp_wormhole.synthetic import vote_test_inputs
    ctx, circ, prover = env
    w = circ.commit(vote_test_inputs())
    gpu = prover.prove_witnesses([w])[0]
    cpu, vd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert prover.verifier_data() == vd
    assert gpu == cpu
    assert verify(vd, gpu) == 0


def test_vote_batch_bit_exact(env):
    from qp_wormhole.synthetic import synthetic_vote_inputs
    ctx, circ, prover = env
    ws = [circ.commit(synthetic_vote_inputs(k, d)) for k, d in ((1, 0), (2, 5), (3, 31), (4, -1), (5, 12))]
    batch = prover.prove_witnesses(ws)
    vd = prover.verifier_data()
    for i, w in enumerate(ws):
        assert verify(vd, batch[i]) == 0, i
    for i in (0, 2):
        cpu, _ = oracle_prove(circ, ws[i].wires(), ws[i].public_inputs())
        assert batch[i] == cpu, i
    assert prover.prove_witnesses([ws[3]])[0] == batch[3]
    # more proofs than max_batch
    many = prover.prove_witnesses(ws + ws)
    assert many[7] == batch[2]


def test_vote_unsatisfied_witness_does_not_verify(env):
    from qp_wormhole.synthetic import vote_test_inputs
    ctx, circ, prover = env
    w = circ.commit(vote_test_inputs())
    wires = w.wires()
    wires[5, 3] ^= 1
    pf = prover.prove_wires(wires[None], w.public_inputs()[None])[0]
    assert verify(prover.verifier_data(), pf) != 0
