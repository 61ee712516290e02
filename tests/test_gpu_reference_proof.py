"""The GPU prover reproduces the reference's own current-circuit proofs byte
for byte (tests/golden/dummy_proof{,_zk}.bin, written by the Rust prover:
wormhole/tests/src/prover/prover_tests.rs:56-82): the native circuit's
preprocessing is the reference's (tests/test_reference_layout.py), the
witness of CircuitInputs::test_inputs() with the PublicInputGate row's random
cells taken from the fixture is the reference's, and the fixture's PoW witness
is forced through the test-only qp_prover_debug_force_pow (the reference's
find_any witness is nondeterministic).  Both the whole-circuit path
(CircuitInputs -> device witness generation -> prove) and the host-witness
path are checked."""
import struct

import pytest

from oracle_lib import golden
from test_reference_layout import PROOFS, fixture_points, reference_pi_cells, reference_test_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def points():
    return fixture_points()


@pytest.mark.parametrize("name", PROOFS)
def test_gpu_proof_is_the_reference_proof(points, name):
    import qp_wormhole
    zk = name.endswith("_zk.bin")
    ref = golden(name)
    pow_w = struct.unpack_from("<Q", ref, len(ref) - 8 * (2 + 16))[0]
    ctx = qp_wormhole.Context(0)
    circ = qp_wormhole.Circuit.wormhole(zero_knowledge=zk)
    prover = qp_wormhole.Prover(ctx, circ, max_batch=2)
    try:
        inp = reference_test_inputs()
        inp.zk_randomness = reference_pi_cells(points, qp_wormhole.Circuit.wormhole(zero_knowledge=False), name)
        prover.debug_force_pow(pow_w)
        # device witness generation from CircuitInputs (the benched path)
        from_inputs = prover.prove_inputs([inp, inp])
        # host witness generation
        from_witness = prover.prove_witnesses([circ.commit(inp)])
        prover.debug_force_pow(0, enable=False)
        assert from_inputs[0] == ref
        assert from_inputs[1] == ref
        assert from_witness[0] == ref
    finally:
        prover.free()
        ctx.close()
