"""End-to-end proving from circuit inputs with witness generation on the device
(WormholeProver::commit + prove, wormhole/prover/src/lib.rs:209-237;
generate_partial_witness = SURVEY.md 8(f) row 3), the zk config, and the
batch-256 configuration (BASELINE configs[2]).

Parity: proofs from qp_prover_prove_{wormhole,voting}_inputs (commit on the
host, every generator on the GPU) are byte-identical to proofs from host-
generated witnesses, which are byte-identical to the CPU oracle prover's; all
verify under the oracle verifier that accepts the reference's own proofs.
"""
import struct

import pytest

import wormhole_inputs as WI
from test_gpu_prover import oracle_prove, verify

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import qp_wormhole
    ctx = qp_wormhole.Context(0)
    circ = qp_wormhole.Circuit.wormhole()
    prover = qp_wormhole.Prover(ctx, circ, max_batch=8)
    yield ctx, circ, prover
    prover.free()
    ctx.close()


def test_device_witness_matches_host_witness(env):
    from qp_wormhole.synthetic import synthetic_inputs
    ctx, circ, prover = env
    inputs = [WI.test_inputs()] + [synthetic_inputs(k, d) for k, d in ((21, 0), (22, 1), (23, 7), (24, 20))]
    dev = prover.prove_inputs(inputs)
    host = prover.prove_witnesses([circ.commit(x) for x in inputs])
    vd = prover.verifier_data()
    for i in range(len(inputs)):
        assert dev[i] == host[i], i
        assert verify(vd, dev[i]) == 0, i
    w = circ.commit(inputs[3])
    cpu, _ = oracle_prove(circ, w.wires(), w.public_inputs())
    assert dev[3] == cpu


def test_device_witness_forms_agree(env, monkeypatch):
    """The two device witness forms -- a launch per dependency level (the
    default up to 32 Wormhole proofs) and one workgroup per proof (larger
    batches; QPGPU_PATHS wit_mode=0 forces it) -- prove the same bytes."""
    from qp_wormhole.synthetic import synthetic_inputs
    ctx, circ, prover = env
    inputs = [WI.test_inputs()] + [synthetic_inputs(k, d) for k, d in ((31, 3), (32, 12))]
    by_level = prover.prove_inputs(inputs)
    monkeypatch.setenv("QPGPU_PATHS", "wit_mode=0")
    per_proof = prover.prove_inputs(inputs)
    monkeypatch.delenv("QPGPU_PATHS")
    assert by_level == per_proof


def test_device_witness_conflict_is_reported(env):
    """storage_proof_tests.rs:30-100 / nullifier_tests.rs:38-48: inconsistent
    inputs make generation fail with "set twice with different values"."""
    import qp_wormhole
    ctx, circ, prover = env
    bad = WI.test_inputs()
    bad.public.nullifier = bytes([1]) + bad.public.nullifier[1:]
    with pytest.raises(qp_wormhole.QpError) as e:
        prover.prove_inputs([WI.test_inputs(), bad])
    assert e.value.code == 5
    assert "proof 1" in str(e.value) and "set twice with different values" in str(e.value)
    # the prover stays usable
    assert verify(prover.verifier_data(), prover.prove_inputs([WI.test_inputs()])[0]) == 0


def test_voting_device_witness():
    import qp_wormhole
    from qp_wormhole.synthetic import synthetic_vote_inputs, vote_test_inputs
    ctx = qp_wormhole.Context(0)
    circ = qp_wormhole.Circuit.voting()
    prover = qp_wormhole.Prover(ctx, circ, max_batch=4)
    inputs = [vote_test_inputs()] + [synthetic_vote_inputs(k, d) for k, d in ((1, 0), (2, 5), (3, 31), (4, -1))]
    dev = prover.prove_inputs(inputs)
    host = prover.prove_witnesses([circ.commit(x) for x in inputs])
    assert dev == host
    vd = prover.verifier_data()
    assert all(verify(vd, p) == 0 for p in dev)
    prover.free()
    ctx.close()


def test_zk_config_proves():
    """standard_recursion_zk_config (the reference prover's default, circuit.rs:68-73):
    same preprocessing and proof shape as the non-zk config (the reference's
    fixture pair, tests/test_zk.py), plus the PublicInputGate row's random cells.
    With the same cells the device-witness path, the host-witness path and the
    oracle prover give the same bytes; other cells give another wires cap, as the
    reference's zk and non-zk proofs of the same inputs do."""
    import dataclasses
    import qp_wormhole
    from qp_wormhole.synthetic import synthetic_inputs
    from test_oracle_golden import current_common_bytes
    zk = qp_wormhole.WormholeProver("standard_recursion_zk_config")
    nz = qp_wormhole.WormholeProver("standard_recursion_config")
    a = zk.commit(WI.test_inputs()).prove().to_bytes()
    b = nz.commit(WI.test_inputs()).prove().to_bytes()
    vd = zk.prover.verifier_data()
    cb = bytearray(current_common_bytes())
    cb[49] = 1
    assert vd.endswith(bytes(cb))
    assert verify(vd, a) == 0 and verify(nz.prover.verifier_data(), b) == 0
    assert a[:512] != b[:512]                    # wires caps differ, as in the fixture pair
    assert a[-8 * 17:] == b[-8 * 17:]            # same public inputs
    circ, prover = zk.circuit, zk.prover
    r = [(0x9e3779b97f4a7c15 * (i + 3)) % 0xFFFFFFFF00000001 for i in range(circ.num_wires - 4)]
    inputs = [dataclasses.replace(WI.test_inputs(), zk_randomness=r),
              dataclasses.replace(synthetic_inputs(31, 2), zk_randomness=r[::-1]), synthetic_inputs(32, 0)]
    dev = prover.prove_inputs(inputs)
    host = prover.prove_witnesses([circ.commit(x) for x in inputs])
    assert dev == host
    w = circ.commit(inputs[0])
    ob, ovd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert dev[0] == ob and ovd == vd
    assert dev[0][:512] != a[:512]               # other random cells, other wires cap
    assert all(verify(vd, p) == 0 for p in dev)


def test_batch_256_two_provers():
    """BASELINE configs[2]: 256 proofs on one GPU, split over two provers (each
    its own context/stream) as bench.py runs them; all verify, 4 are checked
    byte for byte against the oracle prover."""
    import threading

    import qp_wormhole
    from qp_wormhole.synthetic import synthetic_inputs
    circ = qp_wormhole.Circuit.wormhole()
    ctxs = [qp_wormhole.Context(0), qp_wormhole.Context(0)]
    provers = [qp_wormhole.Prover(c, circ, max_batch=128) for c in ctxs]
    inputs = [synthetic_inputs(1000 + k, k % 21) for k in range(256)]
    out = [None, None]

    def run(i):
        out[i] = provers[i].prove_inputs(inputs[128 * i:128 * (i + 1)])

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    proofs = out[0] + out[1]
    assert len(proofs) == 256
    vd = provers[0].verifier_data()
    assert provers[1].verifier_data() == vd
    assert all(verify(vd, p) == 0 for p in proofs)
    for k in (0, 77, 128, 255):
        w = circ.commit(inputs[k])
        cpu, _ = oracle_prove(circ, w.wires(), w.public_inputs())
        assert proofs[k] == cpu, k
    # public inputs round-trip (prover_tests.rs:21-45 layout)
    npi = struct.unpack_from("<Q", proofs[5], len(proofs[5]) - 16 * 8 - 8)[0]
    assert npi == 16
    for p in provers:
        p.free()
    for c in ctxs:
        c.close()
