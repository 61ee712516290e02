"""Recursive aggregation on the MI355X (BASELINE configs[3]):
aggregate_chunk / aggregate_to_tree / WormholeProofAggregator
(wormhole/aggregator/src/circuits/tree.rs:55-143, aggregator.rs:13-92).

Parity: the aggregation circuits' GPU proofs (upstream verify_proof's gate
set, degree 2^13, generic quotient kernel) are byte-identical to the CPU oracle
prover's for the same witness and verify under the oracle verifier.  The
in-circuit verifier itself is pinned by the reference's own leaf proofs
(tests/golden/dummy_proof{,_zk}.bin verify inside it).  The aggregation
circuit's layout is parity-unpinned (no aggregated reference proof exists).
"""
import pytest

from oracle_lib import golden, lib as olib
from test_aggregation import check_census
from test_gpu_prover import oracle_prove

pytestmark = pytest.mark.gpu


def verify(vd, proof):
    return olib().ora_verify(vd, len(vd), proof, len(proof))


@pytest.fixture(scope="module")
def reference_leaves():
    from current_circuit_vd import current_circuit_verifier_data
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    return cb, vd[:len(vd) - len(cb)], [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]


def test_aggregate_reference_proofs_gpu_equals_oracle(reference_leaves):
    """aggregate_chunk over the reference's own two proofs: GPU bytes == oracle
    bytes of the same witness, and the aggregated proof verifies."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    agg = qp_wormhole.aggregate_chunk(leaves, cb, vo)
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    assert circ.degree_bits == 13
    w = circ.commit_proofs(vo, leaves)
    ob, ovd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert agg.proof.to_bytes() == ob
    assert agg.circuit_data.verifier_data() == ovd
    assert verify(ovd, ob) == 0
    # public inputs: the two leaves' 16 each, in order
    from oracle_lib import golden as g
    import struct
    want = []
    for name in ("dummy_proof.bin", "dummy_proof_zk.bin"):
        pf = g(name)
        want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
    assert agg.proof.public_inputs == want


def test_tree_of_eight_native_leaves():
    """WormholeProofAggregator with the default tree (branching 2, depth 3): five
    native leaf proofs + three dummies -> 4 + 2 + 1 aggregation proofs on the GPU;
    the root verifies, its bytes equal the oracle's for the same witness, and the
    leaf public inputs come back out of it (extract_leaf_public_inputs)."""
    import qp_wormhole
    from qp_wormhole.aggregator import public_inputs_from_slice
    from qp_wormhole.synthetic import synthetic_inputs
    wp = qp_wormhole.WormholeProver("standard_recursion_zk_config")
    leaves = [qp_wormhole.WormholeProver("standard_recursion_zk_config").commit(synthetic_inputs(40 + k, k % 3))
              .prove() for k in range(5)]
    agg = qp_wormhole.WormholeProofAggregator.default()
    for p in leaves:
        agg.push_proof(p)
    root = agg.aggregate()
    assert verify(root.circuit_data.verifier_data(), root.proof.to_bytes()) == 0
    pis = agg.extract_leaf_public_inputs(root)
    assert len(pis) == 8
    for k in range(5):
        assert pis[k] == public_inputs_from_slice(leaves[k].public_inputs)
    dummy = public_inputs_from_slice(agg.dummy_proof().public_inputs)
    assert pis[5:] == [dummy] * 3
    del wp


def test_level_two_gpu_equals_oracle(reference_leaves):
    """A level-2 circuit (inner = the aggregation circuit, with RandomAccess gates):
    GPU == oracle bytes; verifies."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    l1 = qp_wormhole.aggregate_chunk(leaves, cb, vo)
    cd = l1.circuit_data
    l2 = qp_wormhole.aggregate_chunk([l1.proof, l1.proof], cd.common, cd.verifier_only)
    circ = qp_wormhole.Circuit.aggregation(cd.common, 2)
    w = circ.commit_proofs(cd.verifier_only, [l1.proof.to_bytes()] * 2)
    ob, ovd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert l2.proof.to_bytes() == ob and verify(ovd, ob) == 0


def test_tampered_leaf_is_rejected(reference_leaves):
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    bad = bytearray(leaves[1])
    bad[3 * 512 + 84 * 16 + 7] ^= 1
    with pytest.raises(qp_wormhole.QpError, match="set twice"):
        qp_wormhole.aggregate_chunk([leaves[0], bytes(bad)], cb, vo)


def test_deep_subtree_root_carries_every_leaf_public_input(reference_leaves):
    """A subtree of 32 leaves (depth 5, as bench.py's per-GPU subtree): the
    root's 512 public inputs (past the 256 the device gather once capped) are
    the leaves' 16 each, in order, and the root verifies."""
    import struct
    import qp_wormhole
    from qp_wormhole.aggregator import TreeAggregationConfig
    cb, vo, leaves = reference_leaves
    ls = [leaves[k % 2] for k in range(32)]
    root = qp_wormhole.aggregate_to_tree(ls, cb, vo, TreeAggregationConfig.new(2, 5))
    assert verify(root.circuit_data.verifier_data(), root.proof.to_bytes()) == 0
    want = []
    for pf in ls:
        want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
    assert root.proof.public_inputs == want


def test_tree_of_2048_leaves_reaches_a_degree15_root(reference_leaves):
    """configs[3] at N = 8 on one GPU: 2048 leaves (the reference's two proofs)
    through 11 levels to one root; the top circuit registers 32,768 public
    inputs and is 2^15 rows (the large-transform path), the root verifies and
    carries every leaf's public inputs in order."""
    import struct
    import qp_wormhole
    from qp_wormhole.aggregator import TreeAggregationConfig
    from qp_wormhole.prover import _common_degree_bits
    cb, vo, leaves = reference_leaves
    ls = [leaves[k % 2] for k in range(2048)]
    root = qp_wormhole.aggregate_to_tree(ls, cb, vo, TreeAggregationConfig.new(2, 11))
    assert _common_degree_bits(root.circuit_data.common) == 15
    assert verify(root.circuit_data.verifier_data(), root.proof.to_bytes()) == 0
    pis = root.proof.public_inputs
    assert len(pis) == 32768
    for k in (0, 1, 2047):
        pf = ls[k]
        assert pis[16 * k:16 * k + 16] == list(struct.unpack_from("<16Q", pf, len(pf) - 128))


@pytest.mark.parametrize("k", [3, 4, 5, 6, 7])
def test_k_ary_depth_two_trees(reference_leaves, k):
    """The reference's tree shapes TreeAggregationConfig::new(k, 2), k = 3..7
    (benches/aggregator.rs:119-123): k^2 of the reference's own leaf proofs
    through k level-1 proofs (degree 2^14 for k = 3, 4; 2^15 for k >= 5) to a
    root (2^14 / 2^15) that verifies and carries every leaf's public inputs in
    order."""
    import struct
    import qp_wormhole
    from qp_wormhole.aggregator import TreeAggregationConfig
    from qp_wormhole.prover import _common_degree_bits
    cb, vo, leaves = reference_leaves
    ls = [leaves[(i * 5 + i // 3) % 2] for i in range(k * k)]
    root = qp_wormhole.aggregate_to_tree(ls, cb, vo, TreeAggregationConfig.new(k, 2))
    assert _common_degree_bits(root.circuit_data.common) == (14 if k == 3 else 15)
    assert verify(root.circuit_data.verifier_data(), root.proof.to_bytes()) == 0
    want = []
    for pf in ls:
        want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
    assert root.proof.public_inputs == want


def _device_vs_host(circ, vo, chunks, zk=None):
    """qp_prover_prove_aggregation (witness generated on the device) vs the host
    witness path (qp_aggregation_commit + qp_prover_prove) of the same chunks."""
    import qp_wormhole
    p = qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=len(chunks))
    dev = p.prove_aggregation(vo, chunks, zk_randomness=zk)
    ws = [circ.commit_proofs(vo, ch, zk_randomness=None if zk is None else zk[i]) for i, ch in enumerate(chunks)]
    host = p.prove_witnesses(ws)
    vd = p.verifier_data()
    p.free()
    return dev, host, vd


def test_degree15_aggregation_gpu_equals_oracle(reference_leaves):
    """A degree-2^15 circuit (aggregate_chunk of five leaves; the root of a
    2048-leaf tree is 2^15 rows too): transforms beyond one workgroup's LDS run
    their first level in HBM (ntt.hip dif_big), Z's scan, the quotient iNTT and
    FRI's divide have large-n forms; proof bytes == the oracle's, verified."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    chunk = [leaves[i % 2] for i in range(5)]
    circ = qp_wormhole.Circuit.aggregation(cb, 5)
    assert circ.degree_bits == 15
    agg = qp_wormhole.aggregate_chunk(chunk, cb, vo)
    w = circ.commit_proofs(vo, chunk)
    ob, ovd = oracle_prove(circ, w.wires(), w.public_inputs())
    assert agg.proof.to_bytes() == ob
    assert agg.circuit_data.verifier_data() == ovd
    assert verify(ovd, ob) == 0


def test_device_witness_equals_host_witness_levels_1_and_2(reference_leaves):
    """The recursive verifier's generators on the device (Poseidon with swap,
    arithmetic, BaseSum, wire split, extension division, RandomAccess): proof
    bytes equal the host-witness path's at level 1 (the reference's own leaf
    proofs, in three chunk orders) and level 2 (inner = the aggregation
    circuit), and verify."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    assert circ.witness_levels > 0
    check_census(circ)
    chunks = [leaves, leaves[::-1], [leaves[0], leaves[0]]]
    dev, host, vd = _device_vs_host(circ, vo, chunks)
    assert dev == host
    assert all(verify(vd, d) == 0 for d in dev)
    l1 = qp_wormhole.aggregate_chunk(leaves, cb, vo)
    cd = l1.circuit_data
    c2 = qp_wormhole.Circuit.aggregation(cd.common, 2)
    dev2, host2, vd2 = _device_vs_host(c2, cd.verifier_only, [[l1.proof.to_bytes()] * 2])
    assert dev2 == host2 and verify(vd2, dev2[0]) == 0


def test_host_chains_off_gives_the_same_proofs(reference_leaves, monkeypatch):
    """The device witness with the input-only Poseidon chains on the host
    (default) and with every generator on the device (QPGPU_PATHS=host_chain=0, a
    circuit built under it: 149 dependency levels instead of 55) prove the
    same bytes, which verify."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    chunks = [leaves, leaves[::-1]]
    c1 = qp_wormhole.Circuit.aggregation(cb, 2)
    monkeypatch.setenv("QPGPU_PATHS", "host_chain=0")
    c0 = qp_wormhole.Circuit.aggregation(cb, 2)
    monkeypatch.delenv("QPGPU_PATHS")
    assert c1.host_chains()[0] and not c0.host_chains()[0] and c0.witness_levels > c1.witness_levels
    out = []
    for c in (c1, c0):
        p = qp_wormhole.Prover(qp_wormhole.Context(0), c, max_batch=2)
        out.append((p.prove_aggregation(vo, chunks), p.verifier_data()))
        p.free()
    (a, vd1), (b, vd0) = out
    assert a == b and vd1 == vd0 and all(verify(vd1, x) == 0 for x in a)


def test_device_witness_zk_aggregation(reference_leaves):
    """Under the zk config the PublicInputGate row's cells are explicit inputs
    (device == host for the same values) or, when not given, OS randomness
    (two runs differ, both verify)."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    zcb = bytearray(cb)
    zcb[49] = 1  # config.zero_knowledge
    circ = qp_wormhole.Circuit.aggregation(bytes(zcb), 2)
    r = [[(0x9E3779B97F4A7C15 * (k + 1) + i) % 0xFFFFFFFF00000001 for i in range(circ.num_wires - 4)]
         for k in range(2)]
    dev, host, vd = _device_vs_host(circ, vo, [leaves, leaves[::-1]], zk=r)
    assert dev == host and all(verify(vd, d) == 0 for d in dev)
    p = qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=1)
    a, = p.prove_aggregation(vo, [leaves])
    b, = p.prove_aggregation(vo, [leaves])
    assert a != b and verify(vd, a) == 0 and verify(vd, b) == 0
    p.free()


@pytest.mark.parametrize("paths", ["wit_mode=0", "wit_mode=1", "merkle_coop=0", "qprefix=0", "leaf_t=0",
                                   "merkle_row=0", "fri_row=0", "open_slices=1", "lde_few=0", "wit_row=0",
                                   "wit_row=0,wit_mode=0"])
def test_latency_paths_prove_the_same_bytes(reference_leaves, monkeypatch, paths):
    """The small-batch paths (device witness one launch per dependency level or
    one workgroup per proof, cooperative Merkle levels in the row or wave form,
    the prefix quotient kernel, the compile-time leaf hash, row-form FRI
    leaves, sliced openings, per-coset LDE of few columns) against their
    alternatives: the same proof bytes, at batch 1 and 3."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    chunks = [leaves, leaves[::-1], [leaves[1], leaves[1]]]
    out = []
    for hook in (None, paths):  # QPGPU_PATHS (csrc/paths.h): force the alternative path
        if hook:
            monkeypatch.setenv("QPGPU_PATHS", hook)
        p = qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=3)
        out.append((p.prove_aggregation(vo, chunks[:1]), p.prove_aggregation(vo, chunks)))
        p.free()
        monkeypatch.delenv("QPGPU_PATHS", raising=False)
    assert out[0] == out[1]


def test_high_priority_context_proves_the_same_bytes(reference_leaves):
    """qp_ctx_set_priority: the level provers' optional high-priority stream."""
    import qp_wormhole
    cb, vo, leaves = reference_leaves
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    res = []
    for high in (False, True):
        ctx = qp_wormhole.Context(0)
        if high:
            ctx.set_priority(True)
        p = qp_wormhole.Prover(ctx, circ, max_batch=1)
        res.append(p.prove_aggregation(vo, [leaves])[0])
        p.free()
    assert res[0] == res[1]


@pytest.mark.parametrize("split", ["2", "4"])
def test_concurrent_subtrees_prove_the_same_root(reference_leaves, monkeypatch, split):
    """aggregate_to_tree's concurrent sub-trees (QP_AGG_SPLIT) take the same
    chunks as the level-by-level order: the same root bytes over 128 leaves,
    and the root verifies."""
    import qp_wormhole
    from qp_wormhole.aggregator import TreeAggregationConfig
    cb, vo, leaves = reference_leaves
    ls = [leaves[(i * 7 + i // 5) % 2] for i in range(128)]
    roots = []
    for s in ("1", split):
        monkeypatch.setenv("QP_AGG_SPLIT", s)
        roots.append(qp_wormhole.aggregate_to_tree(ls, cb, vo, TreeAggregationConfig.new(2, 7)))
    assert roots[0].proof.to_bytes() == roots[1].proof.to_bytes()
    assert roots[0].circuit_data.verifier_only == roots[1].circuit_data.verifier_only
    vd = roots[1].circuit_data.verifier_data()
    pb = roots[1].proof.to_bytes()
    assert olib().ora_verify(vd, len(vd), pb, len(pb)) == 0
