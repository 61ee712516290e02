"""Recursive aggregation on the host (no GPU): the native recursive verifier
(csrc/recursion.cpp — plonky2's verify_proof gadget as aggregate_chunk builds
it, wormhole/aggregator/src/circuits/tree.rs:106-143) and the aggregator API
(tree.rs, aggregator.rs, util.rs, inputs.rs:57-131).

Pinned by the reference's own proofs: the two current-circuit proofs the
reference's Rust prover wrote (tests/golden/dummy_proof{,_zk}.bin) verify
INSIDE the aggregation circuit — its witness (challenger transcript, vanishing
polynomial at zeta over all six gates, permutation argument, FRI queries with
Merkle paths to the caps, coset interpolation, PoW) satisfies every
constraint — and every tampered variant is rejected.  The aggregation
circuit's own layout and proofs are parity-unpinned (the reference commits no
aggregated proof); their proofs are checked by the oracle verifier.
"""
import ctypes
import struct

import pytest

from agg_oracle_backend import oracle_backend
from oracle_lib import U64P, golden, lib as olib


def check_witness(circ, w):
    L = olib()
    L.ora_check_witness.restype = ctypes.c_long
    L.ora_check_witness.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t]
    cb = circ.common_data()
    pis = w.public_inputs()
    return L.ora_check_witness(cb, len(cb), circ.constants_sigmas(), w.wires(), pis, len(pis))


def check_census(circ):
    """The generator schedule against the trace (qp_circuit_census): one
    generator per row of the single-generator gates (Poseidon, PoseidonMds,
    Reducing(Extension), CosetInterpolation, Constant, BaseSum), one per used op
    of the multi-op gates (at most num_ops per row, at least one per row: an
    extension op is ONE ArithmeticExtension / MulExtension generator, not the
    ~4 base-field ops of a base-arithmetic recursive verifier, hence ~16k
    generators for 8k rows), four per RandomAccess row, and their total is the
    schedule the device witness runs (info word 7)."""
    g, r = circ.census()
    assert sum(g.values()) == circ.num_generators and sum(r.values()) == circ.n
    for gk, rk in (("poseidon", "poseidon"), ("poseidon_mds", "poseidon_mds"), ("reducing", "reducing"),
                   ("reducing_ext", "reducing_ext"), ("coset_interp", "coset_interp"), ("constant", "constant"),
                   ("base_split", "base_sum")):
        assert g[gk] == r[rk], (gk, g[gk], r[rk])
    for gk, ops in (("arithmetic", 20), ("arith_ext", 10), ("mul_ext", 13)):
        assert r[gk] <= g[gk] <= ops * r[gk], (gk, g[gk], r[gk])
    assert g["random_access"] == 4 * r["random_access"]
    assert r["public_input"] == 1 and g["equality"] == 0
    return g, r


@pytest.fixture(scope="module")
def ref():
    from current_circuit_vd import current_circuit_verifier_data
    from test_oracle_golden import current_common_bytes
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    return cb, vd[:len(vd) - len(cb)], [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]


@pytest.fixture(scope="module")
def agg_circuit(ref):
    from qp_wormhole import Circuit
    return Circuit.aggregation(ref[0], 2)


def test_aggregation_circuit_shape(agg_circuit):
    """Upstream verify_proof's gate set (plonky2 recursive_verifier.rs /
    fri/recursive_verifier.rs restated; parity unpinned): extension arithmetic
    on ArithmeticExtension / MulExtension ops, PoseidonMds layers for the
    Poseidon gate's in-circuit evaluation, Reducing(Extension) for the alpha
    reductions, CosetInterpolation for the FRI coset checks, RandomAccess for
    caps and coset evaluations -- two degree-13 Wormhole proofs fit 2^13 rows."""
    from qp_wormhole._native import GATE_KINDS, gate_desc
    c = agg_circuit
    assert c.degree_bits == 13 and 4096 < c.gates_used <= 8192
    assert c.num_public_inputs == 32
    g = gate_desc(c)
    kinds = [GATE_KINDS[g.kind[i]] for i in range(g.num_gates)]
    # CommonCircuitData.gates sorted by (degree, id string)
    assert kinds == ["noop", "constant", "poseidon_mds", "public_input", "base_sum", "reducing_extension", "reducing",
                     "arithmetic_extension", "arithmetic", "mul_extension", "random_access", "coset_interpolation",
                     "poseidon"]
    # selectors_info: greedy groups with degree + size < quotient_degree_factor + 1
    assert [g.selector_index[i] for i in range(g.num_gates)] == [0] * 7 + [1] * 4 + [2] * 2
    assert g.num_constants == 3 + 2 and g.num_gate_constraints == 123
    gens, rows = check_census(c)
    # the recursive verifier's every gate kind is present, and its extension
    # arithmetic runs on the extension gates
    assert all(rows[k] > 0 for k in ("random_access", "arith_ext", "mul_ext", "reducing", "reducing_ext",
                                     "poseidon_mds", "coset_interp"))
    assert gens["arith_ext"] + gens["mul_ext"] > gens["arithmetic"]
    cb = c.common_data()
    for tag, params in ((13, (4, 4, 2)), (1, (10,)), (8, (13,)), (15, (43,)), (14, (32,)), (4, (4, 6, 16))):
        assert cb.count(struct.pack("<I", tag) + struct.pack(f"<{len(params)}Q", *params)) == 1


def test_host_chains_cut_the_device_schedule(ref, agg_circuit, monkeypatch):
    """The device witness's host part (CircuitData::host_gens): Poseidon chains
    over inputs alone at least 64 permutations deep -- here the inner proofs'
    transcript sponges -- and the constants they read run on the host, the
    rest of the schedule on the device, 149 dependency levels down to 55;
    QPGPU_PATHS=host_chain=0 keeps every generator on the device.  The leaf circuits
    have no such chain.  (Device == host-witness bytes either way:
    test_gpu_aggregation.)"""
    import qp_wormhole
    g, nslots, chains = agg_circuit.host_chains()
    assert set(g) <= {"poseidon", "constant"} and g["poseidon"] >= 2 * 64
    assert chains == 2  # the two inner proofs' transcripts
    assert agg_circuit.witness_levels == 55
    monkeypatch.setenv("QPGPU_PATHS", "host_chain=0")
    c0 = qp_wormhole.Circuit.aggregation(ref[0], 2)
    g0, n0, ch0 = c0.host_chains()
    assert g0 == {} and ch0 == 0 and c0.witness_levels == 149 and n0 < nslots
    assert c0.num_generators == agg_circuit.num_generators
    monkeypatch.delenv("QPGPU_PATHS")
    for circ in (qp_wormhole.Circuit.wormhole(False), qp_wormhole.Circuit.voting()):
        assert circ.host_chains()[0] == {}


def test_reference_proofs_verify_in_circuit(ref, agg_circuit):
    cb, vo, leaves = ref
    w = agg_circuit.commit_proofs(vo, leaves)
    assert check_witness(agg_circuit, w) == -1
    pis = [int(x) for x in w.public_inputs()]
    want = []
    for pf in leaves:
        want += list(struct.unpack_from("<16Q", pf, len(pf) - 128))
    assert pis == want


@pytest.mark.parametrize("what,off", [
    ("wires cap", 100), ("zs cap", 512 + 8), ("quotient cap", 1024 + 16),
    ("constants opening", 3 * 512 + 3), ("wire opening", 3 * 512 + 84 * 16 + 5),
    ("quotient opening", 3 * 512 + 256 * 16 + 1), ("fri layer cap", 3 * 512 + 257 * 16 + 40),
    ("query leaf", 3 * 512 + 257 * 16 + 2 * 512 + 8), ("merkle sibling", 3 * 512 + 257 * 16 + 2 * 512 + 84 * 8 + 1 + 33),
    ("pow witness", -8 - 128 - 8 - 2), ("final poly", -8 - 128 - 8 - 40), ("public input", -100)])
def test_tampered_reference_proof_is_rejected(ref, agg_circuit, what, off):
    from qp_wormhole import QpError
    cb, vo, leaves = ref
    bad = bytearray(leaves[1])
    bad[off] ^= 1
    try:
        w = agg_circuit.commit_proofs(vo, [leaves[0], bytes(bad)])
    except QpError as e:
        assert "set twice" in str(e) or "deserialize" in str(e) or "canonical" in str(e), str(e)
        return
    assert check_witness(agg_circuit, w) != -1, what


def test_wrong_verifier_data_is_rejected(ref, agg_circuit):
    from qp_wormhole import QpError
    cb, vo, leaves = ref
    bad = bytearray(vo)
    bad[8 + 5 * 32] ^= 1  # one constants||sigmas cap element
    with pytest.raises(QpError, match="set twice"):
        agg_circuit.commit_proofs(bytes(bad), leaves)


def test_aggregation_proof_verifies_and_level_two(ref):
    """aggregate_chunk (CPU prover stand-in) over the reference proofs: the
    aggregation proof verifies; a level-2 circuit over it (its inner gate list
    includes RandomAccess) has a satisfiable witness and a verifying proof."""
    import qp_wormhole
    cb, vo, leaves = ref
    l1 = qp_wormhole.aggregate_chunk(leaves, cb, vo, backend=oracle_backend)
    vd = l1.circuit_data.verifier_data()
    assert olib().ora_verify(vd, len(vd), l1.proof.to_bytes(), len(l1.proof.to_bytes())) == 0
    cd = l1.circuit_data
    c2 = qp_wormhole.Circuit.aggregation(cd.common, 2)
    assert c2.degree_bits == 13
    w2 = c2.commit_proofs(cd.verifier_only, [l1.proof.to_bytes()] * 2)
    assert check_witness(c2, w2) == -1
    assert len(w2.public_inputs()) == 64


def test_public_inputs_roundtrip():
    from qp_wormhole.aggregator import public_inputs_from_aggregated, public_inputs_from_slice
    from qp_wormhole.prover import ProofWithPublicInputs
    pf = golden("dummy_proof.bin")
    pis = list(struct.unpack_from("<16Q", pf, len(pf) - 128))
    p = public_inputs_from_slice(pis)
    assert p.funding_amount == 1_000_000_000_000 and p.exit_account == bytes([4] * 32)
    assert p.nullifier == bytes([169, 76, 150, 35, 66, 248, 76, 193, 57, 204, 106, 33, 169, 160, 248, 113, 235, 144,
                                 212, 48, 9, 232, 146, 7, 105, 125, 170, 24, 33, 54, 135, 28])
    agg = ProofWithPublicInputs(b"", pis * 8)
    assert public_inputs_from_aggregated(agg, 16, 8) == [p] * 8
    with pytest.raises(ValueError, match="should contain"):
        public_inputs_from_aggregated(agg, 16, 4)


def test_tree_config_and_padding():
    from qp_wormhole import TreeAggregationConfig
    from qp_wormhole.aggregator import pad_with_dummy_proofs
    c = TreeAggregationConfig.default()
    assert (c.num_leaf_proofs, c.tree_branching_factor, c.tree_depth) == (8, 2, 3)
    assert TreeAggregationConfig.new(3, 2).num_leaf_proofs == 9
    assert pad_with_dummy_proofs([1, 2], 4, 0) == [1, 2, 0, 0]
    with pytest.raises(ValueError, match="more than the maximum"):
        pad_with_dummy_proofs([1, 2, 3], 2, 0)


def test_unsupported_inner_circuit_is_an_error(ref):
    from qp_wormhole import Circuit, QpError
    cb = bytearray(ref[0])
    cb[-4 - 4] ^= 0xFF  # corrupt the last gate's tag
    with pytest.raises(QpError):
        Circuit.aggregation(bytes(cb), 2)


def test_too_large_level_is_refused_before_proving(ref):
    """aggregate_to_tree sizes every circuit a level builds -- also a lone short
    chunk (fewer proofs than the branching factor): 9 leaf proofs in one chunk
    need 2^16 rows, past the GPU prover's 2^15, so CircuitTooLarge is raised
    before any proving (no GPU needed to see it)."""
    import qp_wormhole
    from qp_wormhole.aggregator import CircuitTooLarge, TreeAggregationConfig
    cb, vo, leaves = ref
    with pytest.raises(CircuitTooLarge, match="2\\^16") as e:
        qp_wormhole.aggregate_to_tree([leaves[0]] * 9, cb, vo, TreeAggregationConfig.new(10, 1))
    assert e.value.proofs == []


def test_subtree_parts(monkeypatch):
    """aggregate_to_tree proves QP_AGG_SPLIT (default 4) complete k-ary
    sub-trees concurrently, only when the leaves split into that many of at
    least SUBTREE_MIN_LEAVES (32) leaves each."""
    from qp_wormhole.aggregator import _subtree_parts
    monkeypatch.delenv("QP_AGG_SPLIT", raising=False)
    monkeypatch.delenv("QP_AGG_PROVERS", raising=False)
    assert _subtree_parts(256, 2) == 4 and _subtree_parts(128, 2) == 4 and _subtree_parts(8, 2) == 1
    assert _subtree_parts(192, 2) == 1 and _subtree_parts(324, 3) == 4 and _subtree_parts(81, 3) == 1
    monkeypatch.setenv("QP_AGG_SPLIT", "2")
    assert _subtree_parts(256, 2) == 2 and _subtree_parts(32, 2) == 1 and _subtree_parts(162, 3) == 2
    monkeypatch.setenv("QP_AGG_SPLIT", "1")
    assert _subtree_parts(256, 2) == 1
