"""GPU parity of the routine-level seams (include/qpgpu.h):
compute_quotient_polys, one fri_committed_trees layer (commit + open), the
coefficient fold and fri_proof_of_work, each bit-exact against the CPU oracle
(oracle/prover.c ora_quotient / ora_fri_layer / ora_fri_fold / ora_pow_grind,
which share or_prove's code pinned by the golden proofs).  The shapes are the
ones plonky2's prove() reaches for the wormhole circuit (degree 13, rate 3,
FRI arities [4, 4], cap height 4) plus smaller and zero-tailed variants."""
import numpy as np
import pytest

from oracle_lib import P, lib as olib

G = 0xC65C18B67785D900


def rand_felts(rng, *shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


def gpow(x, e):
    return pow(int(x), int(e), P)


@pytest.fixture(scope="module")
def circuit():
    from qp_wormhole import Circuit
    return Circuit.wormhole()


def test_gate_desc_matches_common_data(circuit):
    """qp_circuit_gate_desc (host-only) describes the circuit's CommonCircuitData."""
    import qp_wormhole
    g = qp_wormhole.gate_desc(circuit)
    assert g.num_gates == 6
    assert list(g.kind)[:6] == [0, 1, 2, 3, 4, 5]  # Noop, Constant, PI, BaseSum, Arithmetic, Poseidon
    assert g.num_selectors == 2 and (g.group_lo[0], g.group_hi[0], g.group_lo[1], g.group_hi[1]) == (0, 5, 5, 6)
    assert list(g.selector_index)[:6] == [0, 0, 0, 0, 0, 1]
    assert g.num_wires == circuit.num_wires and g.num_routed_wires == circuit.num_routed_wires
    assert g.num_constants == circuit.num_constants
    assert g.num_gate_constraints == circuit.num_gate_constraints
    assert g.quotient_degree_factor == 8 and g.num_challenges == 2


@pytest.fixture(scope="module")
def ctx():
    import qp_wormhole
    c = qp_wormhole.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
def test_quotient_matches_oracle(ctx, circuit):
    import qp_wormhole
    rng = np.random.default_rng(41)
    g = qp_wormhole.gate_desc(circuit)
    n, rb = circuit.n, 3
    cs = circuit.constants_sigmas()
    wires = rand_felts(rng, circuit.num_wires, n)
    nzs = g.num_challenges * ((g.num_routed_wires + g.quotient_degree_factor - 1) // g.quotient_degree_factor)
    zs = rand_felts(rng, nzs, n)
    betas, gammas, alphas, pih = rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 4)
    B = [qp_wormhole.PolynomialBatch.from_values(ctx, v, rb, 4) for v in (cs, wires, zs)]
    got = qp_wormhole.quotient(ctx, B[0], B[1], B[2], g, betas, gammas, alphas, pih)
    want = np.zeros_like(got)
    cb = circuit.common_data()
    assert olib().ora_quotient(cb, len(cb), cs, wires, zs, betas, gammas, alphas, pih, want) == 0
    assert got.shape == (16, n)
    assert (got == want).all(), np.argwhere(got != want)[:4]


@pytest.mark.gpu
def test_quotient_generic_kernel_matches_oracle(ctx, circuit, monkeypatch):
    """The any-gate-list kernels (path hook quotient_parts=1 forces them) on the Wormhole circuit."""
    import qp_wormhole
    monkeypatch.setenv("QPGPU_PATHS", "quotient_parts=1")
    rng = np.random.default_rng(43)
    g = qp_wormhole.gate_desc(circuit)
    n = circuit.n
    cs = circuit.constants_sigmas()
    wires = rand_felts(rng, circuit.num_wires, n)
    zs = rand_felts(rng, 20, n)
    betas, gammas, alphas, pih = rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 4)
    B = [qp_wormhole.PolynomialBatch.from_values(ctx, v, 3, 4) for v in (cs, wires, zs)]
    got = qp_wormhole.quotient(ctx, B[0], B[1], B[2], g, betas, gammas, alphas, pih)
    want = np.zeros_like(got)
    cb = circuit.common_data()
    assert olib().ora_quotient(cb, len(cb), cs, wires, zs, betas, gammas, alphas, pih, want) == 0
    assert (got == want).all()


# the recursive-verifier gate set with standard_recursion_config parameters (plonky2
# *::new_from_config for 135 wires / 80 routed), three selector groups
RECURSION_GATES = [
    ("noop", (), 0), ("constant", (2,), 0), ("public_input", (), 0), ("base_sum", (63,), 0), ("arithmetic", (20,), 0),
    ("poseidon", (), 1), ("arithmetic_extension", (10,), 1), ("mul_extension", (13,), 1),
    ("random_access", (4, 4, 2), 1), ("exponentiation", (66,), 1),
    ("reducing", (43,), 2), ("reducing_extension", (32,), 2), ("poseidon_mds", (), 2),
    ("coset_interpolation", (4, 6), 2),
]


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [8, 10, 15])
def test_quotient_recursion_gate_set_matches_oracle(ctx, log_n):
    """qp_quotient over the aggregator circuits' gate list (generic kernel) vs the
    descriptor-driven oracle; random selector values make every gate's filter
    nonzero, so every constraint of every gate reaches the quotient.  2^15: the
    degree of a 5- to 7-ary level-1 circuit and of a 2048-leaf root (the coset
    iNTT's large-n form)."""
    import ctypes

    import qp_wormhole
    g = qp_wormhole.GateDesc.build(RECURSION_GATES, [(0, 5), (5, 10), (10, 14)], num_gate_constraints=123)
    rng = np.random.default_rng(log_n)
    n = 1 << log_n
    cs = rand_felts(rng, g.num_constants + 80, n)
    wires = rand_felts(rng, 135, n)
    zs = rand_felts(rng, 20, n)
    betas, gammas, alphas, pih = rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 2), rand_felts(rng, 4)
    B = [qp_wormhole.PolynomialBatch.from_values(ctx, v, 3, 4) for v in (cs, wires, zs)]
    got = qp_wormhole.quotient(ctx, B[0], B[1], B[2], g, betas, gammas, alphas, pih)
    want = np.zeros_like(got)
    assert olib().ora_quotient_desc(ctypes.addressof(g), log_n, 3, cs, wires, zs, betas, gammas, alphas, pih,
                                    want) == 0
    assert (got == want).all(), np.argwhere(got != want)[:4]


@pytest.mark.gpu
def test_quotient_rejects_bad_gate_parameters(ctx):
    import qp_wormhole
    rng = np.random.default_rng(44)
    n = 1 << 8
    cs = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, 83, n), 3, 4)
    w = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, 135, n), 3, 4)
    z = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, 20, n), 3, 4)
    two, four = np.ones(2, np.uint64), np.zeros(4, np.uint64)
    for gates in ([("reducing", (70,), 0)],                 # 6 + 70 + 138 wires > 135
                  [("random_access", (7, 1, 0), 0)],         # 2^7-item lists
                  [("exponentiation", (40,), 0)] * 17):      # more than 16 gates
        g = qp_wormhole.GateDesc.build(gates[:16] if len(gates) <= 16 else gates[:16], [(0, 1)],
                                       num_gate_constraints=123)
        if len(gates) > 16:
            g.num_gates = 17
        with pytest.raises(qp_wormhole.QpError, match="QP_ERR_ARG"):
            qp_wormhole.quotient(ctx, cs, w, z, g, two, two, two, four)


@pytest.mark.gpu
def test_quotient_rejects_bad_shapes(ctx, circuit):
    import qp_wormhole
    rng = np.random.default_rng(42)
    g = qp_wormhole.gate_desc(circuit)
    n = circuit.n
    cs = qp_wormhole.PolynomialBatch.from_values(ctx, circuit.constants_sigmas(), 3, 4)
    w = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, circuit.num_wires, n), 3, 4)
    z_bad = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, 5, n), 3, 4)  # needs 2 * 10 polys
    two = np.ones(2, np.uint64)
    with pytest.raises(qp_wormhole.QpError, match="QP_ERR_ARG"):
        qp_wormhole.quotient(ctx, cs, w, z_bad, g, two, two, two, np.zeros(4, np.uint64))
    g.kind[3] = 99
    z = qp_wormhole.PolynomialBatch.from_values(ctx, rand_felts(rng, 20, n), 3, 4)
    with pytest.raises(qp_wormhole.QpError, match="unknown gate kind"):
        qp_wormhole.quotient(ctx, cs, w, z, g, two, two, two, np.zeros(4, np.uint64))


# (nonzero coefficients log, buffer log, values log, shift, arity bits, cap height)
FRI_CASES = [
    (13, 16, 16, G, 4, 4),            # wormhole layer 0: degree < n, zero tail to N (arity 16)
    (14, 17, 17, G, 4, 4),            # aggregation-circuit layer 0 (degree 2^14, rate 3)
    (9, 12, 12, gpow(G, 16), 4, 4),    # wormhole layer 1
    (13, 13, 16, G, 2, 4),            # arity 4, unpadded buffer
    (9, 9, 12, gpow(G, 16), 3, 2),
    (3, 4, 6, 7, 1, 0),               # arity 2: hash_or_noop leaves; generic per-coset LDE; cap height 0
    (1, 1, 5, G, 2, 3),
]


@pytest.mark.gpu
@pytest.mark.parametrize("lnz,lbuf,lv,shift,ab,cap_h", FRI_CASES)
def test_fri_layer_matches_oracle(ctx, lnz, lbuf, lv, shift, ab, cap_h):
    import qp_wormhole
    rng = np.random.default_rng(lnz * 100 + lv)
    coeffs = np.zeros((2, 1 << lbuf), np.uint64)
    coeffs[:, :1 << lnz] = rand_felts(rng, 2, 1 << lnz)
    layer = qp_wormhole.FriLayer(ctx, coeffs, lv, shift, ab, cap_h)
    nleaves = 1 << (lv - ab)
    idx = np.unique(np.concatenate([[0, nleaves - 1], rng.integers(0, nleaves, 28)])).astype(np.uint32)
    evals, sibs = layer.open(idx)
    depth = lv - ab - cap_h
    cap = np.zeros((1 << cap_h, 4), np.uint64)
    w_ev = np.zeros((len(idx), 2 << ab), np.uint64)
    w_sib = np.zeros((len(idx), max(depth, 1) * 4), np.uint64)
    assert olib().ora_fri_layer(np.ascontiguousarray(coeffs), lbuf, lv, shift, ab, cap_h, cap, idx, len(idx),
                                w_ev, w_sib) == 0
    assert (layer.cap == cap).all()
    assert (evals.reshape(len(idx), -1) == w_ev).all()
    assert (sibs.reshape(len(idx), -1) == w_sib[:, :depth * 4]).all()
    layer.free()


@pytest.mark.gpu
def test_fri_layer_errors(ctx):
    import qp_wormhole
    rng = np.random.default_rng(5)
    with pytest.raises(qp_wormhole.QpError, match="more than 2\\^16 nonzero coefficients"):
        qp_wormhole.FriLayer(ctx, rand_felts(rng, 2, 1 << 17), 18, G, 2, 4)
    with pytest.raises(qp_wormhole.QpError, match="QP_ERR_ARG"):
        qp_wormhole.FriLayer(ctx, rand_felts(rng, 2, 1 << 8), 7, G, 2, 4)  # values shorter than coeffs
    layer = qp_wormhole.FriLayer(ctx, rand_felts(rng, 2, 1 << 8), 10, G, 2, 4)
    with pytest.raises(qp_wormhole.QpError, match="out of range"):
        layer.open([1 << 8])


@pytest.mark.gpu
@pytest.mark.parametrize("log_len,ab", [(16, 2), (14, 2), (13, 4), (5, 1), (3, 3)])
def test_fri_fold_matches_oracle(ctx, log_len, ab):
    import qp_wormhole
    rng = np.random.default_rng(log_len + 17 * ab)
    c = rand_felts(rng, 2, 1 << log_len)
    beta = rand_felts(rng, 2)
    got = qp_wormhole.fri_fold(ctx, c, ab, beta)
    want = np.zeros_like(got)
    olib().ora_fri_fold(c, log_len, ab, beta, want)
    assert (got == want).all()


@pytest.mark.gpu
def test_pow_grind_matches_oracle(ctx):
    """Minimal witness for every state, 24 states at once (lanes pos < 8)."""
    import qp_wormhole
    rng = np.random.default_rng(77)
    states = rand_felts(rng, 24, 12)
    pos = (np.arange(24) % 8).astype(np.uint32)
    for bits in (8, 16):
        got = qp_wormhole.pow_grind(ctx, states, pos, bits)
        for b in range(0, 24, 1 if bits == 8 else 6):
            want = olib().ora_pow_grind(np.ascontiguousarray(states[b]), int(pos[b]), bits)
            assert int(got[b]) == want, (bits, b)
            s = states[b].copy()
            s[pos[b]] = got[b]
            olib().ora_permute(s)
            assert int(s[7]) >> (64 - bits) == 0
    with pytest.raises(qp_wormhole.QpError, match="position"):
        qp_wormhole.pow_grind(ctx, states[:1], np.array([8], np.uint32), 8)
