"""GPU parity: NTT/LDE, Poseidon and PolynomialBatch commitments (HIP via the
C ABI) against the CPU oracle, bit-exact.  SURVEY.md section 8 rows a4-a7."""
import numpy as np
import pytest

from oracle_lib import P, commit_values, lib as olib

pytestmark = pytest.mark.gpu

G = 0xC65C18B67785D900


@pytest.fixture(scope="module")
def ctx():
    import qp_wormhole
    c = qp_wormhole.Context(0)
    yield c
    c.close()


def rand_felts(rng, *shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


def test_poseidon_permute(ctx):
    """Every state of a 4096-state batch (random, zero, all p-1, unit lanes,
    small values) equals the oracle's plain-round permutation: exercises the
    device's sparse, grouped partial rounds and their accumulator bounds."""
    import qp_wormhole
    rng = np.random.default_rng(10)
    states = rand_felts(rng, 4096, 12)
    states[0] = 0
    states[1] = P - 1
    for i in range(12):
        states[2 + i] = 0
        states[2 + i, i] = 1
        states[14 + i] = P - 1
        states[14 + i, i] = 0
    states[26:40] = rng.integers(0, 4, size=(14, 12), dtype=np.uint64)
    states[40:60] = P - 1 - rng.integers(0, 2**32, size=(20, 12), dtype=np.uint64)
    got = qp_wormhole.poseidon_permute(ctx, states)
    want = states.copy()
    for i in range(len(want)):
        olib().ora_permute(want[i])
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, bad[:10]


# 15, 16: beyond one workgroup's LDS (HBM levels + 2^14-point LDS blocks)
@pytest.mark.parametrize("log_n", [1, 3, 8, 10, 13, 14, 15, 16])
def test_ifft(ctx, log_n):
    import qp_wormhole
    rng = np.random.default_rng(log_n)
    v = rand_felts(rng, 3, 1 << log_n)
    got = qp_wormhole.ifft(ctx, v)
    for c in range(3):
        e = v[c].copy()
        olib().ora_ifft(e, log_n)
        assert (got[c] == e).all()


@pytest.mark.parametrize("log_n,rate_bits", [(2, 1), (5, 3), (10, 3), (13, 3), (12, 4), (11, 1), (11, 2), (13, 1), (10, 4), (14, 2),
                                            (15, 3), (16, 2), (15, 1)])
def test_lde_leaf_order(ctx, log_n, rate_bits):
    import qp_wormhole
    rng = np.random.default_rng(100 + log_n)
    c = rand_felts(rng, 2, 1 << log_n)
    got = qp_wormhole.lde(ctx, c, rate_bits)
    logN = log_n + rate_bits
    rev = np.array([int(format(i, f"0{logN}b")[::-1], 2) for i in range(1 << logN)])
    for k in range(2):
        e = np.zeros(1 << logN, np.uint64)
        olib().ora_lde(c[k], log_n, rate_bits, G, e)
        assert (got[k] == e[rev]).all()


@pytest.mark.parametrize("npolys,log_n,rate_bits,cap_h,nsalt", [
    (1, 6, 3, 2, 0),     # leaf width 1 -> hash_or_noop pads
    (4, 6, 3, 0, 0),     # width 4 noop, cap height 0
    (5, 7, 3, 4, 0),     # width 5 -> one permutation
    (16, 8, 3, 4, 4),    # salted
    (20, 9, 3, 4, 0),
    (84, 8, 3, 4, 0),    # constants||sigmas width
    (135, 8, 3, 4, 4),   # salted wires width 139
])
def test_commit_values_parity(ctx, npolys, log_n, rate_bits, cap_h, nsalt):
    import qp_wormhole
    rng = np.random.default_rng(npolys * 1000 + log_n)
    vals = rand_felts(rng, npolys, 1 << log_n)
    salt = rand_felts(rng, 1 << (log_n + rate_bits), nsalt) if nsalt else None
    coeffs_o, leaves_o, cap_o = commit_values(vals, log_n, rate_bits, cap_h, salt=salt, want_leaves=True)
    b = qp_wormhole.PolynomialBatch.from_values(ctx, vals, rate_bits, cap_h, salt=salt)
    assert (b.coeffs == coeffs_o).all()
    assert (b.cap == cap_o).all()
    assert (b.lde() == leaves_o[:, :npolys].T).all()
    # openings: leaves + Merkle paths against the oracle's tree
    N = 1 << (log_n + rate_bits)
    idx = np.array([0, 1, N - 1, N // 2, 12345 % N], np.uint32)
    leaves, sibs = b.open(idx)
    assert (leaves == leaves_o[idx]).all()
    depth = log_n + rate_bits - cap_h
    cap2 = np.zeros(((1 << cap_h), 4), np.uint64)
    sib_o = np.zeros((len(idx), depth, 4), np.uint64)
    olib().ora_merkle(np.ascontiguousarray(leaves_o), log_n + rate_bits, leaves_o.shape[1], cap_h, cap2,
                      idx.astype(np.uint64), len(idx), sib_o)
    assert (cap2 == cap_o).all()
    assert (sibs == sib_o).all()
    b.free()


def test_commit_coeffs_parity(ctx):
    import qp_wormhole
    rng = np.random.default_rng(7)
    co = rand_felts(rng, 16, 1 << 9)
    _, _, cap_o = commit_values(co, 9, 3, 4, from_coeffs=True)
    b = qp_wormhole.PolynomialBatch.from_coeffs(ctx, co, 3, 4)
    assert (b.cap == cap_o).all()
    b.free()


def test_commit_full_size_wires(ctx):
    """Full Wormhole wires shape (135 x 2^13, blowup 8, cap 16) bit-exact vs the oracle."""
    import qp_wormhole
    rng = np.random.default_rng(2024)
    vals = rand_felts(rng, 135, 1 << 13)
    coeffs_o, _, cap_o = commit_values(vals, 13, 3, 4)
    b = qp_wormhole.PolynomialBatch.from_values(ctx, vals, 3, 4)
    assert (b.coeffs == coeffs_o).all()
    assert (b.cap == cap_o).all()
    b.free()


def test_bad_shape_is_an_error(ctx):
    """Beyond the twiddle tables (2^16 values at rate 3 = 2^19 points > 2^18):
    an error with the reason, not a wrong result."""
    import qp_wormhole
    with pytest.raises(qp_wormhole.QpError):
        qp_wormhole.PolynomialBatch.from_values(ctx, np.zeros((2, 1 << 16), np.uint64), 3, 4)
