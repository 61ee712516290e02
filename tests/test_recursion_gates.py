"""Recursive-verifier gate constraints (the aggregator
circuits' gates, wormhole/aggregator/src/circuits/tree.rs:106-143) in the CPU
oracle (oracle/gates_impl.h gate_recursion).

Parity UNPINNED: no reference fixture holds a circuit with these gates (the
aggregator's proofs are not committed), so the oracle restates upstream
plonky2's eval_unfiltered layouts.  What is pinned here is semantics: for
every gate a witness built the way the gate's generator defines it (products,
Horner accumulations, x^e by square-and-multiply, a list lookup, the MDS
layer, and the value at a point of the polynomial interpolating a coset,
computed independently by Lagrange interpolation) satisfies every constraint,
and perturbing any wire the constraints read makes some constraint nonzero.
The descriptor-driven oracle quotient is also checked against the
common-data-driven one on the Wormhole circuit."""
import random

import numpy as np
import pytest

from oracle_lib import P, lib as olib

MDS_CIRC = [17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]
MDS_DIAG = [8] + [0] * 11


def inv(a):
    return pow(a % P, P - 2, P)


def emul(a, b):
    return ((a[0] * b[0] + 7 * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def eadd(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def esub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def escale(a, s):
    return (a[0] * s % P, a[1] * s % P)


def root(bits):
    return pow(7277203076849721926, 1 << (32 - bits), P)


def desc(kind, params=()):
    import qp_wormhole
    return qp_wormhole.GateDesc.build([(kind, params, 0)], [(0, 1)], num_gate_constraints=256)


def rnd(rng):
    return rng.randrange(P)


def put(w, i, e):
    w[i], w[i + 1] = e


# ---- witness builders: (wires[135], gate constants[2]) satisfying the gate

def w_arith_ext(rng, n=10):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    for i in range(n):
        o = 8 * i
        m0, m1, ad = (w[o], w[o + 1]), (w[o + 2], w[o + 3]), (w[o + 4], w[o + 5])
        put(w, o + 6, eadd(escale(emul(m0, m1), c[0]), escale(ad, c[1])))
    return w, c


def w_mul_ext(rng, n=13):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    for i in range(n):
        o = 6 * i
        put(w, o + 4, escale(emul((w[o], w[o + 1]), (w[o + 2], w[o + 3])), c[0]))
    return w, c


def w_reducing(rng, n, ext):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    alpha, acc = (w[2], w[3]), (w[4], w[5])
    cw = 2 if ext else 1
    start = 6 + cw * n
    for i in range(n):
        coeff = (w[6 + 2 * i], w[7 + 2 * i]) if ext else (w[6 + i], 0)
        acc = eadd(emul(acc, alpha), coeff)
        put(w, 0 if i == n - 1 else start + 2 * i, acc)
    return w, c


def w_exponentiation(rng, nb=66):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    base, power = w[0], rng.randrange(1 << nb)
    for i in range(nb):
        w[1 + i] = (power >> i) & 1
    cur = 1
    for i in range(nb):  # bits consumed most significant first
        bit = w[1 + nb - 1 - i]
        cur = cur * cur % P * (base if bit else 1) % P
        w[2 + nb + i] = cur
    w[1 + nb] = pow(base, power, P)  # the output is base^power, independent of the gate's recurrence
    assert w[1 + nb] == cur
    return w, c


def mds(v):
    return [(sum(MDS_CIRC[i] * v[(i + r) % 12] for i in range(12)) + MDS_DIAG[r] * v[r]) % P for r in range(12)]


def w_poseidon_mds(rng):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    o0, o1 = mds([w[2 * i] for i in range(12)]), mds([w[2 * i + 1] for i in range(12)])
    for r in range(12):
        w[24 + 2 * r], w[25 + 2 * r] = o0[r], o1[r]
    return w, c


def w_random_access(rng, bits=4, copies=4, extra=2):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    vec = 1 << bits
    routed = (2 + vec) * copies + extra
    for cp in range(copies):
        base = (2 + vec) * cp
        idx = rng.randrange(vec)
        w[base] = idx
        w[base + 1] = w[base + 2 + idx]
        for i in range(bits):
            w[routed + cp * bits + i] = (idx >> i) & 1
    for i in range(extra):
        w[(2 + vec) * copies + i] = c[i]
    return w, c


def w_coset_interp(rng, bits=4, deg=6):
    w, c = [rnd(rng) for _ in range(135)], [rnd(rng), rnd(rng)]
    npts = 1 << bits
    nint = (npts - 2) // (deg - 1)
    sep, sev, si = 1 + 2 * npts, 3 + 2 * npts, 5 + 2 * npts
    ssh = si + 4 * nint
    shift = w[0] = rnd(rng) or 1
    vals = [(w[1 + 2 * i], w[2 + 2 * i]) for i in range(npts)]
    z = (w[sep], w[sep + 1])
    put(w, ssh, escale(z, inv(shift)))
    # value at z of the polynomial through (shift * om^i, vals[i]): Lagrange, independent of the gate
    om = root(bits)
    xs = [shift * pow(om, i, P) % P for i in range(npts)]
    acc = (0, 0)
    for i in range(npts):
        num, den = (1, 0), 1
        for j in range(npts):
            if j != i:
                num = emul(num, esub(z, (xs[j], 0)))
                den = den * (xs[i] - xs[j]) % P
        acc = eadd(acc, escale(emul(vals[i], num), inv(den)))
    put(w, sev, acc)
    # intermediates: the running (eval, prod) of the chunked barycentric fold
    pt = (w[ssh], w[ssh + 1])
    n_inv = inv(npts)
    e, p = (0, 0), (1, 0)
    lo, hi = 0, deg
    for it in range(nint + 1):
        for i in range(lo, hi):
            x = pow(om, i, P)
            t = esub(pt, (x, 0))
            e = eadd(emul(e, t), emul(escale(vals[i], x * n_inv % P), p))
            p = emul(p, t)
        if it == nint:
            break
        put(w, si + 2 * it, e)
        put(w, si + 2 * (nint + it), p)
        lo = 1 + (deg - 1) * (it + 1)
        hi = min(lo + deg - 1, npts)
    assert e == acc  # the fold reproduces the interpolant
    return w, c


CASES = [
    ("arithmetic_extension", (10,), w_arith_ext, 20, list(range(80))),
    ("mul_extension", (13,), w_mul_ext, 26, list(range(78))),
    ("reducing", (43,), lambda r: w_reducing(r, 43, False), 86, list(range(6 + 43 + 84))),
    ("reducing_extension", (32,), lambda r: w_reducing(r, 32, True), 64, list(range(6 + 64 + 62))),
    ("exponentiation", (66,), w_exponentiation, 67, list(range(2 + 132))),
    ("poseidon_mds", (), w_poseidon_mds, 24, list(range(48))),
    # list items other than the indexed one are (correctly) free: access indices, claimed
    # elements, extra constants and bits only (the indexed item: test below)
    ("random_access", (4, 4, 2), w_random_access, 26, [18 * k + o for k in range(4) for o in (0, 1)] + [72, 73] +
     list(range(74, 90))),
    ("coset_interpolation", (4, 6), w_coset_interp, 12, list(range(1 + 32 + 4 + 8 + 2))),
]


def gate_eval(d, w, c):
    out = np.zeros(512, np.uint64)
    k = olib().ora_gate_eval(_addr(d), 0, np.array(c, np.uint64), np.array(w, np.uint64),
                             np.zeros(4, np.uint64), out)
    return [int(x) for x in out[:k]]


def _addr(d):
    import ctypes
    return ctypes.addressof(d)


@pytest.mark.parametrize("kind,params,build,ncons,used", CASES, ids=[c[0] for c in CASES])
def test_recursion_gate_satisfied_and_sensitive(kind, params, build, ncons, used):
    rng = random.Random(sum(map(ord, kind)))
    d = desc(kind, params)
    w, c = build(rng)
    out = gate_eval(d, w, c)
    assert len(out) == ncons
    assert out == [0] * ncons
    # every wire the gate reads changes some constraint
    for j in rng.sample(used, min(len(used), 24)):
        w2 = list(w)
        w2[j] = (w2[j] + 1) % P
        assert any(gate_eval(d, w2, c)), (kind, j)


def test_random_access_reads_the_indexed_item():
    rng = random.Random(5)
    d = desc("random_access", (4, 4, 2))
    w, c = w_random_access(rng)
    w[1] = (w[1] + 1) % P  # claimed element of copy 0 no longer list[index]
    out = gate_eval(d, w, c)
    assert out[5] != 0 and all(x == 0 for i, x in enumerate(out) if i != 5)


def test_quotient_desc_matches_common_data_path():
    """ora_quotient_desc (gate description) == ora_quotient (common data) on the Wormhole circuit."""
    import qp_wormhole
    circ = qp_wormhole.Circuit.wormhole()
    g = qp_wormhole.gate_desc(circ)
    rng = np.random.default_rng(3)
    n = circ.n
    cs = circ.constants_sigmas()
    wires = rng.integers(0, P, (135, n), dtype=np.uint64)
    zs = rng.integers(0, P, (20, n), dtype=np.uint64)
    b, gm, al, pih = (rng.integers(0, P, k, dtype=np.uint64) for k in (2, 2, 2, 4))
    a = np.zeros((16, n), np.uint64)
    bb = np.zeros((16, n), np.uint64)
    cb = circ.common_data()
    assert olib().ora_quotient(cb, len(cb), cs, wires, zs, b, gm, al, pih, a) == 0
    assert olib().ora_quotient_desc(_addr(g), circ.degree_bits, 3, cs, wires, zs, b, gm, al, pih, bb) == 0
    assert (a == bb).all()
