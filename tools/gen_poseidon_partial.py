"""Generate qp-zk-circuits-rm_amd/csrc/poseidon_partial_consts.h: constants of
the sparse ("fast") form of Poseidon's 22 partial rounds (Poseidon paper,
Appendix B; the same factorisation plonky2 ships as FAST_PARTIAL_* tables in
poseidon_goldilocks.rs), derived here from the MDS matrix and the round
constants, then checked against the plain permutation (and, when the oracle
library is built, against oracle/poseidon.c).

Plain partial round r (r = 4..25):  y <- M S(y + c_r), S = x^7 on lane 0 only.
With M = A_r D_r, D_r = diag(1, X_r) (commutes with S) and A_r sparse
(row 0 = [25 | a_hat], column 0 = [25 | b], identity elsewhere), working from
the last partial round back (X of each factorisation merges into the M before
it), the 22 rounds become
    z <- D_4 (y_4 + c_4)                            (merged into round 3's MDS)
    repeat: z0 <- S(z0); z <- A_r z + k_(r+1) e_0   (scalar constants pushed
                                                    forward, the last vector
                                                    folded into round 26's)
so a partial round costs one row dot product and 11 scalar multiply-adds
instead of a dense 12x12 MDS layer.

Device arithmetic: a state value x is split into 22-bit limbs
x = l0 + 2^22 l1 + 2^44 l2, and every constant c of the sparse rows is stored
as the three field elements c 2^(22k) mod p split into 32-bit halves, so a
product-accumulate is 2 v_mad_u64_u32 per limb with all partial sums < 2^60
(one 4-instruction reduction per output).  The lane-0 dot product instead
multiplies the 32-bit halves of the state by 22/22/20-bit pieces of the
constants (AH2: no limb extraction of the 11 inputs), three accumulators at
weights 1, 2^22, 2^44 recombined once per round.

    python tools/gen_poseidon_partial.py   # writes the header, self-checks
"""
import os
import random
import sys

P = 0xFFFFFFFF00000001
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "qp-zk-circuits-rm_amd", "csrc", "poseidon_partial_consts.h")
CIRC = [17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]
W = 12


def round_constants():
    src = open(os.path.join(ROOT, "qp-zk-circuits-rm_amd", "csrc", "poseidon.h")).read()
    body = src[src.index("#define QP_POSEIDON_RC_LIST"):]
    vals = []
    for tok in body.replace("\\", " ").replace(",", " ").split():
        if tok.startswith("0x") and tok.endswith("ULL"):
            vals.append(int(tok[:-3], 16))
        if len(vals) == 360:
            break
    assert len(vals) == 360
    return [vals[r * W:(r + 1) * W] for r in range(30)]


RC = round_constants()
M = [[(CIRC[(c - r) % W] + (8 if r == c == 0 else 0)) for c in range(W)] for r in range(W)]


def matmul(A, B):
    return [[sum(A[i][k] * B[k][j] for k in range(len(B))) % P for j in range(len(B[0]))] for i in range(len(A))]


def matvec(A, v):
    return [sum(a * x for a, x in zip(row, v)) % P for row in A]


def inverse(A):
    n = len(A)
    a = [row[:] + [int(i == j) for j in range(n)] for i, row in enumerate(A)]
    for c in range(n):
        p = next(r for r in range(c, n) if a[r][c])
        a[c], a[p] = a[p], a[c]
        inv = pow(a[c][c], P - 2, P)
        a[c] = [x * inv % P for x in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [(x - f * y) % P for x, y in zip(a[r], a[c])]
    return [row[n:] for row in a]


def sbox(x):
    return pow(x, 7, P)


def permute_plain(s):
    s = list(s)
    for r in range(30):
        s = [(x + c) % P for x, c in zip(s, RC[r])]
        if r < 4 or r >= 26:
            s = [sbox(x) for x in s]
        else:
            s[0] = sbox(s[0])
        s = matvec(M, s)
    return s


def derive():
    A, D = {}, {}
    Q = [row[:] for row in M]
    for r in range(25, 3, -1):
        Qh = [row[1:] for row in Q[1:]]
        Qhi = inverse(Qh)
        ahat = matvec([list(col) for col in zip(*Qhi)], Q[0][1:])  # Q[0,1:] . Qh^-1
        b = [Q[i][0] for i in range(1, W)]
        assert Q[0][0] == M[0][0] == 25
        A[r] = (ahat, b)
        D[r] = [[1] + [0] * (W - 1)] + [[0] + row for row in Qh]
        Q = matmul(D[r], M)
    # init: rows of D_4 M and the constant D_4 c_4
    init_rows = matmul(D[4], M)
    init_k = matvec(D[4], RC[4])
    # forward constant push: v_r = D_r c_r + A_(r-1) (0, v_hat_(r-1)), r = 5..25
    kscalar = {}
    push = [0] * W
    for r in range(5, 26):
        v = [(x + y) % P for x, y in zip(matvec(D[r], RC[r]), push)]
        kscalar[r] = v[0]
        ahat, b = A[r]
        vh = [0] + v[1:]
        push = [sum(a * x for a, x in zip(ahat, vh[1:])) % P] + [(vh[i] + b[i - 1] * 0) % P for i in range(1, W)]
        # A (0, vh): row 0 = ahat . vh[1:], rows i >= 1 = vh[i] + b[i-1] * 0
    c26 = [(x + y) % P for x, y in zip(RC[26], push)]
    return A, init_rows, init_k, kscalar, c26


def permute_fast(s, A, init_rows, init_k, kscalar, c26):
    s = list(s)
    for r in range(4):
        s = [(x + c) % P for x, c in zip(s, RC[r])]
        s = [sbox(x) for x in s]
        if r < 3:
            s = matvec(M, s)
    # round 3's MDS merged with D_4 and c_4
    s = [(x + k) % P for x, k in zip(matvec(init_rows, s), init_k)]
    for r in range(4, 26):
        ahat, b = A[r]
        x0 = sbox(s[0])
        k0 = kscalar[r + 1] if r < 25 else c26[0]
        n0 = (25 * x0 + sum(a * x for a, x in zip(ahat, s[1:])) + k0) % P
        rest = [(s[i] + b[i - 1] * x0 + (c26[i] if r == 25 else 0)) % P for i in range(1, W)]
        s = [n0] + rest
    for r in range(26, 30):
        if r > 26:
            s = [(x + c) % P for x, c in zip(s, RC[r])]
        s = [sbox(x) for x in s]
        s = matvec(M, s)
    return s


def gammas(A):
    """gamma[t][l] = a_hat^(t) . b^(l) (t, l = partial round - 4, l < t): the
    effect of round l's S-box output on round t's lane-0 dot when the lane
    1..11 updates of rounds l..t-1 are deferred"""
    g = [[0] * 22 for _ in range(22)]
    for t in range(22):
        for l in range(t):
            g[t][l] = sum(a * b for a, b in zip(A[t + 4][0], A[l + 4][1])) % P
    return g


def permute_fast_grouped(s, A, init_rows, init_k, kscalar, c26, G):
    """permute_fast with the lane 1..11 updates of G consecutive partial rounds
    applied once per group (lane-0 dots use the group-start lanes + gamma terms)"""
    gam = gammas(A)
    s = list(s)
    for r in range(4):
        s = [(x + c) % P for x, c in zip(s, RC[r])]
        s = [sbox(x) for x in s]
        if r < 3:
            s = matvec(M, s)
    s = [(x + k) % P for x, k in zip(matvec(init_rows, s), init_k)]
    for t0 in range(0, 22, G):
        ts = list(range(t0, min(t0 + G, 22)))
        xs = []
        s0 = s[0]
        for t in ts:
            r = t + 4
            x = sbox(s0)
            k0 = kscalar[r + 1] if r < 25 else c26[0]
            d = 25 * x + sum(a * v for a, v in zip(A[r][0], s[1:])) + k0
            d += sum(gam[t][l] * xl for l, xl in zip(ts, xs))
            xs.append(x)
            s0 = d % P
        rest = []
        for i in range(1, W):
            v = s[i] + sum(A[t + 4][1][i - 1] * x for t, x in zip(ts, xs))
            if ts[-1] == 21:
                v += c26[i]
            rest.append(v % P)
        s = [s0] + rest
    for r in range(26, 30):
        if r > 26:
            s = [(x + c) % P for x, c in zip(s, RC[r])]
        s = [sbox(x) for x in s]
        s = matvec(M, s)
    return s


def limbs_consts(c):
    """c 2^(22k) mod p for k = 0, 1, 2 -> [(lo32, hi32)] * 3"""
    out = []
    for k in range(3):
        v = c * pow(2, 22 * k, P) % P
        out.append((v & 0xFFFFFFFF, v >> 32))
    return out


def emit(A, init_rows, init_k, kscalar, c26):
    L = []
    L.append("// poseidon_partial_consts.h -- GENERATED by tools/gen_poseidon_partial.py (see there).")
    L.append("// Sparse partial-round form of Poseidon-Goldilocks (width 12); every row constant c")
    L.append("// is stored as the 32-bit halves of c * 2^(22k) mod p, k = 0, 1, 2 (one per 22-bit limb).")
    L.append("#pragma once")
    L.append("#include <stdint.h>")
    L.append("namespace pfp {")

    def arr(name, rows):
        flat = []
        for row in rows:
            flat.extend(row)
        L.append(f"constexpr uint32_t {name}[{len(flat)}] = {{")
        for i in range(0, len(flat), 8):
            L.append("    " + ", ".join(f"0x{x:08x}u" for x in flat[i:i + 8]) + ",")
        L.append("};")

    def lc(c):
        return [h for pair in limbs_consts(c) for h in pair]

    # INIT[i][j]: rows i = 1..11 of D_4 M, 12 entries, 6 words each
    arr("INIT", [lc(init_rows[i][j]) for i in range(1, W) for j in range(W)])
    assert init_rows[0] == M[0]
    arr("INIT_K", [[init_k[i] & 0xFFFFFFFF, init_k[i] >> 32] for i in range(W)])
    # AHAT[t][j] (t = r - 4, j = 1..11), B[t][i], S0 = 25
    arr("AHAT", [lc(A[r][0][j]) for r in range(4, 26) for j in range(W - 1)])
    arr("BV", [lc(A[r][1][i]) for r in range(4, 26) for i in range(W - 1)])
    arr("S0C", [lc(25)])
    # AH2[t][j][h]: a_hat_j (h = 0, times the low half) and a_hat_j 2^32 mod p
    # (h = 1, times the high half) as 22/22/20-bit pieces (weights 1, 2^22, 2^44)
    def pieces(c):
        return [c & 0x3FFFFF, (c >> 22) & 0x3FFFFF, c >> 44]
    arr("AH2", [pieces(A[r][0][j] * (1 << (32 * h)) % P) for r in range(4, 26) for j in range(W - 1) for h in range(2)])
    k0 = [kscalar[r + 1] if r < 25 else c26[0] for r in range(4, 26)]
    arr("K0", [[k & 0xFFFFFFFF, k >> 32] for k in k0])
    # CAPZ_K[r]: round 1's constant plus row r of the round-0 MDS applied to
    # the S-box outputs of lanes 8..11 when they enter the permutation as zero
    # (two_to_one / first absorption: sbox(0 + RC[0][j]) is a constant)
    cz = [sbox(RC[0][j]) if j >= 8 else 0 for j in range(W)]
    capz = [(RC[1][r] + sum(M[r][j] * cz[j] for j in range(8, W))) % P for r in range(W)]
    arr("CAPZ_K", [[k & 0xFFFFFFFF, k >> 32] for k in capz])
    # GAM[t][l] (l < t, zero elsewhere): a_hat^(t) . b^(l), as limb halves
    gam = gammas(A)
    arr("GAM", [lc(gam[t][l]) for t in range(22) for l in range(22)])
    arr("KLAST", [[c26[i] & 0xFFFFFFFF, c26[i] >> 32] for i in range(W)])
    L.append("}  // namespace pfp")
    open(HDR, "w").write("\n".join(L) + "\n")


def main():
    A, init_rows, init_k, kscalar, c26 = derive()
    rnd = random.Random(7)
    for _ in range(20):
        s = [rnd.randrange(P) for _ in range(W)]
        assert permute_fast(s, A, init_rows, init_k, kscalar, c26) == permute_plain(s)
        for G in (1, 2, 3, 4, 6):
            assert permute_fast_grouped(s, A, init_rows, init_k, kscalar, c26, G) == permute_plain(s)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle_lib import permute as ora_permute
        for _ in range(5):
            s = [rnd.randrange(P) for _ in range(W)]
            assert [int(x) for x in ora_permute(s)] == permute_plain(s)
        print("oracle permutation agrees")
    except (ImportError, OSError) as e:
        print("oracle not checked:", e)
    emit(A, init_rows, init_k, kscalar, c26)
    print("sparse partial rounds == plain permutation; wrote", HDR)


if __name__ == "__main__":
    main()
