"""plonky2's prove() composed from the routine-level C-ABI seams (INTEGRATION.md
binding A), with the CPU oracle standing in for the host code a patched
qp-plonky2 keeps: the Challenger, wires_permutation_partial_products_and_zs,
OpeningSet::new and the initial FRI polynomial (PolynomialBatch::prove_openings).
Everything else goes through the seams:

    qp_commit_values / qp_commit_coeffs   PolynomialBatch::from_values / from_coeffs
    qp_quotient                           compute_quotient_polys
    qp_fri_layer_commit / qp_fri_fold     fri_committed_trees
    qp_pow_grind                          fri_proof_of_work
    qp_batch_open / qp_fri_layer_open     fri_prover_query_rounds

TEST INFRASTRUCTURE: the proof this builds must be byte-identical to the
oracle's monolithic CPU prover (or_prove) and to the GPU whole-circuit prover,
which shows the seams compose into plonky2's prove() exactly.  Transcript order:
SURVEY.md A.4 (the oracle's or_prove follows the same)."""
import ctypes
import struct

import numpy as np

from oracle_lib import P, U64P, hash_no_pad, lib as olib

GEN = 0xC65C18B67785D900


class Challenger:
    """plonky2 iop/challenger.rs duplex sponge over the oracle's Poseidon."""

    def __init__(self):
        self.state = np.zeros(12, np.uint64)
        self.inp, self.out = [], []

    def duplex(self):
        for i, x in enumerate(self.inp):
            self.state[i] = x
        self.inp = []
        olib().ora_permute(self.state)
        self.out = [int(x) for x in self.state[:8]]

    def observe(self, xs):
        for x in np.asarray(xs, dtype=np.uint64).reshape(-1):
            self.out = []
            self.inp.append(int(x))
            if len(self.inp) == 8:
                self.duplex()

    def get(self):
        if self.inp or not self.out:
            self.duplex()
        return self.out.pop()

    def get_ext(self):
        a = self.get()
        return (a, self.get())

    def pending_state(self):
        """sponge state with the pending inputs written in, and their count (the PoW seam's input)"""
        st = self.state.copy()
        for i, x in enumerate(self.inp):
            st[i] = x
        return st, len(self.inp)


def _bind():
    L = olib()
    if not getattr(L, "_seam_bound", False):
        L.ora_zs_values.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, U64P, U64P]
        L.ora_eval_ext.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, U64P, U64P]
        L.ora_fri_initial.argtypes = [U64P, ctypes.c_uint, U64P, ctypes.c_uint, U64P, ctypes.c_uint, U64P,
                                      ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, U64P, U64P, U64P, U64P]
        L.ora_hash_pad.argtypes = [U64P, ctypes.c_size_t, U64P]
        L._seam_bound = True
    return L


def _ext_mul(a, b):
    return ((a[0] * b[0] + 7 * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _root(log_n):
    return pow(7277203076849721926, 1 << (32 - log_n), P)


def evals_ext(coeffs, x):
    L = _bind()
    c = np.ascontiguousarray(coeffs, dtype=np.uint64)
    out = np.zeros((c.shape[0], 2), np.uint64)
    L.ora_eval_ext(c, c.shape[0], c.shape[1].bit_length() - 1, np.array(x, np.uint64), out)
    return out


def fri_arities(log_n, rate_bits=3, cap_h=4, arity=4, final_poly_bits=5):
    """FriReductionStrategy::ConstantArityBits(4, 5) of standard_recursion_config."""
    out = []
    db = log_n
    while db > final_poly_bits and db + rate_bits - arity >= cap_h:
        out.append(arity)
        db -= arity
    return out, 1 << db


def prove(ctx, circuit, wires, pis, gate_desc=None, cap_h=4, rate_bits=3, num_queries=28, pow_bits=16):
    """One proof of `circuit` (built-in circuit object: constants/sigmas + common data) for
    the witness `wires` [num_wires][n] and public inputs `pis`, through the seams."""
    import qp_wormhole as q
    L = _bind()
    common = circuit.common_data()
    n = circuit.n
    log_n = circuit.degree_bits
    logN = log_n + rate_bits
    N = 1 << logN
    g = gate_desc or q.gate_desc(circuit)
    arity_bits, final_len = fri_arities(log_n, rate_bits, cap_h)
    nc, qdf = g.num_challenges, g.quotient_degree_factor
    cs_vals = circuit.constants_sigmas()
    # preprocessing (build_prover): constants || sigmas commitment and circuit digest
    cs = q.PolynomialBatch.from_values(ctx, cs_vals, rate_bits, cap_h)
    empty = np.zeros(4, np.uint64)
    L.ora_hash_pad(np.zeros(1, np.uint64), 0, empty)
    digest = hash_no_pad(np.concatenate([cs.cap.reshape(-1), empty, np.array([log_n], np.uint64)]))
    pih = hash_no_pad(np.asarray(pis, np.uint64))
    t = Challenger()
    t.observe(digest)
    t.observe(pih)
    # wires commitment
    w = q.PolynomialBatch.from_values(ctx, wires, rate_bits, cap_h)
    t.observe(w.cap)
    betas = [t.get() for _ in range(nc)]
    gammas = [t.get() for _ in range(nc)]
    # partial products and Z (host in plonky2), their commitment
    nchunks = (g.num_routed_wires + qdf - 1) // qdf
    zs_vals = np.zeros((nc * nchunks, n), np.uint64)
    assert L.ora_zs_values(common, len(common), cs_vals, np.ascontiguousarray(wires, np.uint64),
                           np.array(betas, np.uint64), np.array(gammas, np.uint64), zs_vals) == 0
    z = q.PolynomialBatch.from_values(ctx, zs_vals, rate_bits, cap_h)
    t.observe(z.cap)
    alphas = [t.get() for _ in range(nc)]
    # quotient (seam) and its commitment
    qc = q.quotient(ctx, cs, w, z, g, betas, gammas, alphas, pih)
    qb = q.PolynomialBatch.from_coeffs(ctx, qc, rate_bits, cap_h)
    t.observe(qb.cap)
    zeta = t.get_ext()
    # openings (host in plonky2)
    batches = [cs, w, z, qb]
    zeta_next = _ext_mul(zeta, (_root(log_n), 0))
    op = [evals_ext(b.coeffs, zeta) for b in batches]
    z_next = evals_ext(z.coeffs[:nc], zeta_next)
    npp = nc * (nchunks - 1)
    opening_seq = [op[0], op[1], op[2][:nc], op[2][nc:nc + npp], op[3], z_next]
    for o in opening_seq:
        t.observe(o)
    # FRI: initial polynomial (host), then one seam call per reduction layer
    alpha = t.get_ext()
    fin = np.zeros((n, 2), np.uint64)
    L.ora_fri_initial(cs.coeffs, cs.npolys, w.coeffs, w.npolys, z.coeffs, z.npolys, qb.coeffs, qb.npolys, nc, log_n,
                      np.array(alpha, np.uint64), np.array(zeta, np.uint64), np.array(zeta_next, np.uint64), fin)
    coeffs = np.zeros((2, N), np.uint64)  # plonky2 keeps the zero tail: length N
    coeffs[:, :n] = fin.T
    shift, lg = GEN, logN
    layers, layer_caps = [], []
    for ab in arity_bits:
        layer = q.FriLayer(ctx, coeffs, lg, shift, ab, cap_h)
        layers.append(layer)
        layer_caps.append(layer.cap)
        t.observe(layer.cap)
        beta = t.get_ext()
        coeffs = q.fri_fold(ctx, coeffs, ab, beta)
        shift = pow(shift, 1 << ab, P)
        lg -= ab
    final = coeffs[:, :final_len].T.copy()
    t.observe(final)
    # proof of work (seam), then one challenge the verifier draws too
    st, pos = t.pending_state()
    pw = int(q.pow_grind(ctx, st[None, :], [pos], pow_bits)[0])
    t.observe([pw])
    t.get()
    # query rounds
    queries = []
    for _ in range(num_queries):
        xi = t.get() % N
        init = [b.open([xi]) for b in batches]
        steps = []
        for layer, ab in zip(layers, arity_bits):
            li = xi >> ab
            ev, sib = layer.open([li])
            steps.append((ev[0], sib[0]))
            xi = li
        queries.append((init, steps))
    # ProofWithPublicInputs::to_bytes
    out = bytearray()

    def u64s(a):
        out.extend(np.ascontiguousarray(a, dtype=np.uint64).tobytes())
    for b in (w, z, qb):
        u64s(b.cap)
    # openings: constants, wires, zs, zs_next, partial products, quotient
    for o in (op[0], op[1], op[2][:nc], z_next, op[2][nc:nc + npp], op[3]):
        u64s(o)
    for c in layer_caps:
        u64s(c)
    for init, steps in queries:
        for leaves, sibs in init:
            u64s(leaves[0])
            out.append(sibs.shape[1])
            u64s(sibs[0])
        for ev, sib in steps:
            u64s(ev)
            out.append(sib.shape[0])
            u64s(sib)
    u64s(final)
    out.extend(struct.pack("<QQ", pw, len(pis)))
    u64s(np.asarray(pis, np.uint64))
    for layer in layers:
        layer.free()
    return bytes(out)
