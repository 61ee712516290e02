/*
 * oracle/gates_impl.h — plonky2 gate constraints (upstream gates/{arithmetic_base,
 * base_sum, constant, noop, public_input, poseidon}.rs eval_unfiltered) and the
 * selector filter (gates/gate.rs compute_filter), written once over a
 * scalar type T and instantiated for F (prover) and F_ext (verifier at zeta).
 * TEST INFRASTRUCTURE ONLY.  Formulas: SURVEY.md A.5 ([EXT verified] by the
 * zeta-identity on wormhole/bench-data/proof.bin).
 * Required macros: T, T_ADD, T_SUB, T_MUL, T_FROM(u64), T_ZERO, FN(name).
 */
#define UNUSED_SELECTOR 4294967295ULL

static inline T FN(sbox)(T x) { T x2 = T_MUL(x, x); T x3 = T_MUL(x2, x); T x4 = T_MUL(x2, x2); return T_MUL(x3, x4); }

static void FN(mds)(T *s) {
    T o[12];
    for (int r = 0; r < 12; r++) {
        T acc = T_ZERO;
        for (int i = 0; i < 12; i++) acc = T_ADD(acc, T_MUL(s[(i + r) % 12], T_FROM(PS_MDS_CIRC[i])));
        if (PS_MDS_DIAG[r]) acc = T_ADD(acc, T_MUL(s[r], T_FROM(PS_MDS_DIAG[r])));
        o[r] = acc;
    }
    for (int r = 0; r < 12; r++) s[r] = o[r];
}

/* PoseidonGate wire layout: in 0..12, out 12..24, swap 24, delta 25..29,
 * full-round-0 sbox inputs (rounds 1..3) 29..65, partial 65..87, full-1 87..135 */
static unsigned FN(poseidon)(const T *w, T *out) {
    unsigned k = 0;
    T swap = w[24];
    out[k++] = T_MUL(swap, T_SUB(swap, T_FROM(1)));
    for (int i = 0; i < 4; i++) {
        T delta = w[25 + i];
        out[k++] = T_SUB(T_MUL(swap, T_SUB(w[i + 4], w[i])), delta);
    }
    T s[12];
    for (int i = 0; i < 4; i++) { T delta = w[25 + i]; s[i] = T_ADD(w[i], delta); s[i + 4] = T_SUB(w[i + 4], delta); }
    for (int i = 8; i < 12; i++) s[i] = w[i];
    unsigned rc = 0;
    for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = T_ADD(s[i], T_FROM(PS_RC[rc * 12 + i]));
        if (r) for (int i = 0; i < 12; i++) { T sb = w[29 + (r - 1) * 12 + i]; out[k++] = T_SUB(s[i], sb); s[i] = sb; }
        for (int i = 0; i < 12; i++) s[i] = FN(sbox)(s[i]);
        FN(mds)(s);
    }
    for (int r = 0; r < 22; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = T_ADD(s[i], T_FROM(PS_RC[rc * 12 + i]));
        T sb = w[65 + r];
        out[k++] = T_SUB(s[0], sb);
        s[0] = FN(sbox)(sb);
        FN(mds)(s);
    }
    for (int r = 0; r < 4; r++, rc++) {
        for (int i = 0; i < 12; i++) s[i] = T_ADD(s[i], T_FROM(PS_RC[rc * 12 + i]));
        for (int i = 0; i < 12; i++) { T sb = w[87 + r * 12 + i]; out[k++] = T_SUB(s[i], sb); s[i] = sb; }
        for (int i = 0; i < 12; i++) s[i] = FN(sbox)(s[i]);
        FN(mds)(s);
    }
    for (int i = 0; i < 12; i++) out[k++] = T_SUB(s[i], w[12 + i]);
    return k;
}

/* ExtensionAlgebra<T, 2> (F_ext[Y]/(Y^2 - 7) over T): wires in pairs */
static inline void FN(alg_mul)(T a0, T a1, T b0, T b1, T *r0, T *r1) {
    *r0 = T_ADD(T_MUL(a0, b0), T_MUL(T_FROM(7), T_MUL(a1, b1)));
    *r1 = T_ADD(T_MUL(a0, b1), T_MUL(a1, b0));
}

/* recursion gate set (upstream gates/{arithmetic_extension, multiplication_extension,
 * reducing, reducing_extension, exponentiation, poseidon_mds, random_access,
 * coset_interpolation}.rs eval_unfiltered); parity UNPINNED: no reference
 * fixture holds a circuit with these gates (the aggregator's proofs are not
 * committed), so these restate the upstream formulas without a pin. */
static unsigned FN(gate_recursion)(const or_gate_t *g, const T *c, const T *w, T *out) {
    unsigned k = 0;
    switch (g->id) {
    case G_ARITH_EXT: /* per op: m0, m1, addend, output (2 wires each) */
        for (uint64_t i = 0; i < g->p0; i++) {
            const T *o = w + 8 * i;
            T p0, p1;
            FN(alg_mul)(o[0], o[1], o[2], o[3], &p0, &p1);
            out[k++] = T_SUB(o[6], T_ADD(T_MUL(p0, c[0]), T_MUL(o[4], c[1])));
            out[k++] = T_SUB(o[7], T_ADD(T_MUL(p1, c[0]), T_MUL(o[5], c[1])));
        }
        break;
    case G_MUL_EXT: /* per op: m0, m1, output */
        for (uint64_t i = 0; i < g->p0; i++) {
            const T *o = w + 6 * i;
            T p0, p1;
            FN(alg_mul)(o[0], o[1], o[2], o[3], &p0, &p1);
            out[k++] = T_SUB(o[4], T_MUL(p0, c[0]));
            out[k++] = T_SUB(o[5], T_MUL(p1, c[0]));
        }
        break;
    case G_REDUCING: case G_REDUCING_EXT: {
        /* output 0..2, alpha 2..4, old_acc 4..6, coeffs from 6 (base: 1 wire, ext: 2),
         * then the accumulators (the last one is the output) */
        const uint64_t nc = g->p0, cw = g->id == G_REDUCING ? 1 : 2, start_accs = 6 + cw * nc;
        T a0 = w[4], a1 = w[5];
        for (uint64_t i = 0; i < nc; i++) {
            T m0, m1;
            FN(alg_mul)(a0, a1, w[2], w[3], &m0, &m1);
            m0 = T_ADD(m0, w[6 + cw * i]);
            if (cw == 2) m1 = T_ADD(m1, w[7 + 2 * i]);
            const T *acc = i == nc - 1 ? w : w + start_accs + 2 * i;
            out[k++] = T_SUB(m0, acc[0]);
            out[k++] = T_SUB(m1, acc[1]);
            a0 = acc[0]; a1 = acc[1];
        }
        break;
    }
    case G_EXPONENTIATION: { /* base 0, power bits 1..nb+1 (LE), output nb+1, intermediates nb+2.. */
        const uint64_t nb = g->p0;
        const T base = w[0];
        for (uint64_t i = 0; i < nb; i++) {
            T prev = i == 0 ? T_FROM(1) : T_MUL(w[2 + nb + i - 1], w[2 + nb + i - 1]);
            T bit = w[1 + nb - 1 - i];
            T comp = T_MUL(prev, T_ADD(T_MUL(bit, base), T_SUB(T_FROM(1), bit)));
            out[k++] = T_SUB(comp, w[2 + nb + i]);
        }
        out[k++] = T_SUB(w[1 + nb], w[2 + nb + nb - 1]);
        break;
    }
    case G_POSEIDON_MDS: /* inputs 0..24, outputs 24..48, ext pairs */
        for (int r = 0; r < 12; r++) {
            T a0 = T_ZERO, a1 = T_ZERO;
            for (int i = 0; i < 12; i++) {
                a0 = T_ADD(a0, T_MUL(w[2 * ((i + r) % 12)], T_FROM(PS_MDS_CIRC[i])));
                a1 = T_ADD(a1, T_MUL(w[2 * ((i + r) % 12) + 1], T_FROM(PS_MDS_CIRC[i])));
            }
            if (PS_MDS_DIAG[r]) {
                a0 = T_ADD(a0, T_MUL(w[2 * r], T_FROM(PS_MDS_DIAG[r])));
                a1 = T_ADD(a1, T_MUL(w[2 * r + 1], T_FROM(PS_MDS_DIAG[r])));
            }
            out[k++] = T_SUB(w[24 + 2 * r], a0);
            out[k++] = T_SUB(w[25 + 2 * r], a1);
        }
        break;
    case G_RANDOM_ACCESS: { /* p0 bits, p1 copies, p2 extra constants */
        const uint64_t bits = g->p0, copies = g->p1, extra = g->p2, vec = (uint64_t)1 << bits;
        const uint64_t routed = (2 + vec) * copies + extra;
        for (uint64_t cp = 0; cp < copies; cp++) {
            const T *base = w + (2 + vec) * cp;
            const T *bw = w + routed + cp * bits;
            T list[64];
            for (uint64_t i = 0; i < vec; i++) list[i] = base[2 + i];
            for (uint64_t i = 0; i < bits; i++) out[k++] = T_MUL(bw[i], T_SUB(bw[i], T_FROM(1)));
            T idx = T_ZERO;
            for (uint64_t i = bits; i-- > 0;) idx = T_ADD(T_ADD(idx, idx), bw[i]);
            out[k++] = T_SUB(idx, base[0]);
            uint64_t len = vec;
            for (uint64_t i = 0; i < bits; i++) {
                for (uint64_t j = 0; j < len / 2; j++)
                    list[j] = T_ADD(list[2 * j], T_MUL(bw[i], T_SUB(list[2 * j + 1], list[2 * j])));
                len /= 2;
            }
            out[k++] = T_SUB(list[0], base[1]);
        }
        for (uint64_t i = 0; i < extra; i++) out[k++] = T_SUB(c[i], w[(2 + vec) * copies + i]);
        break;
    }
    case G_COSET_INTERP: { /* p0 subgroup bits, p1 degree */
        const uint64_t np = (uint64_t)1 << g->p0, deg = g->p1, nint = (np - 2) / (deg - 1);
        const uint64_t sv = 1, sep = sv + 2 * np, sev = sep + 2, si = sev + 2, sshift = si + 4 * nint;
        gl_t dom[64], wt[64];
        const gl_t om = gl_root_of_unity((unsigned)g->p0);
        dom[0] = 1;
        for (uint64_t i = 1; i < np; i++) dom[i] = gl_mul(dom[i - 1], om);
        for (uint64_t i = 0; i < np; i++) { /* barycentric weights 1 / prod_{j != i} (x_i - x_j) */
            gl_t d = 1;
            for (uint64_t j = 0; j < np; j++) if (j != i) d = gl_mul(d, gl_sub(dom[i], dom[j]));
            wt[i] = gl_inv(d);
        }
        const T shift = w[0];
        const T ep0 = w[sep], ep1 = w[sep + 1], sp0 = w[sshift], sp1 = w[sshift + 1];
        out[k++] = T_SUB(ep0, T_MUL(sp0, shift));
        out[k++] = T_SUB(ep1, T_MUL(sp1, shift));
        T e0 = T_ZERO, e1 = T_ZERO, p0 = T_FROM(1), p1 = T_ZERO;
        uint64_t lo = 0, hi = deg;
        for (uint64_t it = 0; it <= nint; it++) {
            for (uint64_t i = lo; i < hi; i++) { /* eval <- eval * (pt - x_i) + w_i v_i * prod; prod <- prod * (pt - x_i) */
                const T t0 = T_SUB(sp0, T_FROM(dom[i])), t1 = sp1;
                const T v0 = T_MUL(w[sv + 2 * i], T_FROM(wt[i])), v1 = T_MUL(w[sv + 2 * i + 1], T_FROM(wt[i]));
                T a0, a1, b0, b1, n0, n1;
                FN(alg_mul)(e0, e1, t0, t1, &a0, &a1);
                FN(alg_mul)(v0, v1, p0, p1, &b0, &b1);
                FN(alg_mul)(p0, p1, t0, t1, &n0, &n1);
                e0 = T_ADD(a0, b0); e1 = T_ADD(a1, b1);
                p0 = n0; p1 = n1;
            }
            if (it == nint) break;
            const T *ie = w + si + 2 * it, *ip = w + si + 2 * (nint + it);
            out[k++] = T_SUB(ie[0], e0);
            out[k++] = T_SUB(ie[1], e1);
            out[k++] = T_SUB(ip[0], p0);
            out[k++] = T_SUB(ip[1], p1);
            e0 = ie[0]; e1 = ie[1]; p0 = ip[0]; p1 = ip[1];
            lo = 1 + (deg - 1) * (it + 1);
            hi = lo + deg - 1 < np ? lo + deg - 1 : np;
        }
        out[k++] = T_SUB(w[sev], e0);
        out[k++] = T_SUB(w[sev + 1], e1);
        break;
    }
    default: break;
    }
    return k;
}

/* evaluates one gate's unfiltered constraints; returns the count */
static unsigned FN(gate_unfiltered)(const or_gate_t *g, const T *c, const T *w, const gl_t *pi_hash, T *out) {
    unsigned k = 0;
    switch (g->id) {
    case G_NOOP: break;
    case G_CONSTANT:
        for (uint64_t i = 0; i < g->p0; i++) out[k++] = T_SUB(c[i], w[i]);
        break;
    case G_PUBLIC_INPUT:
        for (int i = 0; i < 4; i++) out[k++] = T_SUB(w[i], T_FROM(pi_hash[i]));
        break;
    case G_BASE_SUM: {
        T acc = T_ZERO;
        for (uint64_t i = g->p0; i-- > 0;) acc = T_ADD(T_MUL(acc, T_FROM(2)), w[1 + i]);
        out[k++] = T_SUB(acc, w[0]);
        for (uint64_t i = 0; i < g->p0; i++) out[k++] = T_MUL(w[1 + i], T_SUB(w[1 + i], T_FROM(1)));
        break;
    }
    case G_ARITHMETIC:
        for (uint64_t i = 0; i < g->p0; i++) {
            T comp = T_ADD(T_MUL(T_MUL(w[4 * i], w[4 * i + 1]), c[0]), T_MUL(w[4 * i + 2], c[1]));
            out[k++] = T_SUB(w[4 * i + 3], comp);
        }
        break;
    case G_POSEIDON: k = FN(poseidon)(w, out); break;
    default: k = FN(gate_recursion)(g, c, w, out); break;
    }
    return k;
}

void FN(or_eval_gate_constraints)(const or_common_t *cd, const T *local_constants, const T *local_wires,
                                  const gl_t pi_hash[4], T *out) {
    T tmp[256];
    unsigned nsel = (unsigned)cd->num_groups;
    for (uint64_t j = 0; j < cd->num_gate_constraints; j++) out[j] = T_ZERO;
    for (uint64_t gi = 0; gi < cd->num_gates; gi++) {
        uint64_t si = cd->selector_indices[gi];
        T s = local_constants[si];
        T filter = T_FROM(1);
        for (uint64_t j = cd->groups[si][0]; j < cd->groups[si][1]; j++)
            if (j != gi) filter = T_MUL(filter, T_SUB(T_FROM(j), s));
        if (nsel > 1) filter = T_MUL(filter, T_SUB(T_FROM(UNUSED_SELECTOR), s));
        unsigned k = FN(gate_unfiltered)(&cd->gates[gi], local_constants + nsel + cd->num_lookup_selectors,
                                         local_wires, pi_hash, tmp);
        for (unsigned j = 0; j < k && j < cd->num_gate_constraints; j++) out[j] = T_ADD(out[j], T_MUL(filter, tmp[j]));
    }
}
#undef UNUSED_SELECTOR
