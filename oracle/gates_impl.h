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
    default: break;
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
