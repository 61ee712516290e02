/* oracle/gates.c — instantiates gates_impl.h for F and F_ext.  TEST INFRASTRUCTURE ONLY. */
#include "plonk.h"
#include "poseidon.h"

unsigned or_gate_num_constraints(const or_gate_t *g) {
    switch (g->id) {
    case G_NOOP: return 0;
    case G_CONSTANT: return (unsigned)g->p0;
    case G_PUBLIC_INPUT: return 4;
    case G_BASE_SUM: return (unsigned)g->p0 + 1;
    case G_ARITHMETIC: return (unsigned)g->p0;
    case G_POSEIDON: return 123;
    case G_ARITH_EXT: return 2 * (unsigned)g->p0;
    case G_MUL_EXT: return 2 * (unsigned)g->p0;
    case G_REDUCING: case G_REDUCING_EXT: return 2 * (unsigned)g->p0;
    case G_EXPONENTIATION: return (unsigned)g->p0 + 1;
    case G_POSEIDON_MDS: return 24;
    case G_RANDOM_ACCESS: return (unsigned)((g->p0 + 2) * g->p1 + g->p2);
    case G_COSET_INTERP: return 4 + 4 * (unsigned)(((1u << g->p0) - 2) / (g->p1 - 1));
    default: return 0;
    }
}

/* base field instantiation */
#define T gl_t
#define T_ADD gl_add
#define T_SUB gl_sub
#define T_MUL gl_mul
#define T_FROM(x) gl_reduce((uint64_t)(x))
#define T_ZERO ((gl_t)0)
#define FN(n) base_##n
#include "gates_impl.h"
#undef T
#undef T_ADD
#undef T_SUB
#undef T_MUL
#undef T_FROM
#undef T_ZERO
#undef FN

/* extension instantiation */
static inline glx_t glx_from_u64(uint64_t x) { return glx(gl_reduce(x), 0); }
#define T glx_t
#define T_ADD glx_add
#define T_SUB glx_sub
#define T_MUL glx_mul
#define T_FROM(x) glx_from_u64((uint64_t)(x))
#define T_ZERO glx(0, 0)
#define FN(n) ext_##n
#include "gates_impl.h"

void or_eval_gate_constraints_ext(const or_common_t *c, const glx_t *lc, const glx_t *lw, const gl_t pi[4], glx_t *out) {
    ext_or_eval_gate_constraints(c, lc, lw, pi, out);
}
void or_eval_gate_constraints_base(const or_common_t *c, const gl_t *lc, const gl_t *lw, const gl_t pi[4], gl_t *out) {
    base_or_eval_gate_constraints(c, lc, lw, pi, out);
}

/* one gate's unfiltered constraints in the base field (tests of the gate formulas) */
unsigned or_gate_eval_base(const or_gate_t *g, const gl_t *c, const gl_t *w, const gl_t pi[4], gl_t *out) {
    return base_gate_unfiltered(g, c, w, pi, out);
}
