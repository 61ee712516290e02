/*
 * oracle/challenger.h — plonky2 Challenger (iop/challenger.rs) restated.
 * TEST INFRASTRUCTURE ONLY.  Duplex sponge over Poseidon, rate 8: observe
 * pushes to the input buffer (duplex at 8); get() duplexes if input pending or
 * output empty and pops the LAST of state[0..8].
 */
#ifndef QP_ORACLE_CHALLENGER_H
#define QP_ORACLE_CHALLENGER_H
#include "gl.h"
typedef struct {
    gl_t state[12];
    gl_t in[8]; unsigned nin;
    gl_t out[8]; unsigned nout;
} or_chal_t;
void or_chal_init(or_chal_t *c);
void or_chal_observe(or_chal_t *c, gl_t x);
void or_chal_observe_n(or_chal_t *c, const gl_t *x, size_t n);
void or_chal_observe_ext(or_chal_t *c, glx_t x);
gl_t or_chal_get(or_chal_t *c);
glx_t or_chal_get_ext(or_chal_t *c);
void or_chal_duplex(or_chal_t *c);
#endif
