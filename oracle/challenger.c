/* oracle/challenger.c — see challenger.h.  TEST INFRASTRUCTURE ONLY. */
#include "challenger.h"
#include "poseidon.h"
#include <string.h>

void or_chal_init(or_chal_t *c) { memset(c, 0, sizeof(*c)); }

void or_chal_duplex(or_chal_t *c) {
    for (unsigned i = 0; i < c->nin; i++) c->state[i] = c->in[i];
    c->nin = 0;
    ps_permute(c->state);
    memcpy(c->out, c->state, 8 * sizeof(gl_t));
    c->nout = 8;
}

void or_chal_observe(or_chal_t *c, gl_t x) {
    c->nout = 0;
    c->in[c->nin++] = x;
    if (c->nin == 8) or_chal_duplex(c);
}

void or_chal_observe_n(or_chal_t *c, const gl_t *x, size_t n) {
    for (size_t i = 0; i < n; i++) or_chal_observe(c, x[i]);
}

void or_chal_observe_ext(or_chal_t *c, glx_t x) { or_chal_observe(c, x.c0); or_chal_observe(c, x.c1); }

gl_t or_chal_get(or_chal_t *c) {
    if (c->nin || !c->nout) or_chal_duplex(c);
    return c->out[--c->nout];
}

glx_t or_chal_get_ext(or_chal_t *c) {
    gl_t a = or_chal_get(c);
    gl_t b = or_chal_get(c);
    return glx(a, b);
}
