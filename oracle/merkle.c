/* oracle/merkle.c — see merkle.h.  TEST INFRASTRUCTURE ONLY. */
#include "merkle.h"
#include "poseidon.h"
#include <stdlib.h>
#include <string.h>

or_merkle_t *or_merkle_build(const gl_t *leaves, unsigned log_n, size_t width, unsigned cap_height) {
    if (cap_height > log_n) return NULL;
    size_t n = (size_t)1 << log_n;
    or_merkle_t *t = calloc(1, sizeof(*t));
    t->log_n = log_n; t->cap_height = cap_height; t->leaf_width = width;
    t->leaves = malloc(n * width * sizeof(gl_t) + 8);
    memcpy(t->leaves, leaves, n * width * sizeof(gl_t));
    t->levels = calloc(log_n + 1, sizeof(gl_t *));
    t->levels[0] = malloc(n * 4 * sizeof(gl_t));
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) ps_hash_or_noop(leaves + i * width, width, t->levels[0] + 4 * i);
    for (unsigned k = 1; k <= log_n - cap_height; k++) {
        size_t m = n >> k;
        t->levels[k] = malloc(m * 4 * sizeof(gl_t));
#pragma omp parallel for schedule(static) if (m > 1024)
        for (size_t i = 0; i < m; i++)
            ps_two_to_one(t->levels[k - 1] + 8 * i, t->levels[k - 1] + 8 * i + 4, t->levels[k] + 4 * i);
    }
    return t;
}

void or_merkle_free(or_merkle_t *t) {
    if (!t) return;
    for (unsigned k = 0; k <= t->log_n; k++) free(t->levels[k]);
    free(t->levels); free(t->leaves); free(t);
}

void or_merkle_cap(const or_merkle_t *t, gl_t *cap_out) {
    unsigned d = t->log_n - t->cap_height;
    memcpy(cap_out, t->levels[d], ((size_t)4 << t->cap_height) * sizeof(gl_t));
}

void or_merkle_prove(const or_merkle_t *t, size_t index, gl_t *sib) {
    unsigned d = t->log_n - t->cap_height;
    for (unsigned k = 0; k < d; k++) {
        size_t s = (index >> k) ^ 1;
        memcpy(sib + 4 * k, t->levels[k] + 4 * s, 32);
    }
}

int or_merkle_verify(const gl_t *leaf, size_t width, size_t index, const gl_t *cap, unsigned cap_height,
                     const gl_t *sib, unsigned nsib) {
    gl_t cur[4];
    ps_hash_or_noop(leaf, width, cur);
    for (unsigned k = 0; k < nsib; k++) {
        gl_t o[4];
        if ((index >> k) & 1) ps_two_to_one(sib + 4 * k, cur, o);
        else ps_two_to_one(cur, sib + 4 * k, o);
        memcpy(cur, o, 32);
    }
    size_t ci = index >> nsib;
    if (ci >= ((size_t)1 << cap_height)) return 0;
    return memcmp(cur, cap + 4 * ci, 32) == 0;
}
