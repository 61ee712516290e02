/*
 * oracle/merkle.h — plonky2 MerkleTree (hash/merkle_tree.rs, merkle_proofs.rs)
 * restated.  TEST INFRASTRUCTURE ONLY.  SURVEY.md A.3:
 *   leaf digest = hash_or_noop(leaf); node = two_to_one(L, R);
 *   cap = the 2^h roots of the contiguous subtrees;
 *   proof = log N - h siblings, bit i of the index selects (0: node is left).
 */
#ifndef QP_ORACLE_MERKLE_H
#define QP_ORACLE_MERKLE_H
#include "gl.h"
typedef struct {
    unsigned log_n, cap_height;
    size_t leaf_width;
    gl_t *leaves;   /* N x width, row-major (owned copy) */
    gl_t **levels;  /* levels[0] = N leaf digests, levels[k] = N>>k digests (4 felts each) */
} or_merkle_t;
or_merkle_t *or_merkle_build(const gl_t *leaves, unsigned log_n, size_t width, unsigned cap_height);
void or_merkle_free(or_merkle_t *t);
void or_merkle_cap(const or_merkle_t *t, gl_t *cap_out /* 2^h x 4 */);
void or_merkle_prove(const or_merkle_t *t, size_t index, gl_t *siblings_out /* (logN-h) x 4 */);
/* returns 1 if the path from leaf `index` reaches cap[index >> (depth)] */
int or_merkle_verify(const gl_t *leaf, size_t width, size_t index, const gl_t *cap, unsigned cap_height,
                     const gl_t *siblings, unsigned nsib);
#endif
