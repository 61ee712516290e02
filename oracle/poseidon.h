/*
 * oracle/poseidon.h — Poseidon-Goldilocks (width 12, rate 8, x^7, 8 full + 22
 * partial rounds) and the plonky2 hashing modes.  TEST INFRASTRUCTURE ONLY.
 *
 * Restates qp-plonky2 1.1.1 hash/poseidon.rs + hash/poseidon_goldilocks.rs +
 * hash/hashing.rs (not vendored; SURVEY.md A.2, constants Appendix C).
 * Pinned by the reference's Poseidon KATs:
 *   wormhole/tests/src/prover/prover_tests.rs:21-45 (nullifier bytes),
 *   wormhole/tests/src/circuit/unspendable_account_tests.rs:12-28 (5 pairs),
 *   wormhole/tests/test-helpers/src/lib.rs:68-80 (storage-proof chain).
 */
#ifndef QP_ORACLE_POSEIDON_H
#define QP_ORACLE_POSEIDON_H
#include "gl.h"

#define PS_WIDTH 12
#define PS_RATE 8
#define PS_ROUNDS 30
#define PS_HALF_FULL 4
#define PS_PARTIAL 22

extern const uint64_t PS_RC[PS_ROUNDS * PS_WIDTH];
extern const uint64_t PS_MDS_CIRC[PS_WIDTH];
extern const uint64_t PS_MDS_DIAG[PS_WIDTH];

void ps_permute(gl_t s[PS_WIDTH]);
/* upstream PoseidonHash::hash_no_pad: state=0; per 8-chunk overwrite prefix; permute */
void ps_hash_no_pad(const gl_t *in, size_t n, gl_t out[4]);
/* hash_or_noop: <=4 elements zero-padded, else hash_no_pad */
void ps_hash_or_noop(const gl_t *in, size_t n, gl_t out[4]);
/* two_to_one(a,b) = perm(a||b||0^4)[0..4] */
void ps_two_to_one(const gl_t a[4], const gl_t b[4], gl_t out[4]);
/* hash_pad (used for the circuit digest's domain separator) */
void ps_hash_pad(const gl_t *in, size_t n, gl_t out[4]);
#endif
