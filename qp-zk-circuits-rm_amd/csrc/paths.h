// paths.h — QPGPU_PATHS, the library's one runtime override: test hooks that
// force one of the production paths which the size heuristics pick for other
// shapes, so the GPU tests can prove the same bytes through each of them on a
// small batch ("key=value[,key=value...]", integer values; read per call, so a
// test switches it inside one process).  Nothing here selects an experimental
// form: every path named below runs by default for some circuit or batch.
//   merkle_row=0      Merkle levels one wave per node instead of 16 lanes per node
//   merkle_coop=N     cooperative Merkle forms up to N nodes over the batch (0 = never)
//   merkle_nbat=N     cooperative Merkle forms up to batch N
//   leaf_t=0          the any-width leaf hash instead of the fixed-width (135/20/16) one
//   fri_row=N         FRI-layer leaves in the row form up to N leaves over the batch
//   open_slices=N     openings split over at most N slices per column group
//   lde_few=N         coset LDE one workgroup per coset below N columns x proofs
//   qprefix=0         quotient permutation terms without the routed-wire prefix kernel
//   quotient_parts=1  the per-gate quotient launches for any gate list (the leaf
//                     circuits otherwise take the single-read kernel)
//   wit_mode=0|1      device witness: one workgroup per proof (0) / a launch per level (1)
//   wit_row=0         cooperative witness Poseidons one per wave instead of one per row
//   host_chain=N      host witness chains of depth >= N permutations (0 = none)
#pragma once
#include <stdlib.h>
#include <string.h>

namespace qpk {

// the value of `key` in QPGPU_PATHS, or dflt when absent
inline long path_opt(const char *key, long dflt) {
  const char *e = getenv("QPGPU_PATHS");
  if (!e) return dflt;
  const size_t kl = strlen(key);
  for (const char *p = e; *p;) {
    const char *end = strchr(p, ',');
    const size_t len = end ? (size_t)(end - p) : strlen(p);
    if (len > kl && !strncmp(p, key, kl) && p[kl] == '=') return strtol(p + kl + 1, nullptr, 10);
    p += len + (end ? 1 : 0);
  }
  return dflt;
}

}  // namespace qpk
