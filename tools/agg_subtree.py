"""Per-GPU subtree aggregation timing (configs[3]'s per-GPU share; development
tool): `leaves` leaf proofs (the reference's own two, alternating) -> one root
through aggregate_to_tree (branching 2), one untimed pass that builds and
caches the level circuits, then `reps` timed passes with per-level seconds and
the device stage times of the level provers.  Variants come from the
environment (QP_AGG_PROVERS, QP_AGG_SPLIT, QP_AGG_WITNESS, QPGPU_PATHS).
python tools/agg_subtree.py [leaves] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qp-zk-circuits-rm_amd"), os.path.join(ROOT, "tests")]


def main():
    # torch first (as bench.py): its device context exists before the library's,
    # for the trace-marker spin kernels below
    import torch
    torch.zeros(1, device="cuda").add_(1)
    torch.cuda.synchronize()
    import qp_wormhole
    from qp_wormhole import aggregator as A
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden, lib as olib
    from test_oracle_golden import current_common_bytes
    nl = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    vo = vd[:len(vd) - len(cb)]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    leaves = [fx[i % 2] for i in range(nl)]
    depth = nl.bit_length() - 1
    cfg = A.TreeAggregationConfig.new(2, depth)
    levels = []
    orig = A.aggregate_level

    import resource

    def cpu():
        r = resource.getrusage(resource.RUSAGE_SELF)
        return r.ru_utime + r.ru_stime

    def timed_level(proofs, *a, **k):
        t, c = time.perf_counter(), cpu()
        r = orig(proofs, *a, **k)
        levels.append((len(proofs) // 2, time.perf_counter() - t, cpu() - c))
        return r
    A.aggregate_level = timed_level
    t = time.perf_counter()
    A.aggregate_to_tree(leaves, cb, vo, cfg)
    warm = time.perf_counter() - t
    for lp in A._levels.values():
        for p in lp.provers:
            p.stage_times(reset=True)
    def throttle():
        try:
            d = dict(l.split() for l in open("/sys/fs/cgroup/cpu.stat"))
            return int(d.get("nr_throttled", 0)), int(d.get("throttled_usec", 0))
        except (OSError, ValueError):
            return None
    th0 = throttle()
    res = []
    # trace markers (bench.py's): a spin kernel just outside each end of the
    # timed passes, so tools/kernel_summary.py and tools/agg_trace.py cut a
    # rocprofv3 kernel trace to them
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    for _ in range(reps):
        levels.clear()
        t = time.perf_counter()
        root = A.aggregate_to_tree(leaves, cb, vo, cfg)
        # per level: proofs, wall ms, process CPU ms (all threads; the box gives
        # this job OMP_NUM_THREADS cores)
        res.append({"seconds": time.perf_counter() - t,
                    "levels": [(n, round(s * 1e3, 1), round(c * 1e3, 1)) for n, s, c in levels]})
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    # per level circuit (insertion order = level order): degree, proofs per
    # level prover batch and its device stage times per run
    per_level = []
    for lp in A._levels.values():
        st = {}
        for p in lp.provers:
            for k, v in p.stage_times().items():
                st[k] = round(st.get(k, 0.0) + v / reps, 2)
        per_level.append({"degree_bits": lp.circuit.degree_bits, "npis": lp.circuit.num_public_inputs,
                          "max_batch": lp.max_batch, "provers": len(lp.provers), "stage_ms": st})
    stages = {}
    for lp in A._levels.values():
        for p in lp.provers:
            for k, v in p.stage_times().items():
                stages[k] = stages.get(k, 0.0) + v / reps
    rvd, rp = root.circuit_data.verifier_data(), root.proof.to_bytes()
    env = {k: os.environ.get(k) for k in ("QP_AGG_PROVERS", "QP_AGG_SPLIT", "QP_AGG_WITNESS", "QPGPU_PATHS",
                                        "QP_AGG_THREADS", "OMP_NUM_THREADS")}
    th1 = throttle()
    cg = None
    if th0 and th1:
        cg = {"nr_throttled": th1[0] - th0[0], "throttled_ms": (th1[1] - th0[1]) / 1e3}
    print(json.dumps({"leaves": nl, "env": env, "warm_s": round(warm, 2), "runs": res, "cgroup_throttling": cg,
                      "stage_ms_per_run_all_provers": {k: round(v, 1) for k, v in stages.items()},
                      "per_level": per_level,
                      "root_verified": olib().ora_verify(rvd, len(rvd), rp, len(rp)) == 0}), flush=True)


if __name__ == "__main__":
    main()
