"""Latency of small aggregation batches (development tool; the top levels of a
configs[3] subtree hold 16, 8, 4, 2 and 1 proofs): one level-1 aggregation
circuit (branching 2 over the reference's own leaf proofs), one device prover
per batch size, `reps` timed prove_aggregation calls per size with the
prover's host stage times (qp_prover_stage_times) averaged per call.
Run under `rocprofv3 --kernel-trace` and feed the CSV to tools/gap_summary.py
to see where the GPU idles between launches.
python tools/agg_latency.py [sizes, comma-separated] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qp-zk-circuits-rm_amd"), os.path.join(ROOT, "tests")]


def main():
    import qp_wormhole
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden
    from test_oracle_golden import current_common_bytes
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8,16").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    vo = vd[:len(vd) - len(cb)]
    fx = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    ctx = qp_wormhole.Context(0)
    out = {"circuit": {"degree_bits": circ.degree_bits, "witness_levels": circ.witness_levels}, "sizes": {}}
    for b in sizes:
        p = qp_wormhole.Prover(ctx, circ, max_batch=b)
        chunks = [[fx[i % 2], fx[(i + 1) % 2]] for i in range(b)]
        p.prove_aggregation(vo, chunks)  # warm-up
        p.stage_times(reset=True)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            p.prove_aggregation(vo, chunks)
            ts.append((time.perf_counter() - t) * 1e3)
        st = {k: round(v / reps, 3) for k, v in p.stage_times().items()}
        ts.sort()
        out["sizes"][b] = {"ms_median": round(ts[len(ts) // 2], 2), "ms_min": round(ts[0], 2),
                           "ms_per_proof": round(ts[len(ts) // 2] / b, 2), "stage_ms_per_call": st}
        print(json.dumps({b: out["sizes"][b]}), flush=True)
        p.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
