"""Aggregation level breakdown on the GPU (development tool): host witness
generation (threaded) vs batched GPU proving of aggregate_chunk circuits over
the reference's own two leaf proofs.  python tools/agg_bench.py [chunks] [batch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qp-zk-circuits-rm_amd"), os.path.join(ROOT, "tests")]


def main():
    import qp_wormhole
    from qp_wormhole.aggregator import _witness_pool
    from current_circuit_vd import current_circuit_verifier_data
    from oracle_lib import golden
    from test_oracle_golden import current_common_bytes
    nch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    cb = current_common_bytes()
    vd = current_circuit_verifier_data(cb)[0]
    vo = vd[:len(vd) - len(cb)]
    leaves = [golden("dummy_proof.bin"), golden("dummy_proof_zk.bin")]
    circ = qp_wormhole.Circuit.aggregation(cb, 2)
    ctx = qp_wormhole.Context(0)
    pr = qp_wormhole.Prover(ctx, circ, max_batch=mb)
    pool = _witness_pool()
    ws = list(pool.map(lambda _: circ.commit_proofs(vo, leaves), range(mb)))
    pr.prove_witnesses(ws)
    for w in ws:
        w.free()
    t = time.perf_counter()
    ws = list(pool.map(lambda _: circ.commit_proofs(vo, leaves), range(nch)))
    tw = time.perf_counter() - t
    pr.stage_times(reset=True)
    pr.set_timing(True)
    pr.kernel_stats(reset=True)
    t = time.perf_counter()
    for i in range(0, nch, mb):
        pr.prove_witnesses(ws[i:i + mb])
    tp = time.perf_counter() - t
    print(f"threads {pool._max_workers}: {nch} witnesses {tw * 1e3:.1f} ms ({tw * 1e3 / nch:.2f} ms each); "
          f"prove {tp * 1e3:.1f} ms ({tp * 1e3 / nch:.2f} ms each, batch {mb})")
    print("stages (ms):", {k: round(v, 1) for k, v in pr.stage_times().items() if isinstance(v, float)})
    print("kernels:", pr.kernel_stats())


if __name__ == "__main__":
    main()
