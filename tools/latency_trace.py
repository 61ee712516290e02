"""One Wormhole proof at a time (BASELINE configs[1]): K timed single-proof
calls between the bench's trace markers, for a rocprofv3 kernel trace of
where one proof's latency goes (kernel time vs host gaps).
Usage: python tools/latency_trace.py [K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    import qp_wormhole
    from bench import make_inputs, trace_marker
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    circ = qp_wormhole.Circuit.wormhole(zero_knowledge=False)
    p = qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=1)
    arr = p.inputs_array(make_inputs(circ, 0, 1))
    for _ in range(3):
        p.prove_inputs_array(arr, 1)
    p.stage_times(reset=True)
    torch.cuda.synchronize()
    trace_marker(torch)
    torch.cuda.synchronize()
    ts = []
    for _ in range(K):
        t0 = time.perf_counter()
        p.prove_inputs_array(arr, 1)
        ts.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    trace_marker(torch)
    torch.cuda.synchronize()
    print(json.dumps({"ms_per_proof": ts, "stage_ms_per_proof": {k: round(v / K, 3) for k, v in p.stage_times().items()}}))


if __name__ == "__main__":
    main()
