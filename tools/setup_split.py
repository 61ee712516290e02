"""Aggregation level prover setup on the GPU box: Context creation (stream +
twiddle tables) vs Prover construction (buffers, constants||sigmas
commitment) for the 2^13 aggregation circuit, a few times each.
Usage: python tools/setup_split.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))


def main():
    import torch
    torch.cuda.init()
    import qp_wormhole
    import qp_wormhole.aggregator as A
    base = A.WormholeProofAggregator.default(0)
    circ = A.aggregation_circuit(base.leaf_circuit_data.common, 2)
    res = {"context_ms": [], "prover_b1_ms": [], "prover_b16_ms": []}
    for _ in range(4):
        t0 = time.perf_counter()
        ctx = qp_wormhole.Context(0)
        t1 = time.perf_counter()
        p1 = qp_wormhole.Prover(ctx, circ, max_batch=1)
        t2 = time.perf_counter()
        p16 = qp_wormhole.Prover(ctx, circ, max_batch=16)
        t3 = time.perf_counter()
        res["context_ms"].append(round((t1 - t0) * 1e3, 2))
        res["prover_b1_ms"].append(round((t2 - t1) * 1e3, 2))
        res["prover_b16_ms"].append(round((t3 - t2) * 1e3, 2))
        p1.free()
        p16.free()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
