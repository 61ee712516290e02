"""Where an uncached aggregation call's time goes (the reference's aggregator
bench shapes build their circuits inside every aggregate()): per level, the
aggregation circuit build on the host, the level prover's setup (contexts,
device preprocessing) and the prove itself.  Usage:
python tools/agg_first_call.py [k depth ...]   (default: 2 1  2 5  7 2)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))


def main():
    import torch
    torch.cuda.init()
    import qp_wormhole.aggregator as A
    from qp_wormhole.circuits import Circuit
    args = [int(x) for x in sys.argv[1:]] or [2, 1, 2, 5, 7, 2]
    base = A.WormholeProofAggregator.default(0)
    out = []
    for k, depth in zip(args[0::2], args[1::2]):
        A._levels.clear()
        A._circuits.clear()
        leaves = [base.dummy_proof()] * (k ** depth)
        common = base.leaf_circuit_data.common
        vo = base.leaf_circuit_data.verifier_only
        levels = []
        proofs = leaves
        t_all = time.perf_counter()
        for lvl in range(depth):
            t0 = time.perf_counter()
            circ = A.aggregation_circuit(common, k)
            t1 = time.perf_counter()
            nch = len(proofs) // k
            lp = A._level_prover(common, k, 0, max(1, min(nch, 32)))
            t2 = time.perf_counter()
            proofs = lp.prove_chunks([proofs[i * k:(i + 1) * k] for i in range(nch)], vo)
            t3 = time.perf_counter()
            levels.append({"level": lvl + 1, "degree_bits": circ.degree_bits, "chunks": nch,
                           "circuit_build_ms": (t1 - t0) * 1e3, "prover_setup_ms": (t2 - t1) * 1e3,
                           "prove_ms": (t3 - t2) * 1e3})
            common, vo = proofs[0].circuit_data.common, proofs[0].circuit_data.verifier_only
            proofs = [p.proof for p in proofs]
        out.append({"k": k, "depth": depth, "total_ms": (time.perf_counter() - t_all) * 1e3, "levels": levels})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
