"""Soak check: many Wormhole (or voting) batches through the production path
(three provers -- six for voting -- on their own streams and threads, as bench.py), each step's inputs a fresh
seeded set, and every proof checked by the CPU oracle verifier on a host
thread pool.  A rare kernel or scheduling race would show up as a proof that
does not verify.  Usage: python tools/soak.py [steps] [batch] [wormhole|voting]"""
import concurrent.futures
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    import qp_wormhole
    from bench import make_inputs
    from oracle_lib import lib as olib
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    voting = len(sys.argv) > 3 and sys.argv[3] == "voting"
    NP = 6 if voting else 3  # as bench.py
    circ = qp_wormhole.Circuit.voting() if voting else qp_wormhole.Circuit.wormhole(zero_knowledge=False)
    per = [B // NP + (1 if i < B % NP else 0) for i in range(NP)]
    provers = [qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=per[i]) for i in range(NP)]
    vd = provers[0].verifier_data()
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=16)
    futs = []
    bad = []
    t0 = time.perf_counter()
    for s in range(steps):
        inputs = make_inputs(circ, 100000 + s * B, B)
        first = [sum(per[:i]) for i in range(NP)]
        outs = [None] * NP

        def run(i):
            outs[i] = provers[i].prove_inputs(inputs[first[i]:first[i] + per[i]])

        th = [threading.Thread(target=run, args=(i,)) for i in range(NP)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        proofs = [p for o in outs for p in o]
        assert len(proofs) == B
        for k, p in enumerate(proofs):
            futs.append(((s, k), pool.submit(lambda p=p: olib().ora_verify(vd, len(vd), p, len(p)))))
        print(f"step {s}: {B} proofs, {time.perf_counter() - t0:.1f} s", flush=True)
    for key, f in futs:
        if f.result() != 0:
            bad.append(key)
    print(json.dumps({"circuit": circ.kind, "steps": steps, "batch": B, "proofs": steps * B, "verified": steps * B - len(bad),
                      "failed": bad[:20], "seconds": time.perf_counter() - t0}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
