"""Where a prover's time between two batches goes (voting, 6 provers x 171
proofs, as bench.py --circuit voting): per prove_inputs_array call, the time
inside the C call and the Python time around it, plus the library's stage
times.  Usage: python tools/voting_gaps.py [steps]"""
import ctypes
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
    from qp_wormhole._native import lib
    from bench import make_inputs
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    circ = qp_wormhole.Circuit.voting()
    B, NP = 1024, 6
    per = [B // NP + (1 if i < B % NP else 0) for i in range(NP)]
    first = [sum(per[:i]) for i in range(NP)]
    inputs = make_inputs(circ, 0, B)
    ps = [qp_wormhole.Prover(qp_wormhole.Context(0), circ, max_batch=per[i]) for i in range(NP)]
    cin = [ps[i].inputs_array(inputs[first[i]:first[i] + per[i]]) for i in range(NP)]
    rec = [[] for _ in range(NP)]

    def call(i):
        p = ps[i]
        t0 = time.perf_counter()
        out, lens = p._out_buffers(per[i])
        fn = lib().qp_prover_prove_voting_inputs
        t1 = time.perf_counter()
        rc = fn(p.h, ctypes.cast(cin[i], ctypes.c_void_p), per[i], out, p.proof_size, lens)
        t2 = time.perf_counter()
        assert rc == 0
        proofs = p._proofs(per[i])
        t3 = time.perf_counter()
        return proofs, (t0, t1, t2, t3)

    for i in range(NP):  # warm
        call(i)
    for p in ps:
        p.stage_times(reset=True)
    T0 = time.perf_counter()

    def run(i):
        for _ in range(steps):
            _, t = call(i)
            rec[i].append(t)

    th = [threading.Thread(target=run, args=(i,)) for i in range(NP)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    T1 = time.perf_counter()
    out = {"steps": steps, "proofs_per_s": B * steps / (T1 - T0), "ms_per_step": (T1 - T0) / steps * 1e3,
           "per_prover": []}
    for i in range(NP):
        r = rec[i]
        c_ms = [(t2 - t1) * 1e3 for (t0, t1, t2, t3) in r]
        py_ms = [((t1 - t0) + (t3 - t2)) * 1e3 for (t0, t1, t2, t3) in r]
        between = [(r[k + 1][0] - r[k][3]) * 1e3 for k in range(len(r) - 1)]
        out["per_prover"].append({"c_call_ms": [round(x, 2) for x in c_ms], "python_ms": [round(x, 2) for x in py_ms],
                                  "between_calls_ms": [round(x, 3) for x in between],
                                  "stage_ms_per_call": {k: round(v / steps, 2) for k, v in ps[i].stage_times().items()}})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
