"""Device witness generation of the Wormhole circuit by batch size, in its two
forms (one workgroup per proof / one launch per dependency level, the
QPGPU_PATHS wit_mode hook, read per call): the witness stage and the whole
prove call, per batch.  Usage: python tools/wit_modes.py [batches...]"""
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
    from bench import make_inputs
    batches = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 16, 32, 86]
    circ = qp_wormhole.Circuit.wormhole(zero_knowledge=False)
    ctx = qp_wormhole.Context(0)
    out = []
    for nb in batches:
        p = qp_wormhole.Prover(ctx, circ, max_batch=nb)
        arr = p.inputs_array(make_inputs(circ, 0, nb))
        row = {"batch": nb}
        for mode in (0, 1, 0, 1):
            os.environ["QPGPU_PATHS"] = f"wit_mode={mode}"
            p.prove_inputs_array(arr, nb)  # warm
            p.stage_times(reset=True)
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                p.prove_inputs_array(arr, nb)
            dt = (time.perf_counter() - t0) / reps * 1e3
            st = p.stage_times()
            key = "levels" if mode else "workgroup_per_proof"
            row.setdefault(key, []).append({"call_ms": round(dt, 3), "witness_ms": round(st["witness_gen"] / reps, 3)})
        os.environ.pop("QPGPU_PATHS", None)
        p.free()
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
