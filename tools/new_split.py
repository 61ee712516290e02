"""WormholeProver::new split on the GPU box: the circuit build on the host
(Circuit.wormhole, zk config) and the device prover setup (Prover: buffers,
constants||sigmas commitment), six times.  Usage: python tools/new_split.py"""
import sys, time, json
sys.path.insert(0, "qp-zk-circuits-rm_amd")
import torch
torch.cuda.init()
import qp_wormhole
ctx = qp_wormhole.Context(0)
res = []
for i in range(6):
    t0 = time.perf_counter()
    c = qp_wormhole.Circuit.wormhole(zero_knowledge=True)
    t1 = time.perf_counter()
    p = qp_wormhole.Prover(ctx, c, max_batch=1)
    t2 = time.perf_counter()
    res.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
    p.free()
print(json.dumps({"circuit_build_ms": [round(a, 2) for a, b in res], "prover_new_ms": [round(b, 2) for a, b in res]}))
