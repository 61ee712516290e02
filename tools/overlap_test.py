"""Throughput of one prover over B proofs vs P provers (own context/stream,
own host thread) over B/P proofs each, concurrently.
Usage: python tools/overlap_test.py [B] [P] [steps]"""
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))
sys.path.insert(0, ROOT)
import qp_wormhole  # noqa: E402
from bench import make_witnesses  # noqa: E402


def run(circuit, d_wires, pis, B, P, steps):
    per = B // P
    provers = [qp_wormhole.Prover(qp_wormhole.Context(0), circuit, max_batch=per) for _ in range(P)]
    stride = d_wires[0].numel() * 8

    def one(i):
        provers[i].prove_wires_dev(d_wires.data_ptr() + i * per * stride, pis[i * per:(i + 1) * per], per)

    def step():
        th = [threading.Thread(target=one, args=(i,)) for i in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    for p in provers:
        p.free()
    return B * steps / dt


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    circuit = qp_wormhole.Circuit.wormhole()
    wires, pis = make_witnesses(circuit, 0, B)
    d_wires = torch.from_numpy(wires.view(np.int64)).to("cuda:0")
    for p in (1, P, 4):
        print(f"B={B} provers={p}: {run(circuit, d_wires, pis, B, p, steps):.1f} proofs/s", flush=True)


if __name__ == "__main__":
    main()
