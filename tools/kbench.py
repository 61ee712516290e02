"""Kernel micro-bench for the commit path (iNTT + LDE + leaf hash + tree) with
device-resident inputs.  Usage: python tools/kbench.py [nbat] [iters]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))
import qp_wormhole  # noqa: E402
from qp_wormhole import _native  # noqa: E402

P = 0xFFFFFFFF00000001


def main():
    nbat = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ctx = qp_wormhole.Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    L = _native.lib()
    for npolys in (135, 20):
        n = 1 << 13
        x = torch.randint(0, 2**62, (nbat, npolys, n), dtype=torch.int64, device="cuda")
        cap = torch.zeros((nbat, 16, 4), dtype=torch.int64, device="cuda")
        h = ctypes.c_void_p()
        for it in range(iters + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rc = L.qp_commit_values_dev(ctx.h, x.data_ptr(), nbat, npolys, 13, 3, 4, cap.data_ptr(), ctypes.byref(h))
            assert rc == 0, L.qp_ctx_last_error(ctx.h)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            if it:
                print(f"commit npolys={npolys} nbat={nbat}: {dt*1e3:.2f} ms  ({dt/nbat*1e3:.3f} ms/batch)", flush=True)
        L.qp_batch_free(h)


if __name__ == "__main__":
    main()
