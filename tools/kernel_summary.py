"""Kernel-time summary of a rocprofv3 --kernel-trace CSV of a bench run, for the
bench JSON's measured fields (bench.py reads the JSON this writes):
  kernels:          per kernel name: total ms, launches, share of all kernel time
  gpu_busy_frac:    |union of kernel intervals| / window: the fraction of the
                    window in which some kernel ran (with concurrent provers,
                    kernels of different streams overlap)
  leaf_hash_share:  the leaf-hash kernels' share of all kernel time (k_leaf_hash, k_leaf_hash_t<NC>)
The window is the bench's timed region when the trace holds bench.py's two
trace markers (at::cuda spin kernels launched just outside each end of the
timed steps): kernels that start after the first marker ends and end before the
second starts.  Without markers it is the whole trace (setup, warm-up and the
aggregation pass included), which understates how busy the timed steps keep
the GPU.
Usage: python tools/kernel_summary.py run_kernel_trace.csv out.json [label]"""
import csv
import json
import os
import sys
from collections import defaultdict
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from libhash import lib_sha16  # noqa: E402

MARKER = "spin_kernel"


def union_ms(iv):
    busy, cur_a, cur_b = 0, None, None
    for a, b in sorted(iv):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    return busy


def main():
    path, out = sys.argv[1], sys.argv[2]
    rows = []
    for r in csv.DictReader(open(path)):
        full = r["Kernel_Name"]
        name = MARKER if MARKER in full else full.split("(")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    marks = [(a, b) for a, b, n in rows if MARKER in n]
    if len(marks) >= 2:
        lo, hi = marks[0][1], marks[-1][0]
        scope = "timed region (between bench.py trace markers)"
    else:
        lo, hi = rows[0][0], max(b for _, b, _ in rows)
        scope = "whole trace (no trace markers)"
    sel = [(a, b, n) for a, b, n in rows if a >= lo and b <= hi and MARKER not in n]
    per = defaultdict(lambda: [0.0, 0])
    for a, b, n in sel:
        per[n][0] += (b - a) / 1e6
        per[n][1] += 1
    window = hi - lo
    total = sum(v[0] for v in per.values())
    rec = {"source": path, "label": sys.argv[3] if len(sys.argv) > 3 else "", "scope": scope, "lib_sha16": lib_sha16(),
           "window_ms": window / 1e6, "kernel_ms": total,
           "gpu_busy_frac": union_ms([(a, b) for a, b, _ in sel]) / window,
           # k_leaf_hash and its compile-time column-count forms k_leaf_hash_t<NC>
           "leaf_hash_share": sum(v[0] for k, v in per.items() if k.startswith("qpk::k_leaf_hash")) / total,
           "kernels": {k: {"ms": v[0], "launches": v[1], "share": v[0] / total}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    json.dump(rec, open(out, "w"), indent=1)
    print({k: rec[k] for k in ("scope", "window_ms", "kernel_ms", "gpu_busy_frac", "leaf_hash_share")})


if __name__ == "__main__":
    main()
