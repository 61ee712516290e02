"""Timeline of a rocprofv3 kernel trace cut to its trace markers (tools/agg_subtree.py,
bench.py): GPU busy fraction (union of kernel intervals) per time slice, the
kernel time by (kernel, grid) -- the aggregation levels' batches differ in grid
size, so this splits kernel time by level -- and the overall busy fraction.
Usage: python tools/agg_trace.py <kernel_trace.csv> <out.json> [slice_ms]"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_summary import MARKER, union_ms  # noqa: E402
from libhash import lib_sha16  # noqa: E402


def main():
    path, out = sys.argv[1], sys.argv[2]
    sl = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    rows = []
    for r in csv.DictReader(open(path)):
        full = r["Kernel_Name"]
        name = MARKER if MARKER in full else full.split("(")[0].replace("void ", "")
        grid = "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z")) if "Grid_Size_X" in r \
            else r.get("Grid_Size", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid))
    rows.sort()
    marks = [(a, b) for a, b, n, _ in rows if n == MARKER]
    lo, hi = (marks[0][1], marks[-1][0]) if len(marks) >= 2 else (rows[0][0], max(r[1] for r in rows))
    sel = [r for r in rows if r[0] >= lo and r[1] <= hi and r[2] != MARKER]
    window = (hi - lo) / 1e6
    busy = union_ms([(a, b) for a, b, _, _ in sel]) / (hi - lo)  # union_ms: same unit as its input
    nsl = int(window / sl) + 1
    slices = []
    for k in range(nsl):
        a0, b0 = lo + k * sl * 1e6, lo + (k + 1) * sl * 1e6
        iv = [(max(a, a0), min(b, b0)) for a, b, _, _ in sel if b > a0 and a < b0]
        slices.append(round(union_ms(iv) / min(sl * 1e6, hi - a0), 3) if iv else 0.0)
    per = defaultdict(lambda: [0.0, 0])
    for a, b, n, g in sel:
        per[(n, g)][0] += (b - a) / 1e6
        per[(n, g)][1] += 1
    total = sum(v[0] for v in per.values())
    rec = {"source": path, "lib_sha16": lib_sha16(), "window_ms": window, "kernel_ms": total, "gpu_busy_frac": busy,
           "slice_ms": sl, "busy_per_slice": slices,
           "kernels_by_grid": [{"kernel": n, "grid": g, "ms": round(v[0], 3), "launches": v[1],
                                "share": round(v[0] / total, 4)}
                               for (n, g), v in sorted(per.items(), key=lambda kv: -kv[1][0])][:60]}
    json.dump(rec, open(out, "w"), indent=1)
    print({k: rec[k] for k in ("window_ms", "kernel_ms", "gpu_busy_frac")})
    print("busy per", sl, "ms:", slices)


if __name__ == "__main__":
    main()
