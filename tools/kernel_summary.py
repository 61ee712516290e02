"""Kernel-time summary of a rocprofv3 --kernel-trace CSV of a bench run, for the
bench JSON's measured fields (bench.py reads the JSON this writes):
  kernels:          per kernel name: total ms, launches, share of all kernel time
  gpu_busy_frac:    |union of kernel intervals| / (last end - first start): the
                    fraction of the traced window in which some kernel ran (with
                    concurrent provers, kernels of different streams overlap)
  leaf_hash_share:  k_leaf_hash's share of all kernel time
Usage: python tools/kernel_summary.py run_kernel_trace.csv out.json [label]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    iv = []
    per = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((a, b))
        per[name][0] += (b - a) / 1e6
        per[name][1] += 1
    iv.sort()
    busy, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    busy += cur_b - cur_a
    window = iv[-1][1] - iv[0][0]
    total = sum(v[0] for v in per.values())
    rec = {"source": path, "label": sys.argv[3] if len(sys.argv) > 3 else "",
           "window_ms": window / 1e6, "kernel_ms": total, "gpu_busy_frac": busy / window,
           "leaf_hash_share": per.get("qpk::k_leaf_hash", [0])[0] / total,
           "kernels": {k: {"ms": v[0], "launches": v[1], "share": v[0] / total}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    json.dump(rec, open(out, "w"), indent=1)
    print({k: rec[k] for k in ("window_ms", "kernel_ms", "gpu_busy_frac", "leaf_hash_share")})


if __name__ == "__main__":
    main()
