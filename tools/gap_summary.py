"""Idle time between kernels of a rocprofv3 --kernel-trace CSV (development
tool): kernels sorted by start; every gap above a threshold between the end of
the busy interval so far and the next kernel's start is an idle period, listed
with the kernels on either side (a host sync or transfer sits there).  Prints
the busy fraction of the window [first start, last end] and the gaps grouped by
their (before, after) kernel pair.
python tools/gap_summary.py run_kernel_trace.csv [threshold_us] [skip_first_ms]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    ks = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ks.sort()
    t0 = ks[0][0] + int(skip * 1e6)
    ks = [k for k in ks if k[0] >= t0]
    end = ks[0][1]
    busy = 0
    cur_a, cur_b = ks[0][0], ks[0][1]
    gaps = defaultdict(lambda: [0, 0.0])
    prev = ks[0][2]
    for a, b, name in ks[1:]:
        if a > cur_b:
            busy += cur_b - cur_a
            g = (a - cur_b) / 1e3
            if g >= thr:
                e = gaps[(prev, name)]
                e[0] += 1
                e[1] += g
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
        if b >= end:
            end = b
            prev = name
    busy += cur_b - cur_a
    win = (end - ks[0][0]) / 1e6
    print(f"{path}: {len(ks)} kernels, window {win:.2f} ms, busy {busy / 1e6:.2f} ms ({busy / 1e6 / win:.3f})")
    tot = sum(v[1] for v in gaps.values())
    print(f"gaps >= {thr} us: {sum(v[0] for v in gaps.values())}, {tot / 1e3:.2f} ms")
    for (a, b), (n, g) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {g / 1e3:8.2f} ms  n={n:5d}  {a[:36]:36s} -> {b[:36]}")


if __name__ == "__main__":
    main()
