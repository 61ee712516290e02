"""Per-kernel duration summary of rocprofv3 --kernel-trace CSV files.
Usage: python tools/trace_summary.py run_kernel_trace.csv [...]"""
import csv
import sys
from collections import defaultdict


def main():
    for path in sys.argv[1:]:
        agg = defaultdict(list)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
            agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        print(path)
        for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            if sum(v) < 0.05:
                continue
            v = sorted(v)
            print(f"  {name[:34]:34s} grid {grid:>10s} n={len(v):4d} total {sum(v):9.3f} ms  "
                  f"median {v[len(v) // 2]:8.3f}  min {v[0]:8.3f}")


if __name__ == "__main__":
    main()
