"""Per-kernel mean of every counter in rocprofv3 --pmc output directories.
Usage: python tools/pmc_kernels.py <dir> [<dir> ...]   (each holds run_counter_collection.csv)"""
import csv
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {d}")
    for k, cs in acc.items():
        print(f"  {k[:40]:40s} " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
