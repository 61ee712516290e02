"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one counter per
run, tools/gpu_session.sh pmc_fetch / pmc_write) into per-launch HBM traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
of the bytes of a coalesced streaming read, so hbm_read = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for streaming stores.  Launches are keyed by kernel name
and grid size (the grid identifies the matrix: e.g. the wires LDE is
8 cosets x 135 columns x B proofs workgroups of 512 lanes).

Usage: python tools/pmc_summary.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from libhash import lib_sha16  # noqa: E402


def load(d, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[(name, int(r["Grid_Size"]), int(r["Workgroup_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = []
    for key in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        f = fetch.get(key, [])
        w = write.get(key, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rec = {"kernel": key[0], "grid_lanes": key[1], "wg": key[2], "launches": max(len(f), len(w)),
               "lib_sha16": lib_sha16(),
               "fetch_kib": fk, "write_kib": wk,
               "hbm_read_bytes": 2 * fk * 1024 if fk is not None else None,
               "hbm_write_bytes": wk * 1024 if wk is not None else None}
        if fk is not None and wk is not None:
            rec["hbm_bytes"] = rec["hbm_read_bytes"] + rec["hbm_write_bytes"]
        out.append(rec)
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    for r in out[:20]:
        hb = r.get("hbm_bytes")
        print(f'{r["kernel"][:28]:28s} grid {r["grid_lanes"]:10d} x{r["launches"]:3d} '
              f'read {r["hbm_read_bytes"] or 0:14.0f} write {r["hbm_write_bytes"] or 0:14.0f} '
              f'total {hb or 0:14.0f}')


if __name__ == "__main__":
    main()
