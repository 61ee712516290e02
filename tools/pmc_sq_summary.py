"""Per-kernel SQ issue/stall summary of a rocprofv3 --pmc pass (tools/gpu_session.sh
pmc_sq / pmc_lds): for each (kernel, grid) the mean over its dispatches of the
duration, VALU instructions, VALU-issue utilisation against the guide's wave64
issue of one VALU instruction per 2 cycles per SIMD (MI355X_MICROARCH.md: 1024
SIMDs x 2.4 GHz / 2 = 1228.8 G wave-instructions/s), and the disjoint wave-time
split WAIT_ANY (parked at s_waitcnt/barrier) + WAIT_INST_ANY (issue stall) +
ACTIVE_INST_ANY = WAVE_CYCLES.  (PMC passes serialise dispatches, so durations
run a little long.)
Usage: python tools/pmc_sq_summary.py <pmc_dir> [out.json]"""
import csv
import json
import os
import sys
from collections import defaultdict
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from libhash import lib_sha16  # noqa: E402

PEAK = 1024 * 2.4e9 / 2


def main():
    d = sys.argv[1]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        x = disp[r["Dispatch_Id"]]
        x["kernel"], x["grid"], x["wg"] = name, int(r["Grid_Size"]), int(r["Workgroup_Size"])
        x["vgpr"] = int(r["VGPR_Count"])
        x[r["Counter_Name"]] = float(r["Counter_Value"])
        x["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    groups = defaultdict(list)
    for x in disp.values():
        groups[(x["kernel"], x["grid"], x["wg"])].append(x)
    out = []
    for (k, g, wg), xs in sorted(groups.items(), key=lambda kv: -sum(x["ms"] for x in kv[1])):
        m = {c: sum(x.get(c, 0) for x in xs) / len(xs) for c in xs[0] if c.startswith("SQ_") or c == "ms"}
        rec = {"kernel": k, "grid_lanes": g, "workgroup": wg, "vgpr": xs[0]["vgpr"], "dispatches": len(xs),
               "lib_sha16": lib_sha16(),
               "ms": m["ms"]}
        if "SQ_INSTS_VALU" in m:
            rec["valu_per_lane"] = m["SQ_INSTS_VALU"] * 64 / g
            # the widest dispatch of this (kernel, grid): e.g. the wires leaf hash
            # (135 columns, 17 permutations per leaf) among the zs / quotient ones
            rec["valu_per_lane_max"] = max(x["SQ_INSTS_VALU"] for x in xs) * 64 / g
            rec["valu_issue_util"] = m["SQ_INSTS_VALU"] / (m["ms"] * 1e-3 * PEAK)
        wc = m.get("SQ_WAVE_CYCLES")
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
            if wc and c in m:
                rec[c.lower() + "_frac"] = m[c] / wc
        for c in ("SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAVES"):
            if c in m:
                rec[c.lower()] = m[c]
        out.append(rec)
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    for r in out[:12]:
        print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()})


if __name__ == "__main__":
    main()
