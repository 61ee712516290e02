"""Summary of tools/pmc_calib.sh: per (kernel, grid) mean counters, the clock
the GPU ran at (GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 / duration)
and VALU wave-instructions per SIMD per cycle at that clock.
Usage: python tools/pmc_calib_summary.py gpurun_out/calib_isa [gpurun_out/calib_kb ...]"""
import csv
import sys
from collections import defaultdict


def load(d):
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        x = disp[r["Dispatch_Id"]]
        x["kernel"] = r["Kernel_Name"].split("(")[0].replace("void ", "")
        x["grid"] = int(r["Grid_Size"])
        x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        x["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    return list(disp.values())


for d in sys.argv[1:]:
    print("==", d)
    g = defaultdict(list)
    for x in load(d):
        g[(x["kernel"], x["grid"])].append(x)
    for (k, gr), xs in sorted(g.items(), key=lambda kv: -sum(x["ms"] for x in kv[1]))[:14]:
        m = {c: sum(x.get(c, 0) for x in xs) / len(xs) for c in xs[0] if c.isupper() or c == "ms"}
        ms = m["ms"]
        gui = m.get("GRBM_GUI_ACTIVE", 0)
        # VALU instructions per SIMD per busy cycle: SQ_BUSY_CYCLES counts per SE/XCD, so
        # also report per-SIMD issue against wall time at the GRBM-derived clock
        clk = gui / 8 / (ms * 1e-3) / 1e9 if ms else 0
        ipc_wall = m["SQ_INSTS_VALU"] / 1024 / (ms * 1e-3 * clk * 1e9) if clk else 0
        print(f"{k[:34]:34s} grid {gr:8d} n={len(xs):2d} ms {ms:7.3f} GUI {gui:12.0f} clk~{clk:5.2f} GHz "
              f"VALU/SIMD/cycle {ipc_wall:6.3f} busy {m.get('SQ_BUSY_CYCLES', 0):12.0f} "
              f"act_valu/wavecyc {m.get('SQ_ACTIVE_INST_VALU', 0) / max(m.get('SQ_WAVE_CYCLES', 1), 1):5.3f} "
              f"wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / max(m.get('SQ_WAVE_CYCLES', 1), 1):5.3f}")
