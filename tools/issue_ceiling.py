"""VALU issue ceiling of k_leaf_hash from measured per-class costs.

Per-class cost = wall time per wave-instruction per SIMD of a saturated
single-instruction kernel at 8 waves/SIMD (tools/gen_isa_rates.py chains ->
tools/isa_chains under tools/pmc_calib.sh: SQ_INSTS_VALU and the dispatch
duration of the same counter pass, so no clock assumption; the s_memtime
"cycles" of tools/isa_rates.hip turned out not to be shader cycles).  The
kernel's static instruction mix (one permutation = the absorb-loop body) is
read from its gfx950 assembly; the ceiling is the mix's issue time with every
instruction at its class cost, plus its hazard s_nops at their measured cost.
With a counter pass of tools/kbench.py (third argument) the class costs are
re-priced at the leaf hash's own clock (GRBM_GUI_ACTIVE per dispatch), and the
kernel's own VALU rate in that pass (same dispatches, same clock) gives the
clock-consistent fraction of the ceiling.  The counter pass itself runs the
kernel at a lower clock than the bench (≈2.0 vs ≈2.4 GHz), so the bench's
HIP-event rate is compared with the ceiling at the calibration clock.
Usage: python tools/issue_ceiling.py gpurun_out/calib_isa out.json [gpurun_out/calib_kb]"""
import collections
import csv
import json
import os
import re
import subprocess
import sys
import tempfile
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from libhash import lib_sha16  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "qp-zk-circuits-rm_amd", "csrc")
# kernel ids of tools/gen_isa_rates.py BLOCKS (after the 8 CHAINS kernels; 8
# waves/SIMD grid: 256 CUs x 8 x 256 lanes): 8 instructions per asm statement,
# so no compiler hazard pads
IDS = {"mad": "k8", "mad_nop": "k9", "add": "k10", "mov": "k11", "cndmask": "k12", "sub_co": "k13"}
GRID8 = 256 * 8 * 256
# full-rate class (s_memtime ratio ~0.6 of a VOP3 op, profiles/r02_isa_rates.log)
FAST = {"v_add_u32_e32", "v_sub_u32_e32", "v_xor_b32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_mov_b32_e32",
        "v_lshrrev_b32_e32", "v_not_b32_e32", "v_subrev_u32_e32"}


def dispatches(d):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        x = disp[r["Dispatch_Id"]]
        x["k"] = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        x["grid"] = int(r["Grid_Size"])
        x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        x["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return disp


# GPU clock of a dispatch: GRBM_GUI_ACTIVE counts GPU-clock cycles summed over
# the 8 XCDs (a saturated 2.2 ms dispatch reads ~18.3 G/s = 8 x 2.28 GHz), so
# cycles / 8 / duration is the clock the dispatch actually ran at (DVFS)
XCDS = 8


def clock_ghz(x):
    return x.get("GRBM_GUI_ACTIVE", 0.0) / XCDS / x["ns"] if x.get("GRBM_GUI_ACTIVE") else None


def class_costs(d):
    disp = dispatches(d)
    c, clk = {}, {}
    for name, kid in IDS.items():
        xs = [x for x in disp.values() if x["k"].split("::")[-1] == kid and x["grid"] == GRID8]
        # ns per VALU wave-instruction per SIMD (1024 SIMDs), best of the dispatches
        best = min(xs, key=lambda x: x["ns"] / x["SQ_INSTS_VALU"])
        c[name] = best["ns"] / (best["SQ_INSTS_VALU"] / 1024)
        clk[name] = clock_ghz(best)
    return {"mad": c["mad"], "fast": (c["add"] + c["mov"]) / 2, "vop3": (c["cndmask"] + c["sub_co"]) / 2,
            "s_nop": c["mad_nop"] - c["mad"], "measured": c, "clock_ghz": clk}


def leaf_dispatches(d):
    # the wires leaf hash: k_leaf_hash_t<135u> (compile-time column count), or
    # the run-time form k_leaf_hash of earlier builds
    ds = list(dispatches(d).values())
    xs = [x for x in ds if x["k"].endswith("k_leaf_hash_t<135u>")] or [x for x in ds if x["k"].endswith("k_leaf_hash")]
    if not xs:
        return []
    g = max(x["grid"] for x in xs)
    return [x for x in xs if x["grid"] == g and clock_ghz(x)]


def leaf_clock(d):
    """Clock of the k_leaf_hash dispatches (the wires leaf hash: the largest grid)
    in a counter pass of tools/kbench.py with the same GRBM counters."""
    ck = [clock_ghz(x) for x in leaf_dispatches(d)]
    return sum(ck) / len(ck) if ck else None


def leaf_rate_in_pass(d):
    """The same dispatches' VALU issue rate (SQ_INSTS_VALU wave-instructions
    over their duration): measured at the clock leaf_clock reports, so it
    compares with the ceiling priced at that clock with no clock assumption."""
    xs = [x for x in leaf_dispatches(d) if x.get("SQ_INSTS_VALU")]
    return sum(x["SQ_INSTS_VALU"] / (x["ns"] * 1e-9) for x in xs) / len(xs) if xs else None


def static_mix():
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "merkle.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                        os.path.join(CSRC, "merkle.hip"), "-o", s], check=True, capture_output=True)
        text = open(s).read()
    # the wires form k_leaf_hash_t<135> (compile-time column count), else k_leaf_hash
    m = re.search(r"^(_ZN3qpk13k_leaf_hash_tILj135EE\w*):[^\n]*\n(.*?)\n\s*s_endpgm", text, re.S | re.M) or \
        re.search(r"^(_ZN3qpk11k_leaf_hashE\w*):[^\n]*\n(.*?)\n\s*s_endpgm", text, re.S | re.M)
    ops = collections.Counter()
    for line in m.group(2).split("\n"):
        line = line.strip()
        if line and not line.startswith((";", ".")) and not line.endswith(":"):
            ops[line.split()[0]] += 1
    return ops


def main():
    cost = class_costs(sys.argv[1])
    ops = static_mix()
    valu = {k: v for k, v in ops.items() if k.startswith("v_")}
    n_valu = sum(valu.values())
    t = 0.0
    by = collections.Counter()
    for k, v in valu.items():
        c = cost["mad"] if k.startswith("v_mad_u64_u32") else cost["fast"] if k in FAST else cost["vop3"]
        by["mad" if c == cost["mad"] else "fast" if c == cost["fast"] else "vop3"] += v
        t += v * c
    t += ops["s_nop"] * cost["s_nop"]
    # each class cost was measured at its calibration kernel's clock: re-price
    # it at the leaf hash's own clock (cycles are what an instruction costs;
    # the clock under DVFS differs between kernels, MI355X_MICROARCH.md)
    lclk = leaf_clock(sys.argv[3]) if len(sys.argv) > 3 else None
    lrate = leaf_rate_in_pass(sys.argv[3]) if len(sys.argv) > 3 else None
    t_leaf = None
    if lclk:
        ck = cost["clock_ghz"]
        cyc = {"mad": cost["mad"] * ck["mad"], "fast": (cost["measured"]["add"] * ck["add"] +
                                                        cost["measured"]["mov"] * ck["mov"]) / 2,
               "vop3": (cost["measured"]["cndmask"] * ck["cndmask"] + cost["measured"]["sub_co"] * ck["sub_co"]) / 2,
               "s_nop": cost["measured"]["mad_nop"] * ck["mad_nop"] - cost["mad"] * ck["mad"]}
        t_leaf = (sum(by[k] * cyc[k] for k in ("mad", "fast", "vop3")) + ops["s_nop"] * cyc["s_nop"]) / lclk
    out = {
        "kernel": "qpk::k_leaf_hash",
        "lib_sha16": lib_sha16(),
        "class_ns_per_wave_instr_per_simd": cost,
        "static_mix_per_permutation": {"valu": n_valu, "s_nop": ops["s_nop"], "by_class": dict(by),
                                       "top": dict(collections.Counter(valu).most_common(8))},
        "ceiling_ns_per_wave_permutation_per_simd": t,
        "ceiling_wave_instr_per_s": n_valu / (t * 1e-9) * 1024,
        "leaf_hash_clock_ghz": lclk,
        "ceiling_at_leaf_clock_wave_instr_per_s": n_valu / (t_leaf * 1e-9) * 1024 if t_leaf else None,
        # the kernel's own rate in the same counter pass (same clock as the
        # line above): the clock-consistent fraction of its ceiling
        "leaf_rate_in_counter_pass_wave_instr_per_s": lrate,
        "frac_of_ceiling_in_counter_pass": lrate / (n_valu / (t_leaf * 1e-9) * 1024) if (lrate and t_leaf) else None,
        "sources": {"class costs": "tools/pmc_calib.sh counter pass over tools/isa_chains (8 waves/SIMD)",
                    "mix": "hipcc -S of csrc/merkle.hip (this tree)",
                    "s_nop": "mad+s_nop 0 block minus mad block (same pass)"},
    }
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
