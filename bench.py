"""bench.py — Wormhole proofs/sec on MI355X (BASELINE.json metric).

One step = WormholeProver::commit(inputs) + prove() for one batch of B
synthetic Wormhole CircuitInputs per GPU (BASELINE.json configs[2]: "Batch 256
Wormhole proofs on 1xMI355X"), end to end: commit() (the fragments'
fill_targets) on the host threads, witness generation (generate_partial_witness)
on the device, then the full prover (commitments, permutation argument,
quotient, openings, FRI, PoW, query openings) and the serialized proofs back on
the host.  Only the construction of the CircuitInputs themselves (the API's
input) happens before the timed region.  With N GPUs each rank proves its own
batch (independent proofs, weak scaling) and the leaf proof bytes are gathered
to rank 0 over RCCL (the aggregator's input).  --mode wires-dev times prove()
alone from wire matrices already resident in HBM (round-1 headline, reported as
prove_only for comparison).

Also reported (one JSON line, rank 0):
  roofline      the wires LDE (NTT) kernel: algorithmic bytes 8*(n+N) per column
                / its HIP-event-timed duration, vs the 8 TB/s HBM3E peak
  cpu_baseline  the CPU restatement of the same prover (oracle/prover.c, "port";
                the Rust reference cannot be built here) on a bounded sample
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "qp-zk-circuits-rm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2
# cycles per SIMD): 1024 SIMDs x 2.4 GHz / 2 = 1228.8 G wave-instructions/s
VALU_PEAK_WAVE_INSTR_S = 1024 * 2.4e9 / 2
# measured per-build inputs of the roofline fields, written by the profiling
# session of this build (tools/gpu_session.sh prof3 / pmc_*; tools/kernel_summary.py,
# tools/pmc_sq_summary.py, tools/pmc_summary.py)
PROFILE_TAG = "r06"
PMC_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_hbm_b128.json")
PMC_SQ_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_sq_b128.json")
KSUM_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_kernel_summary_3provers.json")
KSUM1_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_kernel_summary_1prover.json")
# measured issue ceiling of k_leaf_hash's instruction mix (tools/issue_ceiling.py:
# per-class wall-time costs from a counter pass over saturated single-instruction
# kernels, weighted by the kernel's static mix)
CEIL_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_issue_ceiling.json")
UBENCH_FILE = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_leaf_ubench.log")


def register_replay():
    """tools/leaf_ubench: the leaf-hash loop as built (L0) against the same loop
    with the absorbed chunk derived from the lane index instead of loaded (L3),
    back to back in one run: the kernel's instruction stream without memory is
    its own issue ceiling, free of the per-class pricing of mix_ceiling."""
    import re
    try:
        txt = open(UBENCH_FILE).read()
    except OSError:
        return None
    g = {m.group(1): float(m.group(2)) for m in re.finditer(r"^(L\d)\b.*?([\d.]+) Gperm/s", txt, re.M)}
    if "L0" not in g or "L3" not in g:
        return None
    return {"production_gperm_s": g["L0"], "no_load_gperm_s": g["L3"], "frac": g["L0"] / g["L3"],
            "source": os.path.relpath(UBENCH_FILE, ROOT)}


def load_json(path):
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def perm_valu_instr():
    """VALU instructions per Poseidon permutation: SQ_INSTS_VALU x 64 / lanes of the
    wires leaf-hash dispatch (17 permutations per leaf) in this build's PMC pass."""
    recs = load_json(PMC_SQ_FILE) or []
    for r in recs:
        if (r.get("kernel") or "").startswith("qpk::k_leaf_hash") and r.get("valu_per_lane_max"):
            return r["valu_per_lane_max"] / 17.0
    return None


def pmc_traffic(kernel, ncols, log_n, proofs, lanes_per_proof=None):
    """HBM bytes per launch of `kernel` for `proofs` proofs of `ncols` columns, or None."""
    try:
        recs = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None
    for r in recs:
        # template arguments beyond the first (e.g. k_lde_cosets<9, 0>'s twiddle mode) do not matter
        name = r.get("kernel") or ""
        if (name != kernel and not (kernel.endswith(">") and name.startswith(kernel[:-1] + ","))) \
                or not r.get("hbm_bytes"):
            continue
        if lanes_per_proof is None:
            lanes_per_proof = ncols * (1 << log_n) // 16  # one 2^(log_n - 4)-lane workgroup per column
        if r["grid_lanes"] % lanes_per_proof:
            continue
        return r["hbm_bytes"] / (r["grid_lanes"] // lanes_per_proof) * proofs
    return None


def mix_ceiling(ceil):
    """k_leaf_hash's issue ceiling (tools/issue_ceiling.py): its instruction mix at
    the measured per-class costs, at the calibration streams' clock (≈2.38 GHz;
    the bench's HIP-event rate has no clock reading, and the kernel runs near
    that clock outside counter passes)."""
    if not ceil:
        return None
    return ceil["ceiling_wave_instr_per_s"]


def profile_stamp(path):
    """lib_sha16 a profile summary was stamped with (tools/libhash.py), or None."""
    d = load_json(path)
    if isinstance(d, list):
        d = d[0] if d else None
    return d.get("lib_sha16") if isinstance(d, dict) else None


def segregate_profile_fields(rec):
    """Fields read from committed profile summaries (PMC traffic, instructions per
    permutation, mix ceiling, kernel-time share, GPU busy fraction) stay in place
    only when the summary was stamped with the hash of the library this run
    loaded; otherwise they move under rec["from_profile"] with their source and
    stamp, and the in-place value becomes None."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from libhash import lib_sha16
    from qp_wormhole._native import LIB_PATH
    mine = lib_sha16(LIB_PATH)
    moved = {}

    def check(path, owner, keys, label):
        if owner is None:
            return
        st = profile_stamp(path)
        if st == mine:
            return
        for k in keys:
            if owner.get(k) is not None:
                moved[f"{label}.{k}"] = {"value": owner[k], "source": os.path.relpath(path, ROOT), "lib_sha16": st}
                owner[k] = None
    check(PMC_FILE, rec.get("roofline"), ["traffic"], "roofline")
    check(PMC_FILE, rec.get("valu_kernels"), ["quotient_hbm_bytes_per_launch"], "valu_kernels")
    dk = rec.get("dominant_kernel")
    check(PMC_SQ_FILE, dk, ["instr_per_perm", "achieved", "frac", "frac_of_mix_ceiling"], "dominant_kernel")
    check(CEIL_FILE, dk, ["mix_ceiling", "frac_of_mix_ceiling", "frac_of_mix_ceiling_at_own_clock",
                          "own_clock_ghz_in_counter_pass"], "dominant_kernel")
    check(KSUM1_FILE, dk, ["share_of_kernel_time"], "dominant_kernel")
    check(KSUM_FILE, rec.get("gpu_busy_frac"), ["value"], "gpu_busy_frac")
    rec["profile_build"] = {"lib_sha16": mine, "all_profiles_of_this_build": not moved}
    if moved:
        moved["note"] = ("read from profile summaries of another build (their lib_sha16 differs from the loaded "
                         "library's): not this build's measurement")
        rec["from_profile"] = moved


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0,
                    help="proofs per GPU per step (default: 256 Wormhole, 1024 voting)")
    ap.add_argument("--provers", type=int, default=0,
                    help="concurrent provers per GPU (own HIP stream + host thread each, B/provers proofs each): "
                         "one prover's host transcript phases overlap the other's kernels; 0 = the measured best "
                         "per circuit: 3 for Wormhole (2: same, 4: -3 %%), 6 for voting (3: 9.4-10.8 k, 4: "
                         "11.9-12.1 k, 6: 12.4-13.0 k, 8: 12.0-12.5 k proofs/s; profiles/r05_ab_provers.log)")
    ap.add_argument("--circuit", choices=["wormhole", "voting"], default="wormhole",
                    help="wormhole = BASELINE configs[2] (the headline); voting = configs[4]")
    ap.add_argument("--mode", choices=["e2e", "wires-dev"], default="e2e",
                    help="e2e: CircuitInputs -> proofs (headline); wires-dev: prove() from HBM-resident wires")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="join the prover threads after every step (default: each prover runs its share of all "
                         "steps back to back)")
    ap.add_argument("--host-threads", type=int, default=0,
                    help="host threads per prover (caller included); 0 = library default (measured 1.5%% "
                         "faster than a split, profiles/r03_ab_host_threads.log); -1 = split the process's "
                         "cores (OMP_NUM_THREADS, else min(cores, 16)) between the provers")
    ap.add_argument("--agg-leaves", type=int, default=64,
                    help="leaf proofs aggregated (one level, pairs) after the timed region (0 = skip)")
    ap.add_argument("--configs3-steps", type=int, default=4,
                    help="configs[3] also as K batches back to back (leaves of batch k+1 overlapping the "
                         "aggregation of batch k); 0 or 1: the single-batch record only")
    ap.add_argument("--configs3-parts", type=int, default=0,
                    help="configs[3] also with the batch's leaves proved in this many parts, each part's sub-tree "
                         "aggregated as soon as its leaves exist (0 or 1: skip)")
    ap.add_argument("--configs3", type=int, default=1,
                    help="after the headline, time BASELINE configs[3] as one pipeline (every rank: its batch of "
                         "leaves -> its subtree root; roots gathered over RCCL; rank 0: the tree root); 0 = skip")
    ap.add_argument("--ref-shapes", type=int, default=1,
                    help="after the headline, time the reference's own bench shapes: prover_create_proof "
                         "(new + commit + prove, zk config), the aggregator bench trees, one voting pass (0 = skip)")
    ap.add_argument("--cpu-sample", type=int, default=2, help="min proofs in the CPU baseline sample (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="min seconds of CPU baseline proving")
    ap.add_argument("--launch-selftest", choices=["ok", "fail-rank1"], default=None,
                    help="test the --gpus N launcher without a GPU: every rank joins a gloo group and rank 0 prints "
                         "the ranks it saw (fail-rank1: rank 1 exits non-zero first)")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="rehearse the --gpus N path on a one-GPU box: every rank proves on cuda:0, the process "
                         "group is gloo over host tensors (not RCCL); the line says rehearsal (not a measurement)")
    return ap.parse_args()


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) with no WORLD_SIZE in the environment: start N
    rank processes of this script, one per GPU (RANK = LOCAL_RANK = 0..N-1,
    WORLD_SIZE = N, a free 127.0.0.1 port), before anything here imports torch or
    the library -- child processes, never an exec.  Rank 0's stdout is this
    process's (the one JSON line); the other ranks' stdout goes to stderr.  When a
    rank fails the others are stopped (they would wait in a collective).
    Returns the exit status: 0 when every rank succeeded, else the first
    non-zero one."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    try:
        while [p.poll() for p in procs].count(None):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad and not rc:
                rc = bad[0]
                print(f"bench.py launcher: a rank exited with status {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for p in procs:
                    if p.poll() is None:
                        p.send_signal(signal.SIGTERM)
                deadline = time.time() + 30
                while any(p.poll() is None for p in procs) and time.time() < deadline:
                    time.sleep(0.2)
                for p in procs:
                    if p.poll() is None:
                        p.kill()
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    for p in procs:
        p.wait()
    if not rc:
        rc = next((p.returncode for p in procs if p.returncode), 0)
    # a signal-killed rank reports a negative status: exit with 128 + signal
    return rc if rc >= 0 else 128 - rc


def launch_selftest(mode, gpus):
    """One rank of the launcher self-test (no GPU): a gloo group of WORLD_SIZE
    ranks; rank 0 prints one JSON line with every rank's (RANK, LOCAL_RANK,
    WORLD_SIZE) as the group saw them."""
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    if mode == "fail-rank1" and rank == 1:
        sys.exit(5)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        print(f"bench.py: WORLD_SIZE {world} != --gpus {gpus}", file=sys.stderr)
        sys.exit(3)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    me = {"rank": dist.get_rank(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "world": dist.get_world_size()}
    seen = [None] * world
    dist.all_gather_object(seen, me)
    if rank == 0:
        print(json.dumps({"launch_selftest": mode, "gpus": gpus, "world_size": dist.get_world_size(),
                          "ranks": seen}), flush=True)
    dist.destroy_process_group()


def check_world(args, world, torch):
    """Every rank: the process group is the --gpus N the line will report, and
    this node has N devices (before any collective, so every rank fails alike
    instead of one waiting on another)."""
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE {world} != --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(3)
    ndev = torch.cuda.device_count()
    if ndev < (1 if args.rehearse_shared_gpu else args.gpus):
        print(f"bench.py: --gpus {args.gpus} but this node has {ndev} GPU(s)", file=sys.stderr, flush=True)
        sys.exit(3)


def trace_marker(torch):
    """One tiny spin kernel (torch's at::cuda sleep) just outside each end of the
    timed region, so tools/kernel_summary.py can cut a rocprofv3 kernel trace to
    exactly the timed steps (gpu_busy_frac of the timed region)."""
    sleep = getattr(torch.cuda, "_sleep", None)
    if sleep is not None:
        sleep(1000)


def make_inputs(circuit, first, count):
    from qp_wormhole.synthetic import synthetic_inputs, synthetic_vote_inputs
    gen = synthetic_vote_inputs if circuit.kind == "voting" else synthetic_inputs
    return [gen(first + i) for i in range(count)]


def make_witnesses(circuit, inputs):
    n, W = circuit.n, circuit.num_wires
    wires = np.empty((len(inputs), W, n), np.uint64)
    pis = np.empty((len(inputs), circuit.num_public_inputs), np.uint64)
    for i, x in enumerate(inputs):
        w = circuit.commit(x)
        wires[i] = w.wires()
        pis[i] = w.public_inputs()
        w.free()
    return wires, pis


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(circuit, inputs, sample, min_seconds):
    """The GPU line's work on the host cores, proof by proof: commit() + witness
    generation (this library's host generator, circuit.commit: the C++
    restatement of generate_partial_witness) and prove() (oracle/prover.c, the
    C + OpenMP restatement of plonky2's prover), for at least `sample` of the
    bench's own CircuitInputs, continuing (cycling through them) until
    `min_seconds` have been timed."""
    from oracle_lib import U64P, lib as olib
    L = olib()
    L.ora_prove.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64P, U64P, U64P, ctypes.c_size_t, ctypes.c_char_p,
                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), U64P, U64P]
    cores = int(os.environ.get("OMP_NUM_THREADS") or host_cpu_share())
    L.ora_set_threads(cores)
    cb = circuit.common_data()
    cs = circuit.constants_sigmas()
    out = ctypes.create_string_buffer(400000)
    ln = ctypes.c_size_t()
    cap = np.zeros(64, np.uint64)
    dig = np.zeros(4, np.uint64)
    t = time.perf_counter()
    done = 0
    t_wit = 0.0
    while done < sample or time.perf_counter() - t < min_seconds:
        t0 = time.perf_counter()
        w = circuit.commit(inputs[done % len(inputs)])
        wires, pis = w.wires(), w.public_inputs()
        w.free()
        t_wit += time.perf_counter() - t0
        rc = L.ora_prove(cb, len(cb), cs, wires, pis, len(pis), out, 400000, ctypes.byref(ln), cap, dig)
        assert rc == 0
        done += 1
    dt = time.perf_counter() - t
    nproc = os.cpu_count() or 1
    value = done / dt
    # the reference's bench iteration (prover/benches/prover.rs:11-21) on the same
    # cores: WormholeProver::new(standard_recursion_zk_config) = the circuit build
    # (host C++) + the constants||sigmas commitment (oracle ora_commit_values, one
    # thread), then commit(test_inputs()) + prove (oracle/prover.c, OpenMP)
    import wormhole_inputs
    L.ora_commit_values.argtypes = [U64P, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p,
                                    ctypes.c_uint, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, U64P]
    t0 = time.perf_counter()
    zc = type(circuit).wormhole(zero_knowledge=True)
    zcs = np.ascontiguousarray(zc.constants_sigmas())
    zcap = np.zeros(64, np.uint64)
    rc = L.ora_commit_values(zcs, zcs.shape[0], zc.degree_bits, 3, 4, None, 0, 0, None, None, zcap)
    assert rc == 0
    t1 = time.perf_counter()
    w = zc.commit(wormhole_inputs.test_inputs())
    zw, zpis = w.wires(), w.public_inputs()
    w.free()
    t2 = time.perf_counter()
    zcb = zc.common_data()
    assert L.ora_prove(zcb, len(zcb), zcs, zw, zpis, len(zpis), out, 400000, ctypes.byref(ln), cap, dig) == 0
    t3 = time.perf_counter()
    create = {"new_ms": (t1 - t0) * 1e3, "commit_ms": (t2 - t1) * 1e3, "prove_ms": (t3 - t2) * 1e3,
              "iteration_ms": (t3 - t0) * 1e3,
              "note": "one iteration: circuit build (host C++) + constants||sigmas commit (oracle, 1 thread) + "
                      "commit(test_inputs()) + prove (oracle/prover.c, OpenMP)"}
    return {"value": value, "unit": "proofs/s", "cores": cores, "kind": "port",
            "per_core": value / cores, "prover_create_proof": create,
            "sample": f"{done} {circuit.kind} proofs (deg {circuit.degree_bits}, standard_recursion_config) from the "
                      f"bench's CircuitInputs, {dt:.1f} s: commit + witness generation {t_wit:.2f} s (host C++, one "
                      f"thread), prove {dt - t_wit:.1f} s (oracle/prover.c, C + OpenMP, {cores} threads)",
            "host": {"nproc": nproc, "cpu_model": cpu_model(), "omp_threads": cores,
                     "affinity": len(os.sched_getaffinity(0)), "cgroup_cpus": cgroup_cpu_quota(),
                     # the box gives one GPU's job a share of the node's cores
                     # (OMP_NUM_THREADS); all nproc at the measured per-core rate,
                     # an upper bound (commit + witness run on one thread)
                     "whole_node_linear_estimate": value / cores * nproc},
            "note": "the GPU line's work (commit, witness generation, prove) on the host cores this job may use; "
                    "a C restatement of plonky2, not the Rust reference (no cargo here): quote no GPU/CPU ratio"}


def cgroup_cpu_quota():
    """CPUs of this process's cgroup v2 cpu.max quota, or None if unlimited/unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def host_cpu_share():
    """Cores this process may run on: the affinity mask, capped by the cgroup quota."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q))) if q else n


def reference_parity(qp_wormhole, device):
    """The reference's own current-circuit proofs (tests/golden/dummy_proof{,_zk}.bin)
    reproduced byte for byte by the GPU prover: test_inputs() with the proofs'
    PublicInputGate-row cells and PoW witness (tests/golden/reference_pi_cells.json,
    derived from the fixtures by tests/golden/make_pi_cells.py)."""
    import wormhole_inputs
    cells = load_json(os.path.join(ROOT, "tests", "golden", "reference_pi_cells.json"))
    if not cells:
        return None
    out = {}
    for name in ("dummy_proof.bin", "dummy_proof_zk.bin"):
        with open(os.path.join(ROOT, "tests", "golden", name), "rb") as f:
            ref = f.read()
        circ = qp_wormhole.Circuit.wormhole(zero_knowledge=name.endswith("_zk.bin"))
        p = qp_wormhole.Prover(qp_wormhole.Context(device), circ, max_batch=1)
        inp = wormhole_inputs.test_inputs()
        inp.zk_randomness = cells[name]["pi_row_cells"]
        p.debug_force_pow(cells[name]["pow_witness"])
        out[name] = p.prove_inputs([inp])[0] == ref
        p.free()
    out["note"] = ("GPU proof bytes == the reference's own proof of test_inputs() given its PI-row random cells "
                   "and PoW witness (its find_any witness is nondeterministic); after the timed region")
    return out


def cargo_bench_shape(qp_wormhole, local, iters=3):
    """The reference's own benchmark iteration (wormhole/prover/benches/prover.rs:11-21,
    "prover_create_proof"): WormholeProver::new(standard_recursion_zk_config) --
    the circuit build plus the constants||sigmas commitment (prover/src/lib.rs:
    190-202) -- then commit(test_inputs()) and prove(), every iteration from
    scratch (a new device context and prover each time, nothing cached).  One
    untimed iteration first (code objects, allocator); median of `iters`."""
    import wormhole_inputs
    from oracle_lib import lib as olib
    rows = []
    ok = None
    for it in range(iters + 1):
        t0 = time.perf_counter()
        ctx = qp_wormhole.Context(local)
        circ = qp_wormhole.Circuit.wormhole(zero_knowledge=True)
        p = qp_wormhole.Prover(ctx, circ, max_batch=1)
        ctx.synchronize()
        t1 = time.perf_counter()
        w = circ.commit(wormhole_inputs.test_inputs())
        t2 = time.perf_counter()
        proof = p.prove_witnesses([w])[0]
        t3 = time.perf_counter()
        if it:
            rows.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
        if it == iters:
            vd = p.verifier_data()
            ok = olib().ora_verify(vd, len(vd), proof, len(proof)) == 0
        w.free()
        p.free()
        ctx.close()
    med = [sorted(c)[len(c) // 2] * 1e3 for c in zip(*rows)]
    return {"new_ms": med[0], "commit_ms": med[1], "prove_ms": med[2], "iteration_ms": med[3],
            "iterations": iters, "proof_verified": ok,
            "note": "WormholeProver::new(standard_recursion_zk_config) (circuit build on the host + device "
                    "preprocessing: constants||sigmas LDE and Merkle tree) + commit(test_inputs()) + prove(), from "
                    "scratch each iteration; medians; after the timed region"}


# the reference's aggregator benchmark shapes (wormhole/aggregator/benches/aggregator.rs:106-123)
AGG_SHAPES = [(2, 1), (2, 2), (2, 3), (2, 4), (2, 5), (3, 2), (4, 2), (5, 2), (6, 2), (7, 2)]


def aggregator_shapes(qp_wormhole, local):
    """aggregate_proofs_{k}_{depth} of aggregator.rs:22-58: WormholeProofAggregator::default()
    (standard_recursion_zk_config leaves) with TreeAggregationConfig::new(k, depth),
    num_leaf_proofs copies of dummy_proof_zk.bin pushed, aggregate() timed.  The
    reference builds every chunk's circuit inside aggregate() (tree.rs:106-125);
    here level circuits are built once and cached, so each shape reports its
    first call (circuits built + device preprocessing) and the best of two
    cached calls.  Every root is verified by the oracle verifier afterwards."""
    from oracle_lib import lib as olib
    from qp_wormhole import aggregator as A
    out = {}
    base = A.WormholeProofAggregator.default(local)
    dummy = base.dummy_proof()
    for k, depth in AGG_SHAPES:
        cfg = A.TreeAggregationConfig.new(k, depth)
        times, root = [], None
        for _ in range(3):
            agg = A.WormholeProofAggregator(base.leaf_circuit_data, dummy, local).with_config(cfg)
            for _ in range(cfg.num_leaf_proofs):
                agg.push_proof(dummy)
            t0 = time.perf_counter()
            root = agg.aggregate()
            times.append(time.perf_counter() - t0)
        rvd, rp = root.circuit_data.verifier_data(), root.proof.to_bytes()
        from qp_wormhole.prover import _common_degree_bits
        out[f"aggregate_proofs_{k}_{depth}"] = {
            "leaves": cfg.num_leaf_proofs, "first_call_ms": times[0] * 1e3,
            "cached_ms": min(times[1:]) * 1e3,
            "root_degree_bits": _common_degree_bits(root.circuit_data.common),
            "root_verified": olib().ora_verify(rvd, len(rvd), rp, len(rp)) == 0}
        # release this shape's level provers (device workspaces) before the next
        with A._levels_lock:
            A._levels.clear()
    out["note"] = ("the reference's aggregator bench shapes (binary 2..32 leaves, (k,2) for k = 3..7) on the GPU: "
                   "first_call_ms builds the level circuits and their device preprocessing (the reference builds "
                   "them inside every aggregate()); cached_ms (best of two) reuses them; after the timed region")
    return out


def voting_pass(qp_wormhole, local, batch=1024, nprov=6):
    """BASELINE configs[4]: one pass of `batch` voting proofs (voting/src/lib.rs:346-360
    circuit), end to end from the synthetic vote inputs, `nprov` provers in
    parallel on their own streams (the --circuit voting bench's shape), timed
    after one untimed pass."""
    import threading
    from qp_wormhole.synthetic import synthetic_vote_inputs
    circ = qp_wormhole.Circuit.voting()
    per = [batch // nprov + (1 if i < batch % nprov else 0) for i in range(nprov)]
    first = [sum(per[:i]) for i in range(nprov)]
    inputs = [synthetic_vote_inputs(i) for i in range(batch)]
    ps = [qp_wormhole.Prover(qp_wormhole.Context(local), circ, max_batch=per[i]) for i in range(nprov)]
    cin = [ps[i].inputs_array(inputs[first[i]:first[i] + per[i]]) for i in range(nprov)]
    outs = [None] * nprov

    def run(i):
        outs[i] = ps[i].prove_inputs_array(cin[i], per[i])

    def once():
        th = [threading.Thread(target=run, args=(i,)) for i in range(nprov)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if any(o is None for o in outs):
            raise RuntimeError("a voting prover thread failed")
    once()
    t0 = time.perf_counter()
    once()
    dt = time.perf_counter() - t0
    from oracle_lib import lib as olib
    vd = ps[0].verifier_data()
    ok = all(olib().ora_verify(vd, len(vd), pf, len(pf)) == 0 for pf in (outs[0][0], outs[-1][-1]))
    for p in ps:
        p.free()
    return {"proofs": batch, "provers": nprov, "seconds": dt, "proofs_per_s": batch / dt,
            "degree_bits": circ.degree_bits, "proofs_verified": ok,
            "note": "voting circuit, synthetic seeded vote inputs, one timed pass after an untimed one; after the "
                    "timed region"}


def configs3(args, circuit, prover, provers, cin, cin_inputs, per, NP, B, dist, world, rank, local, torch, cdev):
    """BASELINE configs[3] ("Batch 2048 proofs sharded 8xMI355X, RCCL-gather leaves
    into recursive aggregator"; aggregator.rs:74-92, tree.rs:55-103) timed as one
    pipeline (qp_wormhole.distributed.pipeline_aggregate_step): every rank proves
    its batch of leaves end to end (CircuitInputs -> proofs, its provers in
    parallel), aggregates them (branching 2) into its subtree root on its own GPU
    with device witness generation, the roots are gathered to rank 0 over RCCL,
    and rank 0 aggregates them into the tree root.  One untimed pass builds and
    caches every level's circuit; the timed pass is bracketed by barriers and
    device syncs, max over ranks."""
    import threading
    from qp_wormhole.distributed import pipeline_aggregate_step
    ns = 1 << (B.bit_length() - 1)  # leaves per rank: the largest power of two <= B
    vd = prover.verifier_data()
    cb = circuit.common_data()
    vo = vd[:len(vd) - len(cb)]

    def prove_leaves():
        outs = [None] * NP

        def run(i):
            outs[i] = provers[i].prove_inputs_array(cin[i], per[i])
        th = [threading.Thread(target=run, args=(i,)) for i in range(NP)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if any(o is None for o in outs):
            raise RuntimeError("a leaf prover thread failed")
        return [p for o in outs for p in o][:ns]

    dev = cdev  # collective tensors (the rank's GPU; host tensors under --rehearse-shared-gpu)

    def step():
        return pipeline_aggregate_step(prove_leaves, cb, vo, 2, dist, device=dev, gpu=local)

    step()  # untimed: builds and caches every level's circuit and device preprocessing
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    root, tm = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # one batch with its leaves proved in `parts` consecutive parts (the
    # sub-trees' leaf ranges) and each part's sub-tree aggregated as soon as its
    # leaves exist (pipeline_aggregate_step_streamed): the same root
    strm = None
    P = args.configs3_parts
    if P > 1 and ns % P == 0 and ns // P >= 2:
        from qp_wormhole.distributed import pipeline_aggregate_step_streamed
        m = ns // P
        pin = []
        for q in range(P):
            sub = [inp for i in range(NP) for inp in cin_inputs[i]][q * m:(q + 1) * m]
            pp = [m // NP + (1 if i < m % NP else 0) for i in range(NP)]
            pf = [sum(pp[:i]) for i in range(NP)]
            pin.append([(provers[i].inputs_array(sub[pf[i]:pf[i] + pp[i]]), pp[i]) for i in range(NP)])

        def prove_part(q):
            outs = [None] * NP

            def run(i):
                arr, k = pin[q][i]
                outs[i] = provers[i].prove_inputs_array(arr, k) if k else []
            th = [threading.Thread(target=run, args=(i,)) for i in range(NP)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if any(o is None for o in outs):
                raise RuntimeError("a leaf prover thread failed")
            return [p for o in outs for p in o]

        def sstep():
            return pipeline_aggregate_step_streamed(prove_part, P, m, cb, vo, 2, dist, device=dev, gpu=local)
        sstep()  # untimed (the parts' smaller leaf batches)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sroot, stm = sstep()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        sdt = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([sdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            sdt = float(tt.item())
        strm = (sroot, stm, sdt)
    # the same as a stream of batches: batch k+1's leaves proved while batch k
    # is aggregated (pipeline_aggregate_steps), K batches timed end to end
    pipe = None
    K = args.configs3_steps
    if K > 1:
        from qp_wormhole.distributed import pipeline_aggregate_steps
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        proots, ptms = pipeline_aggregate_steps(prove_leaves, K, cb, vo, 2, dist, device=dev, gpu=local)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        pdt = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([pdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            pdt = float(tt.item())
        pipe = (proots, ptms, pdt)
    if rank != 0:
        return None
    from oracle_lib import lib as olib
    from qp_wormhole.prover import _common_degree_bits

    def verified(t):
        vd_, pb = t.circuit_data.verifier_data(), t.proof.to_bytes()
        return olib().ora_verify(vd_, len(vd_), pb, len(pb)) == 0
    tops = root if isinstance(root, list) else [root]
    ok = all(verified(t) for t in tops)
    leaves = world * ns
    pipelined = None
    if pipe is not None:
        proots, ptms, pdt = pipe
        flat = [t for r in proots for t in (r if isinstance(r, list) else [r])]
        pipelined = {"steps": K, "seconds": pdt, "seconds_per_step": pdt / K, "value": K * leaves / pdt,
                     "unit": "leaf proofs/s (each batch proved and aggregated into its root)",
                     "roots_verified": len(proots) == K and all(verified(t) for t in flat),
                     "stages_rank0_s": {k: [round(t[k], 4) for t in ptms] for k in ptms[0]},
                     "note": "K batches back to back, batch k+1's leaves proved on the leaf provers' streams "
                             "while batch k is aggregated on the level provers' (the subtree's narrow top "
                             "levels are latency-bound); leaves_s overlaps the previous batch's subtree"}
    streamed = None
    if strm is not None:
        sroot, stm, sdt = strm
        stops = sroot if isinstance(sroot, list) else [sroot]
        streamed = {"parts": P, "seconds": sdt, "value": leaves / sdt,
                    "unit": "leaf proofs/s (proved and aggregated into one root)",
                    "root_verified": all(verified(t) for t in stops),
                    "same_root_as_batch_step": [t.proof.to_bytes() for t in stops] == [t.proof.to_bytes()
                                                                                         for t in tops],
                    "stages_rank0_s": {k: round(v, 4) for k, v in stm.items() if isinstance(v, float)},
                    "note": f"the batch's leaves proved in {P} parts (the sub-trees' leaf ranges, {ns // P} "
                            "leaves each over the same provers) on a producer thread, each part's sub-tree "
                            "aggregated as soon as its leaves exist; leaves_s = when the last part was proved"}
    return {"workload": f"{leaves}_leaves_as_{world}x{ns}_per_gpu_subtrees_branching2",
            "value": leaves / dt, "unit": "leaf proofs/s (proved and aggregated into one root)"
            if len(tops) == 1 else f"leaf proofs/s (proved and aggregated into {len(tops)} top proofs)",
            "seconds": dt, "leaves": leaves, "aggregation_proofs": leaves - len(tops),
            "stages_rank0_s": tm, "pipelined": pipelined, "streamed": streamed,
            "root_verified" if len(tops) == 1 else "top_proofs_verified": ok,
            "top_circuit_degree_bits": _common_degree_bits(tops[0].circuit_data.common),
            "root_public_inputs": sum(len(t.proof.public_inputs) for t in tops),
            "note": "one timed pass after an untimed one that builds the level circuits; leaves e2e from "
                    "CircuitInputs, per-GPU subtree (device witness generation, batched levels), roots gathered "
                    "over RCCL (world > 1), top levels on rank 0; root verified by the oracle verifier after the "
                    "timed region"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_selftest:
        return launch_selftest(args.launch_selftest, args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    check_world(args, world, torch)
    rehearse = args.rehearse_shared_gpu
    if rehearse:
        local = 0  # every rank's provers on the one GPU
    cdev = "cpu" if rehearse else f"cuda:{local}"
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if rehearse else "nccl")
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: process group of {dist.get_world_size()} ranks != --gpus {args.gpus}",
                  file=sys.stderr, flush=True)
            sys.exit(3)
    import qp_wormhole

    voting = args.circuit == "voting"
    circuit = qp_wormhole.Circuit.voting() if voting else qp_wormhole.Circuit.wormhole(zero_knowledge=False)
    B = args.batch or (1024 if voting else 256)
    inputs = make_inputs(circuit, rank * B, B)
    NP = max(1, min(args.provers or (6 if args.circuit == "voting" else 3), B))
    per = [B // NP + (1 if i < B % NP else 0) for i in range(NP)]
    first = [sum(per[:i]) for i in range(NP)]
    provers = [qp_wormhole.Prover(qp_wormhole.Context(local), circuit, max_batch=per[i]) for i in range(NP)]
    prover = provers[0]
    budget = int(os.environ.get("OMP_NUM_THREADS") or min(os.cpu_count() or 4, 16))
    host_threads = max(2, budget // NP) if args.host_threads < 0 else args.host_threads
    if host_threads:
        for p in provers:
            p.set_host_threads(host_threads)
    # the API input marshalled once into C-ABI structs (CircuitInputs -> qp_wormhole_inputs)
    cin = [prover.inputs_array(inputs[first[i]:first[i] + per[i]]) for i in range(NP)]
    # prove-only comparison path: wire matrices resident in HBM (host-generated)
    wires = pis = d_wires = None
    if args.mode == "wires-dev" or rank == 0:
        wires, pis = make_witnesses(circuit, inputs[:max(per[0], 2)] if args.mode == "e2e" else inputs)
        d_wires = torch.from_numpy(wires.view(np.int64)).to(f"cuda:{local}")
    wstride = wires[0].nbytes if wires is not None else 0
    torch.cuda.synchronize()

    from qp_wormhole.distributed import run_steps

    def prove_share(i):
        if args.mode == "e2e":
            return provers[i].prove_inputs_array(cin[i], per[i])
        return provers[i].prove_wires_dev(d_wires.data_ptr() + first[i] * wstride,
                                          pis[first[i]:first[i] + per[i]], per[i])

    gathered = []  # rank 0: leaf proofs that reached it per timed step (world x B)

    def on_leaves(s, res):
        gathered.append(sum(res[1]) if dist is not None else len(res))

    def steps(k, pipelined):
        # leaf proofs -> aggregator rank over RCCL (raw gather) after every step
        return run_steps(prove_share, NP, k, dist=dist, slot=prover.proof_size, device=cdev,
                         pipelined=pipelined, on_leaves=on_leaves)

    proofs = steps(args.warmup, False) if args.warmup else None
    # proofs of the warmup verify (rank 0 checks the first and last with the oracle verifier)
    verified = None
    if rank == 0 and args.warmup:
        from oracle_lib import lib as olib
        vd = prover.verifier_data()
        verified = all(olib().ora_verify(vd, len(vd), p, len(p)) == 0 for p in (proofs[0], proofs[-1]))
    for p in provers:
        p.set_timing(True)
        p.kernel_stats(reset=True)
        p.stage_times(reset=True)
    if dist is not None:
        dist.barrier()
    gathered.clear()
    trace_marker(torch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps, args.pipeline)
    torch.cuda.synchronize()
    trace_marker(torch)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # kernel statistics summed over the provers (HIP events on each prover's stream)
    ks = provers[0].kernel_stats()
    for p in provers[1:]:
        for k, v in p.kernel_stats().items():
            for f in ("ms", "units", "launches"):
                ks[k][f] += v[f]
    stages = prover.stage_times()
    # the same kernels alone on the GPU (one prover, one step, after the timed region)
    iso = None
    if rank == 0 and NP > 1:
        prover.kernel_stats(reset=True)
        prover.prove_inputs_array(cin[0], per[0])
        iso = prover.kernel_stats()
    # prove() alone from HBM-resident wires (round-1 headline definition), one prover
    prove_only = None
    if rank == 0 and args.mode == "e2e":
        prover.set_timing(False)
        t1 = time.perf_counter()
        prover.prove_wires_dev(d_wires.data_ptr(), pis[:per[0]], per[0])
        prove_only = per[0] / (time.perf_counter() - t1)
    # single-proof latency (BASELINE configs[1]): one proof through the same prover
    lat = None
    if rank == 0:
        prover.set_timing(False)
        ts = []
        one = prover.inputs_array(inputs[:1])
        for _ in range(3):
            t1 = time.perf_counter()
            prover.prove_inputs_array(one, 1)
            ts.append((time.perf_counter() - t1) * 1e3)
        lat = sorted(ts)[1]
    # recursive aggregation of this run's leaf proofs (BASELINE
    # configs[3]'s consumer; wormhole/aggregator/src/circuits/tree.rs): one level of
    # `agg_leaves` leaves (agg_leaves/2 aggregation proofs, degree 2^13, batched) and a
    # default tree (8 leaves, branching 2, depth 3) end to end; after the timed region
    agg = None
    if rank == 0 and not voting and args.agg_leaves and proofs is not None:
        from qp_wormhole.aggregator import TreeAggregationConfig, aggregate_level, aggregate_to_tree
        from qp_wormhole.prover import _common_degree_bits
        from oracle_lib import lib as olib
        vd = prover.verifier_data()
        cb = circuit.common_data()
        vo = vd[:len(vd) - len(cb)]
        nl = min(args.agg_leaves, len(proofs)) // 2 * 2
        cfg2 = TreeAggregationConfig.new(2, 1)
        aggregate_level(proofs[:nl], cb, vo, cfg2)  # circuit build + device preprocessing at this batch (cached)
        t1 = time.perf_counter()
        level = aggregate_level(proofs[:nl], cb, vo, cfg2)
        lvl_s = time.perf_counter() - t1
        aggregate_to_tree(proofs[:8], cb, vo)  # builds the level-2/3 circuits (cached)
        t1 = time.perf_counter()
        root = aggregate_to_tree(proofs[:8], cb, vo)
        tree_ms = (time.perf_counter() - t1) * 1e3
        # one aggregation proof's latency (aggregate_chunk of 2 leaves, batch of one)
        ts = []
        for _ in range(5):
            t1 = time.perf_counter()
            aggregate_level(proofs[:2], cb, vo, cfg2)
            ts.append((time.perf_counter() - t1) * 1e3)
        one_ms = sorted(ts)[2]
        rvd = root.circuit_data.verifier_data()
        rp = root.proof.to_bytes()
        agg = {"level_leaves": nl, "level_aggregation_proofs": len(level),
               "aggregation_proofs_per_s": len(level) / lvl_s, "leaves_per_s_through_one_level": nl / lvl_s,
               "tree8_root_ms": tree_ms, "one_proof_ms": one_ms, "root_verified": olib().ora_verify(rvd, len(rvd), rp, len(rp)) == 0,
               "aggregation_circuit_degree_bits": _common_degree_bits(root.circuit_data.common),
               "proof_bytes": len(rp),
               "note": "aggregate_chunk circuits (recursive verifier of 2 proofs on upstream's gate set, degree "
                       "2^13 at level 1), device "
                       "witness generation + batched GPU prove; one level = nl/2 chunks; tree = 4+2+1 proofs"}
    # BASELINE configs[3] as one measured pipeline (every rank, after the headline):
    # leaves -> per-GPU subtree root -> RCCL gather of the roots -> tree root on rank 0
    c3 = None
    if not voting and args.configs3 and args.mode == "e2e":
        c3 = configs3(args, circuit, prover, provers, cin, [inputs[first[i]:first[i] + per[i]] for i in range(NP)],
                      per, NP, B, dist, world, rank, local, torch, cdev)
    # standard_recursion_zk_config (the reference's cargo-bench and aggregator config):
    # under no_random it proves the same circuit without salts, one prover, one batch
    zk = None
    if rank == 0 and not voting and args.mode == "e2e":
        zc = qp_wormhole.Circuit.wormhole(zero_knowledge=True)
        zp = qp_wormhole.Prover(qp_wormhole.Context(local), zc, max_batch=per[0])
        zin = zp.inputs_array(inputs[:per[0]])
        zp.prove_inputs_array(zin, per[0])
        t1 = time.perf_counter()
        zproofs = zp.prove_inputs_array(zin, per[0])
        zdt = time.perf_counter() - t1
        zok = None
        if args.warmup:
            from oracle_lib import lib as olib
            zvd = zp.verifier_data()
            zok = olib().ora_verify(zvd, len(zvd), zproofs[0], len(zproofs[0])) == 0
        zk = {"proofs_per_s_1prover": per[0] / zdt, "proofs_per_launch": per[0], "proof_verified": zok,
              "note": "standard_recursion_zk_config, e2e, one prover (the headline runs --provers, default 3)"}
        zp.free()
    ref_parity = None
    if rank == 0 and not voting and args.mode == "e2e":
        ref_parity = reference_parity(qp_wormhole, local)
    shapes = None
    if rank == 0 and not voting and args.mode == "e2e" and args.ref_shapes:
        tr = time.perf_counter()
        shapes = {"prover_create_proof": cargo_bench_shape(qp_wormhole, local)}
        tc = time.perf_counter()
        shapes["aggregator"] = aggregator_shapes(qp_wormhole, local)
        ta = time.perf_counter()
        shapes["voting_configs4"] = voting_pass(qp_wormhole, local)
        shapes["wall_s"] = {"prover_create_proof": tc - tr, "aggregator": ta - tc,
                            "voting": time.perf_counter() - ta}
    if rank == 0:
        total = world * B * args.steps
        lde = ks["lde_wires"]
        achieved = lde["units"] / (lde["ms"] * 1e-3) / 1e9 if lde["ms"] else None
        leaf = ks["leaf_hash_wires"]
        rec = {
            "metric": "Voting proofs/sec (whole node)" if voting else "Wormhole proofs/sec (whole node)",
            "value": total / dt,
            "unit": "proofs/s",
            "n_gpus": world,
            "rccl_world_size": dist.get_world_size() if dist is not None else 1,
            "process_group_backend": dist.get_backend() if dist is not None else None,
            "rehearsal": "shared-GPU rehearsal of the N-rank path (gloo, every rank on cuda:0): not a measurement"
                         if rehearse else None,
            "leaf_proofs_gathered_per_step": gathered[-1] if gathered else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64 (Goldilocks field)",
            "data": f"synthetic seeded {circuit.kind} circuit inputs (SURVEY 8d), native circuit, "
                    f"standard_recursion_config; " + ("end to end: commit (host) + witness generation (device) + prove"
                                                      if args.mode == "e2e" else
                                                      "prove() from HBM-resident wire matrices"),
            "config": {"workload": f"batch{B}_{circuit.kind}_proofs_per_gpu",
                       "circuit": f"{circuit.kind} deg{circuit.degree_bits} (135 wires)",
                       "batch_per_gpu": B, "provers_per_gpu": NP, "host_threads_per_prover": host_threads,
                       "step_schedule": "pipelined" if (args.pipeline and NP > 1) else "joined per step",
                       "parallelism": f"proofs sharded x{world}, RCCL gather of leaf proofs"},
            "roofline": {"kernel": f"k_lde (wires LDE, 135 cols x 2^{circuit.degree_bits} -> "
                                   f"2^{circuit.degree_bits + 3})", "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None,
                         "traffic": pmc_traffic("qpk::k_lde_cosets<9>", circuit.num_wires, circuit.degree_bits,
                                                per[0]) if circuit.degree_bits == 13 else None,
                         "traffic_unit": "bytes per launch",
                         "algorithmic_bytes_per_launch": lde["units"] / max(lde["launches"], 1),
                         "traffic_source": f"{os.path.relpath(PMC_FILE, ROOT)} (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE "
                                           "passes of this bench at batch 128), per proof x proofs per launch",
                         "avg_launch_ms": lde["ms"] / max(lde["launches"], 1),
                         "note": "HIP events on the prover stream around each launch of the kernel"},
            "valu_kernels": {"leaf_hash_wires_perms_per_s": leaf["units"] / (leaf["ms"] * 1e-3) if leaf["ms"] else None,
                             "avg_launch_ms": leaf["ms"] / max(leaf["launches"], 1),
                             "quotient_avg_launch_ms": ks["quotient"]["ms"] / max(ks["quotient"]["launches"], 1),
                             # k_quotient_1r: one lane per LDE point; algorithmic = 8 (241 reads + 2 writes) per point
                             "quotient_hbm_bytes_per_launch": pmc_traffic(
                                 "qpk::k_quotient_1r", 0, 0, per[0], lanes_per_proof=8 << circuit.degree_bits)
                             if circuit.degree_bits == 13 else None,
                             "quotient_algorithmic_bytes_per_launch": per[0] * 8 * 243 * (8 << circuit.degree_bits)},
            "stage_ms_per_step": {k: v / args.steps for k, v in stages.items()},
            "proof_bytes": prover.proof_size,
            "latency_1proof_ms": lat,
            "zk_config": zk,
            "aggregation": agg,
            "configs3": c3,
            "prove_only_1prover_proofs_per_s": prove_only,
            "warmup_proof_verified": verified,
            "reference_proof_bytes_equal": ref_parity,
            "reference_bench_shapes": shapes,
        }
        if iso is not None and iso["lde_wires"]["ms"]:
            # with concurrent provers a launch's event-to-event time includes the
            # other prover's kernels; the kernel's own rate is the isolated pass
            il = iso["lde_wires"]
            ia = il["units"] / (il["ms"] * 1e-3) / 1e9
            rl = rec["roofline"]
            rl.update({"timed_region_achieved": rl["achieved"], "timed_region_avg_launch_ms": rl["avg_launch_ms"],
                       "achieved": ia, "frac": ia / HBM_PEAK_GBS,
                       "avg_launch_ms": il["ms"] / max(il["launches"], 1),
                       "algorithmic_bytes_per_launch": il["units"] / max(il["launches"], 1),
                       "note": f"achieved: the kernel alone (one prover, {per[0]} proofs per launch, HIP events on "
                               f"its stream, right after the timed region); timed_region_*: the same events during "
                               f"the timed region, where {NP} provers' kernels share the GPU"})
            lh, qk = iso["leaf_hash_wires"], iso["quotient"]
            if lh["ms"] and qk["ms"]:
                rec["valu_kernels"].update({"leaf_hash_wires_perms_per_s": lh["units"] / (lh["ms"] * 1e-3),
                                            "avg_launch_ms": lh["ms"] / max(lh["launches"], 1),
                                            "quotient_avg_launch_ms": qk["ms"] / max(qk["launches"], 1),
                                            "proofs_per_launch": per[0],
                                            "note": "isolated pass, as roofline.achieved; HBM bytes: PMC file"})
        vk = rec["valu_kernels"]
        ipp = perm_valu_instr()
        ksum, ksum1, ceil = load_json(KSUM_FILE), load_json(KSUM1_FILE), load_json(CEIL_FILE)
        if vk.get("leaf_hash_wires_perms_per_s") and ipp:
            ach = vk["leaf_hash_wires_perms_per_s"] / 64 * ipp
            rr = register_replay()
            rec["dominant_kernel"] = {
                "kernel": "k_leaf_hash (Poseidon Merkle leaves)", "bound": "valu",
                # one prover: kernels do not overlap, so shares are shares of GPU time
                "share_of_kernel_time": ksum1["leaf_hash_share"] if ksum1 else None,
                "achieved": ach, "peak": VALU_PEAK_WAVE_INSTR_S, "unit": "wave-instructions/s",
                "frac": ach / VALU_PEAK_WAVE_INSTR_S, "instr_per_perm": ipp,
                "mix_ceiling": mix_ceiling(ceil),
                "mix_ceiling_priced_at": "the calibration streams' clock" if ceil else None,
                "frac_of_mix_ceiling": ach / mix_ceiling(ceil) if ceil else None,
                # clock-consistent: the kernel's VALU rate and its ceiling re-priced
                # at its own clock, both from the same counter-pass dispatches
                "frac_of_mix_ceiling_at_own_clock": ceil.get("frac_of_ceiling_in_counter_pass") if ceil else None,
                "own_clock_ghz_in_counter_pass": ceil.get("leaf_hash_clock_ghz") if ceil else None,
                # the additive class model underprices this mix (frac > 1 above):
                # the loop replayed from registers is the ceiling that holds
                "frac_of_register_replay": rr["frac"] if rr else None,
                "register_replay": rr,
                "frac_of_ceiling": rr["frac"] if rr else None,
                "ceiling_kind": "the kernel's own instruction stream replayed from registers (tools/leaf_ubench L3 "
                                "vs L0, same run); mix_ceiling* = an additive per-class estimate",
                "sources": {"instr_per_perm": os.path.relpath(PMC_SQ_FILE, ROOT),
                            "mix_ceiling": os.path.relpath(CEIL_FILE, ROOT) if ceil else None,
                            "share": os.path.relpath(KSUM1_FILE, ROOT) if ksum1 else None,
                            "perms_per_s": "this run (HIP events, isolated pass)"},
                "note": "issue-bound 64-bit integer work (no MFMA path); peak = the guide's wave64 issue "
                        "(1 VALU instruction / 2 cycles / SIMD), which v_mad_u64_u32 (59% of the kernel's "
                        "VALU) does not reach: mix_ceiling = the kernel's instruction mix at the measured "
                        "saturated rate of each instruction class"}
        if ksum:
            rec["gpu_busy_frac"] = {"value": ksum["gpu_busy_frac"], "source": os.path.relpath(KSUM_FILE, ROOT),
                                    "scope": ksum.get("scope"),
                                    "note": "union of kernel intervals / window, rocprofv3 kernel trace of this bench "
                                            "(3 provers), cut to the timed steps by the trace markers"}
        rec["stage_ms_per_step"]["note"] = f"prover 0 ({per[0]} proofs), host + device"
        segregate_profile_fields(rec)
        if world == 1 and args.cpu_sample > 0:
            rec["cpu_baseline"] = cpu_baseline(circuit, inputs, args.cpu_sample, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    for p in provers:
        p.free()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
