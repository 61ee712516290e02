"""The N-rank bench path on the one-GPU test box: `bench.py --gpus 2
--rehearse-shared-gpu` starts two rank processes (the launcher), both prove on
cuda:0 and talk over gloo instead of RCCL, and rank 0's line carries the
gathered leaves of both ranks and the configs[3] root over both ranks'
subtrees.  Small batch: this checks the rank != 0 code (gathers, the
timing all-reduce, the roots gather and the top levels), not throughput
(profiles/r06_rehearse_gpus2_shared_gpu.json is the full-size run)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-shared-gpu",
                        "--batch", "8", "--provers", "2", "--steps", "1", "--warmup", "1", "--configs3-steps", "1",
                        "--cpu-sample", "0", "--ref-shapes", "0"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["rccl_world_size"] == 2
    assert rec["process_group_backend"] == "gloo" and rec["rehearsal"]
    assert rec["leaf_proofs_gathered_per_step"] == 2 * 8
    assert rec["warmup_proof_verified"] is True
    c3 = rec["configs3"]
    assert c3["leaves"] == 2 * 8 and c3["aggregation_proofs"] == 2 * 8 - 1
    assert c3["root_verified"] is True
