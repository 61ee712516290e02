#!/bin/bash
# LDE A/B: parity of a variant library (commit tests: LDE log_n 1..14 vs the
# oracle), then commit-path kernel timings of the in-tree library vs the variant.
# Usage (GPU box): bash tools/ab_lde.sh gpurun_ab/libqpgpu_X.so NAME
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
lib=$1; name=$2
QPGPU_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_${name}_pytest.log 2>&1 || { tail -30 gpurun_out/ab_${name}_pytest.log; exit 1; }
tail -1 gpurun_out/ab_${name}_pytest.log
bash tools/ab_kbench.sh 16 base "" $name "QPGPU_LIB=$lib" > gpurun_out/ab_summary.txt 2>&1
