#!/bin/bash
# A/B of a variant library on the full prover: parity tests with the variant,
# then alternating benches (variant, in-tree, variant, in-tree).
# Usage (GPU box): bash tools/ab_bench_lib.sh gpurun_ab/libqpgpu_X.so NAME
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
lib=$1; name=$2
QPGPU_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_prover.py tests/test_gpu_reference_proof.py tests/test_gpu_seams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_${name}_pytest.log 2>&1 || { tail -30 gpurun_out/ab_${name}_pytest.log; exit 1; }
tail -1 gpurun_out/ab_${name}_pytest.log
for r in 1 2; do
  QPGPU_LIB=$lib timeout -k 10 600 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/ab_${name}_$r.log 2>&1 || exit 1
  echo "$name $r: $(grep -o '"value": [0-9.]*\|"quotient_avg_launch_ms": [0-9.]*' gpurun_out/ab_${name}_$r.log | head -2 | tr '\n' ' ')"
  timeout -k 10 600 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/ab_base_$r.log 2>&1 || exit 1
  echo "base $r: $(grep -o '"value": [0-9.]*\|"quotient_avg_launch_ms": [0-9.]*' gpurun_out/ab_base_$r.log | head -2 | tr '\n' ' ')"
done
