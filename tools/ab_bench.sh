#!/bin/bash
# A/B kernel timing of the full prover (bench.py, one prover, 2 steps) under
# rocprofv3 --kernel-trace, one run per library variant.
# Usage (GPU box): bash tools/ab_bench.sh name1 lib1 [name2 lib2 ...]   (lib "" = default build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
dirs=""
while [ $# -ge 2 ]; do
  name=$1; lib=$2; shift 2
  echo "=== ab $name ($lib)"
  ( [ -n "$lib" ] && export QPGPU_LIB=$lib
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/abb_$name" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --provers 1 > "gpurun_out/abb_$name.log" 2>&1 )
  rc=$?
  echo "=== ab $name rc=$rc"
  grep -o '"value": [0-9.]*' "gpurun_out/abb_$name.log" | head -1
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/abb_$name.log"; exit $rc; fi
  dirs="$dirs gpurun_out/abb_$name"
done
python3 tools/trace_summary.py $(for d in $dirs; do echo $d/run_kernel_trace.csv; done)
