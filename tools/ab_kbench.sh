#!/bin/bash
# A/B kernel timing of the commit path under rocprofv3, one run per variant.
# Usage (on the GPU box): bash tools/ab_kbench.sh NBAT name1 "ENV=.. ENV2=.." name2 "..." ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
nbat=$1; shift
while [ $# -ge 2 ]; do
  name=$1; envs=$2; shift 2
  echo "=== ab $name: $envs" | tee -a gpurun_out/session.log
  ( for kv in $envs; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/ab_$name" -o run -- \
      python3 tools/kbench.py "$nbat" 3 > "gpurun_out/ab_$name.log" 2>&1 )
  rc=$?
  echo "=== ab $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab_$name.log"; exit $rc; fi
done
python3 tools/trace_summary.py gpurun_out/ab_*/run_kernel_trace.csv
