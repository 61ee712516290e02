#!/bin/bash
# A/B of bench.py's headline value (default 2 provers) over library variants.
# Usage (GPU box): bash tools/ab_value.sh "<bench args>" name1 lib1 [name2 lib2 ...]   (lib "" = default build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
args=$1; shift
while [ $# -ge 2 ]; do
  name=$1; lib=$2; shift 2
  ( [ -n "$lib" ] && export QPGPU_LIB=$lib
    timeout -k 10 300 python3 bench.py $args --cpu-sample 0 > "gpurun_out/abv_$name.log" 2>&1 )
  rc=$?
  echo "=== $name rc=$rc $(grep -o '"value": [0-9.]*' "gpurun_out/abv_$name.log" | head -1) $(grep -o '"pow": [0-9.]*' "gpurun_out/abv_$name.log")"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/abv_$name.log"; exit $rc; fi
done
