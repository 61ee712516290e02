#!/bin/bash
# PMC A/B of the commit path (tools/kbench.py) over library variants, one
# rocprofv3 --pmc pass per (variant, counter group).
# Usage (GPU box): bash tools/pmc_ab.sh "<counters>" name1 lib1 [name2 lib2 ...]   (lib "" = default build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ctrs=$1; shift
dirs=""
while [ $# -ge 2 ]; do
  name=$1; lib=$2; shift 2
  echo "=== pmc $name ($lib): $ctrs"
  ( [ -n "$lib" ] && export QPGPU_LIB=$lib
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "gpurun_out/pmc_$name" -o run -- \
      python3 tools/kbench.py 8 1 > "gpurun_out/pmc_$name.log" 2>&1 )
  rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc_$name.log"; exit $rc; fi
  dirs="$dirs gpurun_out/pmc_$name"
done
python3 tools/pmc_kernels.py $dirs
