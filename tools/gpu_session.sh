#!/bin/bash
# GPU box session driver: each GPU step under its own timeout; stop at the
# first step that crashes/aborts/times out (exit >= 2 other than pytest's 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    build) step build 600 make -s -C qp-zk-circuits-rm_amd/csrc -j16 ;;
    oracle) step oracle 300 make -s -C oracle ;;
    test) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    kbench) step kbench 300 python tools/kbench.py 8 5 ;;
    prof) export TMPDIR=/tmp; step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 tools/kbench.py 8 3 ;;
    bench) step bench 900 python bench.py ;;
    benchprof) export TMPDIR=/tmp; step rocprof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 ;;
    *) echo "unknown step $s" ;;
  esac
done
