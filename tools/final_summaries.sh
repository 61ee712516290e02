#!/bin/bash
# Summaries of a `gpu_session.sh final5` run, made on the GPU box so only
# small files come back (gpurun copies at most 64 MiB of gpurun_out/): kernel
# summaries of the bench traces (3 provers, 1 prover) and of the aggregation
# subtree, the HBM and SQ PMC summaries, the issue ceiling and the rocprofv3
# --stats tables; the raw traces and counter CSVs are deleted afterwards.
# Usage: bash tools/final_summaries.sh <tag>   (writes gpurun_out/final/<tag>_*)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
tag=${1:-r05}
o=gpurun_out/final
mkdir -p $o
set -e
python3 tools/kernel_summary.py gpurun_out/prof_bench/run_kernel_trace.csv $o/${tag}_kernel_summary_3provers.json "bench, 3 provers"
python3 tools/kernel_summary.py gpurun_out/prof_bench1/run_kernel_trace.csv $o/${tag}_kernel_summary_1prover.json "bench, 1 prover"
python3 tools/kernel_summary.py gpurun_out/prof_agg/run_kernel_trace.csv $o/${tag}_agg_kernel_summary.json "agg_subtree 256, 1 level prover, level by level"
if [ -d gpurun_out/prof_aggd ]; then
  python3 tools/kernel_summary.py gpurun_out/prof_aggd/run_kernel_trace.csv $o/${tag}_agg_kernel_summary_default.json "agg_subtree 256, default (4 concurrent sub-trees), timed pass"
  python3 tools/agg_trace.py gpurun_out/prof_aggd/run_kernel_trace.csv $o/${tag}_agg_trace_default.json 5
  cp gpurun_out/prof_aggd/run_kernel_stats.csv $o/${tag}_rocprof_agg_subtree_default_kernel_stats.csv
fi
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write $o/${tag}_pmc_hbm_b128.json > /dev/null
python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq $o/${tag}_pmc_sq_b128.json > /dev/null
python3 tools/issue_ceiling.py gpurun_out/calib_isa $o/${tag}_issue_ceiling.json gpurun_out/calib_kb > /dev/null
cp gpurun_out/prof_bench/run_kernel_stats.csv $o/${tag}_rocprof_bench_b256_3provers_kernel_stats.csv
cp gpurun_out/prof_bench1/run_kernel_stats.csv $o/${tag}_rocprof_bench_b256_1prover_kernel_stats.csv
cp gpurun_out/prof_agg/run_kernel_stats.csv $o/${tag}_rocprof_agg_subtree_kernel_stats.csv
rm -rf gpurun_out/prof_bench gpurun_out/prof_bench1 gpurun_out/prof_agg gpurun_out/prof_aggd gpurun_out/pmc_fetch gpurun_out/pmc_write \
       gpurun_out/pmc_sq gpurun_out/calib_isa gpurun_out/calib_kb
echo summaries ok
