cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_agg.log 2>&1 || { echo "agg tests rc=$?"; tail -20 gpurun_out/pytest_agg.log; exit 1; }
tail -3 gpurun_out/pytest_agg.log
bash tools/ab_bench.sh base "" qs8 gpurun_ab/libqpgpu_qs8.so qs12 gpurun_ab/libqpgpu_qs12.so > gpurun_out/ab_qstash.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_qstash.log; exit 1; }
tail -30 gpurun_out/ab_qstash.log
