cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
QPGPU_LIB=gpurun_ab/libqpgpu_pm10.so timeout -k 10 600 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pm10_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pm10_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pm10_pytest.log
bash tools/ab_kbench.sh 16 base "" pm10 "QPGPU_LIB=gpurun_ab/libqpgpu_pm10.so" pm10w7 "QPGPU_LIB=gpurun_ab/libqpgpu_pm10w7.so" > gpurun_out/ab_summary.txt 2>&1
