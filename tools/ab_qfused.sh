# A/B of the opt-in fused quotient kernel (QPGPU_QUOTIENT=fused) against k_quotient_1r: parity tests, then two benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_prover.py tests/test_gpu_reference_proof.py tests/test_gpu_seams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qf_pytest.log 2>&1 || { tail -30 gpurun_out/qf_pytest.log; exit 1; }
tail -2 gpurun_out/qf_pytest.log
QPGPU_QUOTIENT=fused timeout -k 10 600 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/qf_fused.log 2>&1 && grep -o '"value": [0-9.]*\|"quotient_avg_launch_ms": [0-9.]*' gpurun_out/qf_fused.log
timeout -k 10 600 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/qf_nofuse.log 2>&1 && grep -o '"value": [0-9.]*\|"quotient_avg_launch_ms": [0-9.]*' gpurun_out/qf_nofuse.log
