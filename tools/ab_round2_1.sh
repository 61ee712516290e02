set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh test
bash tools/ab_kbench.sh 64 carry "" branch "QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_ntt0.so"
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_q1r.log 2>&1
QPGPU_QUOTIENT=rereads timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_qold.log 2>&1
grep -o '"value": [0-9.]*\|"quotient_avg_launch_ms": [0-9.]*\|"achieved": [0-9.]*' gpurun_out/b_q1r.log gpurun_out/b_qold.log
