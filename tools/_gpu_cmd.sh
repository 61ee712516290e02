cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh test || exit 3
bash tools/ab_bench.sh p32 '' nop32 qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_nop32.so > gpurun_out/abb4.log 2>&1 || exit 4
bash tools/gpu_session.sh bench
