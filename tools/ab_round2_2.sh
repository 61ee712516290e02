set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh test_commit
bash tools/ab_kbench.sh 64 r8 "" r16 "QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_r16.so"
bash tools/pmc_ab.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY" r8 "" r16 qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_r16.so
