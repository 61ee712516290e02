#!/bin/bash
# Issue-rate calibration: the same SQ + GRBM counters over the ISA microbench
# (saturated single-instruction kernels) and the commit path (k_leaf_hash), so
# the leaf hash's VALU issue is compared with a measured ceiling in the same
# units.  One counter pass per program (8 SQ + 2 GRBM, within the per-pass limits).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/calib_isa -o run -- tools/isa_chains > gpurun_out/calib_isa.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/calib_kb -o run -- python3 tools/kbench.py 16 1 > gpurun_out/calib_kb.log 2>&1 || exit $?
echo calib ok
