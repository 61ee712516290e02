#!/bin/bash
# PMC passes over the commit-path micro-bench (VALU / LDS / wait cycles of the
# NTT and Poseidon kernels), one counter group per rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_ab.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" g1 "" &&
bash tools/pmc_ab.sh "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" g2 ""
