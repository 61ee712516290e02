#!/bin/bash
# GPU box session driver: each GPU step under its own timeout; stop at the
# first step that crashes/aborts/times out (exit >= 2 other than pytest's 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
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
# PMC passes over a short bench run, one counter group per pass (FETCH_SIZE
# takes 3 of the 4 TCC slots and WRITE_SIZE 2, so they need separate runs)
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step "pmc_$name" 300 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/pmc_$name" -o run -- \
    python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --provers 1 --batch 128 --configs3 0 --ref-shapes 0
}
for s in "$@"; do
  case $s in
    build) step build 600 make -s -C qp-zk-circuits-rm_amd/csrc -j16 ;;
    oracle) step oracle 300 make -s -C oracle ;;
    test) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kbench) step kbench 300 python tools/kbench.py 8 5 ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 tools/kbench.py 8 3 ;;
    bench) step bench 900 python bench.py ;;
    benchprof) step rocprof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 ;;
    benchprof1) step rocprof_bench1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --provers 1 ;;
    pmc_fetch) pmc fetch FETCH_SIZE ;;
    pmc_write) pmc write WRITE_SIZE ;;
    pmc_valu) pmc valu SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES ;;
    pmc_sq) pmc sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY ;;
    pmc_lds) pmc lds SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU ;;
    ab_threads) for r in 1 2; do
             step ab_thr_split_$r 300 python bench.py --cpu-sample 0 --steps 10 &&
             step ab_thr_def_$r 300 python bench.py --cpu-sample 0 --steps 10 --host-threads 0
           done ;;
    test_witness) step pytest_witness 600 python -u -m pytest tests/test_gpu_witness.py -x -v --timeout 300 --timeout-method thread ;;
    test_voting) step pytest_voting 300 python -u -m pytest tests/test_gpu_voting.py -x -v --timeout 120 --timeout-method thread ;;
    bench_voting) step bench_voting 600 python bench.py --circuit voting ;;
    benchprof_voting) step rocprof_bench_voting 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench_voting -o run -- python3 bench.py --circuit voting --steps 3 --warmup 1 --cpu-sample 0 ;;
    test_bins) step pytest_bins 600 python -u -m pytest tests/test_gpu_circuit_bins.py -x -v --timeout 300 --timeout-method thread ;;
    test_seams) step pytest_seams 600 python -u -m pytest tests/test_gpu_seams.py -x -v --timeout 300 --timeout-method thread ;;
    test_commit) step pytest_commit 600 python -u -m pytest tests/test_gpu_commit.py -x -v --timeout 300 --timeout-method thread ;;
    lde_ab) step prof_lde_new 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_new -o run -- python3 tools/kbench.py 16 3 &&
            export QPGPU_LDE_PERCOSET=1 && step prof_lde_old 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_old -o run -- python3 tools/kbench.py 16 3 && unset QPGPU_LDE_PERCOSET ;;
    ab_cw) for r in 1 2; do
             step ab_cw1_$r 300 python bench.py --cpu-sample 0 --steps 10 &&
             step ab_cw0_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_cw0.so python bench.py --cpu-sample 0 --steps 10
           done ;;
    isa) step isa_rates 300 tools/isa_rates ;;
    test_agg) step pytest_agg 900 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_guards.py -x -v --timeout 400 --timeout-method thread ;;
    test_ref) step pytest_ref 600 python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py -x -v --timeout 300 --timeout-method thread ;;
    gpus2) echo "=== gpus2 (expect a refusal: one GPU on this box)" | tee -a gpurun_out/session.log
           timeout -k 10 300 python -u bench.py --gpus 2 --steps 1 --warmup 0 > gpurun_out/gpus2.log 2>&1
           echo "=== gpus2 rc=$?" | tee -a gpurun_out/session.log; tail -5 gpurun_out/gpus2.log ;;
    shapes) step shapes 900 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --configs3 0 --agg-leaves 0 ;;
    benchfull) step benchfull 900 python -u bench.py --steps 20 --warmup 5 ;;
    qlazy) step pytest_q 900 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_aggregation.py tests/test_gpu_seam_prove.py -x -q --timeout 400 --timeout-method thread &&
           step bench5 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --ref-shapes 0 &&
           step agg_subtree 300 python -u tools/agg_subtree.py 256 2 &&
           step pmc_sqq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex "k_quotient|k_lde_cosets" --output-format csv -d gpurun_out/pmc_sqq -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --provers 1 --batch 128 --configs3 0 --agg-leaves 0 --ref-shapes 0 &&
           step pmc_sqq_sum 120 python3 tools/pmc_sq_summary.py gpurun_out/pmc_sqq gpurun_out/pmc_sqq.json && rm -rf gpurun_out/pmc_sqq ;;
    aggprofd) step prof_aggd 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aggd -o run -- python3 tools/agg_subtree.py 256 1 &&
              step aggd_sum 120 python3 tools/agg_trace.py gpurun_out/prof_aggd/run_kernel_trace.csv gpurun_out/agg_trace_default.json 5 &&
              step aggd_ksum 120 python3 tools/kernel_summary.py gpurun_out/prof_aggd/run_kernel_trace.csv gpurun_out/agg_kernel_summary_default.json "agg_subtree 256, default (4 concurrent sub-trees), timed pass" &&
              cp gpurun_out/prof_aggd/run_kernel_stats.csv gpurun_out/agg_default_kernel_stats.csv && rm -rf gpurun_out/prof_aggd ;;
    ldeocc) for r in 1 2; do
             step prof_lde_def_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_def_$r -o run -- python3 tools/kbench.py 86 3 &&
             step prof_lde_lds1_$r 300 env QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_lds1.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_lds1_$r -o run -- python3 tools/kbench.py 86 3 || exit 1
           done; for d in gpurun_out/prof_lde_*; do grep -h "k_lde_cosets\|k_intt\|Name" $d/run_kernel_stats.csv > $d.stats; rm -rf $d; done ;;
    ldeocc_sq) for v in def lds1; do
             if [ $v = def ]; then unset QPGPU_LIB; else export QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_$v.so; fi
             step pmc_lde_sq_$v 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex k_lde_cosets --output-format csv -d gpurun_out/pmc_lde_sq_$v -o run -- python3 tools/kbench.py 86 1 &&
             step pmc_lde_sum_$v 60 python3 tools/pmc_sq_summary.py gpurun_out/pmc_lde_sq_$v gpurun_out/pmc_lde_sq_$v.json && rm -rf gpurun_out/pmc_lde_sq_$v || exit 1
           done; unset QPGPU_LIB ;;
    bsync) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_bsync.so
           for r in 1 2; do
             step bs_agg_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step bs_agg_blk_$r 300 env QPGPU_LIB=$V python -u tools/agg_subtree.py 256 2 &&
             step bs_agg8_blk_$r 300 env QP_AGG_SPLIT=8 QPGPU_LIB=$V python -u tools/agg_subtree.py 256 2 || exit $?
           done
           step bs_bench_def 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 &&
           step bs_bench_blk 300 env QPGPU_LIB=$V python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 ;;
    hipapi) step prof_hipapi 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/prof_hipapi -o run -- python3 tools/agg_subtree.py 256 1 ;;
    votprof) step prof_vot 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vot -o run -- python3 bench.py --circuit voting --steps 2 --warmup 1 --cpu-sample 0 --ref-shapes 0 &&
             step vot_ksum 120 python3 tools/kernel_summary.py gpurun_out/prof_vot/run_kernel_trace.csv gpurun_out/vot_kernel_summary.json "bench voting batch 1024, 6 provers" &&
             step vot_trace 120 python3 tools/agg_trace.py gpurun_out/prof_vot/run_kernel_trace.csv gpurun_out/vot_trace.json ;;
    pyout) P=qp-zk-circuits-rm_amd/qp_wormhole/prover.py
           cp $P /tmp/prover_new.py
           for r in 1 2; do
             cp gpurun_ab_tmp/prover_old.py $P
             step py_old_w_$r 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
             step py_old_v_$r 300 python -u bench.py --circuit voting --steps 5 --cpu-sample 0 --ref-shapes 0 || { cp /tmp/prover_new.py $P; exit 1; }
             cp /tmp/prover_new.py $P
             step py_new_w_$r 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
             step py_new_v_$r 300 python -u bench.py --circuit voting --steps 5 --cpu-sample 0 --ref-shapes 0 || exit $?
           done ;;
    pyagg) P=qp-zk-circuits-rm_amd/qp_wormhole/prover.py
           cp $P /tmp/prover_new.py
           for r in 1 2; do
             cp gpurun_ab_tmp/prover_old.py $P
             step pa_old_$r 300 python -u tools/agg_subtree.py 256 2 || { cp /tmp/prover_new.py $P; exit 1; }
             cp /tmp/prover_new.py $P
             step pa_new_$r 300 python -u tools/agg_subtree.py 256 2 || exit $?
           done
           step pa_bench 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 ;;
    lattrace) step lat_plain 120 python -u tools/latency_trace.py 5 &&
              step prof_lat 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lat -o run -- python3 tools/latency_trace.py 5 &&
              step lat_ksum 120 python3 tools/kernel_summary.py gpurun_out/prof_lat/run_kernel_trace.csv gpurun_out/lat_kernel_summary.json "one proof at a time, 5 timed" &&
              step lat_trace 120 python3 tools/agg_trace.py gpurun_out/prof_lat/run_kernel_trace.csv gpurun_out/lat_trace.json 1 ;;
    latwit) for r in 1 2; do
              step lw_def_$r 120 python -u tools/latency_trace.py 8 &&
              step lw_lvl_$r 120 env QPGPU_PATHS=wit_mode=1 python -u tools/latency_trace.py 8 &&
              step lw_hc16_$r 120 env QPGPU_PATHS=host_chain=16 python -u tools/latency_trace.py 8 &&
              step lw_lvl_hc16_$r 120 env QPGPU_PATHS=wit_mode=1,host_chain=16 python -u tools/latency_trace.py 8 &&
              step lw_lvl_hc8_$r 120 env QPGPU_PATHS=wit_mode=1,host_chain=8 python -u tools/latency_trace.py 8 || exit $?
            done ;;
    witab) for r in 1 2; do
             step wa_w_def_$r 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
             step wa_w_lvl_$r 300 env QPGPU_PATHS=wit_mode=1 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
             step wa_v_def_$r 300 python -u bench.py --circuit voting --steps 5 --cpu-sample 0 --ref-shapes 0 &&
             step wa_v_lvl_$r 300 env QPGPU_PATHS=wit_mode=1 python -u bench.py --circuit voting --steps 5 --cpu-sample 0 --ref-shapes 0 || exit $?
           done ;;
    graphwit) step gw_tests 600 python -u -m pytest tests/test_gpu_witness.py tests/test_gpu_aggregation.py tests/test_gpu_reference_proof.py -x -q --timeout 400 --timeout-method thread &&
              step gw_lat 120 python -u tools/latency_trace.py 8 &&
              step gw_modes 400 python -u tools/wit_modes.py 1 4 16 32 &&
              step gw_agg 300 python -u tools/agg_subtree.py 256 2 &&
              step gw_afc 300 python -u tools/agg_first_call.py ;;
    q1rpm) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_q1rpm.so
           step qp_test 300 env QPGPU_LIB=$V python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py -x -q --timeout 200 --timeout-method thread &&
           for r in 1 2; do
             step qp_def_$r 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
             step qp_pm_$r 300 env QPGPU_LIB=$V python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 || exit $?
           done &&
           step qp_pmc_def 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_quotient_1r --output-format csv -d gpurun_out/qp_pmc_def -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --provers 1 --batch 128 --configs3 0 --ref-shapes 0 &&
           step qp_pmc_pm 300 env QPGPU_LIB=$V rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_quotient_1r --output-format csv -d gpurun_out/qp_pmc_pm -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --provers 1 --batch 128 --configs3 0 --ref-shapes 0 ;;
    qppm) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_qparts_pm.so
          step qpp_test 600 env QPGPU_LIB=$V python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_seams.py tests/test_gpu_prover.py -x -q --timeout 400 --timeout-method thread &&
          step qpp_test_def 300 python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_seams.py -x -q --timeout 300 --timeout-method thread &&
          for r in 1 2; do
            step qpp_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
            step qpp_pm_$r 300 env QPGPU_LIB=$V python -u tools/agg_subtree.py 256 2 || exit $?
          done ;;
    prevab) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_prev.so
            for r in 1 2 3; do
              step pv_new_$r 300 python -u bench.py --steps 10 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
              step pv_old_$r 300 env QPGPU_LIB=$V python -u bench.py --steps 10 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 || exit $?
            done ;;
    pm2) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_pm2.so
         step pm2_test 300 env QPGPU_LIB=$V python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_witness.py -x -q --timeout 300 --timeout-method thread &&
         for r in 1 2 3; do
           step pm2_def_$r 300 python -u bench.py --steps 10 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 &&
           step pm2_new_$r 300 env QPGPU_LIB=$V python -u bench.py --steps 10 --cpu-sample 0 --ref-shapes 0 --configs3 0 --agg-leaves 0 || exit $?
         done ;;
    check) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread &&
           step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
           step bench 900 python -u bench.py ;;
    pinned) V=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_pageable.so
            for r in 1 2; do
              step pin_agg_new_$r 300 python -u tools/agg_subtree.py 256 2 &&
              step pin_agg_old_$r 300 env QPGPU_LIB=$V python -u tools/agg_subtree.py 256 2 || exit $?
            done
            step pin_bench_new 300 python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 &&
            step pin_bench_old 300 env QPGPU_LIB=$V python -u bench.py --steps 5 --cpu-sample 0 --ref-shapes 0 ;;
    hwq) for r in 1 2; do
           step hwq_s4_q4_$r 300 python -u tools/agg_subtree.py 256 2 &&
           step hwq_s8_q4_$r 300 env QP_AGG_SPLIT=8 python -u tools/agg_subtree.py 256 2 &&
           step hwq_s8_q8_$r 300 env QP_AGG_SPLIT=8 GPU_MAX_HW_QUEUES=8 python -u tools/agg_subtree.py 256 2 &&
           step hwq_s4_q8_$r 300 env GPU_MAX_HW_QUEUES=8 python -u tools/agg_subtree.py 256 2 || exit $?
         done ;;
    powocc) for r in 1 2; do for v in pow6 pow5 pow7; do
             if [ $v = pow6 ]; then unset QPGPU_LIB; else export QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_$v.so; fi
             step prof_${v}_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${v}_$r -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --provers 1 --configs3 0 --agg-leaves 0 --ref-shapes 0 &&
             grep -h "k_pow_scan\|Name" gpurun_out/prof_${v}_$r/run_kernel_stats.csv > gpurun_out/prof_${v}_$r.stats && rm -rf gpurun_out/prof_${v}_$r || exit 1
           done; done; unset QPGPU_LIB
           for v in pow6 pow5; do
             if [ $v = pow6 ]; then unset QPGPU_LIB; else export QPGPU_LIB=qp-zk-circuits-rm_amd/qp_wormhole/variants/libqpgpu_$v.so; fi
             step vot_$v 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --ref-shapes 0 --cpu-sample 0 || exit 1
           done; unset QPGPU_LIB ;;
    bench5) step bench5 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 ;;
    agg_ab) step agg_dev2 300 python -u tools/agg_subtree.py 256 2 &&
            step agg_dev1 300 env QP_AGG_PROVERS=1 python -u tools/agg_subtree.py 256 2 &&
            step agg_host1 300 env QP_AGG_PROVERS=1 QP_AGG_WITNESS=host python -u tools/agg_subtree.py 256 2 &&
            step agg_dev2_generic 300 env QPGPU_QUOTIENT=rereads python -u tools/agg_subtree.py 256 2 ;;
    lde_modes) for r in 1 2; do for m in 0 1 2 3; do
             step prof_lde_m${m}_$r 300 env QPGPU_LDE_MODE=$m rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_m${m}_$r -o run -- python3 tools/kbench.py 16 3 || exit 1
           done; done ;;
    lde_pmc) for m in 0 3; do
             export QPGPU_LDE_MODE=$m
             step pmc_lde_fetch_m$m 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lde_fetch_m$m -o run -- python3 tools/kbench.py 16 1 &&
             step pmc_lde_sq_m$m 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_lde_sq_m$m -o run -- python3 tools/kbench.py 16 1 || exit 1
           done; unset QPGPU_LDE_MODE ;;
    aggprof) step prof_agg 300 env QP_AGG_PROVERS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_agg -o run -- python3 tools/agg_subtree.py 256 1 ;;
    aggpmc) step pmc_agg_wit 300 env QP_AGG_PROVERS=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex k_witness_gen --output-format csv -d gpurun_out/pmc_agg_wit -o run -- python3 tools/agg_subtree.py 256 1 ;;
    lde_batch) for nb in 16 43 86; do
             step prof_lde_b$nb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde_b$nb -o run -- python3 tools/kbench.py $nb 2 || exit 1
           done ;;
    wit_ab) step wit_def 300 python -u tools/agg_subtree.py 256 2 &&
            step wit_wp0 300 env QPGPU_LIB=gpurun_ab/libqpgpu_wp0.so python -u tools/agg_subtree.py 256 2 &&
            step wit_wp2 300 env QPGPU_LIB=gpurun_ab/libqpgpu_wp2.so python -u tools/agg_subtree.py 256 2 &&
            step wit_wp2_test 600 env QPGPU_LIB=gpurun_ab/libqpgpu_wp2.so python -u -m pytest tests/test_gpu_aggregation.py -x -q --timeout 400 --timeout-method thread ;;
    wit_ab2) step wit_t256 300 python -u tools/agg_subtree.py 256 2 &&
             step wit_t512 300 env QPGPU_WIT_THREADS=512 python -u tools/agg_subtree.py 256 2 &&
             step wit_t512_test 600 env QPGPU_WIT_THREADS=512 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_witness.py -x -q --timeout 400 --timeout-method thread ;;
    wit_prof) step prof_wit2 300 env QP_AGG_PROVERS=1 QPGPU_WIT_TWICE=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wit2 -o run -- python3 tools/agg_subtree.py 256 1 &&
              step agg_p4 300 env QP_AGG_PROVERS=4 python -u tools/agg_subtree.py 256 2 &&
              step agg_p3 300 env QP_AGG_PROVERS=3 python -u tools/agg_subtree.py 256 2 ;;
    coop_ab) step coop_def 300 python -u tools/agg_subtree.py 256 2 &&
             step coop_off 300 env QPGPU_WIT_COOP=0 python -u tools/agg_subtree.py 256 2 &&
             step coop_16 300 env QPGPU_WIT_COOP=16 python -u tools/agg_subtree.py 256 2 &&
             step coop_t512 300 env QPGPU_WIT_THREADS=512 python -u tools/agg_subtree.py 256 2 ;;
    lde_mulk) for r in 1 2; do
             step prof_lde86_def_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86_def_$r -o run -- python3 tools/kbench.py 86 2 &&
             step prof_lde86_mulk0_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_mulk0.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86_mulk0_$r -o run -- python3 tools/kbench.py 86 2 &&
             step prof_lde86_m1_$r 300 env QPGPU_LDE_MODE=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86_m1_$r -o run -- python3 tools/kbench.py 86 2 || exit 1
           done ;;
    aggpmc_q) step pmc_agg_q 300 env QP_AGG_PROVERS=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex k_quotient --output-format csv -d gpurun_out/pmc_agg_q -o run -- python3 tools/agg_subtree.py 256 1 ;;
    calib) step pmc_calib 600 bash tools/pmc_calib.sh ;;
    qgen_ab) for r in 1 2; do
             step qgen_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step qgen_qpc_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_qpc.so python -u tools/agg_subtree.py 256 2 &&
             step qgen_qpc3_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_qpc3.so python -u tools/agg_subtree.py 256 2 || exit 1
           done ;;
    lde_alds) for r in 1 2; do
             step prof_lde86b_def_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86b_def_$r -o run -- python3 tools/kbench.py 86 2 &&
             step prof_lde86b_alds3_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_alds3.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86b_alds3_$r -o run -- python3 tools/kbench.py 86 2 &&
             step prof_lde86b_alds2_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_alds2.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde86b_alds2_$r -o run -- python3 tools/kbench.py 86 2 || exit 1
           done &&
           step test_alds3 300 env QPGPU_LIB=gpurun_ab/libqpgpu_alds3.so python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 120 --timeout-method thread ;;
    agglog) step agg_subtree 300 python -u tools/agg_subtree.py 256 3 ;;
    qpart_ab) for r in 1 2; do
             step qpart_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step qpart_onepass_$r 300 env QPGPU_QUOTIENT=onepass python -u tools/agg_subtree.py 256 2 || exit 1
           done ;;
    qpart_prof) step prof_qpart 300 env QP_AGG_PROVERS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_qpart -o run -- python3 tools/agg_subtree.py 256 1 &&
                step prof_qone 300 env QP_AGG_PROVERS=1 QPGPU_QUOTIENT=onepass rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_qone -o run -- python3 tools/agg_subtree.py 256 1 ;;
    agglat) step agg_latency 300 python -u tools/agg_latency.py 1,2,4,8,16 5 ;;
    agglatprof) step prof_agglat 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_agglat -o run -- python3 tools/agg_latency.py 1,16 3 ;;
    test_seamprove) step pytest_seamprove 600 python -u -m pytest tests/test_gpu_seam_prove.py tests/test_gpu_seams.py -x -v --timeout 300 --timeout-method thread ;;
    aggthr) step agg_thr_def 300 python -u tools/agg_subtree.py 256 2 &&
            step agg_thr4 300 env QP_AGG_THREADS=4 python -u tools/agg_subtree.py 256 2 &&
            step agg_thr8 300 env QP_AGG_THREADS=8 python -u tools/agg_subtree.py 256 2 &&
            step agg_thr16_p1 300 env QP_AGG_PROVERS=1 python -u tools/agg_subtree.py 256 2 &&
            cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat > gpurun_out/cgroup.txt ;;
    c3q) step c3_q4 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --agg-leaves 0 &&
         step c3_q16 300 env GPU_MAX_HW_QUEUES=16 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --agg-leaves 0 ;;
    c3prio) step c3_prio0 300 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --agg-leaves 0 &&
            step c3_prio1 300 env QP_AGG_PRIORITY=1 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --agg-leaves 0 ;;
    aggtrace) step prof_aggsub 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_aggsub -o run -- python3 tools/agg_subtree.py 256 2 ;;
    qprefix) step pytest_qprefix 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_seams.py tests/test_gpu_seam_prove.py -x -q --timeout 400 --timeout-method thread &&
             for r in 1 2; do
               step qp_new_$r 300 python -u tools/agg_subtree.py 256 2 &&
               step qp_off_$r 300 env QPGPU_QPREFIX=0 python -u tools/agg_subtree.py 256 2 &&
               step qp_w3_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_qpw3.so python -u tools/agg_subtree.py 256 2 || exit 1
             done &&
             step prof_qprefix 300 env QP_AGG_PROVERS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_qprefix -o run -- python3 tools/agg_subtree.py 256 1 &&
             step prof_qoff 300 env QP_AGG_PROVERS=1 QPGPU_QPREFIX=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_qoff -o run -- python3 tools/agg_subtree.py 256 1 ;;
    ilv) step pytest_ilv 900 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_aggregation.py tests/test_gpu_seams.py -x -q --timeout 400 --timeout-method thread &&
         for r in 1 2; do
           step prof_ilv1_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ilv1_$r -o run -- python3 tools/kbench.py 86 2 &&
           step prof_ilv0_$r 300 env QPGPU_LIB=gpurun_ab/libqpgpu_ilv0.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ilv0_$r -o run -- python3 tools/kbench.py 86 2 || exit 1
         done &&
         step bench_ilv1 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 &&
         step bench_ilv0 300 env QPGPU_LIB=gpurun_ab/libqpgpu_ilv0.so python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 ;;
    mcoop) step pytest_mcoop 900 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_aggregation.py tests/test_gpu_seams.py tests/test_gpu_witness.py -x -q --timeout 400 --timeout-method thread &&
           step agglat_coop 300 python -u tools/agg_latency.py 1,2,4,8,16 5 &&
           step agglat_nocoop 300 env QPGPU_MERKLE_COOP=0 python -u tools/agg_latency.py 1,2,4,8,16 5 &&
           for r in 1 2; do
             step sub_coop_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step sub_nocoop_$r 300 env QPGPU_MERKLE_COOP=0 python -u tools/agg_subtree.py 256 2 || exit 1
           done &&
           step bench_coop 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 &&
           step bench_nocoop 300 env QPGPU_MERKLE_COOP=0 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 ;;
    leafub) step leaf_ubench 300 tools/leaf_ubench 86 5 ;;
    witrow) step pytest_witrow 900 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_witness.py tests/test_gpu_reference_proof.py -x -q --timeout 400 --timeout-method thread &&
            step wr_lat_new 300 python -u tools/agg_latency.py 1,8,32 5 &&
            step wr_lat_off 300 env QPGPU_WIT_ROW=0 python -u tools/agg_latency.py 1,8,32 5 &&
            step wr_sub_new 300 python -u tools/agg_subtree.py 256 2 &&
            step wr_sub_off 300 env QPGPU_WIT_ROW=0 python -u tools/agg_subtree.py 256 2 &&
            step wr_sub_new2 300 python -u tools/agg_subtree.py 256 2 &&
            step wr_bench 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 &&
            step wr_bench_off 600 env QPGPU_WIT_ROW=0 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 ;;
    agg32prof) step prof_agg32 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_agg32 -o run -- python3 tools/agg_latency.py 32 3 ;;
    split) step pytest_split 900 python -u -m pytest tests/test_gpu_aggregation.py tests/test_distributed.py -x -q --timeout 400 --timeout-method thread &&
           step sp_sub_2 300 python -u tools/agg_subtree.py 256 3 &&
           step sp_sub_1 300 env QP_AGG_SPLIT=1 python -u tools/agg_subtree.py 256 3 &&
           step sp_sub_4 300 env QP_AGG_SPLIT=4 QP_AGG_PROVERS=4 python -u tools/agg_subtree.py 256 3 &&
           step sp_sub_4p2 300 env QP_AGG_SPLIT=4 python -u tools/agg_subtree.py 256 3 &&
           step sp_bench 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 ;;
    split4) step pytest_split4 900 python -u -m pytest tests/test_gpu_aggregation.py -x -q --timeout 400 --timeout-method thread &&
           step sp4_sub 300 python -u tools/agg_subtree.py 256 3 &&
           step sp4_sub_8 300 env QP_AGG_SPLIT=8 python -u tools/agg_subtree.py 256 3 &&
           step sp4_sub_4p3 300 env QP_AGG_PROVERS=3 python -u tools/agg_subtree.py 256 3 &&
           step sp4_bench 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 ;;
    qrest) step pytest_qrest 900 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_seams.py tests/test_gpu_seam_prove.py -x -q --timeout 400 --timeout-method thread &&
           step qr_lat_1 300 python -u tools/agg_latency.py 1,8,32 5 &&
           step qr_lat_0 300 env QPGPU_QREST=0 python -u tools/agg_latency.py 1,8,32 5 &&
           step qr_lat_2 300 env QPGPU_QREST=2 python -u tools/agg_latency.py 1,8,32 5 &&
           step qr_sub_1 300 python -u tools/agg_subtree.py 256 3 &&
           step qr_sub_0 300 env QPGPU_QREST=0 python -u tools/agg_subtree.py 256 3 &&
           step qr_sub_2 300 env QPGPU_QREST=2 python -u tools/agg_subtree.py 256 3 &&
           step prof_qr1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_qr1 -o run -- python3 tools/agg_latency.py 32 3 &&
           step prof_qr2 300 env QPGPU_QREST=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_qr2 -o run -- python3 tools/agg_latency.py 32 3 &&
           step prof_qr0 300 env QPGPU_QREST=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_qr0 -o run -- python3 tools/agg_latency.py 32 3 ;;
    splitab) for r in 1 2; do
             step sab_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step sab_m8k_$r 300 env QPGPU_MERKLE_COOP=8192 python -u tools/agg_subtree.py 256 2 &&
             step sab_m2k_$r 300 env QPGPU_MERKLE_COOP=2048 python -u tools/agg_subtree.py 256 2 &&
             step sab_wg_$r 300 env QPGPU_WIT_MODE=wg python -u tools/agg_subtree.py 256 2 &&
             step sab_fri2k_$r 300 env QPGPU_FRI_ROW=2048 python -u tools/agg_subtree.py 256 2 &&
             step sab_lde0_$r 300 env QPGPU_LDE_FEW=0 python -u tools/agg_subtree.py 256 2 &&
             step sab_open1_$r 300 env QPGPU_OPEN_SLICES=1 python -u tools/agg_subtree.py 256 2 || exit 1
             done ;;
    qrestpmc) for m in 0 1 2; do
             step pmc_qr${m}_fetch 300 env QPGPU_QREST=$m rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_quotient --output-format csv -d gpurun_out/pmc_qr${m}_fetch -o run -- python3 tools/agg_latency.py 32 2 &&
             step pmc_qr${m}_write 300 env QPGPU_QREST=$m rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_quotient --output-format csv -d gpurun_out/pmc_qr${m}_write -o run -- python3 tools/agg_latency.py 32 2 || exit 1
             done ;;
    provab) for r in 1 2; do
             step pv3_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
             step pv4_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 --provers 4 &&
             step pv2_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 --provers 2 || exit 1
             done ;;
    final6) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread &&
            step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
            step bench 900 python -u bench.py &&
            step rocprof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --ref-shapes 0 &&
            step rocprof_bench1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --provers 1 --ref-shapes 0 &&
            pmc fetch FETCH_SIZE && pmc write WRITE_SIZE &&
            pmc sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY &&
            step pmc_calib 600 bash tools/pmc_calib.sh &&
            step prof_agg 300 env QP_AGG_PROVERS=1 QP_AGG_SPLIT=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_agg -o run -- python3 tools/agg_subtree.py 256 1 &&
            step prof_aggd 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aggd -o run -- python3 tools/agg_subtree.py 256 1 &&
            step leaf_ubench 300 tools/leaf_ubench 86 5 &&
            step agg_subtree 300 python -u tools/agg_subtree.py 256 3 &&
            step bench_voting 600 python -u bench.py --circuit voting &&
            step final_summaries 300 bash tools/final_summaries.sh r06 ;;
    final5) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread &&
            step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
            step bench 900 python -u bench.py &&
            step rocprof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 &&
            step rocprof_bench1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --provers 1 &&
            pmc fetch FETCH_SIZE && pmc write WRITE_SIZE &&
            pmc sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY &&
            step pmc_calib 600 bash tools/pmc_calib.sh &&
            step prof_agg 300 env QP_AGG_PROVERS=1 QP_AGG_SPLIT=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_agg -o run -- python3 tools/agg_subtree.py 256 1 &&
            step leaf_ubench 300 tools/leaf_ubench 86 5 &&
            step agg_subtree 300 python -u tools/agg_subtree.py 256 3 &&
            step bench_voting 600 python -u bench.py --circuit voting &&
            step final_summaries 300 bash tools/final_summaries.sh r05 ;;
    votab) step vot_def 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 &&
           step vot_split 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --host-threads -1 &&
           step vot_p2 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --provers 2 &&
           step vot_p4 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --provers 4 &&
           step vot_prof 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_vot -o run -- python3 bench.py --circuit voting --steps 3 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step vot_sum 120 python3 tools/kernel_summary.py gpurun_out/prof_vot/run_kernel_trace.csv gpurun_out/vot_ksum.json "voting bench, 3 provers" &&
           rm -rf gpurun_out/prof_vot ;;
    votab2) for r in 1 2; do
           step vot3_$r 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 &&
           step vot4_$r 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --provers 4 &&
           step vot6_$r 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --provers 6 &&
           step vot8_$r 600 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 --provers 8 || exit 1
           done ;;
    powab) step pytest_pow 600 python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_voting.py -x -q --timeout 300 --timeout-method thread &&
           for r in 1 2; do
           step pw1_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step pw0_$r 300 env QPGPU_POW_WAVE=0 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step vw1_$r 300 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 &&
           step vw0_$r 300 env QPGPU_POW_WAVE=0 python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 || exit 1
           done ;;
    cptab) step pytest_cpt 600 env QPGPU_POW_CPT=4 python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_voting.py -x -q --timeout 300 --timeout-method thread &&
           for r in 1 2; do for c in 1 2 4; do
           step cl${c}_$r 300 env QPGPU_POW_CPT=$c python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step cv${c}_$r 300 env QPGPU_POW_CPT=$c python -u bench.py --circuit voting --agg-leaves 0 --configs3 0 || exit 1
           done; done ;;
    nbatab) for r in 1 2; do
           step nb32_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step nb128_$r 300 env QPGPU_MERKLE_NBAT=128 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
           step nb128c8_$r 300 env QPGPU_MERKLE_NBAT=128 QPGPU_MERKLE_COOP=12000 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 || exit 1
           done ;;
    witab3) for r in 1 2; do
             step w3_def_$r 300 python -u tools/agg_subtree.py 256 2 &&
             step w3_lev_$r 300 env QPGPU_WIT_MODE=levels python -u tools/agg_subtree.py 256 2 &&
             step w3_t256_$r 300 env QPGPU_WIT_THREADS=256 python -u tools/agg_subtree.py 256 2 || exit 1
             done ;;
    wlab) step pytest_wl 900 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_seams.py -x -q --timeout 400 --timeout-method thread &&
          for r in 1 2; do
          step wl_kb1_$r 300 python -u tools/kbench.py 16 5 &&
          step wl_kb0_$r 300 env QPGPU_LIB=ab_libs/libqpgpu_wl0.so python -u tools/kbench.py 16 5 &&
          step wl_b1_$r 300 python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 &&
          step wl_b0_$r 300 env QPGPU_LIB=ab_libs/libqpgpu_wl0.so python -u bench.py --steps 10 --warmup 1 --cpu-sample 0 --agg-leaves 0 --configs3 0 || exit 1
          done ;;
    wlprof) for r in 1 2; do
          step wlp1_$r 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wlp1_$r -o run -- python3 tools/kbench.py 32 5 &&
          step wlp0_$r 300 env QPGPU_LIB=ab_libs/libqpgpu_wl0.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wlp0_$r -o run -- python3 tools/kbench.py 32 5 || exit 1
          done &&
          step wlsq1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex k_lde_cosets --output-format csv -d gpurun_out/wlsq1 -o run -- python3 tools/kbench.py 32 2 &&
          step wlsq0 300 env QPGPU_LIB=ab_libs/libqpgpu_wl0.so rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex k_lde_cosets --output-format csv -d gpurun_out/wlsq0 -o run -- python3 tools/kbench.py 32 2 ;;
    esprof) step pytest_es 900 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_seams.py -x -q --timeout 400 --timeout-method thread &&
          for r in 1 2; do
          step esp1_$r 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/esp1_$r -o run -- python3 tools/kbench.py 32 5 &&
          step esp0_$r 300 env QPGPU_LIB=ab_libs/libqpgpu_es0.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/esp0_$r -o run -- python3 tools/kbench.py 32 5 &&
          step espw_$r 300 env QPGPU_LIB=ab_libs/libqpgpu_wl0.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/espw_$r -o run -- python3 tools/kbench.py 32 5 || exit 1
          done ;;
    lat5) step pytest_lat5 900 python -u -m pytest tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_aggregation.py tests/test_gpu_seams.py tests/test_gpu_seam_prove.py -x -q --timeout 400 --timeout-method thread &&
          step lat_new 300 python -u tools/agg_latency.py 1,2,4,8,16,32 5 &&
          step lat_off 300 env QPGPU_MERKLE_ROW=0 QPGPU_FRI_ROW=0 QPGPU_OPEN_SLICES=1 QPGPU_LDE_FEW=0 python -u tools/agg_latency.py 1,2,4,8,16,32 5 &&
          step lat_nomrow 300 env QPGPU_MERKLE_ROW=0 python -u tools/agg_latency.py 1,8,32 5 &&
          step lat_nofri 300 env QPGPU_FRI_ROW=0 python -u tools/agg_latency.py 1,8,32 5 &&
          step lat_noopen 300 env QPGPU_OPEN_SLICES=1 python -u tools/agg_latency.py 1,8,32 5 &&
          step lat_nolde 300 env QPGPU_LDE_FEW=0 python -u tools/agg_latency.py 1,8,32 5 &&
          step sub_new 300 python -u tools/agg_subtree.py 256 2 &&
          step sub_off 300 env QPGPU_MERKLE_ROW=0 QPGPU_FRI_ROW=0 QPGPU_OPEN_SLICES=1 QPGPU_LDE_FEW=0 python -u tools/agg_subtree.py 256 2 &&
          step sub_m8k 300 env QPGPU_MERKLE_COOP=8192 python -u tools/agg_subtree.py 256 2 &&
          step sub_m32k 300 env QPGPU_MERKLE_COOP=32768 python -u tools/agg_subtree.py 256 2 &&
          step bench_lat5 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 ;;
    leaft) step pytest_leaft 600 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_reference_proof.py tests/test_gpu_prover.py tests/test_gpu_voting.py -x -q --timeout 400 --timeout-method thread &&
           for r in 1 2; do
             step prof_leaft1_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_leaft1_$r -o run -- python3 tools/kbench.py 86 2 &&
             step prof_leaft0_$r 300 env QPGPU_LEAF_T=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_leaft0_$r -o run -- python3 tools/kbench.py 86 2 || exit 1
           done &&
           for r in 1 2; do
             step bench_leaft1_$r 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 &&
             step bench_leaft0_$r 300 env QPGPU_LEAF_T=0 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --configs3 0 --agg-leaves 0 || exit 1
           done ;;
    witlev) step pytest_witlev 900 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_witness.py tests/test_gpu_seam_prove.py -x -q --timeout 400 --timeout-method thread &&
            step agglat_lev 300 python -u tools/agg_latency.py 1,2,4,8,16,32 5 &&
            step agglat_wg 300 env QPGPU_WIT_MODE=wg python -u tools/agg_latency.py 1,2,4,8,16,32 5 &&
            for r in 1 2; do
              step sub_lev_$r 300 python -u tools/agg_subtree.py 256 2 &&
              step sub_wg_$r 300 env QPGPU_WIT_MODE=wg python -u tools/agg_subtree.py 256 2 || exit 1
            done ;;
    *) echo "unknown step $s" ;;
  esac
done
