#!/bin/bash
# The GPU steps of this round's runs, by name:  tools/gpu_suite.sh STEP [STEP ...]
# Each step runs under its own time limit through tools/gpu_step.sh (log: gpurun_out/STEP.log);
# the suite stops at the first step that fails, times out or faults.
#   gpurun -- 'tools/gpu_suite.sh tests smoke bench profbench pmc'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
run() { tools/gpu_step.sh "$@" || exit $?; }
for s in "$@"; do
  case $s in
    tests)      run tests 900 $T tests ;;
    t_zw)       run t_zw 400 $T tests/test_gpu_headline.py tests/test_gpu_epochs.py tests/test_gpu_ordered_frontier.py tests/test_gpu_parity.py ;;
    t_ff)       run t_ff 600 $T tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_runs.py tests/test_gpu_sharded.py tests/test_gpu_ordered_frontier.py tests/test_gpu_epochs.py -k "ff or FF or keyed or headline or config5 or sharded" ;;
    b_c3ff)     run b_c3ff 150 python bench.py --mode ca_ff --hosts 100000 --tasks 1000 $NB ;;
    t_ffe)      run t_ffe 500 $T tests/test_gpu_ff_epochs.py ;;
    t_runs)     run t_runs 400 $T tests/test_gpu_runs.py ;;
    t_vbp)      run t_vbp 400 $T tests/test_gpu_band.py tests/test_gpu_headline.py tests/test_gpu_parity.py -k "vbp or VBP or band or headline or config5" ;;
    t_opp)      run t_opp 500 $T tests/test_gpu_opp_walk.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sharded.py tests/test_gpu_batch.py -k "opp or OPP or opportunistic" ;;
    t_multi)    run t_multi 600 $T tests/test_bench_multirank.py tests/test_gpu_batch.py ;;
    smoke)      run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)      run bench 400 python bench.py ;;
    b_cabf)     run b_cabf 150 python bench.py $NB --steps 20 ;;
    b_vbpff)    run b_vbpff 150 python bench.py --mode vbp_ff $NB ;;
    b_caff)     run b_caff 150 python bench.py --mode ca_ff $NB ;;
    b_vbpbf)    run b_vbpbf 200 python bench.py --mode vbp_bf $NB ;;
    b_vbpbf1)   PVT_AHEAD=1 run b_vbpbf1 200 python bench.py --mode vbp_bf $NB ;;
    b_prof)     for m in ${BM:-vbp_bf ca_bf}; do BENCH_PROF=0 run b_p0_$m 200 python bench.py --mode $m $NB && run b_p2_$m 200 python bench.py --mode $m $NB; done ;;
    b_c3)       for m in ${C3M:-ca_bf ca_ff opp vbp_ff vbp_bf}; do run b_c3_$m 150 python bench.py --mode $m --hosts 100000 --tasks 1000 $NB --steps 20; done ;;
    b_segs)     for sg in ${SEGS:-8 32}; do PVT_BAND_SEGS=$sg run b_vbpbf_s$sg 200 python bench.py --mode vbp_bf $NB; done ;;
    b_opp)      run b_opp 200 python bench.py --mode opp $NB ;;
    b_c4)       for w in ${C4W:-4 2}; do for m in ca_bf ca_ff opp vbp_ff vbp_bf; do PVT_RES_WAVES=$w run b_c4_${m}_w$w 120 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 10 $NB; done; done ;;
    t_res)      run t_res 600 $T tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_policies.py tests/test_sim_replay.py tests/test_lockstep.py tests/test_gpu_fused.py tests/test_anchor.py ;;
    r_split)    run r_split 300 python tools/replay_split.py sim_c1_cost_aware sim_c2a1000_cost_aware sim_c2a1000_opportunistic sim_c2a1000_vbp_ff ;;
    b_replay)   run b_replay 300 python bench.py --extra 0 --replay 1 --cpu-baseline-seconds 0 --steps 3 ;;
    b_shard)    run b_shard 200 python bench.py --shard hosts $NB ;;
    st_zw)      for m in ca_bf vbp_ff ca_ff; do run st_$m 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so $m; done ;;
    st_var)     for v in ${VARS:-stamps}; do for m in ${STM:-ca_bf}; do TAILN=13 run st_${v}_$m 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_$v.so $m; done; done ;;
    b_var)      for v in ${VARS:-u8}; do for m in ${BM:-ca_bf}; do PIVOT_PLACE_LIB=pivot-scheduling_amd/diag/libpivot_place_$v.so run b_${v}_$m 150 python bench.py --mode $m $NB --steps 20; done; done ;;
    st_ord)     TAILN=6 run st_ord 120 python tools/order_stamps.py ;;
    tl)         mkdir -p gpurun_out/tl && run tl 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 10 $NB && python tools/api_timeline.py gpurun_out/tl/run_hip_api_trace.csv gpurun_out/tl/run_kernel_trace.csv 0.7 > gpurun_out/tl_summary.txt ;;
    kt_vbf)     mkdir -p gpurun_out/ktv && run kt_vbf 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktv -o a -- python tools/walk_probe.py --mode vbp_bf --hosts 1000000 --tasks 10000 --reps 3 && PVT_AHEAD=0 run kt_vbf0 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktv -o b -- python tools/walk_probe.py --mode vbp_bf --hosts 1000000 --tasks 10000 --reps 3 && python tools/trace_gaps.py gpurun_out/ktv/a_kernel_trace.csv 8 20 > gpurun_out/ktv_a.txt && python tools/trace_gaps.py gpurun_out/ktv/b_kernel_trace.csv 8 20 > gpurun_out/ktv_b.txt ;;
    st_lw)      run st_lw 150 python tools/lwalk_stamps.py 1000000 10000 ;;
    t_new)      run t_new 600 $T tests/test_gpu_restore.py tests/test_gpu_fused.py tests/test_gpu_epochs.py tests/test_gpu_headline.py ;;
    t_sh)       run t_sh 600 $T tests/test_gpu_sharded.py tests/test_gpu_runs.py tests/test_gpu_band.py ;;
    t_batch)    run t_batch 300 $T tests/test_gpu_batch.py ;;
    t_rw)       run t_rw 400 $T tests/test_gpu_resident_walk.py tests/test_gpu_batch.py ;;
    b_c4w)      for m in ${C4M:-ca_bf ca_ff vbp_ff}; do run b_c4w_$m 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 10 $NB; done ;;
    b_c4ab)     for m in ${C4M:-ca_bf ca_ff vbp_ff}; do PVT_RWALK=0 run b_c4nw_$m 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 10 $NB; done ;;
    hb_split)   TAILN=6 run hb_split 300 python tools/host_batch_split.py ;;
    hb_ab)      PVT_HOSTBATCH=0 TAILN=6 run hb_split0 300 python tools/host_batch_split.py && TAILN=6 run hb_split 300 python tools/host_batch_split.py ;;
    t_host)     run t_host 400 $T tests/test_gpu_host_batch.py tests/test_lockstep.py tests/test_gpu_fused.py ;;
    b_lock)     run b_lock 300 python -c "import bench, json; from pivot_place.engine import PlacementEngine; e = PlacementEngine(0); bench.replay_workloads(e); print(json.dumps(bench.lockstep_workload(e)))" ;;
    st_res)     for m in ${RES_MODES:-ca_bf vbp_bf vbp_ff ca_ff}; do run st_res_$m 120 python tools/resident_stamps.py $m; done ;;
    st_rw)      for m in ca_bf vbp_ff ca_ff; do TAILN=12 run st_rw_$m 120 python tools/resident_stamps.py $m; PVT_RWALK=0 TAILN=12 run st_rw0_$m 120 python tools/resident_stamps.py $m; done ;;
    st_rw1)     for m in ${RWM:-vbp_ff}; do TAILN=14 run st_rw_$m 120 python tools/resident_stamps.py $m; done ;;
    st_opp)     run st_opp 150 python tools/commit_stamps.py 2 1000000 10000 ;;
    profbench)  mkdir -p gpurun_out/prof; run profbench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 $NB ;;
    pmc)        run pmc 1100 tools/pmc_all.sh "${PMC_TAG:-r04z}" ;;
    pstep)      run pstep 400 python tools/pmc_step.py --tag "${PMC_TAG:-r05z}_c5_ca_bf" -- --mode ca_bf --hosts 1000000 --tasks 10000 ;;
    pmc_c4)     run pmc_c4 400 tools/pmc_all.sh "${PMC_TAG:-r04z}" c4 ;;
    *)          echo "unknown step $s"; exit 2 ;;
  esac
done
