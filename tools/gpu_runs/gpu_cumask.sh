#!/bin/bash
# Experiment: walker CU reservation on the side stream (PVT_WALK_CUS) for pipelined windows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
for n in 0 1 8 32; do
  PVT_WALK_CUS=$n timeout -k 10 200 python -u bench.py --mode ca_bf --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/bench_cus$n.log 2>&1 || exit $?
done
PVT_WALK_CUS=8 timeout -k 10 200 python -u bench.py --mode vbp_bf --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/bench_vbp_cus8.log 2>&1 || exit $?
