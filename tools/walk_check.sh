#!/bin/bash
# Resident walk fast path: parity of the resident paths, config-4 timings, and the kernel trace of
# the config-1 drop-in replay (fused host batch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
tools/gpu_step.sh walk_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resident_walk.py tests/test_gpu_batch.py tests/test_gpu_host_batch.py tests/test_sim_replay.py || exit $?
for m in ca_bf ca_ff vbp_bf; do
  timeout -k 10 120 python tools/walk_probe.py --hosts 1000 --tasks 1000 --reps 4 --mode $m --batch 512 \
    > gpurun_out/wc_c4_$m.log 2>&1 || exit 1
  echo "c4 $m: $(grep -h resident_kernel gpurun_out/wc_c4_$m.log)"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/c1kt" -o c1 -- python "$R/tools/replay_split.py" sim_c1_cost_aware \
  > "$R/gpurun_out/c1kt.log" 2>&1
echo "c1kt rc=$?"
