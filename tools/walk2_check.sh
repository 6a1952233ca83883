#!/bin/bash
# Resident walk with the zero-cost window: parity of every resident path, config-4 timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh walk2_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resident_walk.py tests/test_gpu_batch.py tests/test_gpu_host_batch.py tests/test_sim_replay.py \
  tests/test_lockstep.py "tests/test_gpu_headline.py::test_config4_batch_per_gpu_matches_oracle" || exit $?
for m in ca_bf ca_ff; do
  timeout -k 10 120 python tools/walk_probe.py --hosts 1000 --tasks 1000 --reps 4 --mode $m --batch 512 \
    > gpurun_out/w2_c4_$m.log 2>&1 || exit 1
  echo "c4 $m: $(grep -h resident_kernel gpurun_out/w2_c4_$m.log)"
done
tools/gpu_step.sh c1split3 200 python tools/replay_split.py sim_c1_cost_aware || exit $?
