#!/bin/bash
# Fused host batch with batched PCIe copies: parity, config-1 split; resident walk stamps; the
# config-5 default step's kernel timeline (gaps between launches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
tools/gpu_step.sh fused2_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_batch.py tests/test_lockstep.py tests/test_sim_replay.py tests/test_policies.py || exit $?
tools/gpu_step.sh c1split2 200 python tools/replay_split.py sim_c1_cost_aware || exit $?
tools/gpu_step.sh rstamps2_ca_bf 120 python tools/resident_stamps.py ca_bf || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d "$R/gpurun_out/c5kt" -o c5 -- python "$R/tools/walk_probe.py" --mode ca_bf --hosts 1000000 --tasks 10000 --reps 6 \
  > "$R/gpurun_out/c5kt.log" 2>&1
echo "c5kt rc=$?"
