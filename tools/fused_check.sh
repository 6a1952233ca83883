#!/bin/bash
# The fused host batch (one launch per pvt_place_host_batch call): parity tests of every path that
# goes through it, then the config-1 / config-2 drop-in replays fused and staged (PVT_FUSED=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh fused_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_batch.py tests/test_lockstep.py tests/test_sim_replay.py tests/test_policies.py \
  tests/test_gpu_resident_walk.py tests/test_anchor.py tests/test_trace.py || exit $?
tools/gpu_step.sh c1split_fused 200 python tools/replay_split.py sim_c1_cost_aware sim_c2a1000_cost_aware || exit $?
PVT_FUSED=0 tools/gpu_step.sh c1split_staged 200 python tools/replay_split.py sim_c1_cost_aware sim_c2a1000_cost_aware || exit $?
