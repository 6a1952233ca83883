#!/bin/bash
# Zone-table cache of host-array rounds: parity of the drop-in paths, config-1/2 replay split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh ztc_tests 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_batch.py tests/test_lockstep.py tests/test_sim_replay.py tests/test_policies.py \
  tests/test_gpu_fused.py tests/test_anchor.py tests/test_trace.py || exit $?
TAILN=8 tools/gpu_step.sh c1split4 300 python tools/replay_split.py sim_c1_cost_aware sim_c2a1000_cost_aware sim_c2a1000_opportunistic sim_c2a1000_vbp_ff || exit $?
