#!/bin/bash
# Phase stamps (diagnostic build): the fused host-batch kernel over the config-1 replay, the
# opportunistic speculative-range walk at configs 5 and 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh fstamps 200 python tools/fused_stamps.py sim_c1_cost_aware || exit $?
tools/gpu_step.sh ostamps_c5 200 python tools/commit_stamps.py 2 1000000 10000 || exit $?
tools/gpu_step.sh ostamps_c3 200 python tools/commit_stamps.py 2 100000 1000 || exit $?
