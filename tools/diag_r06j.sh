#!/bin/bash
# Default line A/B, interleaved, 100 steps each: prebuilt windows only (10) vs with the by-value
# chain tables (11), three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0 --steps 100"
for rep in a b c; do
  PVT_CHAIN_TAB=0 tools/gpu_step.sh j10${rep} 200 python bench.py $NB || exit $?
  tools/gpu_step.sh j11${rep} 200 python bench.py $NB || exit $?
done
