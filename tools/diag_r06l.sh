#!/bin/bash
# Config-4 resident kernel: per-phase stamps of block 0 and the per-round cycle distribution.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for m in ca_bf vbp_bf ca_ff opp vbp_ff; do
  TAILN=16 tools/gpu_step.sh rs_$m 120 python tools/resident_stamps.py $m || exit $?
done
