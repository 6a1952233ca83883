#!/bin/bash
# Opportunistic window sweep at the config-5 shape (pipelined count/walk), one line per window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
for w in 64 128 192; do
  timeout -k 10 200 python -u bench.py --mode opp --window $w --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/opp_w$w.log 2>&1 || exit $?
done
