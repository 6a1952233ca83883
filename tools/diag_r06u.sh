#!/bin/bash
# Run lists: config-4 vbp best-fit thresholds 2 / 4 / 8; cost_aware first-fit and best-fit with
# lists for every policy (PVT_RWALK bit 64) against without, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0"
T="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
PVT_RWALK=$((64 + (8 << 8))) TAILN=12 tools/gpu_step.sh u_probe 200 python -u tools/sticky_probe.py 64 || exit $?
for rep in a b; do
  for t in 2 4 8; do
    PVT_RWALK=$((9 + (t << 8))) tools/gpu_step.sh u_t${t}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
  done
  for m in ca_ff ca_bf; do
    PVT_RWALK=$((9 + 64 + (8 << 8))) tools/gpu_step.sh u_all_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB || exit $?
    tools/gpu_step.sh u_def_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB || exit $?
  done
done
