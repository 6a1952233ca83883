#!/bin/bash
# Config-4 vbp_ff / ca_bf: this build against the previous commit's (diag/libpivot_place_prev.so), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0"
for rep in a b; do
  for m in ca_bf; do
    tools/gpu_step.sh n_cur_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB || exit $?
    PIVOT_PLACE_LIB=pivot-scheduling_amd/diag/libpivot_place_prev.so tools/gpu_step.sh n_prev_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB || exit $?
  done
done
