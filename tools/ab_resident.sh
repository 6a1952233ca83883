#!/bin/bash
# A/B of resident variants at config 4 (run on the GPU box)
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
for v in main noskip noscreen noboth; do
  lib=""
  [ "$v" != main ] && lib="pivot-scheduling_amd/diag/libpivot_place_$v.so"
  for m in ${MODES:-ca_bf vbp_ff ca_ff vbp_bf opp}; do
    PIVOT_PLACE_LIB=$lib timeout -k 10 120 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 10 --extra 0 --cpu-baseline-seconds 0 --parity 1 > gpurun_out/ab_${v}_$m.log 2>&1 || { echo "fail $v $m"; exit 1; }
    echo "$v $m $(grep -o "\"ms_per_step\": [0-9.]*\|\"parity\": [a-z]*" gpurun_out/ab_${v}_$m.log | tr "\n" " ")"
  done
done
