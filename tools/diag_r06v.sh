#!/bin/bash
# Run lists: 4 / 8 (default) / 16 hosts per wave (-DPVT_RES_LK variant builds), config-4 vbp
# best-fit, interleaved; a parity probe of each variant first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0"
D=pivot-scheduling_amd/diag
for k in k4 k16; do
  PIVOT_PLACE_LIB=$D/libpivot_place_$k.so TAILN=3 tools/gpu_step.sh v_probe_$k 200 python -u tools/sticky_probe.py || exit $?
done
for rep in a b; do
  tools/gpu_step.sh v_k8_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
  for k in k4 k16; do
    PIVOT_PLACE_LIB=$D/libpivot_place_$k.so tools/gpu_step.sh v_${k}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
  done
done
