#!/bin/bash
# Config-4 resident kernel A/B (one GPU call): batch sizes (are co-resident workgroups sharing a
# CU's issue?), the walking wave (PVT_RWALK=2: rotated by workgroup), waves per round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
run() {   # NAME ENV... -- ARGS
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 120 python tools/walk_probe.py --hosts 1000 --tasks 1000 --reps 4 "$@" \
    > "gpurun_out/c4ab_$name.log" 2>&1 || { echo "$name failed"; return 1; }
  echo "$name: $(grep -h resident_kernel gpurun_out/c4ab_$name.log)"
}
for m in ca_bf vbp_bf ca_ff; do
  for b in 512 256 128; do run ${m}_b$b PVT_RWALK=1 -- --mode $m --batch $b || exit 1; done
done
run ca_bf_rot PVT_RWALK=2 -- --mode ca_bf --batch 512 || exit 1
run ca_bf_nowalk PVT_RWALK=0 -- --mode ca_bf --batch 512 || exit 1
for w in 2 8; do
  for m in vbp_bf ca_ff ca_bf; do run ${m}_w$w PVT_RES_WAVES=$w -- --mode $m --batch 512 || exit 1; done
done
