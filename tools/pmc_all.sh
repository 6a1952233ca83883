#!/bin/bash
# PMC profiles of the kernels that can dominate every bench.py line, on THIS build, indexed for
# bench.py (profiles/pmc_index.json; entries carry the library's sha256, so bench.py uses them
# only for the binary they were collected on). Run on the GPU box:  tools/pmc_all.sh TAG [SET..]
# Sets: c5 (config 5, 1M x 10k, five policies), c5l (loaded config 5), c3 (100k x 1k), c4 (512
# scenarios of 1000 x 1000, resident kernel); default all. Each tools/pmc_profile.py pass is its
# own `rocprofv3 --pmc` child under a hard time limit (two passes per config for the kernels, two
# for the whole step's FETCH_SIZE / WRITE_SIZE: tools/pmc_step.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r04}
shift
sets=${*:-c5 c5l c3 c4}
set -e
WALKS=zwalk_kernel,commit_kernel,lwalk_kernel,opp_commit_kernel
PARS=score_kernel,band_score_kernel,opp_count_kernel,perm_scan_kernel,ordered_kernel,merge_kernel,merge_small_kernel,merge_path_kernel
idx=()
prof() {   # prof NAME MODE HOSTS TASKS KEYSUFFIX KERNELS PROBE-ARGS...
  local name=$1 mode=$2 h=$3 t=$4 suf=$5 kern=$6
  shift 6
  python tools/pmc_profile.py --tag "${tag}_${name}" --kernel "$kern" --secs 150 -- \
    tools/walk_probe.py --mode "$mode" --hosts "$h" --tasks "$t" --reps 2 "$@" \
    > "gpurun_out/pmc_${tag}_${name}.log" 2>&1
  # the whole step's HBM bytes (every dispatch of a round; bench.py hbm_GBs_measured)
  python tools/pmc_step.py --tag "${tag}_${name}" --secs 150 -- \
    --mode "$mode" --hosts "$h" --tasks "$t" "$@" > "gpurun_out/pmcstep_${tag}_${name}.log" 2>&1
  for f in gpurun_out/pmc_${tag}_${name}_*.json; do
    [ -e "$f" ] && idx+=("$mode:$h:$t$suf:$f")
  done
  echo "pmc $name ok"
}
for s in $sets; do
  case $s in
    c5)  for m in ca_bf vbp_ff ca_ff vbp_bf opp; do prof "c5_$m" $m 1000000 10000 "" "$WALKS,$PARS"; done ;;
    c5l) prof c5_ca_bf_loaded ca_bf 1000000 10000 _loaded "$WALKS,$PARS" --loaded 1 ;;
    c3)  for m in ca_bf vbp_ff ca_ff vbp_bf opp; do prof "c3_$m" $m 100000 1000 "" "$WALKS,$PARS"; done ;;
    c4)  for m in ca_bf vbp_ff ca_ff vbp_bf opp; do prof "c4_$m" $m 1000 1000 _b512 resident_kernel --batch 512; done ;;
    *)   echo "unknown set $s"; exit 2 ;;
  esac
done
python tools/pmc_index.py --dest "profiles/$tag" gpurun_out/pmc_index.json "${idx[@]}"
