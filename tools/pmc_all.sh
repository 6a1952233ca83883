#!/bin/bash
# PMC profiles of every hot kernel of the bench lines on THIS build, indexed for bench.py
# (profiles/pmc_index.json; entries carry the library's sha256, so bench.py uses them only for
# the binary they were collected on). Run on the GPU box:  tools/pmc_all.sh TAG
# Each tools/pmc_profile.py pass is its own `rocprofv3 --pmc` child under a hard time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r03}
H=1000000 T=10000
set -e
prof() {   # prof MODE KERNELS
  python tools/pmc_profile.py --tag "${tag}_$1" --kernel "$2" --secs 120 -- \
    tools/walk_probe.py --mode "$1" --hosts $H --tasks $T --reps 2 > "gpurun_out/pmc_${tag}_$1.log" 2>&1
  echo "pmc $1 ($2) ok"
}
prof ca_bf zwalk_kernel
prof vbp_ff zwalk_kernel
prof ca_ff zwalk_kernel
prof vbp_bf band_score_kernel,lwalk_kernel
prof opp opp_count_kernel,opp_commit_kernel
args=()
for m in ca_bf vbp_ff ca_ff; do args+=("$m:$H:$T:gpurun_out/pmc_${tag}_$m.json"); done
for k in band_score_kernel lwalk_kernel; do args+=("vbp_bf:$H:$T:gpurun_out/pmc_${tag}_vbp_bf_$k.json"); done
for k in opp_count_kernel opp_commit_kernel; do args+=("opp:$H:$T:gpurun_out/pmc_${tag}_opp_$k.json"); done
python tools/pmc_index.py gpurun_out/pmc_index.json "${args[@]}"
