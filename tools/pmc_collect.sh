#!/bin/bash
# Build container side: copy a tools/pmc_all.sh run's PMC summaries (gpurun_out/pmc_TAG_*) into
# profiles/TAG/ and index them in profiles/pmc_index.json (sources pointing at profiles/TAG/).
#   tools/pmc_collect.sh r03f
cd "$(dirname "$0")/.." || exit 2
tag=$1; H=1000000; T=10000
mkdir -p profiles/$tag
cp gpurun_out/pmc_${tag}_*.json gpurun_out/pmc_${tag}_*.csv profiles/$tag/ || exit 1
args=()
for m in ca_bf vbp_ff ca_ff; do args+=("$m:$H:$T:profiles/$tag/pmc_${tag}_$m.json"); done
for k in band_score_kernel lwalk_kernel; do args+=("vbp_bf:$H:$T:profiles/$tag/pmc_${tag}_vbp_bf_$k.json"); done
for k in opp_count_kernel opp_commit_kernel; do args+=("opp:$H:$T:profiles/$tag/pmc_${tag}_opp_$k.json"); done
rm -f profiles/pmc_index.json
python tools/pmc_index.py profiles/pmc_index.json "${args[@]}"
