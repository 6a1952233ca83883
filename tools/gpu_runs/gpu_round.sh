#!/bin/bash
# Round-end evidence: GPU tests, smoke, rocprofv3 kernel stats + PMC traffic + default bench line
# (with CPU baseline), scenario-batch lines. Summaries land in gpurun_out/ (copy to profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01c}
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0
f=$(find gpurun_out/prof_$TAG -name "bench_kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_ca_bf_kernel_stats.csv
run pmc 300 python tools/pmc_traffic.py ca_bf 1000000 10000
cp gpurun_out/traffic.json gpurun_out/${TAG}_traffic.json
run bench 600 python bench.py --traffic-json gpurun_out/traffic.json
for m in ca_bf ca_ff opp vbp_ff vbp_bf; do
  run batch_$m 200 python -u bench.py --mode $m --batch 512 --hosts 1000 --tasks 1000 --steps 5 --warmup 2 --cpu-baseline-seconds 0
done
run anchor_prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_anchor -o anchor -- python tools/anchor_bench.py
f=$(find gpurun_out/prof_${TAG}_anchor -name "anchor_kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_anchor_kernel_stats.csv
