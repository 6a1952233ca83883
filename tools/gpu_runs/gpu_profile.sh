#!/bin/bash
# Profiling session: rocprofv3 kernel-trace stats of the default bench, PMC traffic passes
# (each its own run), then the full default bench line (with CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=${TAG:-r01}
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0
f=$(find gpurun_out/prof_$TAG -name "bench_kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_ca_bf_kernel_stats.csv
run pmc 300 python tools/pmc_traffic.py ca_bf 1000000 10000
cp gpurun_out/traffic.json gpurun_out/${TAG}_traffic.json
run bench 600 python bench.py --traffic-json gpurun_out/traffic.json
