#!/bin/bash
# Bench lines for BASELINE config 3 (100k hosts x 1k tasks, 20 zones) in every policy, and the
# config-5 shape through the host-sharded path at world 1 (exchange code path on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
TAG=${TAG:-r01g}
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
for m in ca_bf ca_ff opp vbp_ff vbp_bf; do
  run ${TAG}_c3_$m 200 python -u bench.py --mode $m --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --cpu-baseline-seconds 5
done
run ${TAG}_c5_shard_hosts_w1 300 python -u bench.py --shard hosts --steps 3 --warmup 1 --cpu-baseline-seconds 0
