#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
for m in ca_bf vbp_bf ca_ff; do
  timeout -k 10 200 python -u bench.py --mode $m --steps 3 --warmup 1 --cpu-baseline-seconds 0 --pipeline 0 > gpurun_out/bench_pf_${m}.log 2>&1 || exit $?
done
