#!/bin/bash
# Bench sweep: list modes pipelined and sequential (no CPU baseline), optional stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "gpurun_out/$name.log"; exit $rc; fi; }
for m in ${MODES:-ca_bf vbp_bf ca_ff}; do
  for p in 1 0; do run bench_${m}_p$p 300 python -u bench.py --mode $m --pipeline $p --steps 3 --warmup 1 --cpu-baseline-seconds 0; done
done
