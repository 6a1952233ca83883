#!/bin/bash
# Pipelined vs sequential windows, per mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in ${MODES:-vbp_bf ca_bf ca_ff vbp_ff}; do
  for p in 1 0; do
    timeout -k 10 200 python -u bench.py --mode $m --pipeline $p --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/pipe_${m}_p$p.log 2>&1
    rc=$?; echo "=== $m p$p rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pipe_${m}_p$p.log; exit $rc; fi
  done
done
