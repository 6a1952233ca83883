#!/bin/bash
# Iteration session: parity tests, then bench for every mode (no CPU baseline), then stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
TAILN=3 run tests 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x
for m in ${MODES:-ca_bf vbp_bf ca_ff vbp_ff opp}; do
  TAILN=1 run bench_$m 300 python -u bench.py --mode $m --steps 3 --warmup 1 --cpu-baseline-seconds 0
done
for m in ${STAMPS:-}; do TAILN=7 run stamps_$m 300 python -u tools/commit_stamps.py $m; done
