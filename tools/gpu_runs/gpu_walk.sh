#!/bin/bash
# Walk iteration: all GPU tests, bench of the list-based modes, commit-walk stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=12 run tests 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x
for m in ca_bf vbp_bf ca_ff vbp_ff; do
  TAILN=1 run bench_$m 300 python -u bench.py --mode $m --steps 3 --warmup 1 --cpu-baseline-seconds 0
done
for m in 1 4 0; do TAILN=7 run stamps_$m 300 python -u tools/commit_stamps.py $m; done
