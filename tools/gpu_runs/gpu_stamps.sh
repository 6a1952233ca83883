#!/bin/bash
# Commit-walk phase stamps (diagnostic build) + rocprofv3 kernel stats of the scenario batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for m in ${SMODES:-1 4 0}; do TAILN=7 run stamps_$m 300 python -u tools/commit_stamps.py $m; done
if [ -n "$PROF" ]; then
run trace_batch 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_batch -o batch -- python bench.py --mode ca_bf --batch 512 --hosts 1000 --tasks 1000 --steps 5 --warmup 2 --cpu-baseline-seconds 0
fi
