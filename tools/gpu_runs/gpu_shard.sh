#!/bin/bash
# Sharded-path session: sharded parity tests, all GPU tests, bench unsharded vs host-sharded x1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=15 run tests_sharded 600 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread
TAILN=3 run tests 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x
TAILN=1 run bench_hosts1 300 python -u bench.py --shard hosts --steps 3 --warmup 1 --cpu-baseline-seconds 0
