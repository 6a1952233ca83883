#!/bin/bash
# Diagnostics session: commit-walk phase stamps + a rocprofv3 kernel trace of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -12 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run stamps_ca_bf 300 python -u tools/commit_stamps.py 1
run stamps_vbp_bf 300 python -u tools/commit_stamps.py 4
run stamps_ca_ff 300 python -u tools/commit_stamps.py 0
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 3 --warmup 1 --cpu-baseline-seconds 0
find gpurun_out/prof -name "*stats*" | head
