#!/bin/bash
# One step of a GPU call: tools/gpu_step.sh NAME SECONDS CMD... runs CMD under its own time limit
# (timeout -k 10), logs to gpurun_out/NAME.log, prints the log's last lines and returns CMD's exit
# status, so steps chain with && and the call stops at the first failure, timeout or fault.
#   gpurun -- 'tools/gpu_step.sh tests 600 python -u -m pytest tests -m gpu -x -q && \
#              tools/gpu_step.sh bench 300 python bench.py'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1 secs=$2
shift 2
echo "=== $name"
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "=== $name rc=$rc"
tail -"${TAILN:-3}" "gpurun_out/$name.log" | cut -c1-400
exit $rc
