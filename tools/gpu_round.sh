#!/bin/bash
# One GPU-box session: parity tests, smoke, bench. Each step has its own time limit; a fault,
# abort, segfault or time limit (rc other than 0/1) ends the session before the next GPU step.
# Usage: tools/gpu_round.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py "$@"
