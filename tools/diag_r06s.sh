#!/bin/bash
# Run lists (vbp best-fit): the minimum remaining run that builds a list, config 4, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0"
T="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
TAILN=12 tools/gpu_step.sh s_probe 200 python -u tools/sticky_probe.py || exit $?
tools/gpu_step.sh s_tests 300 $T tests/test_gpu_sticky_runs.py tests/test_gpu_headline.py -k "not config5" || exit $?
for rep in a b; do
  for t in 4 8 16 24 48; do
    PVT_RWALK=$((9 + (t << 8))) tools/gpu_step.sh s_t${t}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
  done
done
