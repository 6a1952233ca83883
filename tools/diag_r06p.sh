#!/bin/bash
# Bulk sticky runs in the 4-wave resident path: a probe, parity, then config-4 bench lines with the
# bulk step on (default) and off (PVT_RWALK=25), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
TAILN=12 tools/gpu_step.sh p_probe 200 python -u tools/sticky_probe.py || exit $?
tools/gpu_step.sh p_tests 700 $T tests/test_gpu_sticky_runs.py tests/test_gpu_resident_walk.py tests/test_gpu_batch.py \
  tests/test_gpu_host_batch.py tests/test_gpu_headline.py -k "not config5" || exit $?
for rep in a b; do
  for m in vbp_bf ca_ff ca_bf; do
    tools/gpu_step.sh p_on_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB --parity 0 || exit $?
    PVT_RWALK=25 tools/gpu_step.sh p_off_${m}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 20 $NB --parity 0 || exit $?
  done
done
