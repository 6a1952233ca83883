#!/bin/bash
# Run lists merged on the fly (8 hosts per wave): parity, then config-4 vbp best-fit with the
# list threshold 8 / 16 / 24 and without lists (PVT_RWALK=41), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0 --parity 0"
T="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
TAILN=12 tools/gpu_step.sh t_probe 200 python -u tools/sticky_probe.py || exit $?
tools/gpu_step.sh t_tests 400 $T tests/test_gpu_sticky_runs.py tests/test_gpu_resident_walk.py tests/test_gpu_batch.py tests/test_gpu_headline.py -k "not config5" || exit $?
for rep in a b; do
  for t in 8 16 24; do
    PVT_RWALK=$((9 + (t << 8))) tools/gpu_step.sh t_t${t}_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
  done
  PVT_RWALK=41 tools/gpu_step.sh t_nol_$rep 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_bf --steps 20 $NB || exit $?
done
