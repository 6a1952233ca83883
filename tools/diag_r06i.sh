#!/bin/bash
# Frontier-walk prologue: first chain positions from the by-value segments (stamps, A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_step.sh i_tests 400 $T tests/test_gpu_headline.py tests/test_gpu_epochs.py tests/test_gpu_ff_epochs.py tests/test_gpu_sharded.py || exit $?
for v in 00 11; do
  PVT_ZPRE=${v:0:1} PVT_CHAIN_TAB=${v:1:1} TAILN=14 tools/gpu_step.sh st_zw$v 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so ca_bf || exit $?
done
for rep in a b; do
  PVT_ZPRE=0 PVT_CHAIN_TAB=0 tools/gpu_step.sh i00${rep}_ca_bf 200 python bench.py $NB || exit $?
  tools/gpu_step.sh i11${rep}_ca_bf 200 python bench.py $NB || exit $?
done
