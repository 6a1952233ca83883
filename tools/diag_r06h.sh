#!/bin/bash
# The frontier walk with the chain map written by the walk's own blocks (by-value tables), phases
# and default-line A/B; vbp best-fit with the default sort and the record gather.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_step.sh h_tests 400 $T tests/test_gpu_headline.py tests/test_gpu_epochs.py tests/test_gpu_ff_epochs.py tests/test_gpu_band.py tests/test_gpu_restore.py || exit $?
for v in 00 11; do
  PVT_ZPRE=${v:0:1} PVT_CHAIN_TAB=${v:1:1} TAILN=14 tools/gpu_step.sh st_zw$v 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so ca_bf || exit $?
done
for rep in a b; do
  PVT_ZPRE=0 PVT_CHAIN_TAB=0 tools/gpu_step.sh h00${rep}_ca_bf 200 python bench.py $NB || exit $?
  tools/gpu_step.sh h11${rep}_ca_bf 200 python bench.py $NB || exit $?
done
tools/gpu_step.sh h_vbpbf 200 python bench.py --mode vbp_bf $NB || exit $?
tools/gpu_step.sh h_caff 200 python bench.py --mode ca_ff $NB || exit $?
