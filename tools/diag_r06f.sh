#!/bin/bash
# The frontier walk without generic pointers (chain map from the by-value tables), default line
# A/B; vbp best-fit kernel statistics after the onesweep band sort and record gather.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_step.sh f_tests 400 $T tests/test_gpu_headline.py tests/test_gpu_epochs.py tests/test_gpu_ff_epochs.py tests/test_gpu_band.py || exit $?
PVT_ZPRE=0 PVT_CHAIN_TAB=0 tools/gpu_step.sh f00_ca_bf 200 python bench.py $NB || exit $?
tools/gpu_step.sh f11_ca_bf 200 python bench.py $NB || exit $?
PVT_ZPRE=0 PVT_CHAIN_TAB=0 tools/gpu_step.sh f00b_ca_bf 200 python bench.py $NB || exit $?
tools/gpu_step.sh f11b_ca_bf 200 python bench.py $NB || exit $?
mkdir -p gpurun_out/fvk
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/fvk" -o run -- python "$R/tools/walk_probe.py" --mode vbp_bf --hosts 1000000 --tasks 10000 --reps 3 > "$R/gpurun_out/fvk.log" 2>&1) || { echo "fvk failed"; exit 1; }
python tools/trace_gaps.py gpurun_out/fvk/run_kernel_trace.csv 8 20 > gpurun_out/fvk_gaps.txt 2>&1
echo "fvk ok"
