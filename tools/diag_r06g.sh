#!/bin/bash
# Frontier-walk phases (stamps build) with the prebuilt window / by-value chain tables on and off;
# vbp best-fit bench line (record gather, per-block key bits) and its bench-mode kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
for v in 00 10 01 11; do
  PVT_ZPRE=${v:0:1} PVT_CHAIN_TAB=${v:1:1} TAILN=14 tools/gpu_step.sh st_zw$v 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so ca_bf || exit $?
done
tools/gpu_step.sh g_band 300 $T tests/test_gpu_band.py tests/test_gpu_headline.py -k "band or vbp or VBP" || exit $?
tools/gpu_step.sh g_vbpbf 200 python bench.py --mode vbp_bf $NB || exit $?
mkdir -p gpurun_out/gvk
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/gvk" -o run -- python "$R/bench.py" --mode vbp_bf --steps 10 $NB > "$R/gpurun_out/gvk.log" 2>&1) || { echo "gvk failed"; exit 1; }
python tools/trace_gaps.py gpurun_out/gvk/run_kernel_trace.csv 8 25 > gpurun_out/gvk_gaps.txt 2>&1
echo "gvk ok"
