#!/bin/bash
# Round-6 session 2 baseline: the default line's device timeline and host API calls under the
# bench's own profiling setting (events around the dominant kernel only), then the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
mkdir -p gpurun_out/tl6
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv \
  -d "$R/gpurun_out/tl6" -o run -- python "$R/bench.py" --steps 30 $NB > "$R/gpurun_out/tl6.log" 2>&1) || { echo "tl6 failed"; exit 1; }
echo "tl6 ok"
python tools/trace_gaps.py gpurun_out/tl6/run_kernel_trace.csv 1.5 20 > gpurun_out/tl6_gaps.txt 2>&1
python tools/api_timeline.py gpurun_out/tl6/run_hip_api_trace.csv gpurun_out/tl6/run_kernel_trace.csv 0.5 > gpurun_out/tl6_api.txt 2>&1
tools/gpu_step.sh bench6 400 python bench.py
