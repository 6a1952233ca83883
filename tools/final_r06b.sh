#!/bin/bash
# Round-6 final library, part 2: PMC profiles of every bench line's hot kernels (indexed for
# bench.py with this library's sha256), then the full bench and the default line's kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
tools/gpu_step.sh fin_pmc 1000 tools/pmc_all.sh "${1:-r06e}" || exit $?
cp gpurun_out/pmc_index.json profiles/pmc_index.json
tools/gpu_step.sh fin_bench 500 python bench.py || exit $?
mkdir -p gpurun_out/fin_prof
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/fin_prof" -o run -- python "$R/bench.py" --steps 20 --extra 0 --replay 0 --cpu-baseline-seconds 0 \
  > "$R/gpurun_out/fin_profbench.log" 2>&1) || { echo "fin_prof failed"; exit 1; }
echo "fin_prof ok"
