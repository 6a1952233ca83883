#!/bin/bash
# Round-6 diagnostics (one GPU call): refined band-list invariant checks on the two check
# builds; resident-kernel phase stamps at config 4 (ca_bf, vbp_bf); where a config-1 drop-in
# round's time goes (engine call vs Python; then a HIP API + kernel trace of the same replay).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
tools/band_variants.sh bandcheck bandhelpck || exit $?
tools/gpu_step.sh rstamps_ca_bf 120 python tools/resident_stamps.py ca_bf || exit $?
tools/gpu_step.sh rstamps_vbp_bf 120 python tools/resident_stamps.py vbp_bf || exit $?
tools/gpu_step.sh rstamps_ca_ff 120 python tools/resident_stamps.py ca_ff || exit $?
tools/gpu_step.sh c1split 200 python tools/replay_split.py sim_c1_cost_aware || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv \
  -d "$R/gpurun_out/c1trace" -o c1 -- python "$R/tools/replay_split.py" sim_c1_cost_aware \
  > "$R/gpurun_out/c1trace.log" 2>&1
echo "c1trace rc=$?"
