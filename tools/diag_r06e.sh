#!/bin/bash
# Round-6 launch-overhead changes, each with an A/B switch: events bound to the timed kernel's
# dispatch (PVT_BIND_EVENTS), the first epoch's windows prebuilt by the grouped order's launch
# (PVT_ZPRE), chain tables passed by value to the frontier walk (PVT_CHAIN_TAB); and the band
# sort by onesweep over the varying key bits (vbp best-fit). Parity tests first, then bench lines,
# then a kernel trace of the default line (bound events' kernel time vs rocprofv3's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_step.sh ev_tests 600 $T tests/test_gpu_restore.py tests/test_gpu_headline.py tests/test_gpu_epochs.py \
  tests/test_gpu_ff_epochs.py tests/test_gpu_band.py tests/test_gpu_parity.py || exit $?
PVT_ZPRE=0 PVT_BIND_EVENTS=0 PVT_CHAIN_TAB=0 tools/gpu_step.sh ab000_ca_bf 200 python bench.py $NB || exit $?
PVT_ZPRE=0 PVT_BIND_EVENTS=1 PVT_CHAIN_TAB=0 tools/gpu_step.sh ab010_ca_bf 200 python bench.py $NB || exit $?
PVT_ZPRE=1 PVT_BIND_EVENTS=1 PVT_CHAIN_TAB=0 tools/gpu_step.sh ab110_ca_bf 200 python bench.py $NB || exit $?
tools/gpu_step.sh ab111_ca_bf 200 python bench.py $NB || exit $?
tools/gpu_step.sh ab111_ca_ff 200 python bench.py --mode ca_ff $NB || exit $?
for m in vbp_bf opp; do
  PVT_BIND_EVENTS=0 tools/gpu_step.sh ev0_$m 200 python bench.py --mode $m $NB || exit $?
  PVT_BIND_EVENTS=1 tools/gpu_step.sh ev1_$m 200 python bench.py --mode $m $NB || exit $?
done
mkdir -p gpurun_out/ev1kt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/ev1kt" -o run -- python "$R/bench.py" --steps 30 $NB > "$R/gpurun_out/ev1kt.log" 2>&1) || { echo "ev1kt failed"; exit 1; }
echo "ev1kt ok"
