#!/bin/bash
# Resident walk with bulk runs: parity (resident, batch, fused, lock-step, replays), config-4
# stamps and bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
NB="--extra 0 --replay 0 --cpu-baseline-seconds 0"
T="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_step.sh m_tests 700 $T tests/test_gpu_resident_walk.py tests/test_gpu_batch.py tests/test_gpu_fused.py \
  tests/test_gpu_host_batch.py tests/test_sim_replay.py tests/test_lockstep.py tests/test_gpu_parity.py tests/test_gpu_headline.py -k "not config5" || exit $?
TAILN=16 tools/gpu_step.sh rs_ca_bf 120 python tools/resident_stamps.py ca_bf || exit $?
TAILN=16 tools/gpu_step.sh rs_vbp_ff 120 python tools/resident_stamps.py vbp_ff || exit $?
for m in ca_bf vbp_bf vbp_ff; do
  tools/gpu_step.sh m_c4_$m 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode $m --steps 10 $NB || exit $?
done
PVT_RWALK=1 tools/gpu_step.sh m_c4nw_vbp_ff 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode vbp_ff --steps 10 $NB || exit $?
PVT_RWALK=0 tools/gpu_step.sh m_c4nw_ca_bf 150 python bench.py --batch 512 --hosts 1000 --tasks 1000 --mode ca_bf --steps 10 $NB || exit $?
