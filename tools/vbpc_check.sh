#!/bin/bash
# vbp best-fit s2 cache in the resident kernel: parity of the resident paths, config-4 timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh vbpc_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resident_walk.py tests/test_gpu_batch.py tests/test_gpu_host_batch.py tests/test_sim_replay.py \
  tests/test_gpu_parity.py "tests/test_gpu_headline.py::test_config4_batch_per_gpu_matches_oracle" || exit $?
for m in vbp_bf ca_bf; do
  timeout -k 10 120 python tools/walk_probe.py --hosts 1000 --tasks 1000 --reps 4 --mode $m --batch 512 \
    > gpurun_out/vc_c4_$m.log 2>&1 || exit 1
  echo "c4 $m: $(grep -h resident_kernel gpurun_out/vc_c4_$m.log)"
done
