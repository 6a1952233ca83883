#!/bin/bash
# GPU tests, then cost_aware first-fit (sort_hosts) bench lines at config 3 and config 5 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/kscan_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --mode ca_ff --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/kscan_c3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode ca_ff --steps 5 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/kscan_c5.log 2>&1
