#!/bin/bash
# Opportunistic parity tests, then the config-5 and config-3 opportunistic bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "opp or OPP or opportunistic or 2-" tests > gpurun_out/opp_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode opp --steps 5 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/opp_c5.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --mode opp --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/opp_c3.log 2>&1
