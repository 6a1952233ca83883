# r02 session 39: keyed frontier walk launched with the prefix length on the device, one synchronisation per group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g39_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_policies.py tests/test_sim_replay.py tests/test_lockstep.py tests/test_gpu_sharded.py || exit 1
step g39_bench_ca_ff 300 python bench.py --mode ca_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g39_bench_c3_ca_ff 300 python bench.py --mode ca_ff --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
