# r02 session 5: chain epochs (one walk per zero-cost component) -- parity and bench sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g5_epochs 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_epochs.py || exit 1
step g5_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lockstep.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_policies.py tests/test_sim_replay.py || exit 1
step g5_bench_ca_bf 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
for S in 1 4 8; do PVT_SEGMENTS=$S step g5_bench_ca_bf_S$S 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1; done
step g5_bench_c3 300 python bench.py --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
PVT_SEGMENTS=4 step g5_bench_c3_S4 300 python bench.py --hosts 100000 --tasks 1000 --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
