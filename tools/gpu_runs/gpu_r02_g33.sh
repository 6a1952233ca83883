# r02 session 33: opportunistic walk fast path whenever the draw holds and c_0 is unaffected.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g33_tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_opp_walk.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sharded.py tests/test_policies.py tests/test_sim_replay.py || exit 1
step g33_stamps_opp 200 python -u tools/commit_stamps.py 2 || exit 1
step g33_bench_opp 300 python bench.py --mode opp --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
