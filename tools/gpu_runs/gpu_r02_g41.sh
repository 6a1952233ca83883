# r02 session 41: ordered frontier walk (vbp first-fit / unsorted cost_aware first-fit) --
# its parity tests, vbp_ff bench, then the full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step g41_ord 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ordered_frontier.py || exit 1
step g41_vbpff 300 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g41_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
