# r02 session 13: zero-cost frontier walk (pvt_zwalk.hip) -- epoch tests both ways, parity, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step g13_epochs 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_epochs.py || exit 1
step g13_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g13_parity 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_sharded.py || exit 1
