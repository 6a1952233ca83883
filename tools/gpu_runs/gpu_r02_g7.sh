# r02 session 7: fixed gather, fast validation and walk shortcuts -- GPU suite, stamps, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g7_epochs 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_epochs.py tests/test_gpu_batch.py || exit 1
step g7_tests 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ || exit 1
step g7_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g7_stamps_ca_bf 300 python -u tools/commit_stamps.py 1 || exit 1
step g7_stamps_vbp_bf 300 python -u tools/commit_stamps.py 4 || exit 1
