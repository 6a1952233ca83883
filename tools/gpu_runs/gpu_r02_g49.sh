# r02 session 49: keyed / ordered frontier walk without the per-task anchor test -- walk parity
# tests, vbp_ff and ca_ff lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*\|"kernels_ms_per_step": {[^}]*}\|"parity": [a-z]*\|passed.*\|failed.*' | tr '\n' ' '; echo; return $rc; }
step g49_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ordered_frontier.py tests/test_gpu_parity.py tests/test_gpu_headline.py || exit 1
step g49_vbpff 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g49_caff 200 python bench.py --mode ca_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g49_vbpff2 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
