# r02 session 47: round evidence at HEAD (ordered frontier walk, pipelined task-record loads) -- full GPU suite, smoke, default bench with extras +
# CPU baseline, 20-step bench, kernel-trace stats (the frontier walk kernel is unchanged since
# the PMC profile in profiles/r02p).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g47_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
step g47_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step g47_bench 600 python bench.py || exit 1
step g47_bench20 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g47_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g47 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
step g47_vbpff 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g47_caff 200 python bench.py --mode ca_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
