# r02 session 36: device-side epoch accept + apply, pinned group-info staging; one host
# synchronisation for group info, optimistic epoch validation; full suite, bench, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g36_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
step g36_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g36_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g36 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
