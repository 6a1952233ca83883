# r02 session 17: frontier walk -- epoch tests, stamps, bench, kernel-trace stats of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g17_epochs 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_epochs.py || exit 1
step g17_zstamps 200 python -u tools/zwalk_stamps.py || exit 1
step g17_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g17_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g17 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
