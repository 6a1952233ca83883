# r02 session 16: register-resident frontier walk -- epoch tests, stamps, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g16_epochs 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_epochs.py || exit 1
step g16_zstamps 200 python -u tools/zwalk_stamps.py || exit 1
step g16_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
