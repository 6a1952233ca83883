# r02 session 14: frontier-walk stamps + bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g14_zstamps 200 python -u tools/zwalk_stamps.py || exit 1
step g14_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
