# r02 session 15: frontier-walk stamps with / without the per-task log stores.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -5 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g15_zstamps 200 python -u tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so || exit 1
