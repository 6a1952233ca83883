# r02 session 48: frontier-walk stamps (diagnostic build): vbp_ff ordered frontier and ca_bf chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run g48_stamps_vbpff 200 python -u tools/commit_stamps.py 3
PVT_OF_TASKS=4096 run g48_stamps_vbpff_4096 200 python -u tools/commit_stamps.py 3
ZWALK=1 run g48_stamps_cabf 200 python -u tools/commit_stamps.py 1
