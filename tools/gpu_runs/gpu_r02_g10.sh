# r02 session 10: full GPU suite (sharding, DPP scout selection); default bench; walk stamps;
# sharded benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g10_tests 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
step g10_bench 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g10_stamps_ca_bf 300 python -u tools/commit_stamps.py 1 || exit 1
for m in ca_bf vbp_bf ca_ff; do
  step g10_bench_shard_$m 300 python bench.py --mode $m --shard hosts --steps 5 --warmup 2 --extra 0 --cpu-baseline-seconds 0 || exit 1
done
