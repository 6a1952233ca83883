# r02 session 8: host sharding (pipelined list windows, opportunistic super-chunk shards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g8_sharded 900 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gpu_sharded.py || exit 1
for m in ca_bf vbp_bf ca_ff opp; do
  step g8_bench_shard_$m 300 python bench.py --mode $m --shard hosts --steps 5 --warmup 2 --extra 0 --cpu-baseline-seconds 0 || exit 1
done
step g8_bench_shard_ca_bf_nopipe 300 python bench.py --mode ca_bf --shard hosts --pipeline 0 --steps 5 --warmup 2 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
