# r02 session 3: group-parallel epochs (cost_aware best-fit) parity + bench; side-stream
# priority variants for the pipelined list walk and the opportunistic pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g3_epochs 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_epochs.py || exit 1
step g3_parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_policies.py tests/test_sim_replay.py || exit 1
step g3_bench_ca_bf 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
for S in 4 8 16; do PVT_SEGMENTS=$S step g3_bench_ca_bf_S$S 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1; done
step g3_bench_ca_bf_noep 300 python bench.py --epochs 0 --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
for prio in 1 0; do
  for m in opp vbp_bf; do
    PVT_SIDE_PRIO=$prio step g3_bench_${m}_prio$prio 300 python bench.py --mode $m --steps 5 --warmup 2 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
  done
done
