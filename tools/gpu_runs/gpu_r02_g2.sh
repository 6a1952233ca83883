# r02 session 2: event-ordered pipeline (no in-kernel start flag) on a CU-masked side stream.
# Parity of the pipelined paths, then the walk under rocprofv3 PMC (pipelined, list walk and
# opportunistic), a commit_kernel PMC profile at 1M x 10k, and the default bench with and
# without the CU reservation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
step g2_parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py || exit 1
step g2_pmc_walk1 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_walk1 -o p -- python tools/walk_probe.py --pipeline 1 --hosts 100000 --tasks 2000 || exit 1
step g2_pmc_opp1 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_opp1 -o p -- python tools/walk_probe.py --mode opp --pipeline 1 --hosts 100000 --tasks 2000 || exit 1
step g2_pmc_commit 600 python tools/pmc_profile.py --tag r02_commit_ca_bf --secs 150 --kernel commit_kernel -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 1 || exit 1
step g2_bench_cus8 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
PVT_WALK_CUS=0 step g2_bench_cus0 300 python bench.py --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g2_bench_opp 300 python bench.py --mode opp --steps 5 --warmup 2 --extra 0 --cpu-baseline-seconds 0 || exit 1
