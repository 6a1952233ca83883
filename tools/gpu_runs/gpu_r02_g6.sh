# r02 session 6: realtime_bw + chain epochs parity (full GPU suite), default bench with extras
# and CPU baseline, PMC profiles of the epoch-mode score kernel, the chain walks and validation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
step g6_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ || exit 1
step g6_bench 600 python bench.py --steps 20 --warmup 5 || exit 1
step g6_pmc_score 600 python tools/pmc_profile.py --tag r02c_score_ca_bf --secs 150 --kernel score_kernel --candidates-per-launch 1e10 -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 1 || exit 1
step g6_pmc_commit 600 python tools/pmc_profile.py --tag r02c_commit_ca_bf --secs 150 --kernel commit_kernel -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 1 || exit 1
step g6_pmc_validate 600 python tools/pmc_profile.py --tag r02c_validate_ca_bf --secs 150 --kernel epoch_validate -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c5" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --extra 0 --cpu-baseline-seconds 0 --parity 0 > "$GRAFT_REPO_ROOT/gpurun_out/g6_prof.log" 2>&1; echo "prof rc=$?"
