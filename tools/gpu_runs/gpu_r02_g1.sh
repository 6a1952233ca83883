# r02 first GPU session: counter list, headline-size parity, default bench (parity + extra keys),
# score-kernel PMC profile + diag counters, then walk PMC probes (pipeline off, then on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
step g1_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_headline.py "tests/test_gpu_parity.py::test_score_instances_both_tasks_per_wave" || exit 1
step g1_bench 600 python bench.py --steps 20 --warmup 5 || exit 1
step g1_diag 120 python tools/score_probe.py --diag --mode ca_bf --reps 2 || exit 1
step g1_pmc_score 600 python tools/pmc_profile.py --tag r02_ca_bf --kernel score_kernel -- tools/score_probe.py --mode ca_bf --reps 2 || exit 1
step g1_pmc_walk0 100 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_walk0 -o p -- python tools/walk_probe.py --pipeline 0 --hosts 100000 --tasks 2000 || exit 1
step g1_pmc_walk1 100 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_walk1 -o p -- python tools/walk_probe.py --pipeline 1 --hosts 100000 --tasks 2000 || exit 1
