# r02 session 35: round evidence at HEAD -- PMC of the frontier walk (all passes; the bench's
# issue roofline reads it), full GPU suite, smoke, default bench with extras + CPU baseline,
# kernel-trace stats of the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step g35_pmc 600 python -u tools/pmc_profile.py --tag r02p_zwalk --kernel zwalk_kernel --passes sq,sq2,fetch,write -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 3 || exit 1
cp gpurun_out/pmc_r02p_zwalk.json gpurun_out/pmc_r02p_zwalk.csv profiles/r02p/ || exit 1
step g35_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
step g35_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step g35_bench 600 python bench.py || exit 1
step g35_bench20 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 || exit 1
step g35_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g35 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 --parity 0 || exit 1
