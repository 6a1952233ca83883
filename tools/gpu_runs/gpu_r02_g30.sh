# r02 session 30: PMC counters of the zero-cost frontier walk (instruction mix, waits) at config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pmc_profile.py --tag r02l_zwalk --kernel zwalk_kernel --passes sq,sq2,fetch,write -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 3 > gpurun_out/g30_pmc_zwalk.log 2>&1; rc=$?; tail -30 gpurun_out/g30_pmc_zwalk.log; exit $rc
