# r02 session 34: PMC counters of the current zero-cost walk (for the issue roofline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pmc_profile.py --tag r02p_zwalk --kernel zwalk_kernel --passes sq,sq2 -- tools/walk_probe.py --mode ca_bf --hosts 1000000 --tasks 10000 --reps 3 > gpurun_out/g34_pmc_zwalk.log 2>&1; rc=$?; tail -3 gpurun_out/g34_pmc_zwalk.log | cut -c1-300; exit $rc
