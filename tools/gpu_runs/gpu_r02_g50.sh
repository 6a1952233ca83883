# r02 session 50: ordered frontier walk tuning sweep (task prefix x first host span), vbp_ff at
# config 5 and config 3, unsorted ca_ff at config 5 shape via bench env knobs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo -n "=== $name "; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo -n "rc=$rc "; tail -1 "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo; return $rc; }
for t in 768 1024 1536; do for h in 8192 65536; do
  PVT_OF_TASKS=$t PVT_OF_HOSTS=$h step g50_c5_t${t}_h${h} 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
  PVT_OF_TASKS=$t PVT_OF_HOSTS=$h step g50_c3_t${t}_h${h} 200 python bench.py --mode vbp_ff --hosts 100000 --tasks 1000 --steps 20 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
done; done
