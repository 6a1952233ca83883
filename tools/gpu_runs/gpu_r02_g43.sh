# r02 session 43: ordered frontier walk with per-batch suffix minima and an adaptive host span --
# parity tests, vbp_ff task-prefix / host-span sweep, unsorted ca_ff.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*\|"frontier_chains_per_step": [0-9.]*\|"windows_per_step": [0-9.]*\|"kernels_ms_per_step": {[^}]*}\|"parity": [a-z]*\|passed.*\|failed.*' | tr '\n' ' '; echo; return $rc; }
step g43_ord 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ordered_frontier.py || exit 1
for k in 512 1024 2048 4096; do
  PVT_OF_TASKS=$k step g43_vbpff_$k 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
done
PVT_OF_HOSTS=2000000 step g43_vbpff_fullspan 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
PVT_OF_HOSTS=8192 step g43_vbpff_span8k 200 python bench.py --mode vbp_ff --steps 10 --warmup 3 --extra 0 --cpu-baseline-seconds 0 || exit 1
PYTHONPATH=$PWD/pivot-scheduling_amd step g43_caff_unsorted 200 python - <<'PY' || exit 1
import time, numpy as np, torch
from pivot_place import _abi, synthetic
from pivot_place.engine import default_engine
e = default_engine()
r = synthetic.make_round(_abi.PVT_CA_FF, 1_000_000, 10_000, seed=0, sort_hosts=False)
for zw in (True, False):
    e.set_zero_walk(zw); e.place(r); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5): e.place(r)
    torch.cuda.synchronize()
    print("ca_ff unsorted zero_walk", zw, "ms", (time.perf_counter() - t) / 5 * 1e3, e.epoch_stats(), e.last_stats())
PY
cat gpurun_out/g43_caff_unsorted.log
