#!/bin/bash
# Resident kernel / scenario batches: GPU tests of the new path, then bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -z "$NOTEST" ]; then
run t_batch 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread
run t_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
fi
for w in ${WAVES:-1 4}; do
for m in ${MODES:-ca_bf ca_ff opp vbp_ff vbp_bf}; do
  PVT_RES_WAVES=$w run bb_${m}_w$w 200 python -u bench.py --mode $m --batch ${B:-512} --hosts ${H:-1000} --tasks ${T:-1000} --steps 3 --warmup 1 --cpu-baseline-seconds 0
done
done
