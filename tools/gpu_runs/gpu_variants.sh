#!/bin/bash
# Commit-walk build variants (producer waves x lookahead): bench lines per variant library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ${LIBS:-p3_l3 p7_l3 p3_l2 p7_l2}; do
  for m in ${MODES:-ca_bf vbp_ff}; do
    PIVOT_PLACE_LIB=$PWD/pivot-scheduling_amd/build/libpivot_place_$lib.so timeout -k 10 200 python -u bench.py --mode $m --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/var_${lib}_$m.log 2>&1
    rc=$?; echo "=== $lib $m rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/var_${lib}_$m.log; exit $rc; fi
  done
done
