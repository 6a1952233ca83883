# r02 session 12: scout-split variants (PVT_SPLIT_CA / PVT_SPLIT_VBP builds in build/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local lib=$1 m=$2 name=g12_$1_$2; if [ "$lib" = main ]; then L=$PWD/pivot-scheduling_amd/pivot_place/libpivot_place.so; else L=$PWD/pivot-scheduling_amd/build/libpivot_place_$lib.so; fi
  PIVOT_PLACE_LIB=$L timeout -k 10 200 python -u bench.py --mode $m --steps 20 --warmup 5 --extra 0 --cpu-baseline-seconds 0 > gpurun_out/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"commit": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"parity": [a-z]*' gpurun_out/$name.log | head -1)"; return $rc; }
for lib in main ca0 ca3 ca5 ca6 main; do run $lib ca_bf || exit 1; done
for lib in main vbp2 vbp4; do run $lib vbp_bf || exit 1; done
