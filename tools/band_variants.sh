#!/bin/bash
# Band-list kernel variants A/B on the GPU: the band tests (and the config-5 vbp best-fit parity
# test) against each diagnostic build in diag/ named on the command line ("default" = the shipped
# library). Test failures (rc 1) go on to the next variant; any other status (fault, abort,
# timeout) ends the call there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in "$@"; do
  if [ "$v" = default ]; then unset PIVOT_PLACE_LIB; else export PIVOT_PLACE_LIB=$PWD/pivot-scheduling_amd/diag/libpivot_place_$v.so; fi
  TAILN=6 tools/gpu_step.sh band_$v 240 python -u -m pytest -s -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_band.py "tests/test_gpu_headline.py::test_config5_round_matches_oracle" -k "band or vbp_bf"
  rc=$?
  [ $rc -le 1 ] || exit $rc
done
