#!/bin/bash
# Config-4 vbp_bf phase stamps (PVT_STAMPS build): where the 4-wave resident round spends its cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh rs_vbp_bf 120 python tools/resident_stamps.py vbp_bf || exit $?
tools/gpu_step.sh rs_ca_ff 120 python tools/resident_stamps.py ca_ff || exit $?
