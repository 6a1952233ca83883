#!/bin/bash
# Round-6 final library, part 1: the whole GPU suite and smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh fin_tests 1100 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests || exit $?
tools/gpu_step.sh fin_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
