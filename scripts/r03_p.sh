#!/bin/bash
# Round 3: new headless tests, then VALU / traffic PMC of the moment-path kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03p}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_sequence.py tests/test_noise.py -m gpu -q --timeout 120 --timeout-method thread -k "overlap or noise or maximize" > gpurun_out/$T/pytest_new.log 2>&1
echo "pytest rc=$? $(tail -n 1 gpurun_out/$T/pytest_new.log)"
timeout -k 10 800 bash scripts/r03_wzpmc.sh $T/pmc
echo "pmc rc=$?"
