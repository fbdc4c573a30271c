#!/bin/bash
# Round 4: feathering masks (compute_masks / stack_read_block_data mask
# planes / -feather= sequence stacks) and the suites the ABI-4 options
# struct touches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04f}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_feather.py tests/test_capi_c.py tests/test_sequence.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
exit $rc
