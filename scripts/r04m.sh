#!/bin/bash
# Round 4: striped rejection totals (one atomic pair per wave on one address
# serialises across XCDs): parity, then A/B on the sorted and moment paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04m}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py tests/test_distributed.py tests/test_capi_c.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in winsorized100 sigma100 sigma400 percentile100; do
  timeout -k 10 400 bash scripts/ab_env.sh $T $c "-" "SGPU_COUNT_STRIPES=0" || exit $?
done
