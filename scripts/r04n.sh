#!/bin/bash
# Round 4: wave-aggregated fallback appends + striped totals: parity, the
# headline, and the small-N routing re-measured now that the sorted kernels
# no longer pay per-wave same-address atomics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04n}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py tests/test_sum_order.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash scripts/ab_env.sh $T winsorized100 "-" "-" || exit $?
for c in sigma12 percentile12 sigmedian12 winsorized12 winsorized12_s1 sigma24; do
  timeout -k 10 300 bash scripts/ab_env.sh $T $c "-" "SGPU_SMALL_ALL=0" || exit $?
done
timeout -k 10 300 bash scripts/ab_env.sh $T winsorized24 "-" "SGPU_SMALL_ALL=32" || exit $?
