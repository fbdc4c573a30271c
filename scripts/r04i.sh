#!/bin/bash
# Round 4: the 16-bit small-column kernel and X-Trans nongreen: parity, then
# the small-N routing A/B (sorted + deferred vs every pixel on the
# small-column kernel) on float and 16-bit master cases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04i}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_cfa.py tests/test_stack_gpu.py tests/test_sequence.py tests/test_demosaic.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in winsorized12 sigma12 winsorized12_u16 winsorized12_s1_u16; do
  timeout -k 10 300 bash scripts/ab_env.sh $T $c "-" "SGPU_SMALL_ALL=16" || exit $?
done
