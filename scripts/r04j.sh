#!/bin/bash
# Round 4: X-Trans interpolation by Jacobi passes (parity), small-column
# routing at N = 17..32 (A/B), and the default routing's small-N lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04j}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_cfa.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in winsorized24 sigma24 winsorized32_s1; do
  timeout -k 10 300 bash scripts/ab_env.sh $T $c "-" "SGPU_SMALL_ALL=32" || exit $?
done
for c in winsorized12_s1 winsorized12 sigma12; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/$T/b_$c.log 2>&1
  echo "$c rc=$? $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
