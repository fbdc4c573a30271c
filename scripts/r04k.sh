#!/bin/bash
# Round 4: PERCENTILE / SIGMEDIAN on the small-column kernels (parity of the
# stack suites) and their routing A/B; sigma24 default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04k}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py tests/test_sequence.py tests/test_capi_c.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in percentile12 sigmedian12; do
  timeout -k 10 300 bash scripts/ab_env.sh $T $c "-" "SGPU_SMALL_ALL=0" || exit $?
done
timeout -k 10 300 python bench.py --config sigma24 --steps 5 --warmup 2 > gpurun_out/$T/b_sigma24.log 2>&1
echo "sigma24 rc=$? $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/$T/b_sigma24.log | tr '\n' ' ')"
