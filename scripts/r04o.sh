#!/bin/bash
# Round 4: striped totals in the sequential kernels, small-N routing off:
# parity suites, then bench lines of the stack configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04o}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_stack_gpu.py tests/test_sum_order.py tests/test_sequence.py tests/test_capi_c.py tests/test_distributed.py tests/test_feather.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in winsorized100 winsorized12_s1 winsorized12 sigma12 percentile100 winsorized100_u16 winsorized100_u16_norm sigma100; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > gpurun_out/$T/b_$c.log 2>&1
  echo "$c rc=$? $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
