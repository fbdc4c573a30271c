#!/bin/bash
# Round 4: real-slot sort networks in the default build (prep kernel and
# float SIGMA, rs_pick): stack parity suites, bench lines; interleaved SIGMA
# columns at G = 4 (variants/il) as an A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04r}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_stack_gpu.py tests/test_sum_order.py tests/test_sequence.py tests/test_capi_c.py tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
for c in winsorized100 sigma400 sigma100 winsorized400 winsorized12_s1 percentile100; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
[ -f variants/il/libsirilgpu.so ] || exit 0
for c in sigma400 sigma100 percentile100; do
  SGPU_LIB=variants/il/libsirilgpu.so timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/il_$c.log 2>&1 || exit $?
  echo "il $c $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/il_$c.log | tr '\n' ' ')"
done
