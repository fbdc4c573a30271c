#!/bin/bash
# Round 4: the small-column exact kernel (k_stack_exact_small) and the
# two-kernel RCD: parity suites, then winsorized12_s1 A/B (LDS kernel; all
# small columns on the new kernel) and rcd A/B (multi-pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04h}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py tests/test_sum_order.py tests/test_capi_c.py tests/test_demosaic.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash scripts/ab_env.sh $T winsorized12_s1 "-" "SGPU_EXACT_SMALL=0" "SGPU_SMALL_ALL=16" || exit $?
timeout -k 10 300 bash scripts/ab_env.sh $T rcd "-" "SGPU_RCD_FUSED=0" "-" "SGPU_RCD_FUSED=0" || exit $?
timeout -k 10 300 python bench.py --config winsorized12_s1 --steps 5 --warmup 2 > gpurun_out/$T/bench_w12.log 2>&1
echo "bench rc=$? $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*\|"exact_kernel_ms": [0-9.]*' gpurun_out/$T/bench_w12.log | tr '\n' ' ')"
