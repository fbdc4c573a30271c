#!/bin/bash
# Round 5 session a: streaming mean kernel (unrolled non-temporal loads,
# order guard, 16-bit twin): mean parity suite + stack suite, mean100 /
# mean100_u16 / median100 lines, rocprofv3 kernel stats of mean100.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05a}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_mean_gpu.py tests/test_stack_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
grep "order guard" gpurun_out/$T/pytest.log | head
[ $rc -eq 0 ] || exit $rc
for c in mean100 mean100_u16 median100 winsorized100; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python bench.py --config mean100 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1 || exit $?
find gpurun_out/$T/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/mean100_kernel_stats.csv \;
head -5 gpurun_out/$T/mean100_kernel_stats.csv
