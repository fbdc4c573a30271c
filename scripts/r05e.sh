#!/bin/bash
# Round 5 session e: two-pass bayerfast, pipelined exact kernel (gather in
# flight, Lomuto read-ahead), threaded FITS output, fused kernel removed:
# GPU suites, then the affected bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05e}
mkdir -p gpurun_out/$T
timeout -k 10 1100 python -u -m pytest tests/test_demosaic.py tests/test_stack_gpu.py tests/test_mean_gpu.py tests/test_sequence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/$T/pytest.log | head -60; exit $rc; }
line() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"exact_kernel_ms": [0-9.]*\|"pipeline_ms": [0-9.]*\|"frac": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/$1.log | tr '\n' ' ')"; }
for c in bayerfast sigma400 winsorized100 winsorized12_s1; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  line b_$c
done
timeout -k 10 300 python bench.py --config sigma400 --band-rows 500 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/band_sigma400.log 2>&1 || exit $?
line band_sigma400
for c in seq100 seq100_ser fits10; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"achieved": [0-9.]*\|"peak": [0-9.]*\|"end_to_end_input_gbs": [0-9.]*\|"h2d_ms": [0-9.]*\|"loop_s": [0-9.]*\|"setup_s": [0-9.]*\|"write_s": [0-9.]*\|"call_s": [0-9.]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
