#!/bin/bash
# Round 5 session d: the legs of session c after the bench.py aux-config fix
# (_dist_setup): demosaic lines, sigma400, per-rank band A/B, the fused
# moment-path kernel (SGPU_WZ=7) suite and lines, end-to-end sequence stacks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05d}
mkdir -p gpurun_out/$T
line() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"pipeline_ms": [0-9.]*\|"frac": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/$1.log | tr '\n' ' ')"; }
for c in bayerfast rcd sigma400; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  line b_$c
done
for c in winsorized100 sigma400; do
  timeout -k 10 300 python bench.py --config $c --band-rows 500 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/band_$c.log 2>&1 || exit $?
  line band_$c
  SGPU_WZ_MINCH=1 timeout -k 10 300 python bench.py --config $c --band-rows 500 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/band1_$c.log 2>&1 || exit $?
  line band1_$c
done
SGPU_WZ=7 timeout -k 10 600 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q -k "golden or block_parity or full_frame or winsorized or sum_order or u16_winsorized" --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_wz7.log 2>&1
rc=$?; echo "pytest wz7 rc=$rc $(tail -n 1 gpurun_out/$T/pytest_wz7.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/$T/pytest_wz7.log | head -60; exit $rc; }
for c in winsorized100 winsorized100_u16 winsorized400; do
  SGPU_WZ=7 timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/wz7_$c.log 2>&1 || exit $?
  line wz7_$c
done
SGPU_WZ=7 timeout -k 10 300 python bench.py --config winsorized100 --band-rows 500 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/wz7_band_winsorized100.log 2>&1 || exit $?
line wz7_band_winsorized100
for c in seq100 seq100_ser fits10; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"achieved": [0-9.]*\|"peak": [0-9.]*\|"end_to_end_input_gbs": [0-9.]*\|"kernel_ms": [0-9.]*\|"h2d_ms": [0-9.]*\|"readers_s": [0-9.]*\|"loop_s": [0-9.]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
