#!/bin/bash
# Round 5 session f: 16-bit exact gather in flight, result rows streamed to
# the output file during the block loop (suites + sequence lines), and the
# rank-record size A/B (variants/kt20km8, kt24km8: KT ranks per end, KM
# around the median; default KT = 24, KM = 16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05f}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_stack_gpu.py tests/test_sequence.py tests/test_feather.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/$T/pytest.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/$T/pytest.log | head -60; exit $rc; }
line() { echo "$1 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"exact_kernel_ms": [0-9.]*\|"frac": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/$1.log | tr '\n' ' ')"; }
for c in seq100 seq100_ser fits10; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 > gpurun_out/$T/b_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"achieved": [0-9.]*\|"peak": [0-9.]*\|"end_to_end_input_gbs": [0-9.]*\|"h2d_ms": [0-9.]*\|"loop_s": [0-9.]*\|"setup_s": [0-9.]*\|"write_s": [0-9.]*\|"call_s": [0-9.]*' gpurun_out/$T/b_$c.log | tr '\n' ' ')"
done
for rep in 1 2; do
  for v in default kt20km8 kt24km8; do
    L=""; [ $v != default ] && L="SGPU_LIB=variants/$v/libsirilgpu.so"
    [ $v != default ] && [ ! -f variants/$v/libsirilgpu.so ] && continue
    env $L timeout -k 10 300 python bench.py --config winsorized100 --steps 10 --warmup 3 --cpu-seconds 4 > gpurun_out/$T/ab_${v}_$rep.log 2>&1 || exit $?
    line ab_${v}_$rep
  done
done
for v in default kt20km8 kt24km8; do
  L=""; [ $v != default ] && L="SGPU_LIB=variants/$v/libsirilgpu.so"
  [ $v != default ] && [ ! -f variants/$v/libsirilgpu.so ] && continue
  env $L timeout -k 10 300 python bench.py --config winsorized400 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/ab400_$v.log 2>&1 || exit $?
  line ab400_$v
done
