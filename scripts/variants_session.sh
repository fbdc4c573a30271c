#!/bin/bash
# A/B of tuning variants (variants/<name>/libsirilgpu.so vs the default lib):
# bench of each config + the stack parity tests, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; mkdir -p "$O"
for rep in 1 2; do
  for v in default $(ls variants); do
    if [ "$v" = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
    for cfg in ${CONFIGS:-winsorized100}; do
      SGPU_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.$cfg.$rep.log 2>&1 || { echo "FAIL $v $cfg rc=$?"; exit 1; }
      python -c "import json; d=json.loads([l for l in open('$O/$v.$cfg.$rep.log') if l.startswith('{')][-1]); print('$rep $v $cfg', d['value'], d['roofline']['kernel_ms'], d['exact_pixels'])"
    done
  done
done
for v in default $(ls variants); do
  if [ "$v" = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
  SGPU_LIB=$lib timeout -k 10 300 python -m pytest tests/test_stack_gpu.py -q -x -k "${TESTK:-golden or full_size or block_parity or aggressive or u16}" --timeout 120 > $O/check_$v.log 2>&1
  echo "check $v rc=$? $(tail -1 $O/check_$v.log)"
done
