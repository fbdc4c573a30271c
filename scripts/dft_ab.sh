#!/bin/bash
# DFT variants (variants/<name>/libsirilgpu.so): DFT/quality GPU tests, then dft100 twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-dftab}; mkdir -p "$O"
for v in default $(ls variants); do
  if [ "$v" = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
  SGPU_LIB=$lib timeout -k 10 300 python -m pytest tests/test_dft_gpu.py tests/test_quality.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/check_$v.log 2>&1
  echo "check $v rc=$? $(tail -1 $O/check_$v.log)"
done
for rep in 1 2; do
  for v in default $(ls variants); do
    if [ "$v" = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
    SGPU_LIB=$lib timeout -k 10 300 python bench.py --config dft100 --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.$rep.log 2>&1 || { echo "FAIL $v"; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/$v.$rep.log') if l.startswith('{')][-1]); print('$rep $v', d['value'], d['ms_per_step'], d['roofline']['pipeline_ms'])"
  done
done
