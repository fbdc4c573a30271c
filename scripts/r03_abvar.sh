#!/bin/bash
# Round 3: A/B of the gather stop and the late pixel index (variant libraries)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03n}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u -m pytest tests/test_noise.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_noise.log 2>&1
echo "pytest noise rc=$? $(tail -n 1 gpurun_out/$T/pytest_noise.log)"
for cfg in sigma400 winsorized400 sigma100 winsorized100; do
  timeout -k 10 400 bash scripts/ab_env.sh $T $cfg "-" "SGPU_LIB=variants/nostop/libsirilgpu.so" "SGPU_LIB=variants/nolate/libsirilgpu.so" "-" || exit $?
done
