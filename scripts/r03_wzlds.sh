#!/bin/bash
# Round 3: rounds kernel with LDS-staged ranks (SGPU_WZ_RW=64) vs the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03k}
timeout -k 10 400 bash scripts/ab_env.sh $T winsorized100 "SGPU_WZ_RW=5" "SGPU_WZ_RW=64" "SGPU_WZ_RW=5" "SGPU_WZ_RW=64" || exit $?
timeout -k 10 300 env SGPU_WZ_RW=64 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or full_size or stress" > gpurun_out/$T/pytest_lds.log 2>&1
echo "pytest rc=$? $(tail -1 gpurun_out/$T/pytest_lds.log)"
mkdir -p gpurun_out/$T/prof
SGPU_WZ_RW=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
find gpurun_out/$T -name "*kernel_trace.csv" -delete
