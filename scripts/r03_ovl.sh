#!/bin/bash
# Round 3: overlapped prep / rounds on two streams (SGPU_WZ=3) vs one stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03s}
mkdir -p gpurun_out/$T
SGPU_WZ=3 timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or full_size or stress or multi" > gpurun_out/$T/pytest_ovl.log 2>&1
echo "pytest ovl rc=$? $(tail -n 1 gpurun_out/$T/pytest_ovl.log)"
timeout -k 10 400 bash scripts/ab_env.sh $T winsorized100 "SGPU_WZ=2" "SGPU_WZ=3" "SGPU_WZ=2" "SGPU_WZ=3" || exit $?
timeout -k 10 300 bash scripts/ab_env.sh $T winsorized400 "SGPU_WZ=2" "SGPU_WZ=3" || exit $?
mkdir -p gpurun_out/$T/prof
SGPU_WZ=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
find gpurun_out/$T -name "*kernel_trace.csv" -delete
