#!/bin/bash
# Round 3: round-wise rounds kernel (SGPU_WZ_RW=100) vs the one-launch nest
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03q}
mkdir -p gpurun_out/$T
SGPU_WZ_RW=100 timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or full_size or stress" > gpurun_out/$T/pytest_rw.log 2>&1
echo "pytest rc=$? $(tail -n 1 gpurun_out/$T/pytest_rw.log)"
timeout -k 10 500 bash scripts/ab_env.sh $T winsorized100 "SGPU_WZ_RW=5" "SGPU_WZ_RW=100" "SGPU_WZ_RW=5" "SGPU_WZ_RW=100" || exit $?
timeout -k 10 300 bash scripts/ab_env.sh $T winsorized400 "SGPU_WZ_RW=5" "SGPU_WZ_RW=100" || exit $?
mkdir -p gpurun_out/$T/prof
SGPU_WZ_RW=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
find gpurun_out/$T -name "*kernel_trace.csv" -delete
timeout -k 10 400 bash scripts/ab_env.sh $T dft100 "SGPU_DFT_REMAP=0" "SGPU_DFT_REMAP=1" "SGPU_DFT_REMAP=0" "SGPU_DFT_REMAP=1" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_dft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_dft.log 2>&1
echo "pytest dft rc=$? $(tail -n 1 gpurun_out/$T/pytest_dft.log)"
