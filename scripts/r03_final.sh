#!/bin/bash
# Round 3 closing session: GPU tests, smoke, headline bench, A/B of the
# round-wise rounds and the DFT block order, per-step traffic at HEAD, the
# secondary bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03r}
mkdir -p gpurun_out/$T
bash scripts/r03_session.sh $T tests smoke bench || exit $?
timeout -k 10 400 bash scripts/ab_env.sh $T winsorized100 "SGPU_WZ_RW=5" "SGPU_WZ_RW=100" "SGPU_WZ_RW=5" "SGPU_WZ_RW=100" || exit $?
timeout -k 10 400 bash scripts/ab_env.sh $T dft100 "SGPU_DFT_REMAP=0" "SGPU_DFT_REMAP=1" "SGPU_DFT_REMAP=0" "SGPU_DFT_REMAP=1" || exit $?
SGPU_WZ_RW=100 timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or full_size or stress" > gpurun_out/$T/pytest_rw.log 2>&1
echo "pytest rw rc=$? $(tail -n 1 gpurun_out/$T/pytest_rw.log)"
SGPU_DFT_REMAP=1 timeout -k 10 300 python -u -m pytest tests/test_dft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_remap.log 2>&1
echo "pytest remap rc=$? $(tail -n 1 gpurun_out/$T/pytest_remap.log)"
bash scripts/r03_session.sh $T traffic_winsorized100 traffic_sigma400 traffic_dft100 traffic_rl63 bench_sigma400 bench_dft100 bench_rl63 bench_rcd prof_dft100
