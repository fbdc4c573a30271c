#!/bin/bash
# Round 4: config 2 after the fetch-address and clamp-width trims (A/B vs the
# tails build), Winsorized parity, VALU PMC of every moment-path kernel of one
# step and the step's HBM traffic at this source hash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04e}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or golden or block_parity or full_frame or stress" > gpurun_out/$T/pytest_wz.log 2>&1
rc=$?; echo "pytest wz rc=$rc $(tail -n 1 gpurun_out/$T/pytest_wz.log)"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 bash scripts/ab_env.sh $T winsorized100 "-" "SGPU_LIB=variants/tails/libsirilgpu.so" "-" "SGPU_LIB=variants/tails/libsirilgpu.so" || exit $?
timeout -k 10 900 bash scripts/pmc_session.sh $T/pmc_w winsorized100 k_stack || exit $?
bash scripts/r03_session.sh $T traffic_winsorized100
