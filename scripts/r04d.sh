#!/bin/bash
# Round 4: per-chunk tails of the moment path on a third stream (A/B against
# SGPU_WZ_TAILS=0), parity of the Winsorized suite with the tails.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04d}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or golden or block_parity or full_frame or stress or aggressive" > gpurun_out/$T/pytest_wz.log 2>&1
rc=$?; echo "pytest wz rc=$rc $(tail -n 1 gpurun_out/$T/pytest_wz.log)"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 bash scripts/ab_env.sh $T winsorized100 "-" "SGPU_WZ_TAILS=0" "-" "SGPU_WZ_TAILS=0" || exit $?
