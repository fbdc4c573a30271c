#!/bin/bash
# Round 4, first GPU session: GPU tests (full-frame parity, compiled C caller,
# advisor regressions, 16-bit normalized sorted path, partial-sum guard,
# 16-bit DFT, apply_reg), smoke, headline bench with full-frame parity,
# kernel stats, A/B of the batched rank walks, MALL-sized chunks and the
# one-lane-per-pixel fused kernels (SGPU_WZ=5 / 6), 16-bit bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04a}
bash scripts/r03_session.sh $T smoke tests bench prof || exit $?
timeout -k 10 900 bash scripts/ab_env.sh $T winsorized100 "-" "SGPU_LIB=variants/nobatch/libsirilgpu.so" \
  "SGPU_WZ_CHUNK=1048576" "SGPU_WZ_CHUNK=524288" "SGPU_WZ=6" "SGPU_WZ=5" "-" || exit $?
SGPU_WZ=6 timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or golden or block_parity" > gpurun_out/$T/pytest_wz6.log 2>&1
echo "pytest wz6 rc=$? $(tail -n 1 gpurun_out/$T/pytest_wz6.log)"
bash scripts/r03_session.sh $T bench_winsorized100_u16 bench_winsorized100_u16_norm
