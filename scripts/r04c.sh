#!/bin/bash
# Round 4, headline A/B: batched rank walks at 5 (spilling) and 4 waves/SIMD,
# the unbatched form, MALL-sized chunks, the fused one-lane-per-pixel kernels
# (SGPU_WZ=5 / 6); GPU parity of the fused column kernel; 16-bit bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04c}
mkdir -p gpurun_out/$T
timeout -k 10 900 bash scripts/ab_env.sh $T winsorized100 "-" "SGPU_WZ_RW=4" "SGPU_LIB=variants/nobatch/libsirilgpu.so" \
  "SGPU_WZ=6" "SGPU_WZ_RW=4 SGPU_WZ_CHUNK=1048576" "SGPU_WZ=5" "SGPU_WZ_RW=4" "SGPU_WZ=6" || exit $?
SGPU_WZ=6 timeout -k 10 300 python -u -m pytest tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winsor or Winsor or golden or block_parity or full_frame" > gpurun_out/$T/pytest_wz6.log 2>&1
echo "pytest wz6 rc=$? $(tail -n 1 gpurun_out/$T/pytest_wz6.log)"
bash scripts/r03_session.sh $T bench_winsorized100_u16 bench_winsorized100_u16_norm
