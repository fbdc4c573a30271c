#!/bin/bash
# Round 4, first GPU session: GPU tests (full-frame parity, compiled C caller,
# advisor regressions), smoke, headline bench with full-frame parity, kernel
# stats, A/B of the batched rank walks and of MALL-sized chunks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04a}
bash scripts/r03_session.sh $T smoke tests bench prof || exit $?
timeout -k 10 600 bash scripts/ab_env.sh $T winsorized100 "-" "SGPU_LIB=variants/nobatch/libsirilgpu.so" \
  "SGPU_WZ_CHUNK=1048576" "SGPU_WZ_CHUNK=524288" "SGPU_WZ_CHUNK=262144" "-" "SGPU_LIB=variants/nobatch/libsirilgpu.so"
bash scripts/r03_session.sh $T bench_winsorized100_u16 bench_winsorized100_u16_norm
