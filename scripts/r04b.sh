#!/bin/bash
# Round 4, secondary measurements at HEAD: bench lines of BASELINE configs 3,
# 4, 5 (FFT and MFMA-direct), RCD, norm, fits10 and the deferral-heavy small-N
# master case; per-step HBM traffic of each; MFMA utilisation of the direct
# RL convolution.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04b}
bash scripts/r03_session.sh $T bench_sigma400 bench_winsorized12_s1 bench_dft100 bench_rl63 bench_rl63_direct bench_rcd bench_norm100 bench_fits10 || exit $?
bash scripts/r03_session.sh $T traffic_sigma400 traffic_dft100 traffic_rl63 traffic_rcd traffic_winsorized12_s1 || exit $?
timeout -k 10 400 bash scripts/pmc_mfma.sh $T/mfma_rl63_direct
