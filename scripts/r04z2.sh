#!/bin/bash
# Round 4 closing session, part 2: config-2 VALU PMC and per-step HBM
# traffic at this kernel-source hash, traffic of the secondary configs whose
# sources changed this round, and their bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04z}
timeout -k 10 600 bash scripts/pmc_session.sh $T/pmc_w winsorized100 k_stack || exit $?
bash scripts/r03_session.sh $T traffic_winsorized100 traffic_sigma400 traffic_dft100 traffic_rcd traffic_winsorized12_s1 bench_sigma400 bench_winsorized12_s1 bench_dft100 bench_rcd bench_norm100 bench_fits10
