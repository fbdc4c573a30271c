#!/bin/bash
# Round 3: WINSORIZED moment-path A/B (SGPU_WZ mode, rounds-kernel form /
# occupancy), then the kernel split of the default under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r03j}
timeout -k 10 500 bash scripts/ab_env.sh $T winsorized100 "SGPU_WZ=0" "SGPU_WZ=2 SGPU_WZ_RW=4" "SGPU_WZ=2 SGPU_WZ_RW=5" "SGPU_WZ=2 SGPU_WZ_RW=6" || exit $?
timeout -k 10 300 bash scripts/ab_env.sh $T winsorized400 "SGPU_WZ=0" "SGPU_WZ=2" || exit $?
mkdir -p gpurun_out/$T/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
find gpurun_out/$T -name "*kernel_trace.csv" -delete
