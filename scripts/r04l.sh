#!/bin/bash
# Round 4: why the sorted kernel costs ~9 ms at N = 12 whatever the type:
# VALU PMC of the NP = 16 SIGMA kernel (routing off) and of sigma100.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04l}
mkdir -p gpurun_out/$T
SGPU_SMALL_ALL=0 timeout -k 10 600 bash scripts/pmc_session.sh $T/pmc_s12 sigma12 k_stack_sorted || exit $?
timeout -k 10 600 bash scripts/pmc_session.sh $T/pmc_s100 sigma100 k_stack_sorted || exit $?
export TMPDIR=/tmp
SGPU_SMALL_ALL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/kt_s12 -o run --output-format csv -- python3 bench.py --config sigma12 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/kt_s12.log 2>&1
echo "kt rc=$?"
