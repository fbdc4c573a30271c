#!/bin/bash
# Round 4: kernel breakdown of the deferral-heavy small-N master case
# (winsorized12_s1) and of config 4 (sigma400).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04g}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for c in winsorized12_s1 sigma400; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 > gpurun_out/$T/prof_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
