#!/bin/bash
# Round 5 session ap: config 3, final plan (5 x 8 x 10 x 10) vs the round's
# starting plan (SGPU_DFT_PLAN=8,5,5,5,4), alternating, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ap}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_dft100_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"pipeline_ms": [0-9.]*' "$O/ab_dft100_$name.log" | tr '\n' ' ')"
}
for i in 1 2; do ab final SGPU_X=0; ab start SGPU_DFT_PLAN=8,5,5,5,4; done
echo "session done"
