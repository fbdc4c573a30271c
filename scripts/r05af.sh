#!/bin/bash
# Round 5 session af: DFT (config 3) knobs re-measured after the
# transpose-free layout: frame-fastest XCD-contiguous column order
# (SGPU_DFT_REMAP=1) and the split column passes (SGPU_DFT_FUSED=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05af}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_dft100_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_dft100_$name.log")"
}
for i in 1 2; do ab def SGPU_X=0; ab remap SGPU_DFT_REMAP=1; ab split SGPU_DFT_FUSED=0; done
echo "session done"
