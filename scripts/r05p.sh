#!/bin/bash
# Round 5 session p: config 2 with the moment path's prep / rounds overlap on
# (SGPU_WZ=2, default at N <= 128) and off (SGPU_WZ=4), chunk sizes, tails.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05p}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_$name.log")"
}
ab def SGPU_X=0
ab wz4 SGPU_WZ=4
ab wz3 SGPU_WZ=3
ab wz4_tails0 SGPU_WZ=4 SGPU_WZ_TAILS=0
ab def_tails0 SGPU_WZ_TAILS=0
ab wz4_c6m SGPU_WZ=4 SGPU_WZ_CHUNK=6000000
ab def2 SGPU_X=0
echo "session done"
