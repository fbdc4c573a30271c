#!/bin/bash
# Round 5 session ab: config 2's chunking with the smaller records (6 chunks
# of 4 M pixels by default): at most 3 M / 2 M / 1.5 M pixels per chunk
# (SGPU_WZ_CHUNK), and the 500-row band (one chunk) split in 2 / 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ab}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $extra > "$O/ab_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_$name.log")"
}
for i in 1 2; do
  ab def "" SGPU_X=0
  ab c3m "" SGPU_WZ_CHUNK=3000000
  ab c2m "" SGPU_WZ_CHUNK=2000000
  ab c1500k "" SGPU_WZ_CHUNK=1500000
done
ab band "--band-rows 500" SGPU_X=0
ab band_min2 "--band-rows 500" SGPU_WZ_MINCH=2
ab band_min4 "--band-rows 500" SGPU_WZ_MINCH=4
echo "session done"
