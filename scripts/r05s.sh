#!/bin/bash
# Round 5 session s: rank records of 16 / 8 ranks with LDS-staged rounds (the
# new default) against the round-4 records (24 / 16, global reads; variant
# kt24km16 with SGPU_WZ_RW=5) and 24 / 16 staged in LDS, at N = 100 (float,
# 16-bit) and N = 128.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05s}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1 lib=$2 cfg=$3; shift 3
  env SGPU_LIB=$PWD/$lib "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $name $cfg"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log")"
}
M=siril_amd/libsirilgpu.so
V=variants/kt24km16/libsirilgpu.so
for cfg in winsorized100 winsorized128 winsorized100_u16 winsorized400; do
  ab new $M $cfg SGPU_X=0
  ab old $V $cfg SGPU_WZ_RW=5
  ab old_lds $V $cfg SGPU_WZ_RW=64
done
echo "session done"
