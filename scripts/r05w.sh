#!/bin/bash
# Round 5 session w: 14 / 8-rank records (variant kt14km8: 36 slots, 9 KB per
# wave of LDS) against the 16 / 8 default, LDS rounds both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05w}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1 lib=$2 cfg=$3; shift 3
  env SGPU_LIB=$PWD/$lib "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $name $cfg"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log")"
}
for cfg in winsorized100 winsorized128 winsorized100_u16; do
  ab kt16 siril_amd/libsirilgpu.so $cfg SGPU_X=0
  ab kt14 variants/kt14km8/libsirilgpu.so $cfg SGPU_X=0
done
echo "session done"
