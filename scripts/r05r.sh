#!/bin/bash
# Round 5 session r: config 2 with smaller rank records (KT / KM variants)
# and the rounds kernel reading them from LDS (SGPU_WZ_RW=64) instead of
# dependent global loads; full-frame parity on the LDS legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05r}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1 lib=$2 extra=$3; shift 3
  env SGPU_LIB=$PWD/$lib "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 $extra > "$O/ab_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_$name.log") $(grep -o '"mismatches": [0-9]*' "$O/ab_$name.log")"
}
M=siril_amd/libsirilgpu.so
ab def $M --no-cpu-baseline SGPU_X=0
ab def_rw64 $M --no-cpu-baseline SGPU_WZ_RW=64
ab kt16km8 variants/kt16km8/libsirilgpu.so --no-cpu-baseline SGPU_X=0
ab kt16km8_rw64 variants/kt16km8/libsirilgpu.so --no-cpu-baseline SGPU_WZ_RW=64
ab kt20km8 variants/kt20km8/libsirilgpu.so --no-cpu-baseline SGPU_X=0
ab kt20km8_rw64 variants/kt20km8/libsirilgpu.so --no-cpu-baseline SGPU_WZ_RW=64
ab def2 $M --no-cpu-baseline SGPU_X=0
ab kt16km8_rw64_parity variants/kt16km8/libsirilgpu.so "" SGPU_WZ_RW=64
ab kt20km8_rw64_parity variants/kt20km8/libsirilgpu.so "" SGPU_WZ_RW=64
echo "session done"
