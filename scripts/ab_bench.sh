#!/bin/bash
# A/B timing of one bench config across variant libraries (main = in-tree).
# usage: scripts/ab_bench.sh TAG CONFIG variant...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for v in "$@"; do
  if [ "$v" = main ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
  SGPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config "$CFG" --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${CFG}_$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${CFG}_$v.log")"
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac
done
