#!/bin/bash
# Round 5 session al / am: pass order of the 4000-point plan (SGPU_DFT_PLAN), config 3.
# usage: r05al.sh TAG [am]  (am: the second set, the small radix first)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05al}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_dft100_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"pipeline_ms": [0-9.]*' "$O/ab_dft100_$name.log" | tr '\n' ' ')"
}
if [ "${2:-al}" = am ]; then
for i in 1 2; do
  ab p5_10_10_8 SGPU_DFT_PLAN=5,10,10,8
  ab p5_8_10_10 SGPU_DFT_PLAN=5,8,10,10
  ab p5_10_8_10 SGPU_DFT_PLAN=5,10,8,10
  ab p10_10_5_8 SGPU_DFT_PLAN=10,10,5,8
done
echo "session done"
exit 0
fi
for i in 1 2; do
  ab def SGPU_X=0
  ab p10_10_8_5 SGPU_DFT_PLAN=10,10,8,5
  ab p5_10_10_8 SGPU_DFT_PLAN=5,10,10,8
  ab p8_5_10_10 SGPU_DFT_PLAN=8,5,10,10
  ab p4_10_10_10 SGPU_DFT_PLAN=4,10,10,10
  ab p10_4_10_10 SGPU_DFT_PLAN=10,4,10,10
done
echo "session done"
