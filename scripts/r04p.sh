#!/bin/bash
# Round 4: moment-path levers re-measured without the rejection-total
# atomics floor (chunk size, fused one-lane kernel, round-wise rounds,
# overlap at NP = 512).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04p}
mkdir -p gpurun_out/$T
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/ab_$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $* $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/$T/ab_$n.log | tr '\n' ' ')"
  return $rc
}
run w100_def winsorized100 X=0 &&
run w100_c256k winsorized100 SGPU_WZ_CHUNK=262144 &&
run w100_c512k winsorized100 SGPU_WZ_CHUNK=524288 &&
run w100_c1m winsorized100 SGPU_WZ_CHUNK=1048576 &&
run w100_wz6 winsorized100 SGPU_WZ=6 &&
run w100_rw100 winsorized100 SGPU_WZ_RW=100 &&
run w100_wz0 winsorized100 SGPU_WZ=0 &&
run w400_def winsorized400 X=0 &&
run w400_ovl winsorized400 SGPU_WZ=3 &&
run w400_c512k winsorized400 SGPU_WZ_CHUNK=524288 &&
run w400_wz0 winsorized400 SGPU_WZ=0
for c in sigma400 sigma100; do
  SGPU_LIB=variants/prof/libsirilgpu.so SGPU_PROF=1 timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$T/prof_$c.log 2>&1 || exit $?
  echo "prof $c: $(grep -A3 SGPU_PROF gpurun_out/$T/prof_$c.log | head -8 | tr '\n' ' ')"
done
