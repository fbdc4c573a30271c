#!/bin/bash
# Round 4: sort networks pruned by a compile-time real-slot bound
# (variants/rs: SGPU_RS64=52, SGPU_RS128=100) against the default build;
# parity of the variant from the bench line's full-frame oracle comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04q}
mkdir -p gpurun_out/$T
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/$T/ab_$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $* $(grep -o '"ms_per_step": [0-9.]*\|"mismatches": [0-9]*\|"exact_pixels": [0-9]*' gpurun_out/$T/ab_$n.log | tr '\n' ' ')"
  return $rc
}
for c in winsorized100 sigma400 sigma100 percentile100; do
  run ${c}_def $c X=0 && run ${c}_rs $c SGPU_LIB=variants/rs/libsirilgpu.so || exit $?
done
