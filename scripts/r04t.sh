#!/bin/bash
# Round 4: the prep kernel's gather bounded at the real-slot bound too
# (variants/pg, SGPU_PREP_GATHER_RS=1) vs the default (runtime gather stop
# only), and the rounds kernel at 6 / 4 waves per SIMD (SGPU_WZ_RW),
# alternated three times in one session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04t}
mkdir -p gpurun_out/$T
for i in 1 2 3; do
  for v in def pg rw6 rw4 w5; do
    L=siril_amd/libsirilgpu.so; E=X=0
    case $v in pg) L=variants/pg/libsirilgpu.so;; w5) L=variants/w5/libsirilgpu.so;; rw6) E=SGPU_WZ_RW=6;; rw4) E=SGPU_WZ_RW=4;; esac
    env SGPU_LIB=$L $E timeout -k 10 300 python bench.py --config winsorized100 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/ab_${v}_$i.log 2>&1 || exit $?
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/ab_${v}_$i.log)"
  done
done
