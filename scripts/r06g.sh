#!/bin/bash
# Round 6 session g: the prep-kernel A/B in isolation -- kernel stats of the
# main library and of the pre-change variant with prep and rounds serialised
# (SGPU_WZ=4) and overlapped (default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p "$O"
for v in main old_prep gbuf_only gather_only; do
  if [ "$v" = main ]; then lib=$PWD/siril_amd/libsirilgpu.so; else lib=$PWD/variants/$v/libsirilgpu.so; fi
  for wz in 2; do
    SGPU_LIB=$lib SGPU_WZ=$wz timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/p_${v}_$wz" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$O/p_${v}_$wz.log" 2>&1
    rc=$?
    echo "$v wz=$wz rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/p_${v}_$wz.log")"
    case $rc in 0) ;; *) echo FATAL; exit $rc;; esac
  done
done
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
