#!/bin/bash
# Round 5 session ak: per-kernel DFT times of the radix-10 plan and the old
# plan (SGPU_DFT_R10=0) on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ak}
O=gpurun_out/$T; mkdir -p "$O"
for v in r10 old; do
  if [ $v = old ]; then export SGPU_DFT_R10=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$v" -o run --output-format csv -- python bench.py --config dft100 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; echo "FATAL prof $v"; exit 1; }
  cp "$O/prof_$v/run_kernel_stats.csv" "$O/kstats_$v.csv"
  rm -rf "$O/prof_$v"
done
echo "session done"
