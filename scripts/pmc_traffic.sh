#!/bin/bash
# HBM traffic of every library kernel of one bench step (secondary configs:
# dft100, rl63, rcd, norm100): two rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass), one step, no warmup; then the per-kernel
# summary.  usage: scripts/pmc_traffic.sh OUTDIR CONFIG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; CFG=$2
mkdir -p "$O"
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  echo "pass $i: $c ($CFG)"
  timeout -s KILL 240 rocprofv3 --pmc $c -d "$O/t$i" -o run --output-format csv -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline > "$O/t$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$O/t$i.log"; fi
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
python scripts/pmc_traffic_summary.py "$CFG" "$O"/t1 "$O"/t2 > "$O/traffic.json" 2>&1; tail -25 "$O/traffic.json"
rm -rf "$O"/t[0-9]/
