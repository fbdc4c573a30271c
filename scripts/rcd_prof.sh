#!/bin/bash
# RCD kernel stats (fused vs step kernels) and a PMC pass of the fused kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rcdprof}; mkdir -p "$O"
for m in 1 0; do
  SGPU_RCD_FUSED=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/k$m" -o run --output-format csv -- python bench.py --config rcd --steps 10 --warmup 2 --no-cpu-baseline > "$O/k$m.log" 2>&1 || { echo "prof $m failed"; tail -5 "$O/k$m.log"; exit 1; }
done
SGPU_RCD_FUSED=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$O/pmc" -o run --output-format csv -- python bench.py --config rcd --steps 1 --warmup 0 --no-cpu-baseline > "$O/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$O/pmc.log"; }
find "$O" -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -12; done
find "$O" -name "*counter_collection.csv" | while read f; do python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'rcd' in r.get('Kernel_Name', ''):
        acc[r['Counter_Name']] += float(r['Counter_Value'])
print(dict(acc))
PY
done
find "$O" -name "*kernel_trace.csv" -delete
