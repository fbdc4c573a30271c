#!/bin/bash
# Round 5 session aj: radix-10 passes in the LDS FFT (4000 = 8 x 10 x 10 x 5,
# 4 passes instead of 5): DFT tests (incl. the new peak-value test) with and
# without them, the RL tests, then config 3 A/B (SGPU_DFT_R10=0 is the old plan).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05aj}
O=gpurun_out/$T; mkdir -p "$O"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_dft_gpu.py > "$O/test_dft.log" 2>&1 || { tail -30 "$O/test_dft.log"; echo "FATAL dft tests"; exit 1; }
tail -2 "$O/test_dft.log"
SGPU_DFT_R10=0 timeout -k 10 300 $PT tests/test_dft_gpu.py -k peak > "$O/test_dft_old.log" 2>&1 || { tail -30 "$O/test_dft_old.log"; echo "FATAL old-plan peak tests"; exit 1; }
tail -2 "$O/test_dft_old.log"
timeout -k 10 400 $PT tests/test_rl_gpu.py > "$O/test_rl.log" 2>&1 || { tail -30 "$O/test_rl.log"; echo "FATAL rl tests"; exit 1; }
tail -2 "$O/test_rl.log"
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_dft100_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"pipeline_ms": [0-9.]*' "$O/ab_dft100_$name.log" | tr '\n' ' ')"
}
for i in 1 2; do ab r10 SGPU_X=0; ab old SGPU_DFT_R10=0; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python bench.py --config dft100 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; echo "FATAL prof"; exit 1; }
cp "$O/prof/run_kernel_stats.csv" "$O/kstats.csv"
python3 - "$O/prof/run_kernel_trace.csv" > "$O/vgpr.txt" <<'EOF'
import csv, sys
seen = {}
for r in csv.DictReader(open(sys.argv[1])):
    if 'dft::' in r['Kernel_Name']:
        seen[r['Kernel_Name'].split('(')[0]] = (r['VGPR_Count'], r['Scratch_Size'], r['LDS_Block_Size'])
for k, v in seen.items():
    print(k, v)
EOF
rm -rf "$O/prof"
cat "$O/vgpr.txt"
echo "session done"
