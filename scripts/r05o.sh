#!/bin/bash
# Round 5 session o: kernel stats of the DFT registration (config 3) and RL
# deconvolution (config 5) lines -- where the step goes before touching the
# transposes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05o}
O=gpurun_out/$T; mkdir -p "$O"
for c in dft100 rl63; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$c" -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_$c.log" 2>&1 || exit $?
done
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
find "$O" -name "*kernel_stats.csv" | while read f; do d=$(basename $(dirname "$f")); cp "$f" "$O/${d}_kernel_stats.csv"; done
for c in dft100 rl63; do echo "== $c"; head -12 "$O/prof_${c}_kernel_stats.csv" | cut -d, -f1-4; done
echo "session done"
