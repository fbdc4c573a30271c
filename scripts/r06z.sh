#!/bin/bash
# Round 6 session z: the measurement record at the final round-6 kernel sources --
# full GPU suite, smoke, the headline line, rocprofv3 kernel stats of the
# headline and of mean100, VALU / wait PMC passes of config 2 and config 4,
# FETCH / WRITE traffic of every line bench.py attaches it to, the bench
# lines of the secondary configs (part 2), and (part 3) the MFMA PMC of the
# direct RL convolution, one rank's row bands and the frame-sharded line.  Merges run on the host afterwards
# (scripts/merge_pmc.py, scripts/merge_traffic.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06z}
PART=${2:-all}
O=gpurun_out/$T; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if fatal $rc; then echo "FATAL rc=$rc in $name"; exit $rc; fi
  return 0
}
if [ "$PART" = all ] || [ "$PART" = 1 ]; then
run pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 20 --warmup 5
run prof 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run prof_mean100 600 rocprofv3 --kernel-trace --stats -d "$O/prof_mean100" -o run --output-format csv -- python bench.py --config mean100 --steps 20 --warmup 5 --no-cpu-baseline
run pmc_w 900 bash scripts/pmc_session.sh "$T/pmc_w" winsorized100 k_stack
run pmc_s400 900 bash scripts/pmc_session.sh "$T/pmc_s400" sigma400 k_stack
fi
# part 2 = 2a + 2b (each within one gpurun call's limit)
if [ "$PART" = all ] || [ "$PART" = 2 ] || [ "$PART" = 2a ]; then
for c in winsorized100 sigma400 mean100 median100 dft100 rl63 rcd bayerfast norm100; do
  run tr_$c 600 bash scripts/pmc_traffic.sh "$T/tr_$c" "$c"
done
fi
if [ "$PART" = all ] || [ "$PART" = 2 ] || [ "$PART" = 2b ]; then
for c in sigma400 mean100 median100 winsorized100_u16 winsorized128 winsorized12_s1 dft100 rl63 rl63_direct rcd bayerfast norm100 fits10 seq100; do
  run b_$c 600 python bench.py --config $c --steps 10 --warmup 3
done
fi
if [ "$PART" = all ] || [ "$PART" = 3 ]; then
run mfma 400 bash scripts/pmc_mfma.sh "$T/mfma"
run band_winsorized100_500 600 python bench.py --config winsorized100 --band-rows 500 --steps 10 --warmup 3 --no-cpu-baseline
run band_sigma400_500 600 python bench.py --config sigma400 --band-rows 500 --steps 10 --warmup 3 --no-cpu-baseline
run band_sigma400_100 600 python bench.py --config sigma400 --band-rows 100 --steps 10 --warmup 3 --no-cpu-baseline
run fs_sigma400_p4 600 python bench.py --config sigma400 --input frame-sharded --pipeline 4 --steps 3 --warmup 1 --no-cpu-baseline
fi
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
find "$O" -name "*kernel_stats.csv" | while read f; do d=$(basename $(dirname "$f")); cp "$f" "$O/${d}_kernel_stats.csv"; done
echo "session done"
