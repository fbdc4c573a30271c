#!/bin/bash
# GPU session runner: smoke, GPU tests, headline bench, rocprof kernel stats,
# PMC passes.  usage: scripts/session.sh TAG [steps]
# Every GPU step has its own time limit; a fault / abort / time-out ends the
# session, an ordinary test failure does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03}; shift
STEPS=${*:-smoke tests bench}
O=gpurun_out/$TAG; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log" | cut -c1-600
  if fatal $rc; then echo "FATAL rc=$rc in $name"; exit $rc; fi
  return 0
}
rocm-smi --showclocks > "$O/clocks.txt" 2>&1 || true
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf --durations=15;;
    tests_k) run pytest_k 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -s -k "${PYTEST_K}";;
    tests_stack) run pytest_stack 900 python -u -m pytest tests/test_stack_gpu.py tests/test_distributed_gpu.py tests/test_mean_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -rf;;
    fscheck) run fscheck 400 python scripts/fs_check.py 100 4000 6000;;
    fs_*) x=${s#fs_}; cfg=${x%_p*}; k=${x##*_p}; run "fs_${cfg}_p$k" 600 python bench.py --config "$cfg" --input frame-sharded --pipeline "$k" --steps 3 --warmup 1 --no-cpu-baseline;;
    band_*) x=${s#band_}; cfg=${x%_*}; r=${x##*_}; run "band_${cfg}_$r" 600 python bench.py --config "$cfg" --band-rows "$r" --steps 10 --warmup 3 --no-cpu-baseline;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline;;
    pmc) run pmc 900 bash scripts/pmc_session.sh "$TAG/pmc_w" winsorized100 k_stack_sorted;;
    pmc_s400) run pmc_s400 900 bash scripts/pmc_session.sh "$TAG/pmc_s400" sigma400 k_stack_sorted;;
    bench_*) cfg=${s#bench_}; run "b_$cfg" 600 python bench.py --config "$cfg" --steps 5 --warmup 2;;
    traffic_*) cfg=${s#traffic_}; run "tr_$cfg" 600 bash scripts/pmc_traffic.sh "$TAG/tr_$cfg" "$cfg";;
    sprof_*) cfg=${s#sprof_}; run "sp_$cfg" 300 env SGPU_LIB=variants/prof/libsirilgpu.so SGPU_PROF=1 python bench.py --config "$cfg" --steps 1 --warmup 1 --no-cpu-baseline;;
    prof_*) cfg=${s#prof_}; run "p_$cfg" 600 rocprofv3 --kernel-trace --stats -d "$O/p_$cfg" -o run --output-format csv -- python bench.py --config "$cfg" --steps 5 --warmup 2 --no-cpu-baseline;;
  esac
done
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
echo "session done"
