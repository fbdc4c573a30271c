#!/bin/bash
# Round 5 session k: the one-wave-per-pixel exact kernel (stack_exact_wave.hip)
# suite, then config 4 (whole frame and one rank's 500-row band) with and
# without it (SGPU_EXACT_WAVE=0), the headline and the N = 12 master case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05k}
O=gpurun_out/$T; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if fatal $rc; then echo "FATAL rc=$rc in $name"; exit $rc; fi
  return 0
}
run pytest_stack 600 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 300 --timeout-method thread -rf
run b_sigma400 300 python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run b_sigma400_oldexact 300 env SGPU_EXACT_WAVE=0 python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run band_sigma400 300 python bench.py --config sigma400 --band-rows 500 --steps 10 --warmup 3 --no-cpu-baseline
run band_sigma400_oldexact 300 env SGPU_EXACT_WAVE=0 python bench.py --config sigma400 --band-rows 500 --steps 10 --warmup 3 --no-cpu-baseline
run b_winsorized100 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run b_winsorized12_s1 300 python bench.py --config winsorized12_s1 --steps 10 --warmup 3 --no-cpu-baseline
echo "session done"
