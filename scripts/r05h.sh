#!/bin/bash
# Round 5 session h: the SIGMA moment path (stack_wz.h SIG form, k_stack_wz
# for float SIGMA columns of 129..1024 samples) -- parity suites, then
# config 4 (sigma400) against the register-resident kernel (SGPU_SIGM=0) and
# the G = 8 variant, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05h}
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
run pytest_sigma 400 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 200 --timeout-method thread -rf \
  -k "sigma_moment or block_parity or sum_order or full_frame or aggressive or normalization or nan_inf or golden or kats or drizzle"
run b_sigma400 300 python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run b_sigma400_reg 300 env SGPU_SIGM=0 python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run b_sigma400_g8w3 300 env SGPU_LIB=$PWD/variants/sigm_g8w3/libsirilgpu.so python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run prof_sigma400 300 rocprofv3 --kernel-trace --stats -d "$O/prof_sigma400" -o run --output-format csv -- python bench.py --config sigma400 --steps 5 --warmup 2 --no-cpu-baseline
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
find "$O" -name "*kernel_stats.csv" | while read f; do d=$(basename $(dirname "$f")); cp "$f" "$O/${d}_kernel_stats.csv"; done
echo "session done"
