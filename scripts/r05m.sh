#!/bin/bash
# Round 5 session m: the wave exact kernel without scratch traffic (helpers
# inlined, tape pointers by value, unrolled pointer jumping) -- its GPU tests,
# config 4 whole frame and 500-row band (exact tail), config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05m}
O=gpurun_out/$T; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if fatal $rc; then echo "FATAL rc=$rc in $name"; exit $rc; fi
  return 0
}
run pytest_wave 400 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 300 --timeout-method thread -rf -k "exact_wave or sum_order or aggressive or full_frame or exact_only or kats"
run b_sigma400 300 python bench.py --config sigma400 --steps 10 --warmup 3 --no-cpu-baseline
run band_sigma400 300 python bench.py --config sigma400 --band-rows 500 --steps 10 --warmup 3 --no-cpu-baseline
run b_winsorized100 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
for f in b_sigma400 band_sigma400 b_winsorized100; do python -c "
import json; l=[x for x in open('$O/$f.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$f', d['ms_per_step'], r.get('kernel_ms'), r.get('exact_kernel_ms'), d.get('exact_pixels'))"; done
echo "session done"
