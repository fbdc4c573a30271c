#!/bin/bash
# Round 5 session v: config 2's per-chunk exact tails on the one-wave kernel
# (default) vs the one-thread LDS kernel (SGPU_EXACT_WAVE=0), and the stack
# suites that route deferred Winsorized pixels through the tails.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05v}
O=gpurun_out/$T; mkdir -p "$O"
ab() {
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $name $cfg"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log") $(grep -o '"exact_pixels": [0-9]*' "$O/ab_${cfg}_$name.log")"
}
timeout -k 10 400 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 300 --timeout-method thread -rf -k "sum_order or aggressive or block_parity or full_frame" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for i in 1 2; do
  ab wave winsorized100 SGPU_X=0
  ab thread winsorized100 SGPU_EXACT_WAVE=0
done
echo "session done"
