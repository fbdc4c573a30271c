#!/bin/bash
# Round 5 session ac: per-chunk tails for the 16-bit Winsorized moment path
# (the 16-bit sorted kernel and LDS exact kernel on the third stream under
# the next chunks) vs tails after the last chunk (SGPU_WZ_TAILS=0); the 16-bit
# and Winsorized GPU suites, full-frame parity on the 16-bit line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ac}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py tests/test_sequence.py -x -q --timeout 300 --timeout-method thread -rf -m gpu -k "u16 or winsorized or sequence or block_parity" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
ab() {
  local cfg=$1 name=$2 extra=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 $extra > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $cfg $name"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log") $(grep -o '"mismatches": [0-9]*' "$O/ab_${cfg}_$name.log" | head -1)"
}
for i in 1 2; do
  ab winsorized100_u16 tails --no-cpu-baseline SGPU_X=0
  ab winsorized100_u16 notails --no-cpu-baseline SGPU_WZ_TAILS=0
done
ab winsorized100_u16 parity "" SGPU_X=0
ab winsorized100_u16_norm tails --no-cpu-baseline SGPU_X=0
ab winsorized100 tails --no-cpu-baseline SGPU_X=0
echo "session done"
