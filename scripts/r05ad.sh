#!/bin/bash
# Round 5 session ad: the SIGMA window sum carried through the rounds when it
# is exact (no sum pass after a round that removed <= 2 samples, no final sum
# pass) vs the previous library (variants/pre_sigmas): the stack GPU suite,
# then sigma400 / sigma100 / the 500-row band, with full-frame parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ad}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 300 --timeout-method thread -rf -m gpu > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
ab() {
  local cfg=$1 name=$2 lib=$3 extra=$4
  env SGPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 $extra > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $cfg $name"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log") $(grep -o '"mismatches": [0-9]*' "$O/ab_${cfg}_$name.log" | head -1)"
}
M=siril_amd/libsirilgpu.so; V=variants/pre_sigmas/libsirilgpu.so
for i in 1 2; do
  ab sigma400 new $M --no-cpu-baseline; ab sigma400 old $V --no-cpu-baseline
  ab sigma100 new $M --no-cpu-baseline; ab sigma100 old $V --no-cpu-baseline
done
ab sigma400 band_new $M "--band-rows 500 --no-cpu-baseline"; ab sigma400 band_old $V "--band-rows 500 --no-cpu-baseline"
ab sigma400 parity $M ""
ab sigma100 parity $M ""
echo "session done"
