#!/bin/bash
# Round 5 session aq: radix 10 in place with one butterfly per thread (row
# kernels 87 -> 79 VGPRs): DFT / RL / CFA tests, smoke, config 3 A/B against
# the old radices in the odd-first order, traffic of configs 3 and 5 at the
# final aux hashes, their bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05aq}
O=gpurun_out/$T; mkdir -p "$O"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 500 $PT tests/test_dft_gpu.py tests/test_rl_gpu.py tests/test_cfa.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; echo "FATAL tests"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; echo "FATAL smoke"; exit 1; }
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_dft100_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"pipeline_ms": [0-9.]*' "$O/ab_dft100_$name.log" | tr '\n' ' ')"
}
for i in 1 2; do ab final SGPU_X=0; ab old_radices SGPU_DFT_PLAN=5,8,5,5,4; done
for c in dft100 rl63; do
  timeout -k 10 600 bash scripts/pmc_traffic.sh "$T/tr_$c" "$c" > "$O/tr_$c.log" 2>&1 || { tail -20 "$O/tr_$c.log"; echo "FATAL traffic $c"; exit 1; }
done
for c in dft100 rl63; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > "$O/b_$c.log" 2>&1 || { tail -20 "$O/b_$c.log"; echo "FATAL bench $c"; exit 1; }
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' "$O/b_$c.log" | tr '\n' ' ')"
done
echo "session done"
