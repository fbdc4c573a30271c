#!/bin/bash
# Round 5 session z: XCD-contiguous tile order of the demosaic stencil kernels
# (default) vs the dispatcher's order (SGPU_DM_REMAP=0): demosaic GPU tests,
# then rcd and bayerfast lines, and their FETCH / WRITE traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05z}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_demosaic.py -x -q --timeout 300 --timeout-method thread -rf -m gpu > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
ab() {
  local cfg=$1 name=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $cfg $name"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log")"
}
for i in 1 2; do
  ab rcd remap SGPU_X=0; ab rcd plain SGPU_DM_REMAP=0
  ab bayerfast remap SGPU_X=0; ab bayerfast plain SGPU_DM_REMAP=0
done
timeout -k 10 300 bash scripts/pmc_traffic.sh "$T/tr_rcd" rcd > "$O/tr_rcd.log" 2>&1 && tail -3 "$O/tr_rcd.log"
echo "session done"
