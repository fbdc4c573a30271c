#!/bin/bash
# Round 5 session x: DFT registration and RL deconvolution with the half
# spectra stored straight into the column-major layout the column passes
# read (no rectangular transposes) vs the transpose kernels
# (SGPU_DFT_TRANSPOSE=1 / SGPU_RL_TRANSPOSE=1): GPU tests, then configs 3 / 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05x}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_dft_gpu.py tests/test_rl_gpu.py -x -q --timeout 300 --timeout-method thread -rf -m gpu > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
ab() {
  local cfg=$1 name=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${cfg}_$name.log" 2>&1 || { echo "FATAL $cfg $name"; exit 1; }
  echo "$cfg $name $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${cfg}_$name.log")"
}
for i in 1 2; do
  ab dft100 direct SGPU_X=0; ab dft100 transpose SGPU_DFT_TRANSPOSE=1
  ab rl63 direct SGPU_X=0; ab rl63 transpose SGPU_RL_TRANSPOSE=1
done
echo "session done"
