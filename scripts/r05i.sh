#!/bin/bash
# Round 5 session i: VALU / wait PMC of the SIGMA moment-path kernel at
# config 4 (G = 4 / W = 2 default build, G = 8 / W = 3 variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05i}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 600 bash scripts/pmc_session.sh "$T/pmc_sigm" sigma400 "k_stack_wz<" > "$O/pmc_sigm.log" 2>&1 || exit $?
tail -30 "$O/pmc_sigm.log"
SGPU_LIB=$PWD/variants/sigm_g8w3/libsirilgpu.so timeout -k 10 600 bash scripts/pmc_session.sh "$T/pmc_sigm_g8" sigma400 "k_stack_wz<" > "$O/pmc_sigm_g8.log" 2>&1 || exit $?
tail -30 "$O/pmc_sigm_g8.log"
echo "session done"
