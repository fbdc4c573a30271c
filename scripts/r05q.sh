#!/bin/bash
# Round 5 session q: VALU / wait PMC of config 2's two moment-path kernels
# separately (prep: gather + sort + rank records; rounds: the scalar rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05q}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 600 bash scripts/pmc_session.sh "$T/pmc_prep" winsorized100 "k_stack_wz_prep" > "$O/pmc_prep.log" 2>&1 || exit $?
timeout -k 10 600 bash scripts/pmc_session.sh "$T/pmc_rounds" winsorized100 "k_stack_wz_rounds" > "$O/pmc_rounds.log" 2>&1 || exit $?
for k in prep rounds; do echo "== $k"; python3 -c "
import json; d=json.load(open('$O/pmc_$k/summary.json')); p=d['per_dispatch']
print({k: p.get(k) for k in ['SQ_WAVES','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_WAVE_CYCLES','SQ_ACTIVE_INST_ANY','SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_INSTS_VMEM_RD','SQ_INSTS_LDS','GRBM_GUI_ACTIVE','FETCH_SIZE','WRITE_SIZE']}, d.get('valu_insts_per_wave'), d.get('valu_lane_utilisation'))"; done
echo "session done"
