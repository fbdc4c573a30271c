#!/bin/bash
# Where the direct RL convolution's MFMA pipe waits (LDS
# operand feed vs MFMA dependency chains): two rocprofv3 --pmc passes over
# the rl63_direct bench config (wait / active cycles by kind, then the LDS
# array's conflict and FIFO counters), summarised per dispatch of
# k_conv2d_mfma.  usage: scripts/pmc_mfma_stall.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
i=0
for grp in "$P1" "$P2"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp -d "$O/s$i" -o run --output-format csv -- python bench.py --config rl63_direct --steps 1 --warmup 0 --no-cpu-baseline > "$O/s$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -3 "$O/s$i.log"; exit $rc;; esac
done
PMC_SOURCE_CONFIG=rl63_direct python scripts/pmc_summary.py k_conv2d_mfma rl63_direct "$O"/s1 "$O"/s2 > "$O/summary.json" 2>&1; cat "$O/summary.json"
rm -rf "$O"/s1/ "$O"/s2/
