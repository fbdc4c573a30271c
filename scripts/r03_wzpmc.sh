#!/bin/bash
# PMC passes of the WINSORIZED two-kernel moment path (prep + rounds kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03h}; mkdir -p $O
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY"
i=0
for grp in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
for k in k_stack_wz_prep k_stack_wz_rounds; do
  python scripts/pmc_summary.py $k winsorized100 $O/p* > $O/$k.summary.json 2>&1
done
rm -rf $O/p[0-9]*/
