#!/bin/bash
# PMC A/B of the dominant kernel across library variants (one rocprofv3 run
# per counter group and variant).  usage: scripts/pmc_ab.sh OUT CONFIG "lib1 lib2 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; CFG=$2; LIBS=$3
mkdir -p "$O"
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY"
for lib in $LIBS; do
  name=$(basename $(dirname $lib))
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    SGPU_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $grp -d "$O/$name.p$i" -o run --output-format csv -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline > "$O/$name.p$i.log" 2>&1
    rc=$?; echo "$name pass $i rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
  python scripts/pmc_summary.py k_stack_sorted "$CFG" "$O"/$name.p* > "$O/$name.summary.json" 2>&1
  rm -rf "$O"/$name.p[0-9]/
done
