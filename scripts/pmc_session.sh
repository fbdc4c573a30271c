#!/bin/bash
# PMC passes of one bench config's dominant kernel, one rocprofv3 run per
# counter group (MI355X_MICROARCH.md: no multi-pass counter splitting; <= 8 SQ,
# 4 TCC, 2 GRBM per pass), then the summary keyed to the kernel sources.
# usage: scripts/pmc_session.sh OUTDIR CONFIG KERNEL_SUBSTRING
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; CFG=$2; K=$3
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/avail_full.txt" 2>&1 || true
grep -o "\bSQ_[A-Z0-9_]*\|\bTCC_[A-Z0-9_]*\|\bGRBM_[A-Z0-9_]*\|FETCH_SIZE\|WRITE_SIZE" "$O/avail_full.txt" | sort -u > "$O/avail.txt" || true
rm -f "$O/avail_full.txt"
have() { grep -qx "$1" "$O/avail.txt"; }
pick() { local out=""; for c in "$@"; do have "$c" && out="$out $c"; done; echo $out; }
G1=$(pick SQ_WAVES SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE)
G2=$(pick SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD)
G3=$(pick SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SMEM)
i=0
for grp in "$G1" "$G2" "$G3" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  [ -z "$grp" ] && continue
  echo "pass $i: $grp"
  timeout -s KILL 180 rocprofv3 --pmc $grp -d "$O/p$i" -o run --output-format csv -- python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline > "$O/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$O/p$i.log"; fi
  case $rc in 124|134|137|139) echo "fatal rc, stopping"; exit $rc;; esac
done
python scripts/pmc_summary.py "$K" "$CFG" "$O"/p* > "$O/summary.json" 2>&1; cat "$O/summary.json"
rm -rf "$O"/p[0-9]*/
