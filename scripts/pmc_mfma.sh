#!/bin/bash
# Matrix-core utilisation of the direct RL convolution (BASELINE config 5's
# "MFMA blur GEMM"): one rocprofv3 --pmc pass with the MFMA busy counter on
# the rl63_direct bench config, summarised per dispatch of k_conv2d_mfma.
# usage: scripts/pmc_mfma.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/avail_full.txt" 2>&1 || true
grep -o "\bSQ_[A-Z0-9_]*\|\bGRBM_[A-Z0-9_]*" "$O/avail_full.txt" | sort -u > "$O/avail.txt" || true
rm -f "$O/avail_full.txt"
have() { grep -qx "$1" "$O/avail.txt"; }
pick() { local out=""; for c in "$@"; do have "$c" && out="$out $c"; done; echo $out; }
G=$(pick SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE)
echo "pass: $G"
timeout -s KILL 240 rocprofv3 --pmc $G -d "$O/m1" -o run --output-format csv -- python bench.py --config rl63_direct --steps 1 --warmup 0 --no-cpu-baseline > "$O/m1.log" 2>&1
rc=$?
echo "pass rc=$rc"
[ $rc -ne 0 ] && tail -3 "$O/m1.log"
case $rc in 0) ;; *) exit $rc;; esac
PMC_SOURCE_CONFIG=rl63_direct python scripts/pmc_summary.py k_conv2d_mfma rl63_direct "$O"/m1 > "$O/summary.json" 2>&1; cat "$O/summary.json"
rm -rf "$O"/m1/
