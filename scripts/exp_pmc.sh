# PMC counters for the main stack kernel (one pass per counter group)
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${1:-pmc}; mkdir -p $O; CFG=${2:-winsorized100}
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INST_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1 || echo "pass $i rc=$?"
done
python scripts/pmc_summary.py k_stack_sorted $O/p* > $O/summary.json 2>&1; cat $O/summary.json
# raw per-dispatch CSVs (every torch kernel of the run) are large: keep the summary
rm -rf $O/p[0-9]*/ $O/avail.txt
