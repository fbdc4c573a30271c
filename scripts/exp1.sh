set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/exp1; mkdir -p $O
timeout -k 10 300 python bench.py --config median100 --steps 3 --warmup 1 --no-cpu-baseline > $O/med.log 2>&1 &&
timeout -k 10 300 python bench.py --config mean100 --steps 3 --warmup 1 --no-cpu-baseline > $O/mean.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $O/pmc1 -o run --output-format csv -- python bench.py --config sigma100 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $O/pmc2 -o run --output-format csv -- python bench.py --config median100 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc2.log 2>&1
echo done rc=$?
