# Round-end evidence on one MI355X: smoke, full GPU tests, every bench config,
# rocprof kernel stats of the headline config, PMC passes of the stack kernel.
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; TAG=${1:-r01_final}
bash scripts/gpu_session.sh $TAG smoke tests bench prof prof_s400 prof_dft prof_rcd || exit $?
O=gpurun_out/$TAG/cfg; mkdir -p $O
for cfg in sigma400 sigma100 median100 mean100 winsorized100_u16 dft100 rl63 rcd fits10; do
  timeout -k 10 600 python bench.py --config $cfg --steps 3 --warmup 1 > $O/$cfg.log 2>&1 || { echo "bench $cfg rc=$?"; exit 1; }
  tail -1 $O/$cfg.log | cut -c1-400
done
bash scripts/exp_pmc.sh $TAG/pmc_w winsorized100 > /dev/null 2>&1 || exit $?
cat gpurun_out/$TAG/pmc_w/summary.json | tail -6
echo final_session done
