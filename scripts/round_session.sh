# Round-end evidence: smoke, GPU tests, benches, rocprof kernel stats, PMC passes.
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; TAG=${1:-r01_final}
bash scripts/gpu_session.sh $TAG smoke tests bench prof || exit $?
CONFIGS="sigma400 sigma100 median100 mean100" bash scripts/exp_variants.sh $TAG/cfg || exit $?
bash scripts/exp_pmc.sh $TAG/pmc_w winsorized100 || exit $?
bash scripts/exp_pmc.sh $TAG/pmc_s400 sigma400 || exit $?
echo round_session done
