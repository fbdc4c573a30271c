#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a fault / abort / time-out ends the
# session (no further GPU step), an ordinary test failure does not.
# usage: scripts/gpu_session.sh TAG [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
STEPS=${*:-smoke tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; grep -m1 "model name" /proc/cpuinfo >> "$OUT/nproc.txt" || true
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run pytest_gpu 1500 python -m pytest tests -m gpu -q --timeout=600 -rf;;
    bench) run bench 900 python bench.py --steps 5 --warmup 1;;
    rltests) run pytest_rl 900 python -m pytest tests/test_rl_gpu.py -m gpu -q --timeout=300 -rf;;
    dfttests) run pytest_dft 900 python -m pytest tests/test_dft_gpu.py -m gpu -q --timeout=300 -rf;;
    bench_rl) run bench_rl 900 python bench.py --steps 3 --warmup 1 --config rl63;;
    newtests) run pytest_new 900 python -m pytest tests/test_cfa.py tests/test_demosaic.py -m gpu -q --timeout=300 -rf;;
    bench_rcd) run bench_rcd 600 python bench.py --steps 10 --warmup 2 --config rcd;;
    bench_dft) run bench_dft 900 python bench.py --steps 3 --warmup 1 --config dft100;;
    prof_rl) run prof_rl 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rl" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --config rl63 --no-cpu-baseline;;
    prof_dft) run prof_dft 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dft" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --config dft100 --no-cpu-baseline;;
    prof_rcd) run prof_rcd 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rcd" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --config rcd --no-cpu-baseline;;
    pmc_aux) for cfg in rl63 dft100 rcd; do
               run pmc_fetch_$cfg 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$cfg" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --config $cfg --no-cpu-baseline
               run pmc_write_$cfg 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$cfg" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --config $cfg --no-cpu-baseline
             done;;
    stacktests) run pytest_stack 900 python -m pytest tests/test_stack_gpu.py -m gpu -q --timeout=300 -rf;;
    fullcheck) run fullcheck_wins 600 python scripts/check_full_parity.py 100 4000 6000 WINSORIZED
               run fullcheck_sigma 600 python scripts/check_full_parity.py 100 4000 6000 SIGMA;;
    bench_sigma100) run bench_sigma100 900 python bench.py --steps 3 --warmup 1 --config sigma100 --no-cpu-baseline;;
    bench_sigma400) run bench_sigma400 900 python bench.py --steps 3 --warmup 1 --config sigma400 --no-cpu-baseline;;
    prof_s400) run prof_s400 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_s400" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --config sigma400 --no-cpu-baseline;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline;;
    pmc) run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
         run pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline;;
    variants)
        for v in default $(ls variants 2>/dev/null); do
          if [ "$v" = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
          run bench_var_$v 600 env SGPU_LIB=$lib python bench.py --steps 3 --warmup 1 --no-cpu-baseline
          run check_var_$v 600 env SGPU_LIB=$lib python -m pytest tests/test_stack_gpu.py -q -k "golden or full_size or block_parity" --timeout=300
        done;;
    sq) run pmc_sq1 900 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES -d "$OUT/pmc_sq1" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline
        run pmc_sq2 900 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/pmc_sq2" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline;;
  esac
done
# keep the per-kernel statistics, drop the (large) per-dispatch traces
find "$OUT" -name "*kernel_trace.csv" -delete 2>/dev/null
find "$OUT" -name "*counter_collection.csv" -size +2M -delete 2>/dev/null
echo "session done" | tee -a "$OUT/session.log"
