#!/bin/bash
# Round 6 session e: where the config-2 step goes after the prep-kernel
# instruction cuts -- kernel stats with prep and rounds serialised on one
# stream (SGPU_WZ=4: each kernel's isolated time), and PMC passes of the prep
# and rounds kernels at the new kernel hash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06e}
O=gpurun_out/$T; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if fatal $rc; then echo "FATAL rc=$rc in $name"; exit $rc; fi
  return 0
}
SGPU_WZ=4 run prof_serial 600 rocprofv3 --kernel-trace --stats -d "$O/prof_serial" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run pmc_prep 900 bash scripts/pmc_session.sh "$T/pmc_prep" winsorized100 k_stack_wz_prep
run pmc_rounds 900 bash scripts/pmc_session.sh "$T/pmc_rounds" winsorized100 k_stack_wz_rounds_lds
find "$O" -name "*kernel_trace.csv" -delete 2>/dev/null
echo "session done"
