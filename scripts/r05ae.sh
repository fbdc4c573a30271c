#!/bin/bash
# Round 5 session ae: closing check at HEAD -- the whole GPU suite, smoke, the
# headline line, and the bayerfast traffic at the demosaic sources' new hash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ae}
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
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 20 --warmup 5
run tr_bayerfast 300 bash scripts/pmc_traffic.sh "$T/tr_bayerfast" bayerfast
run b_bayerfast 300 python bench.py --config bayerfast --steps 10 --warmup 3
run b_rcd 300 python bench.py --config rcd --steps 10 --warmup 3
echo "session done"
