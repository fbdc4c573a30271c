#!/bin/bash
# RCD variants: parity tests, then the rcd bench line per SGPU_RCD_FUSED mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rcd}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_demosaic.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit 1; }
for m in 1 2 0 1; do
  SGPU_RCD_FUSED=$m timeout -k 10 300 python bench.py --config rcd --steps 20 --warmup 3 --no-cpu-baseline > $O/rcd_$m.log 2>&1 || { echo "FAIL $m"; tail -5 $O/rcd_$m.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/rcd_$m.log') if l.startswith('{')][-1]); r=d['roofline']; print('mode $m', d['value'], d['ms_per_step'], r.get('kernel_ms'), r['frac'])"
done
