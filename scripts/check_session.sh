#!/bin/bash
# GPU check: stack parity tests, then one bench line per config in $CONFIGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-check}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_stack_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit 1; }
for cfg in ${CONFIGS:-}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > $O/$cfg.log 2>&1 || { echo "FAIL $cfg rc=$?"; tail -20 $O/$cfg.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/$cfg.log') if l.startswith('{')][-1]); print('$cfg', d['value'], d['unit'], d['ms_per_step'], d.get('exact_pixels'))"
done
