#!/bin/bash
# A/B parity: run the given pytest selection against each variant library.
# usage: scripts/ab_tests.sh TAG "pytest args" variant...   ("main" = siril_amd/libsirilgpu.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for v in "$@"; do
  if [ "$v" = main ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
  echo "== $v"
  SGPU_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest $ARGS -q --timeout 120 --timeout-method thread > "$O/$v.log" 2>&1
  rc=$?; tail -3 "$O/$v.log"
  case $rc in 0|1) ;; *) echo "FATAL rc=$rc"; exit $rc;; esac
done
