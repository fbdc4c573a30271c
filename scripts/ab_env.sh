#!/bin/bash
# A/B timing of one bench config under environment settings.
# usage: scripts/ab_env.sh TAG CONFIG "VAR=VALUE" ...   ("-" = no extra setting)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
i=0
for e in "$@"; do
  i=$((i+1))
  if [ "$e" = - ]; then envs=(); else read -r -a envs <<< "$e"; fi
  env "${envs[@]}" timeout -k 10 300 python bench.py --config "$CFG" --steps 10 --warmup 3 --no-cpu-baseline > "$O/ab_${CFG}_$i.log" 2>&1
  rc=$?
  echo "$e rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/ab_${CFG}_$i.log")"
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac
done
