# Tuning sweep: bench each variants/<name>/libsirilgpu.so (and the default lib)
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${1:-expv}; mkdir -p $O
for v in default $(ls variants); do
  if [ $v = default ]; then lib=siril_amd/libsirilgpu.so; else lib=variants/$v/libsirilgpu.so; fi
  for cfg in ${CONFIGS:-winsorized100 sigma100}; do
    SGPU_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/$v.$cfg.log 2>&1 || { echo "FAIL $v $cfg rc=$?"; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$O/$v.$cfg.log') if l.startswith('{')][-1]); print('$v $cfg', d['value'], d['roofline']['kernel_ms'], d['exact_pixels'])"
  done
done
