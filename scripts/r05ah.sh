#!/bin/bash
# Round 5 session ah: RCCL on hardware (world-1 nccl group): the new
# tests/test_distributed_gpu.py, the frame-sharded bench line of config 2
# (all-to-all inside the step) under a kernel trace that lists the RCCL
# kernels, and config 3 priced on the transpose-free 24 B/px model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ah}
O=gpurun_out/$T; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_distributed_gpu.py > "$O/test_dist.log" 2>&1 || { tail -30 "$O/test_dist.log"; echo "FATAL tests"; exit 1; }
tail -3 "$O/test_dist.log"
timeout -k 10 300 python bench.py --config winsorized100 --input frame-sharded --steps 5 --warmup 2 --no-cpu-baseline > "$O/b_winsorized100_fs.log" 2>&1 || { tail -20 "$O/b_winsorized100_fs.log"; echo "FATAL fs"; exit 1; }
grep '^{' "$O/b_winsorized100_fs.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_fs" -o run --output-format csv -- python bench.py --config winsorized100 --input frame-sharded --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof_fs.log" 2>&1 || { tail -20 "$O/prof_fs.log"; echo "FATAL prof"; exit 1; }
find "$O/prof_fs" -name "*kernel_trace.csv" -delete
cp "$O/prof_fs/run_kernel_stats.csv" "$O/fs_kernel_stats.csv"
timeout -k 10 300 python bench.py --config dft100 --steps 10 --warmup 3 --no-cpu-baseline > "$O/b_dft100.log" 2>&1 || { tail -20 "$O/b_dft100.log"; echo "FATAL dft"; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' "$O/b_dft100.log"
echo "session done"
