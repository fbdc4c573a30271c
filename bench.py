#!/usr/bin/env python3
"""Benchmark of the MI355X rejection stack (BASELINE.json metric).

One step = one pass of the hot path (sgpu_stack_rows_device: gather +
Winsorized 3/3 rejection + mean, Siril's mean_and_reject per pixel) over a
synthetic 100 x 6000 x 4000 fp32 frame stack already resident in HBM
(BASELINE config 2).  With N GPUs each rank stacks its own stack of that size
(weak scaling: independent images / row-band shards, no data-path
collective; the rejection totals are all-reduced once at the end).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config winsorized100]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  `roofline` uses the dominant kernel's time
measured with HIP events on its own stream (sgpu_last_timing); `cpu_baseline`
times the oracle (C restatement, OpenMP) on a bounded sample of the same
workload, on rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (rejection, sig, nframes, width, height, method)
    "winsorized100": ("WINSORIZED", (3.0, 3.0), 100, 6000, 4000, 0),   # BASELINE config 2
    "sigma400": ("SIGMA", (3.0, 3.0), 400, 6000, 4000, 0),             # BASELINE config 4 (per rank)
    "sigma100": ("SIGMA", (3.0, 3.0), 100, 6000, 4000, 0),
    "median100": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 1),
    "mean100": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 0),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="winsorized100", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(frames, rtype, sig, method, target_s):
    """Oracle (C restatement of Siril's per-pixel stack, OpenMP) on a bounded
    sample of rows of the same stack, timed on this host's cores."""
    import numpy as np
    from oracle import oracle as O
    O.build()
    n, h, w = frames.shape
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    rows = 32
    sample = np.ascontiguousarray(frames[:, :rows, :].cpu().numpy())
    t0 = time.perf_counter()
    O.stack_rows(sample, rtype, sig, method=method, nthreads=threads)
    dt = time.perf_counter() - t0
    rate = rows * w / dt
    rows = int(max(4, min(h, target_s * rate / w)))
    sample = np.ascontiguousarray(frames[:, :rows, :].cpu().numpy())
    t0 = time.perf_counter()
    O.stack_rows(sample, rtype, sig, method=method, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(rows * w / dt / 1e6, 4), "unit": "Mpix/s", "cores": threads,
            "kind": "port",
            "sample": f"{rows} rows x {w} px x {n} frames of the benchmark stack ({dt:.1f} s)"}


def pmc_traffic(config):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(config, {}).get("bytes_per_launch")
    except Exception:
        return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from siril_amd import stacking as S, synth
    rname, sig, n, w, h, method = CONFIGS[a.config]
    rt = S.Rejection[rname]
    frames = synth.frames_torch(n, h, w, dev, seed=20260821 + 1000 * rank)
    out = torch.empty((h, w), dtype=torch.float32, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    ctx = S.Context(local)
    args = S.StackingArgs(rt, sig)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.stack_device(frames, args, method, out=out, counts=counts, stream=stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    exact_px = ctx.last_exact_pixels()

    ctx.set_timing(True)
    kern_ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        kern_ms.append(ctx.last_timing())   # syncs the stream after each step
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(counts)          # rejection totals (tiny, once)
    elapsed = float(t.item())
    ms_per_step = elapsed / a.steps * 1e3
    total_pix = world * w * h * a.steps
    value = total_pix / elapsed / 1e6

    main_ms = sum(k[0] for k in kern_ms) / len(kern_ms)
    exact_ms = sum(k[1] for k in kern_ms) / len(kern_ms)
    alg_bytes = n * w * h * 4 + w * h * 4          # frames read once + output written
    achieved = alg_bytes / (main_ms / 1e3) / 1e9
    res = {
        "metric": "Mpix/s stacked (100x6000x4000 fp32 sigma-clip) at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded BASELINE config-2 recipe, generated in HBM)",
        "config": {"workload": f"{rname} {sig[0]:g}/{sig[1]:g} {'median' if method else 'mean'} stack "
                               f"{n}x{w}x{h} fp32 per GPU (BASELINE config 2)" if a.config == "winsorized100"
                               else f"{a.config}: {rname} {n}x{w}x{h} fp32 per GPU",
                   "frames": n, "width": w, "height": h, "rejection": rname, "sig": list(sig),
                   "method": "median" if method else "mean",
                   "parallelism": f"one independent {n}x{w}x{h} stack per GPU" if world > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic(a.config),
                     "kernel": "k_stack_sorted" if rname != "NO_REJEC" or method else "k_stack_mean",
                     "kernel_ms": round(main_ms, 3), "exact_kernel_ms": round(exact_ms, 3),
                     "alg_bytes_per_launch": alg_bytes},
        "exact_pixels": int(exact_px),
        "rejected": [int(x) for x in counts.tolist()],
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(frames, int(rt), sig, method, a.cpu_seconds)
        res["cpu_baseline"]["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
