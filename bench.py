#!/usr/bin/env python3
"""Benchmark of the MI355X rejection stack (BASELINE.json metric).

One step = one pass of the hot path (sgpu_stack_rows_device: gather +
Winsorized 3/3 rejection + mean, Siril's mean_and_reject per pixel) over a
synthetic 100 x 6000 x 4000 fp32 frame stack already resident in HBM
(BASELINE config 2).  With N GPUs the SAME stack is split by pixel rows
(strong scaling): rank r holds rows [y0_r, y1_r) of every frame,
stacks them, and the output bands are all-gathered over RCCL inside the
timed step (the assembled image is on every rank at the end of each step);
the rejection totals are all-reduced once at the end.

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
    "sigma400": ("SIGMA", (3.0, 3.0), 400, 6000, 4000, 0),             # BASELINE config 4 (row bands)
    "sigma100": ("SIGMA", (3.0, 3.0), 100, 6000, 4000, 0),
    "winsorized400": ("WINSORIZED", (3.0, 3.0), 400, 6000, 4000, 0),
    "winsorized128": ("WINSORIZED", (3.0, 3.0), 128, 6000, 4000, 0),
    "median100": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 1),
    "mean100": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 0),
    "mean100_u16": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 0),
    "median100_u16": ("NO_REJEC", (3.0, 3.0), 100, 6000, 4000, 1),
    # DATA_USHORT twin of config 2 (raw 16-bit lights): apply_rejection_ushort
    "winsorized100_u16": ("WINSORIZED", (3.0, 3.0), 100, 6000, 4000, 0),
    # ... with -norm=addscale coefficients (round_to_WORD in the 16-bit gather)
    "winsorized100_u16_norm": ("WINSORIZED", (3.0, 3.0), 100, 6000, 4000, 0),
    # the other rejection types at the config-2 size
    "mad100": ("MAD", (3.0, 3.0), 100, 6000, 4000, 0),
    "linearfit100": ("LINEARFIT", (3.0, 3.0), 100, 6000, 4000, 0),
    "percentile100": ("PERCENTILE", (0.2, 0.1), 100, 6000, 4000, 0),
    "sigmedian100": ("SIGMEDIAN", (3.0, 3.0), 100, 6000, 4000, 0),
    "gesdt100": ("GESDT", (0.3, 0.05), 100, 6000, 4000, 0),
    "percentile100_u16": ("PERCENTILE", (0.2, 0.1), 100, 6000, 4000, 0),
    "sigmedian100_u16": ("SIGMEDIAN", (3.0, 3.0), 100, 6000, 4000, 0),
    # deferral-heavy: a 12-frame master with low sigmas
    "winsorized12_s1": ("WINSORIZED", (1.0, 1.0), 12, 6000, 4000, 0),
    # the small-N master cases with the usual sigmas (stack dark|bias rej 3 3),
    # float and raw 16-bit
    "winsorized12": ("WINSORIZED", (3.0, 3.0), 12, 6000, 4000, 0),
    "sigma12": ("SIGMA", (3.0, 3.0), 12, 6000, 4000, 0),
    "winsorized12_u16": ("WINSORIZED", (3.0, 3.0), 12, 6000, 4000, 0),
    "winsorized12_s1_u16": ("WINSORIZED", (1.0, 1.0), 12, 6000, 4000, 0),
    "winsorized24": ("WINSORIZED", (3.0, 3.0), 24, 6000, 4000, 0),
    "sigma24": ("SIGMA", (3.0, 3.0), 24, 6000, 4000, 0),
    "winsorized32_s1": ("WINSORIZED", (1.0, 1.0), 32, 6000, 4000, 0),
    "percentile12": ("PERCENTILE", (0.2, 0.1), 12, 6000, 4000, 0),
    "sigmedian12": ("SIGMEDIAN", (3.0, 3.0), 12, 6000, 4000, 0),
}
AUX_CONFIGS = {
    # BASELINE config 3: DFT registration of 100 frames 6000x4000, S = 4000 centred selection
    "dft100": ("DFT", 100, 6000, 4000, 4000),
    # BASELINE config 5: RL 50 iterations (rl -mul), 6000x4000, 64x64 PSF -> 63x63 (crop)
    "rl63": ("RL", 50, 6000, 4000, 63),
    # the same on the matrix cores: direct circular convolution as a GEMM on
    # v_mfma_f32_16x16x4_f32 (SGPU_RL_DIRECT=1; BASELINE config 5's "MFMA blur GEMM")
    "rl63_direct": ("RL", 50, 6000, 4000, 63),
    # RCD demosaic of one 6000x4000 RGGB frame (debayer_buffer_new_float)
    "rcd": ("RCD", 1, 6000, 4000, 0),
    # BAYER_BILINEAR = librtprocess bayerfast (forced for colour SER frames, io/ser.c:1177-1182)
    "bayerfast": ("RCD", 1, 6000, 4000, 0),
    # BASELINE config 1: headless `stack synth_ rej n -nonorm -32b` of 10 FITS 1024x1024 (plumbing)
    "fits10": ("FITS", 10, 1024, 1024, 0),
    # end-to-end `stack <seq> rej w 3 3 -nonorm -32b` of 100 FITS 6000x4000 float frames
    # (9.6 GB) from the page cache: block reads, pinned H2D, Winsorized stack, output write
    "seq100": ("SEQ", 100, 6000, 4000, 0),
    # the same as one 16-bit SER file (raw camera sequences; 4.8 GB)
    "seq100_ser": ("SEQ", 100, 6000, 4000, 16),
    # -norm=addscale estimators (median, MAD, IKSS) of 100 frames 6000x4000
    "norm100": ("NORM", 100, 6000, 4000, 0),
}
# Every stack config is ONE N x 6000 x 4000 stack split over the GPUs by
# pixel rows: strong scaling, output bands all-gathered over RCCL.
STRONG_CONFIGS = set(CONFIGS)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_F32_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="winsorized100", choices=sorted(CONFIGS) + sorted(AUX_CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--band-rows", type=int, default=0,
                    help="stack configs, one GPU: time one rank's row band of this many rows (e.g. 500 = "
                         "an 8-GPU rank's band of a 4000-row frame) instead of the whole frame")
    ap.add_argument("--input", default="row-bands", choices=["row-bands", "frame-sharded"],
                    help="stack configs at N>1: each rank holds a row band of every frame (default) or "
                         "N/world whole frames, moved to row bands by an all-to-all inside the step")
    ap.add_argument("--contexts", type=int, default=3,
                    help="frame-sharded, pipelined: contexts (streams) the sub-chunk stacks alternate over")
    ap.add_argument("--pipeline", type=int, default=4,
                    help="frame-sharded input: row sub-chunks of the transpose pipelined under the stack "
                         "(stack_frame_sharded_pipelined); 0 or 1 = one all-to-all of the whole band, then the stack")
    return ap.parse_args()


def host_cpu():
    """Host description for the CPU baseline: CPU
    model, nproc, the CPUs this process may run on, and the thread count used
    (OMP_NUM_THREADS when set -- the GPU box sets it to the box's CPU share --
    else every CPU of the affinity mask)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = nproc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail
    return {"cpu_model": model, "nproc": nproc, "affinity_cpus": avail, "threads": threads}


def norm_coefficients(n, seed=5):
    """Per-frame -norm=addscale coefficients of the *_norm configs (scale near
    1, offsets of a few hundred ADU): (normalization, scale, offset)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 300.0 * rng.standard_normal(n)
    return 3, scale, offset


def cpu_baseline(frames, rtype, sig, method, target_s, u16=False, norm=None):
    """Oracle (C restatement of Siril's per-pixel stack, OpenMP with dynamic
    row scheduling like median_and_mean.c:1551) on a bounded sample of rows
    of the same stack, timed on this host's cores.  Returns (baseline dict,
    (rows, out, rej_lo, rej_hi, counts) of the timed sample): the caller
    compares the sample with the GPU image bit for bit."""
    import numpy as np
    from oracle import oracle as O
    O.build()
    n, h, w = frames.shape
    host = host_cpu()
    threads = host["threads"]
    box = {}

    def run(rows):
        sample = np.ascontiguousarray(frames[:, :rows, :].cpu().numpy())
        t0 = time.perf_counter()
        kw = {} if norm is None else {"norm": norm[0], "scale": norm[1], "offset": norm[2]}
        if u16:
            r = O.stack_rows_u16(sample.view(np.uint16), rtype, sig, method=method, nthreads=threads, **kw)
        else:
            r = O.stack_rows(sample, rtype, sig, method=method, nthreads=threads, **kw)
        dt = time.perf_counter() - t0
        box["res"] = (rows,) + tuple(r[:4])
        return dt

    rows = 32
    dt = run(rows)
    rate = rows * w / dt
    rows = int(max(4, min(h, target_s * rate / w)))
    dt = run(rows)
    return ({"value": round(rows * w / dt / 1e6, 4), "unit": "Mpix/s", "cores": threads,
             "kind": "port", **{k: host[k] for k in ("cpu_model", "nproc", "affinity_cpus")},
             "sample": f"{rows} rows x {w} px x {n} frames of the benchmark stack ({dt:.1f} s, "
                       f"{threads} OpenMP threads)"}, box["res"])


def parity_vs_oracle(ctx, S, frames, args, method, ref, u16=False):
    """One extra (untimed) GPU stack of the rows the CPU baseline stacked, with
    both rejection maps, compared bit for bit with the oracle's output of the
    same rows: output float bits, low / high rejection maps, totals."""
    import numpy as np
    import torch
    rows, out_o, rl_o, rh_o, cnt_o = ref
    band = frames[:, :rows, :]
    dev = frames.device
    out = torch.empty((rows, frames.shape[2]), dtype=torch.float32, device=dev)
    rl = torch.zeros((rows, frames.shape[2]), dtype=torch.int16, device=dev)
    rh = torch.zeros_like(rl)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ctx.stack_device(band, args, method, out=out, rej_lo=rl, rej_hi=rh, counts=cnt)
    torch.cuda.synchronize()
    g = out.cpu().numpy().view(np.uint32)
    o = np.asarray(out_o, np.float32).view(np.uint32)
    bad = int(np.count_nonzero(g != o))
    maps = method == 0 and rtype_has_maps(args)
    bad_l = int(np.count_nonzero(rl.cpu().numpy().view(np.uint16) != rl_o)) if maps else None
    bad_h = int(np.count_nonzero(rh.cpu().numpy().view(np.uint16) != rh_o)) if maps else None
    cnt_ok = [int(x) for x in cnt.tolist()] == [int(x) for x in cnt_o]
    return {"pixels": int(g.size), "rows": int(rows), "mismatches": bad, "rejmap_low_mismatches": bad_l,
            "rejmap_high_mismatches": bad_h, "counts_equal": bool(cnt_ok),
            "scope": ("full frame" if rows == frames.shape[1] else f"first {rows} rows") +
                     ": GPU (one extra untimed stack with rejection maps) vs the CPU-baseline oracle run, bit for bit"}


def rtype_has_maps(args):
    return int(args.type_of_rejection) != 0


class ClockSampler:
    """Shader clock (sclk) of this process's GPU sampled every 20 ms from
    sysfs (pp_dpm_sclk: the current level carries '*') while the timed steps
    run: VALU-bound kernels run at the clock the card holds under load, so
    the bench line records it (min / median / max MHz).  None fields when the
    file is not readable."""

    def __init__(self, dev):
        import glob
        self.path, self.mhz, self._stop = None, [], None
        cands = []
        try:
            import torch
            pr = torch.cuda.get_device_properties(dev)
            bus = getattr(pr, "pci_bus_id", None)
            dom = getattr(pr, "pci_domain_id", 0) or 0
            did = getattr(pr, "pci_device_id", 0) or 0
            if bus is not None:
                cands.append(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{did:02x}.0/pp_dpm_sclk")
        except Exception:
            pass
        found = [p for p in cands if os.access(p, os.R_OK)]
        if not found:   # one card visible to the process: the only readable sclk file
            found = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))
            found = found if len(found) == 1 else []
        self.path = found[0] if found else None

    def _read(self):
        try:
            for line in open(self.path):
                if "*" in line:
                    return int("".join(c for c in line.split(":", 1)[1] if c.isdigit()))
        except Exception:
            return None
        return None

    def __enter__(self):
        import threading
        if self.path is None:
            return self
        self._stop = threading.Event()

        def loop():
            while not self._stop.wait(0.02):
                v = self._read()
                if v:
                    self.mhz.append(v)
        self._t = threading.Thread(target=loop, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        if self._stop is not None:
            self._stop.set()
            self._t.join()

    def summary(self):
        if not self.mhz:
            return {"sclk_mhz_min": None, "sclk_mhz_median": None, "sclk_mhz_max": None, "samples": 0}
        s = sorted(self.mhz)
        return {"sclk_mhz_min": s[0], "sclk_mhz_median": s[len(s) // 2], "sclk_mhz_max": s[-1],
                "samples": len(s)}


def kernel_source_hash():
    """Hash of every source and build flag the stack kernels are compiled
    from: a committed PMC profile is used only when it was taken from the
    same kernel code (scripts/pmc_summary.py records this hash)."""
    import hashlib
    import glob
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "siril_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "stack_sorted*")) +
                   [os.path.join(csrc, n) for n in ("stack_wz.h", "stack_exact.hip", "stack_exact_wave.hip",
                                                    "stack_mean.hip", "sgpu_kparams.h", "sgpu_capi.cpp")] +
                   [os.path.join(ROOT, "siril_amd", "build.py")])
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


# kernels each secondary config's roofline covers (scripts/pmc_traffic_summary.py)
AUX_TRAFFIC_SCOPE = {"rl63": r"^sgpu::(rl|dft)::", "rl63_direct": r"^sgpu::", "dft100": r"^sgpu::dft::", "rcd": r"^sgpu::dm::",
                     "bayerfast": r"^sgpu::dm::",
                     "norm100": r"^sgpu::ns::", **{c: r"^sgpu::k_stack" for c in CONFIGS}}
AUX_SOURCES = {"rl63": ["rl_fft.hip", "rl_conv.hip", "rl_conv.h", "fft_lds.h", "dft_register.hip", "sgpu_rl.cpp"],
               "rl63_direct": ["rl_conv.hip", "rl_conv.h", "sgpu_rl.cpp"],
               "dft100": ["dft_register.hip", "fft_lds.h", "sgpu_dft.cpp", "quality.hip"],
               "rcd": ["demosaic.hip", "sgpu_demosaic.cpp"],
               "bayerfast": ["demosaic.hip", "sgpu_demosaic.cpp"],
               "norm100": ["norm_stats.hip"]}


def aux_source_hash(config):
    """Hash of the sources a config's kernels are built from (the stack
    configs: kernel_source_hash)."""
    if config in CONFIGS:
        return kernel_source_hash()
    import hashlib
    h = hashlib.sha256()
    for n in AUX_SOURCES.get(config, []):
        h.update(n.encode())
        h.update(open(os.path.join(ROOT, "siril_amd", "csrc", n), "rb").read())
    h.update(open(os.path.join(ROOT, "siril_amd", "build.py"), "rb").read())
    return h.hexdigest()[:16]


def aux_traffic(config):
    """(HBM bytes per step of the roofline's kernels, source profile) from
    profiles/pmc_traffic_aux.json when it was taken from these sources."""
    try:
        ent = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_aux.json"))).get(config, {})
    except Exception:
        return None, None
    if ent.get("source_hash") != aux_source_hash(config):
        return None, None
    return ent.get("bytes_per_step_scope"), ent.get("source")


def pmc_info(config):
    """Per-launch PMC figures of the dominant kernel from the committed
    rocprofv3 summaries (profiles/pmc_traffic.json, written by
    scripts/pmc_summary.py): HBM bytes (FETCH_SIZE doubled per
    MI355X_MICROARCH.md §HBM, + WRITE_SIZE) and VALU issue counts.  Empty
    when the profile was taken from different kernel sources."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        ent = json.load(open(path)).get(config, {})
    except Exception:
        return {}
    if ent.get("kernel_source_hash") != kernel_source_hash():
        return {}
    return ent


def main():
    a = parse()
    if a.config in AUX_CONFIGS:
        return bench_aux(a)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # frame-sharded input always goes through the process group (RCCL), also
    # on one GPU: the all-to-all transpose then runs with a single rank, which
    # exercises the collective path on a 1-GPU box
    use_pg = world > 1 or a.input == "frame-sharded"
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from siril_amd import stacking as S, synth
    from siril_amd.distributed import (row_bands, frame_shards, transpose_frames_to_bands,
                                       stack_frame_sharded_pipelined)
    if a.input == "frame-sharded" and world == 1:
        import siril_amd.distributed as _D
        _D.COLLECTIVE_AT_WORLD1 = True     # one GPU: still run the exchange through RCCL (capped pieces)
    rname, sig, n, w, h, method = CONFIGS[a.config]
    rt = S.Rejection[rname]
    strong = a.config in STRONG_CONFIGS
    sharded = a.input == "frame-sharded"
    y0, y1 = row_bands(h, world)[rank] if strong else (0, h)
    if a.band_rows:                                # one rank's band, timed alone (DESIGN §6 prediction)
        if world > 1 or sharded:
            raise SystemExit("--band-rows is a one-GPU measurement")
        y0, y1 = 0, min(h, a.band_rows)
    hb = y1 - y0                                   # rows this rank stacks
    u16 = "_u16" in a.config
    norm = norm_coefficients(n) if a.config.endswith("_norm") else None
    if sharded:   # rank r holds frames [f0, f1) whole (BASELINE config 4: "frame-sharded across 8")
        f0, f1 = frame_shards(n, world)[rank]
        frames = synth.frames_torch(f1 - f0, h, w, dev, seed=20260821 + 13 * f0)
    else:
        frames = synth.frames_torch(n, hb, w, dev, seed=20260821 + (1000 * rank if not strong else 7 * y0))
    if u16:   # same recipe quantised to 16 bits (0 stays 0 = missing)
        frames = torch.round(frames * 65535.0).to(torch.int32).to(torch.int16)
    out = torch.empty((hb, w), dtype=torch.float32, device=dev)
    full = torch.empty((h, w), dtype=torch.float32, device=dev) if strong and world > 1 else None
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    ctx = S.Context(local)
    # pipelined frame-sharded stacks alternate their sub-chunks over contexts
    ctxs = [ctx] + [S.Context(local) for _ in range(max(0, a.contexts - 1))] if sharded and a.pipeline > 1 else [ctx]
    args = (S.StackingArgs(rt, sig) if norm is None else
            S.StackingArgs(rt, sig, normalize=S.Normalization(norm[0]), scale=norm[1], offset=norm[2]))
    stream = torch.cuda.current_stream(dev)
    xev = []                                       # (start, end) events of the all-to-all per step
    pipelined = sharded and a.pipeline > 1
    pev = []                                       # pipelined: per step, the sub-chunks' stack events
    prej = [0, 0]

    def step():
        if pipelined:
            # transpose in a.pipeline row sub-chunks under the stack, then
            # the all-gather of the output bands (inside the function)
            st = {}
            _, rej = stack_frame_sharded_pipelined(frames, n, args, method, ctx=ctx, subchunks=a.pipeline, stats=st,
                                                   ctxs=ctxs)
            pev.append(st["events"])
            prej[0] += rej[0]
            prej[1] += rej[1]
            return
        if sharded:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            band = transpose_frames_to_bands(frames, n)
            e1.record(stream)
            xev.append((e0, e1))
        else:
            band = frames
        ctx.stack_device(band, args, method, out=out, counts=counts, stream=stream)
        if full is not None:             # assemble the image: one all-gather of the bands
            dist.all_gather_into_tensor(full, out)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    exact_px = ctx.last_exact_pixels()
    counts.zero_()                       # rejection totals of the timed steps only
    xev.clear()
    pev.clear()
    prej[0] = prej[1] = 0

    ctx.set_timing(True)
    kern_ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    with ClockSampler(dev) as clk:
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
            if not pipelined:
                kern_ms.append(ctx.last_timing())   # syncs the stream after each step
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    a2a_ms = sum(e0.elapsed_time(e1) for e0, e1 in xev) / len(xev) if xev else None
    if pipelined:
        # kernel time of a step = the sum of its sub-chunk stacks (HIP events
        # on the stack stream); the exchange of the first sub-chunk is the
        # pipeline's fill (side-stream start to the first stack's start)
        kern_ms = [(sum(e1.elapsed_time(e2) for _, e1, e2 in evs), 0.0) for evs in pev]
        fill = [evs[0][0].elapsed_time(evs[0][1]) for evs in pev if evs and evs[0][0] is not None]
        a2a_ms = sum(fill) / len(fill) if fill else None
        counts = torch.tensor(prej, dtype=torch.int64, device=dev)
        if world > 1:
            counts //= world             # every rank returns the all-reduced totals

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(counts)          # rejection totals of the bands (tiny, once)
    elapsed = float(t.item())
    ms_per_step = elapsed / a.steps * 1e3
    total_pix = (1 if strong else world) * w * (hb if a.band_rows else h) * a.steps
    value = total_pix / elapsed / 1e6

    main_ms = sum(k[0] for k in kern_ms) / len(kern_ms)
    exact_ms = sum(k[1] for k in kern_ms) / len(kern_ms)
    alg_bytes = n * w * hb * (2 if u16 else 4) + w * hb * 4   # frames read once + output written (per rank)
    achieved = alg_bytes / (main_ms / 1e3) / 1e9
    pmc = pmc_info(a.config)
    # every stack kernel of one step, when profiled -- the profile is of the
    # whole-frame, row-band step: not attached to a band or frame-sharded line
    step_traffic, step_traffic_src = ((None, None) if (a.band_rows or sharded) else aux_traffic(a.config))
    valu = None
    if pmc.get("valu_wave_insts") and pmc.get("valu_peak_wave_insts_per_s") and not (a.band_rows or sharded):
        # VALU issue roofline: wave-instructions issued per second vs the chip's
        # issue peak (1024 SIMDs x clock / 2 cycles per wave64 f32 op), and the
        # same rate weighted by the active-lane fraction (divergence waste);
        # multi-kernel steps (the moment path) use the per-step totals
        insts = pmc.get("valu_wave_insts_step") or pmc["valu_wave_insts"]
        if pmc.get("valu_lane_utilisation_step"):
            pmc["valu_lane_utilisation"] = pmc["valu_lane_utilisation_step"]
        rate = insts / (main_ms / 1e3)
        valu = {"bound": "valu", "achieved": round(rate / 1e9, 1), "unit": "Gwave-inst/s",
                "peak": round(pmc["valu_peak_wave_insts_per_s"] / 1e9, 1),
                "frac": round(rate / pmc["valu_peak_wave_insts_per_s"], 4),
                "lane_utilisation": pmc.get("valu_lane_utilisation"),
                "useful_frac": (round(rate * pmc["valu_lane_utilisation"] / pmc["valu_peak_wave_insts_per_s"], 4)
                                if pmc.get("valu_lane_utilisation") else None),
                "wave_insts_per_step": insts, "wait_any_frac": pmc.get("wait_any_frac_step"),
                "profile": pmc.get("source")}
    res = {
        "metric": "Mpix/s stacked (100x6000x4000 fp32 sigma-clip) at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u16" if u16 else "f32",
        "data": "synthetic (seeded BASELINE config-2 recipe, generated in HBM)",
        "config": {"workload": (f"{rname} {sig[0]:g}/{sig[1]:g} {'median' if method else 'mean'} stack "
                                f"{n}x{w}x{h} {'u16' if u16 else 'fp32'}"
                                + (" -norm=addscale" if norm is not None else "")
                                + {"winsorized100": " (BASELINE config 2)",
                                   "sigma400": " (BASELINE config 4)"}.get(a.config, "")),
                   "frames": n, "width": w, "height": h, "rejection": rname, "sig": list(sig),
                   "method": "median" if method else "mean",
                   "input": "frame-sharded" if sharded else "row-bands",
                   "pipeline": a.pipeline if sharded else None,
                   "contexts": len(ctxs) if sharded and a.pipeline > 1 else None,
                   "band_rows": a.band_rows or None,
                   "parallelism": ((f"{n} frames sharded by frame over {world} GPUs, RCCL all-to-all to row bands "
                                    f"({hb} rows per GPU"
                                    + (f", in {a.pipeline} row sub-chunks pipelined under the stack" if pipelined
                                       else "")
                                    + "), stack, all-gather of the output bands, all inside the step")
                                   if sharded else
                                   f"one rank's row band ({hb} of {h} rows) on one GPU, no collective"
                                   if a.band_rows else
                                   f"row bands of one {n}x{w}x{h} stack ({hb} rows per GPU), RCCL all-gather "
                                   "of the output bands inside the step" if world > 1 else "single GPU")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     # HBM bytes per launch from the PMC profile of these kernel sources
                     "traffic": (step_traffic if step_traffic is not None else
                                 None if (a.band_rows or sharded) else pmc.get("bytes_per_launch")),
                     "traffic_profile": step_traffic_src if step_traffic is not None else pmc.get("source"),
                     "kernel": (("k_stack_wz_prep + k_stack_wz_rounds (moment path, chunked) + k_stack_sorted over "
                                 "its fallbacks" if os.environ.get("SGPU_WZ", "2") == "2" else "k_stack_sorted")
                                if rname == "WINSORIZED" and not u16 and 64 < n <= 1024 else
                                "k_stack_sorted" if rname != "NO_REJEC" or method else "k_stack_mean"),
                     "kernel_ms_scope": "HIP events around every kernel of the stack launch (sgpu_last_timing ms[0])",
                     "kernel_ms": round(main_ms, 3), "exact_kernel_ms": round(exact_ms, 3),
                     "alg_bytes_per_launch": alg_bytes,
                     # exact rejection is VALU-issue bound, not HBM-bound
                     "valu": valu},
        "exact_pixels": int(exact_px),
        "all_to_all_ms": None if a2a_ms is None else round(a2a_ms, 3),
        "all_to_all_scope": (None if not sharded else
                             f"pipelined ({a.pipeline} row sub-chunks): staging + exchange of the first sub-chunk "
                             "(pipeline fill), the rest runs under the stacks" if pipelined else
                             "the whole band's transpose (staging copy + all_to_all_single), before the stack"),
        "gpu_clock": clk.summary(),
        # rejection totals per step (one stack); summed over the bands of all ranks
        "rejected_per_step": [int(x) // a.steps for x in counts.tolist()],
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"], ref = cpu_baseline(frames, int(rt), sig, method, a.cpu_seconds, u16, norm)
        res["cpu_baseline"]["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
        res["parity"] = parity_vs_oracle(ctx, S, frames, args, method, ref, u16)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    for c in ctxs[1:]:
        c.close()
    ctx.close()
    if use_pg:
        dist.destroy_process_group()


def _dist_setup(a):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # frame-sharded input always goes through the process group (RCCL), also
    # on one GPU: the all-to-all transpose then runs with a single rank, which
    # exercises the collective path on a 1-GPU box
    use_pg = world > 1 or a.input == "frame-sharded"
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    return world, rank, local, dev


_LAST_CLOCK = None


def _write_seq_only(d, n, name="synth_"):
    """The .seq of n regular FITS frames already written in d (synth names)."""
    from siril_amd.sequence import write_seq
    path = os.path.join(d, name + ".seq")
    write_seq(path, name, n)
    return path


def _timed(step, steps, warmup, world, ctx, dev):
    """W untimed steps, then K steps between barrier + synchronize; returns
    (max-over-ranks elapsed s, per-step sgpu_last_timing list)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    kern = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    global _LAST_CLOCK
    with ClockSampler(dev) as clk:
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
            kern.append(ctx.last_timing())
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    _LAST_CLOCK = clk.summary()
    ctx.set_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), kern


def _rl_observed(h, w, ks, dev, seed=5):
    """Star field blurred (circularly) by the benchmark PSF + noise, in HBM."""
    import numpy as np
    import torch
    from siril_amd import synth
    from siril_amd.deconvolution import moffat_psf
    K = moffat_psf(ks, fwhm=6.0, ellipticity=1.2, angle=0.2)
    img = torch.from_numpy(synth.star_field(h, w, nstars=4000, sigma=1.2, seed=seed).astype(np.float32)).to(dev)
    pad = torch.zeros((h, w), dtype=torch.float32, device=dev)
    kt = torch.from_numpy(K).to(dev)
    r = ks // 2
    for ky in range(ks):                       # padcirc: centre at the origin
        rows = torch.arange(ks, device=dev)
        pad[(ky - r) % h, (rows - r) % w] = kt[ky]
    obs = torch.fft.ifft2(torch.fft.fft2(img) * torch.fft.fft2(pad)).real
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    obs = obs + 0.002 * torch.randn(obs.shape, device=dev, generator=g)
    return obs.clamp_(1e-4, None).float().contiguous(), K


class _ThreadedFFT:
    """fft2 / ifft2 through scipy.fft with `workers` threads (pocketfft, as
    numpy): the CPU baselines of the FFT restatements run on the host's cores."""

    def __init__(self, workers):
        import scipy.fft as sf
        self.sf, self.workers = sf, workers

    def fft2(self, x):
        return self.sf.fft2(x, workers=self.workers)

    def ifft2(self, x):
        return self.sf.ifft2(x, workers=self.workers)


def _fft_threads():
    return max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))


def cpu_baseline_rl(obs, K, iters, target_s):
    """numpy restatement (oracle/rl_ref.py, complex128, pocketfft through
    scipy.fft on the host's cores) on a crop of the benchmark image, all
    iterations."""
    import numpy as np
    from oracle import rl_ref as R
    threads = _fft_threads()
    saved, R.FFT = R.FFT, _ThreadedFFT(threads)
    try:
        h = w = 256
        crop = np.ascontiguousarray(obs[:h, :w].cpu().numpy())[None]
        t0 = time.perf_counter()
        R.fft_richardson_lucy(crop, K[None], maxiter=iters, regtype=R.REG_NONE_MULT)
        dt = time.perf_counter() - t0
        scale = max(1.0, (target_s / max(dt, 1e-3)) ** 0.5)
        h = min(obs.shape[0], int(h * scale))
        w = min(obs.shape[1], int(w * scale))
        crop = np.ascontiguousarray(obs[:h, :w].cpu().numpy())[None]
        t0 = time.perf_counter()
        R.fft_richardson_lucy(crop, K[None], maxiter=iters, regtype=R.REG_NONE_MULT)
        dt = time.perf_counter() - t0
    finally:
        R.FFT = saved
    return {"value": round(h * w / dt / 1e6, 5), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{w}x{h} crop, {iters} iterations, complex128 FFT restatement, scipy.fft "
                      f"{threads} workers ({dt:.1f} s)"}


def cpu_baseline_dft(frames, S, target_s):
    """numpy restatement (oracle/dft_ref.py, complex128, pocketfft through
    scipy.fft on the host's cores) on a few frames of the benchmark stack;
    Mpix/s of S x S selections, as the GPU line counts."""
    import numpy as np
    from oracle import dft_ref
    threads = _fft_threads()
    n, h, w = frames.shape
    y0, x0 = (h - S) // 2, (w - S) // 2
    ref = frames[0, y0:y0 + S, x0:x0 + S].cpu().numpy()
    saved, dft_ref.FFT = dft_ref.FFT, _ThreadedFFT(threads)
    try:
        done, t0 = 0, time.perf_counter()
        while done < n - 1 and (done == 0 or time.perf_counter() - t0 < target_s):
            dft_ref.dft_shift(ref, frames[1 + done, y0:y0 + S, x0:x0 + S].cpu().numpy())
            done += 1
        dt = time.perf_counter() - t0
    finally:
        dft_ref.FFT = saved
    return {"value": round(done * S * S / dt / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{done} frames, {S}x{S} selection, complex128 FFT restatement, scipy.fft "
                      f"{threads} workers ({dt:.1f} s)"}


def aux_pmc(config):
    """PMC record (profiles/pmc_traffic.json, scripts/pmc_summary.py) of a
    secondary config when it was taken from these sources."""
    try:
        ent = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json"))).get(config, {})
    except Exception:
        return {}
    return ent if ent.get("kernel_source_hash") == aux_source_hash(config) else {}


def bench_aux(a):
    """BASELINE configs 3 (DFT registration) and 5 (RL deconvolution): the
    path does not shard (one image / one reference): replicas only, each
    rank runs its own copy of the workload."""
    if a.config == "rl63_direct":
        os.environ["SGPU_RL_DIRECT"] = "1"          # read once by the library, before its first RL call
    import torch
    import torch.distributed as dist
    world, rank, local, dev = _dist_setup(a)
    from siril_amd import stacking as S
    kind = AUX_CONFIGS[a.config][0]
    ctx = S.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    res = {"n_gpus": world, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32"}
    if kind == "RL":
        from siril_amd import deconvolution as D
        from siril_amd._lib import lib
        _, iters, w, h, ks = AUX_CONFIGS[a.config]
        obs, K = _rl_observed(h, w, ks, dev, seed=5 + rank)
        work = torch.empty_like(obs)

        def step():
            work.copy_(obs)
            rc = D.fft_richardson_lucy(work, K, maxiter=iters, regtype=D.REG_NONE_MULT, ctx=ctx)
            assert rc == 0

        elapsed, kern = _timed(step, a.steps, a.warmup, world, ctx, dev)
        flops = lib().sgpu_rl_last_iter_flops(ctx.h)
        fft_convs = int(lib().sgpu_rl_last_fft_convs(ctx.h))
        it_bytes = lib().sgpu_rl_last_iter_bytes(ctx.h)
        it_ms = sum(k[0] for k in kern) / len(kern)
        taper_ms = sum(k[1] for k in kern) / len(kern)
        achieved = flops / (it_ms / 1e3) / 1e12
        if fft_convs:
            # FFT convolution (rl_fft.hip): HBM-bound passes over half spectra
            gbs = it_bytes / (it_ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                    "kernel": "k_rlf_rows_fwd / k_rlf_cols / k_rlf_rows_inv + transposes (FFT convolution)",
                    "iteration_ms": round(it_ms, 3), "taper_ms": round(taper_ms, 3),
                    "alg_bytes_per_step": it_bytes,
                    "direct_equivalent_tflops": round(achieved, 3)}
        else:
            roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": MFMA_F32_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": round(achieved / MFMA_F32_PEAK_TFS, 4), "traffic": None,
                    "kernel": "k_conv2d_mfma", "iteration_ms": round(it_ms, 3),
                    "taper_ms": round(taper_ms, 3), "alg_flops_per_step": flops}
            pm = aux_pmc(a.config)
            if pm.get("mfma_busy_frac") is not None:
                # rocprof: SQ_VALU_MFMA_BUSY_CYCLES over the dispatch's cycles x 1024 SIMDs
                roof["mfma_util_pmc"] = pm["mfma_busy_frac"]
                roof["mfma_util_profile"] = pm.get("source")
        res.update({
            "metric": f"RL deconvolution Mpix/s ({iters} iters, {w}x{h} fp32, 64x64 PSF cropped to {ks}x{ks})",
            "value": round(world * w * h * a.steps / elapsed / 1e6, 4), "unit": "Mpix/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "data": "synthetic star field blurred by a Moffat PSF + noise, generated in HBM",
            "config": {"workload": f"BASELINE config 5: rl -mul, {iters} iterations, {w}x{h}, PSF {ks}x{ks}",
                       "parallelism": "replicas only" if world > 1 else "single GPU",
                       "conv_launches_per_step": int(lib().sgpu_rl_last_conv_launches(ctx.h)),
                       "fft_convs_per_step": fft_convs},
            "roofline": roof,
        })
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_rl(obs, K, iters, a.cpu_seconds)
    elif kind == "RCD":
        import numpy as np
        from siril_amd import demosaic as Dm, synth
        _, _, w, h, _ = AUX_CONFIGS[a.config]
        base = torch.from_numpy(synth.star_field(h, w, nstars=4000, seed=13 + rank).astype(np.float32)).to(dev)
        yy = torch.arange(h, device=dev)[:, None] & 1
        xx = torch.arange(w, device=dev)[None, :] & 1
        gain = torch.where((yy ^ xx) == 1, 1.0, torch.where(yy == 0, 0.8, 0.6))   # RGGB site gains
        mos = (base * gain * 60000.0 + 100.0).float().contiguous()
        rgb = torch.empty((3, h, w), dtype=torch.float32, device=dev)

        interp = Dm.BAYER_BILINEAR if a.config == "bayerfast" else Dm.BAYER_RCD

        def step():
            Dm.debayer(mos, pattern=0, out=rgb, ctx=ctx, interpolation=interp)

        elapsed, kern = _timed(step, a.steps, a.warmup, world, ctx, dev)
        pipe_ms = sum(k[0] for k in kern) / len(kern)
        alg_bytes = 16 * w * h            # read the CFA frame once, write 3 planes
        achieved = alg_bytes / (pipe_ms / 1e3) / 1e9
        res.update({
            "metric": f"{'bayerfast (BAYER_BILINEAR)' if a.config == 'bayerfast' else 'RCD'} demosaic Mpix/s "
                      f"({w}x{h} fp32 CFA -> planar RGB)",
            "value": round(world * w * h * a.steps / elapsed / 1e6, 3), "unit": "Mpix/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "data": "synthetic star field mosaicked RGGB, generated in HBM",
            "config": {"workload": f"SURVEY 8 D1: debayer_buffer_new_float "
                                   f"{'BAYER_BILINEAR' if a.config == 'bayerfast' else 'RCD'}, {w}x{h} RGGB",
                       "parallelism": "replicas only" if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "min/max + k_bayerfast (one stencil pass)" if a.config == "bayerfast" else {
                                    "1": "RCD pipeline (min/max + one LDS-tiled k_rcd_fused)",
                                    "2": "RCD pipeline (min/max + one LDS-tiled k_rcd_fused, 32x32)",
                                    "0": "RCD pipeline (min/max, 7 stencil passes)"}.get(
                                        os.environ.get("SGPU_RCD_FUSED", "0"),
                                        "RCD pipeline (min/max + k_rcd_a / k_rcd_b, LDS halos)"),
                         "pipeline_ms": round(pipe_ms, 3),
                         "alg_bytes_per_step": alg_bytes},
        })
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            from oracle import demosaic_ref as Do
            crop = mos[:1000, :1500].cpu().numpy()
            t0 = time.perf_counter()
            reps = 0
            while reps == 0 or time.perf_counter() - t0 < a.cpu_seconds:
                Do.debayer_buffer_new_float(crop, Do.BAYER_BILINEAR if a.config == "bayerfast" else Do.BAYER_RCD,
                                            Do.RGGB)
                reps += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": round(reps * crop.size / dt / 1e6, 4), "unit": "Mpix/s", "cores": 1,
                                   "kind": "port",
                                   "sample": f"{reps} x 1500x1000 crop, numpy restatement ({dt:.1f} s)"}
    elif kind == "NORM":
        import numpy as np
        from siril_amd import normalization as Nz, synth
        _, n, w, h, _ = AUX_CONFIGS[a.config]
        frames = synth.frames_torch(n, h, w, dev, seed=20260821 + 1000 * rank)

        def step():
            st = Nz.norm_stats_device(ctx, frames, lite=False)
            assert not st.status.any()

        elapsed, _ = _timed(step, a.steps, a.warmup, world, ctx, dev)
        # 9 streaming passes over every frame: 4 count/min/max, 4 histogram, 1 bwmv
        # (median -> MAD -> IKSS median -> IKSS MAD -> bwmv are data-dependent)
        passes = 9
        alg_bytes = passes * 4 * n * w * h
        achieved = alg_bytes / (elapsed / a.steps) / 1e9
        res.update({
            "metric": f"normalization estimators Mpix/s (STATS_NORM: median, MAD, IKSS; {n}x{w}x{h} fp32)",
            "value": round(world * n * w * h * a.steps / elapsed / 1e6, 3), "unit": "Mpix/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "data": "synthetic (seeded BASELINE config-2 recipe, generated in HBM)",
            "config": {"workload": f"SURVEY 8f rank 1: -norm=addscale statistics of {n} frames {w}x{h}",
                       "parallelism": "replicas only" if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "norm_stats pipeline (k_minmax x4, k_hist x4, k_bwmv, k_select x4)",
                         "alg_bytes_per_step": alg_bytes, "passes": passes},
        })
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            from oracle import oracle as O
            O.build()
            one = frames[0].cpu().numpy()
            t0 = time.perf_counter()
            reps = 0
            while reps == 0 or time.perf_counter() - t0 < min(a.cpu_seconds, 10.0):
                O.norm_stats(one)
                reps += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": round(reps * w * h / dt / 1e6, 3), "unit": "Mpix/s", "cores": 1,
                                   "kind": "port",
                                   "sample": f"{reps} x one {w}x{h} frame, C restatement single thread ({dt:.1f} s)"}
    elif kind == "SEQ":
        import shutil
        import tempfile
        import numpy as np
        from siril_amd import sequence as Q, synth
        _, n, w, h, bits = AUX_CONFIGS[a.config]
        d = tempfile.mkdtemp(prefix=f"sgpu_{a.config}_r{rank}_")
        try:
            # the frames: the config-2 recipe generated in HBM, written through
            # the native FITS / SER writers (outside the timed region)
            t_w = time.perf_counter()
            if bits == 16:
                allf = np.empty((n, h, w), np.uint16)
                for f0 in range(0, n, 10):
                    t = synth.frames_torch(min(10, n - f0), h, w, dev, seed=20260821 + f0)
                    allf[f0:f0 + t.shape[0]] = torch.round(t * 65535.0).to(torch.int32).cpu().numpy().astype(np.uint16)
                    del t
                seq = synth.write_sequence(d, allf, kind="ser")
                del allf
            else:
                from siril_amd.sequence import frame_name, write_fits, write_seq
                for f0 in range(0, n, 10):
                    t = synth.frames_torch(min(10, n - f0), h, w, dev, seed=20260821 + f0).cpu().numpy()
                    for k in range(t.shape[0]):
                        write_fits(os.path.join(d, frame_name("synth_", f0 + k + 1, 5)), t[k])
                    del t
                seq = _write_seq_only(d, n)
            torch.cuda.empty_cache()
            t_w = time.perf_counter() - t_w
            # the link's pinned H2D rate, measured here (the PCIe figure the
            # pipeline is compared with)
            hb = torch.empty(1 << 28, dtype=torch.float32, pin_memory=True)
            db = torch.empty_like(hb, device=dev)
            for _ in range(2):
                db.copy_(hb, non_blocking=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                db.copy_(hb, non_blocking=True)
            e1.record()
            torch.cuda.synchronize()
            pcie = 4 * hb.numel() * 4 / (e0.elapsed_time(e1) / 1e3) / 1e9
            del hb, db
            torch.cuda.empty_cache()
            outp = os.path.join(d, "result.fit")
            stats = []

            def step():
                Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -out={outp}", ctx)
                stats.append(ctx.last_seq_stats())

            elapsed, _ = _timed(step, a.steps, a.warmup, world, ctx, dev)
            st = stats[-a.steps:]
            mean = lambda k: sum(x[k] for x in st) / len(st)
            h2d_gbs = mean("h2d_bytes") / (mean("h2d_ms") / 1e3) / 1e9 if mean("h2d_ms") else None
            in_bytes = n * w * h * (2 if bits == 16 else 4)
            e2e_in_gbs = in_bytes / (elapsed / a.steps) / 1e9
            kern_ms = mean("kernel_ms")
            res.update({
                "metric": f"headless sequence stack Mpix/s ({n}x{w}x{h} {'16-bit SER' if bits == 16 else 'fp32 FITS'}, "
                          "Winsorized 3/3, read + H2D + stack + write)",
                "value": round(world * w * h * a.steps / elapsed / 1e6, 3), "unit": "Mpix/s",
                "ms_per_step": round(elapsed / a.steps * 1e3, 3),
                "data": "synthetic config-2 recipe written as a sequence (page cache)",
                "config": {"workload": f"SURVEY 8f rank 2: stack synth_ rej w 3 3 -nonorm -32b, {n} "
                                       f"{'frames in one SER file' if bits == 16 else 'FITS files'} {w}x{h}",
                           "parallelism": "replicas only" if world > 1 else "single GPU",
                           "blocks": int(mean("blocks")), "readers": int(mean("readers")),
                           "pinned": bool(st[-1]["pinned"]), "write_s_untimed": round(t_w, 1)},
                "roofline": {"bound": "pcie", "achieved": None if h2d_gbs is None else round(h2d_gbs, 2),
                             "peak": round(pcie, 2), "unit": "GB/s",
                             "frac": None if h2d_gbs is None else round(h2d_gbs / pcie, 4),
                             "end_to_end_input_gbs": round(e2e_in_gbs, 2),
                             "end_to_end_frac_of_pcie": round(e2e_in_gbs / pcie, 4),
                             "traffic": None,
                             "kernel": "per block: H2D copy stream -> k_stack_wz_* on the context stream",
                             "kernel_ms": round(kern_ms, 3), "h2d_ms": round(mean("h2d_ms"), 3),
                             "readers_s": round(mean("read_s"), 3), "loop_s": round(mean("loop_s"), 3),
                             "setup_s": round(mean("setup_s"), 3), "write_s": round(mean("write_s"), 3),
                             "call_s": round(mean("call_s"), 3),
                             "note": "peak = pinned 1 GiB torch H2D measured in this run; achieved = the "
                                     "pipeline's H2D bytes over its copy-stream event time"},
            })
        finally:
            shutil.rmtree(d, ignore_errors=True)
        res["cpu_baseline"] = None
    elif kind == "FITS":
        import shutil
        import tempfile
        import numpy as np
        from siril_amd import sequence as Q, synth
        _, n, w, h, _ = AUX_CONFIGS[a.config]
        d = tempfile.mkdtemp(prefix=f"sgpu_fits10_r{rank}_")
        frames = synth.config1_frames(n, h, w, seed=20260821 + 100 * rank)
        seq = synth.write_sequence(d, frames)        # outside the timed region
        outp = os.path.join(d, "result.fit")

        def step():
            Q.run_command(f"stack {seq} rej n -nonorm -32b -out={outp}", ctx)

        elapsed, kern = _timed(step, a.steps, a.warmup, world, ctx, dev)
        kern_ms = sum(k[0] for k in kern) / len(kern)
        alg_bytes = n * w * h * 4 + w * h * 4
        res.update({
            "metric": f"headless FITS stack Mpix/s ({n}x{w}x{h} fp32 FITS, mean, read+stack+write)",
            "value": round(world * w * h * a.steps / elapsed / 1e6, 3), "unit": "Mpix/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "data": "synthetic BASELINE config-1 frames written as a FITS sequence (page cache)",
            "config": {"workload": f"BASELINE config 1: stack synth_ rej n -nonorm -32b, {n} FITS {w}x{h}",
                       "parallelism": "replicas only" if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": round(alg_bytes / (kern_ms / 1e3) / 1e9, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg_bytes / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "k_stack_mean (per block, last block timed)", "kernel_ms": round(kern_ms, 4),
                         "note": "end-to-end step is host I/O bound (FITS read/convert, PCIe)"},
        })
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            from oracle import oracle as O
            O.build()
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            t0 = time.perf_counter()
            reps = 0
            while reps == 0 or time.perf_counter() - t0 < min(a.cpu_seconds, 5.0):
                O.stack_rows(frames, 0, (3.0, 3.0), nthreads=threads)
                reps += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": round(reps * w * h / dt / 1e6, 3), "unit": "Mpix/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{reps} x the full {n}x{w}x{h} in-memory stack (no FITS I/O), {dt:.1f} s"}
        shutil.rmtree(d, ignore_errors=True)
    else:
        from siril_amd import synth, registration as Rg
        _, n, w, h, Ssel = AUX_CONFIGS[a.config]
        base = synth.star_field(h, w, nstars=6000, seed=9 + rank)
        import numpy as np
        rng = np.random.default_rng(3 + rank)
        frames = torch.empty((n, h, w), dtype=torch.float32, device=dev)
        bt = torch.from_numpy(base.astype(np.float32)).to(dev)
        for f in range(n):
            dx, dy = (0, 0) if f == 0 else (int(rng.integers(-80, 81)), int(rng.integers(-80, 81)))
            frames[f] = torch.roll(bt, (dy, dx), (0, 1)) + 0.002 * torch.randn((h, w), device=dev)
        sel = ((w - Ssel) // 2, (h - Ssel) // 2, Ssel, Ssel)
        box = {}

        def step():
            # shifts + per-frame QualityEstimate + normalizeQualityData, as register_shift_dft does
            box["s"] = Rg.register_shift_dft_full(frames, 0, sel, ctx)

        # the pipeline time comes from HIP events the library records on the
        # stream it launches on (sgpu_last_timing ms[0])
        elapsed, kern = _timed(step, a.steps, a.warmup, world, ctx, dev)
        gpu_ms = sum(k[0] for k in kern) / len(kern)
        # DESIGN.md 4.4 traffic model, B per selection pixel (a half-spectrum
        # plane is 4 B/px): per frame rows fwd 4 + 4, fused columns (plane,
        # reference spectrum, write back) 12, C2R + argmax 4 = 24; the
        # reference frame once: rows 8 + columns 8.  The A/B layouts add
        # their passes: two transposes 16 (SGPU_DFT_TRANSPOSE=1), the split
        # column passes 8 (SGPU_DFT_FUSED=0)
        transposed = os.environ.get("SGPU_DFT_TRANSPOSE", "0") not in ("", "0")
        split = os.environ.get("SGPU_DFT_FUSED", "1") == "0"
        per_frame = 24 + (16 if transposed else 0) + (8 if split else 0)
        alg_bytes = (per_frame * (n - 1) + 16 + (16 if transposed else 0)) * Ssel * Ssel
        achieved = alg_bytes / (gpu_ms / 1e3) / 1e9
        res.update({
            # pixels of the S x S selections the path actually transforms
            "metric": f"DFT registration Mpix/s of {Ssel}x{Ssel} selections ({n} frames {w}x{h} fp32)",
            "value": round(world * n * Ssel * Ssel * a.steps / elapsed / 1e6, 3), "unit": "Mpix/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "data": "synthetic star field, integer-shifted frames + noise, generated in HBM",
            "config": {"workload": f"BASELINE config 3: REG_DFT of {n} frames {w}x{h}, centred {Ssel}^2 selection"
                                   " (integer shifts + frame quality + best frame)",
                       "parallelism": "replicas only" if world > 1 else "single GPU"},
            # roofline of the FFT pipeline alone (DFT events); the quality
            # kernels of the same step are outside pipeline_ms
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "scope": "DFT kernels only",
                         "kernel": ("DFT half-spectrum pipeline (row pairs fwd, transpose, columns fwd, xpow + columns bwd, transpose, C2R row pairs + argmax)"
                                    if transposed else
                                    "DFT half-spectrum pipeline (row pairs fwd into the column layout, columns fwd + xpow + columns bwd, C2R row pairs + argmax)"),
                         "pipeline_ms": round(gpu_ms, 3), "alg_bytes_per_step": alg_bytes},
        })
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_dft(frames, Ssel, a.cpu_seconds)
    res["gpu_clock"] = _LAST_CLOCK
    traffic, src = aux_traffic(a.config)
    if traffic is not None and "roofline" in res:
        res["roofline"]["traffic"] = traffic
        res["roofline"]["traffic_unit"] = "HBM bytes per step (FETCH_SIZE x 2 + WRITE_SIZE, rocprofv3 --pmc)"
        res["roofline"]["traffic_profile"] = src
    if rank == 0:
        if res.get("cpu_baseline"):
            res["cpu_baseline"]["gpu_over_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
