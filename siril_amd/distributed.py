"""Multi-GPU rejection stack: pixel-row bands, one process per GPU.

Every output pixel is a function of its own N-sample column only, so the
exact decomposition is by rows (finding F3): rank r stacks the
rows [y0_r, y1_r) of all N frames -- the same row blocks Siril hands to its
OpenMP threads (stack_compute_parallel_blocks, median_and_mean.c:295-356) --
with no exchange during compute.  Afterwards:
  * the output bands are all-gathered (RCCL over xGMI with backend "nccl"),
  * the low/high rejection totals are all-reduced.
Frame sharding + partial-sum all-reduce would only be exact for the
no-rejection mean; sigma / Winsorized / median need whole columns.

The per-band compute is `Context.stack_device` by default; tests inject a
CPU compute function to check the decomposition with the gloo backend.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple


def row_bands(height: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced row bands [y0, y1) covering [0, height)."""
    base, extra = divmod(height, world)
    bands, y = [], 0
    for r in range(world):
        h = base + (1 if r < extra else 0)
        bands.append((y, y + h))
        y += h
    return bands


def stack_row_band(frames_band, args, method, ctx=None, compute: Optional[Callable] = None):
    """Stack one band; returns (out [rows, W] float32 tensor, counts [2] int64 tensor)."""
    import torch
    if compute is not None:
        return compute(frames_band, args, method)
    out, _, _, counts = ctx.stack_device(frames_band, args, method)
    return out, counts


def stack_distributed(frames_band, height: int, args, method: int = 0, ctx=None,
                      compute: Optional[Callable] = None, group=None):
    """Collective over the default process group.  `frames_band` holds this
    rank's rows [y0, y1) of every frame ([N, y1-y0, W], on this rank's device
    for backend nccl).  Returns (full image [height, W] on every rank,
    (rejected_low, rejected_high) totals)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bands = row_bands(height, world)
    y0, y1 = bands[rank]
    n, rows, W = frames_band.shape
    if rows != y1 - y0:
        raise ValueError(f"rank {rank} holds {rows} rows, band is {y1 - y0}")
    out, counts = stack_row_band(frames_band, args, method, ctx, compute)
    # pad every band to the largest one so all_gather sees equal shapes
    hmax = max(b1 - b0 for b0, b1 in bands)
    pad = torch.zeros((hmax, W), dtype=out.dtype, device=out.device)
    pad[:rows] = out
    gathered = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad, group=group)
    full = torch.cat([g[: b1 - b0] for g, (b0, b1) in zip(gathered, bands)], dim=0)
    counts = counts.to(torch.int64).clone()
    dist.all_reduce(counts, group=group)
    return full, (int(counts[0]), int(counts[1]))
