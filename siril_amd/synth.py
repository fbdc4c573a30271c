"""Seeded synthetic frame stacks (BASELINE.md config 2/4 recipe).

Frame f: b(x, y) = 0.05 + 0.02*x/W + N(0, 0.005); 1 % of samples get a cosmic
ray +U(0.2, 0.6); 0.1 % are cold pixels (x0.1); clipped to [1e-6, 1] so no
sample is an exact zero (zero = missing in Siril, rejection_float.c:128-135).
Layout: frame-major [N, H, W] float32, as Siril's block buffers
(median_and_mean.c:1503-1512).
"""
from __future__ import annotations

import numpy as np


def frames_numpy(n: int, h: int, w: int, seed: int = 20260821, shift_max: int = 0) -> np.ndarray:
    out = np.empty((n, h, w), np.float32)
    xs = (np.arange(w, dtype=np.float32) / np.float32(w))[None, :]
    for f in range(n):
        rng = np.random.default_rng(seed + f)
        a = np.float32(0.05) + np.float32(0.02) * xs + rng.normal(0, 0.005, (h, w)).astype(np.float32)
        cr = rng.random((h, w)) < 0.01
        a[cr] += rng.uniform(0.2, 0.6, int(cr.sum())).astype(np.float32)
        cold = rng.random((h, w)) < 0.001
        a[cold] *= np.float32(0.1)
        out[f] = np.clip(a, 1e-6, 1.0)
    return out


def frames_torch(n: int, h: int, w: int, device, seed: int = 20260821):
    """Same recipe generated directly in HBM (torch RNG, not bit-identical to
    the numpy variant)."""
    import torch
    out = torch.empty((n, h, w), dtype=torch.float32, device=device)
    xs = (torch.arange(w, dtype=torch.float32, device=device) / w)[None, :]
    g = torch.Generator(device=device)
    for f in range(n):
        g.manual_seed(seed + f)
        a = out[f]
        a.normal_(0.0, 0.005, generator=g)
        a.add_(0.05 + 0.02 * xs)
        u = torch.rand((h, w), device=device, generator=g)
        amp = torch.rand((h, w), device=device, generator=g) * 0.4 + 0.2
        a.add_(torch.where(u < 0.01, amp, torch.zeros_like(amp)))
        a.mul_(torch.where(u > 0.999, torch.full_like(amp, 0.1), torch.ones_like(amp)))
        a.clamp_(1e-6, 1.0)
        del u, amp
    return out
