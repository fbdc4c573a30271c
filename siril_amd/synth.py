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


def star_field(h: int, w: int, nstars: int = 2000, sigma: float = 1.5, seed: int = 7,
               background: float = 0.05) -> np.ndarray:
    """Base star field for the DFT registration config (BASELINE config 3):
    Gaussian PSFs (sigma 1.5 px) of random flux on a flat background."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w), background, np.float64)
    ys = rng.uniform(0, h, nstars)
    xs = rng.uniform(0, w, nstars)
    flux = rng.uniform(0.05, 0.9, nstars)
    r = int(np.ceil(4 * sigma))
    gy, gx = np.mgrid[-r:r + 1, -r:r + 1]
    for y, x, f in zip(ys, xs, flux):
        iy, ix = int(y), int(x)
        fy, fx = y - iy, x - ix
        k = f * np.exp(-((gy - fy) ** 2 + (gx - fx) ** 2) / (2 * sigma * sigma))
        y0, y1, x0, x1 = iy - r, iy + r + 1, ix - r, ix + r + 1
        ky0, kx0 = max(0, -y0), max(0, -x0)
        ky1, kx1 = k.shape[0] - max(0, y1 - h), k.shape[1] - max(0, x1 - w)
        if ky1 <= ky0 or kx1 <= kx0:
            continue
        img[max(0, y0):min(h, y1), max(0, x0):min(w, x1)] += k[ky0:ky1, kx0:kx1]
    return img


def shifted_frames(base: np.ndarray, shifts, noise: float = 0.002, seed: int = 11) -> np.ndarray:
    """Frames = base translated by integer (dx, dy) (np.roll, wrap-around) + noise."""
    rng = np.random.default_rng(seed)
    out = np.empty((len(shifts),) + base.shape, np.float32)
    for i, (dx, dy) in enumerate(shifts):
        out[i] = (np.roll(base, (dy, dx), axis=(0, 1)) + rng.normal(0, noise, base.shape)).astype(np.float32)
    return out


def config1_frames(n: int = 10, h: int = 1024, w: int = 1024, seed: int = 20260821) -> np.ndarray:
    """BASELINE config 1 / SURVEY 8d: values 0.1 + 0.01*N(0,1) clipped to
    [1e-6, 1] (no exact zeros), seed 20260821 + f per frame."""
    out = np.empty((n, h, w), np.float32)
    for f in range(n):
        rng = np.random.default_rng(seed + f)
        out[f] = np.clip(0.1 + 0.01 * rng.standard_normal((h, w)), 1e-6, 1.0).astype(np.float32)
    return out


def write_sequence(directory: str, frames: np.ndarray, name: str = "synth_", fixed: int = 5,
                   shifts=None, included=None, kind: str = "fits", reference: int = 0, reg_layer: int = 0,
                   fwhm=None, quality=None, regdata=None, stackcnt=None) -> str:
    """Write frames [N, H, W] or [N, 3, H, W] (float32 or uint16; row 0 =
    first FITS row) as a sequence plus <name>.seq; returns the .seq path.
    kind: "fits" (regular: <name>00001.fit ...), "fitseq" (one <name>.fit
    holding every frame) or "ser" (<name>.ser, uint16 only; RGB frames
    interleaved, rows stored top-down as SER does)."""
    import os
    from .sequence import SER_MONO, SER_RGB, frame_name, write_fits, write_fitseq, write_seq, write_ser
    os.makedirs(directory, exist_ok=True)
    n = frames.shape[0]
    nl = 3 if frames.ndim == 4 else 1
    if kind == "fits":
        for f in range(n):
            write_fits(os.path.join(directory, frame_name(name, f + 1, fixed)), frames[f],
                       stackcnt=None if stackcnt is None else int(stackcnt[f]))
    elif kind == "fitseq":
        write_fitseq(os.path.join(directory, name + ".fit"), frames)
    elif kind == "ser":
        if frames.dtype != np.uint16:
            raise ValueError("SER frames are 8/16-bit")
        top_down = frames[..., ::-1, :]                      # FITS row q = SER row H-1-q
        if nl == 3:
            top_down = np.moveaxis(top_down, 1, -1)          # [N, H, W, 3] interleaved
        write_ser(os.path.join(directory, name + ".ser"), np.ascontiguousarray(top_down),
                  SER_RGB if nl == 3 else SER_MONO)
    else:
        raise ValueError(kind)
    seq = os.path.join(directory, name + ".seq")
    write_seq(seq, name, n, fixed=fixed, shifts=shifts, included=included, reference=reference,
              kind={"fits": None, "fitseq": "F", "ser": "S"}[kind], nb_layers=nl, reg_layer=reg_layer,
              fwhm=fwhm, quality=quality, **(regdata or {}))
    return seq
