"""Host-side mirror of Siril's Richardson-Lucy entry points over the C-ABI.

  * `fft_richardson_lucy`   -- filters/deconvolution/deconvolve.cpp:56-84
  * `naive_richardson_lucy` -- filters/deconvolution/deconvolve.cpp:86-114
  * `deconvolve_rl`         -- the dispatch of deconvolution.c:806-817
                               (RL_MULT -> REG_NONE_MULT, ks < fft_cutoff ->
                               naive) plus the even-PSF crop of :236-244

Same argument meaning and return values as the reference: planar float
data deconvolved in place, 0 on success, 1 when a channel's maximum is 0.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ._lib import check, lib

REG_TV_GRAD, REG_FH_GRAD, REG_NONE_GRAD, REG_TV_MULT, REG_FH_MULT, REG_NONE_MULT = range(6)
FFT_CUTOFF = 15          # deconvolution.c: fft_cutoff default
STEPSIZE = 0.0003        # deconvolution.c:112-177 defaults
STOPCRITERION = 0.002
ALPHA = float(np.float32(1.0) / np.float32(3000.0))   # args->alpha default (1.f / 3000.f) (deconvolution.c:172): the entry points' lambda


def _planar(fdata: np.ndarray) -> np.ndarray:
    if fdata.dtype != np.float32 or not fdata.flags.c_contiguous:
        raise TypeError("fdata must be a C-contiguous float32 array (modified in place)")
    if fdata.ndim == 2:
        return fdata[None]
    if fdata.ndim != 3:
        raise ValueError("fdata must be (ry, rx) or (nchans, ry, rx)")
    return fdata


def _kernel(kernel) -> np.ndarray:
    k = np.ascontiguousarray(kernel, np.float32)
    if k.ndim == 2:
        k = k[None]
    if k.ndim != 3 or k.shape[1] != k.shape[2]:
        raise ValueError("kernel must be (ks, ks) or (kchans, ks, ks)")
    return k


def crop_even_psf(kernel: np.ndarray) -> np.ndarray:
    """deconvolution.c:236-244: an even PSF loses its last row and column."""
    k = _kernel(kernel)
    ks = k.shape[-1]
    if ks % 2 == 0:
        k = np.ascontiguousarray(k[:, :ks - 1, :ks - 1])
    return k


def _call(name: str, fdata, kernel, maxiter, regtype, stepsize, stopcriterion, stop_active, ctx, device,
          lam=ALPHA):
    f = fdata if device else _planar(fdata)
    k = _kernel(kernel)
    ks = k.shape[-1]
    if device:
        import torch
        if f.dtype != torch.float32 or not f.is_contiguous():
            raise TypeError("device fdata must be a contiguous float32 tensor")
        shp = tuple(f.shape)
        nch, ry, rx = (1,) + shp if len(shp) == 2 else shp
        ctx.set_stream(torch.cuda.current_stream(f.device).cuda_stream)
        ptr = C.c_void_p(f.data_ptr())
    else:
        nch, ry, rx = f.shape
        ptr = f.ctypes.data_as(C.c_void_p)
    rc = getattr(lib(), name)(ctx.h, ptr, rx, ry, nch, k.ctypes.data_as(C.c_void_p), ks, k.shape[0], float(lam),
                              int(maxiter), float(stopcriterion), int(regtype), float(stepsize), int(stop_active))
    if rc < 0:
        check(rc, name)
    return rc


def fft_richardson_lucy(fdata, kernel, maxiter: int = 10, regtype: int = REG_NONE_GRAD,
                        stepsize: float = STEPSIZE, stopcriterion: float = STOPCRITERION,
                        stopcriterion_active: int = 0, ctx=None, lam: float = ALPHA) -> int:
    """deconvolve.cpp:56-84 on host data (numpy, modified in place) or, for a
    torch.cuda tensor, on HBM-resident data.  `lam` is the entry point's
    lambda (args->alpha: 1/3000 by default, 1/X for `-alpha=X`)."""
    from .stacking import default_context
    ctx = ctx or default_context()
    device = not isinstance(fdata, np.ndarray)
    return _call("sgpu_rl_fft_device" if device else "sgpu_rl_fft", fdata, kernel, maxiter, regtype, stepsize,
                 stopcriterion, stopcriterion_active, ctx, device, lam)


def naive_richardson_lucy(fdata, kernel, maxiter: int = 10, regtype: int = REG_NONE_GRAD,
                          stepsize: float = STEPSIZE, stopcriterion: float = STOPCRITERION,
                          stopcriterion_active: int = 0, ctx=None, lam: float = ALPHA) -> int:
    """deconvolve.cpp:86-114 (direct zero-border correlation)."""
    from .stacking import default_context
    ctx = ctx or default_context()
    device = not isinstance(fdata, np.ndarray)
    return _call("sgpu_rl_naive_device" if device else "sgpu_rl_naive", fdata, kernel, maxiter, regtype,
                 stepsize, stopcriterion, stopcriterion_active, ctx, device, lam)


def deconvolve_rl(fdata, kernel, maxiter: int = 10, multiplicative: bool = False, stepsize: float = STEPSIZE,
                  stopcriterion: float = STOPCRITERION, stopcriterion_active: int = 0,
                  fft_cutoff: int = FFT_CUTOFF, ctx=None, regularisation: str | None = None,
                  alpha: float | None = None) -> int:
    """deconvolution.c:806-817: `rl [-mul] [-tv|-fh] [-alpha=X]` with a loaded
    PSF (option parsing: core/command.c:2451-2540; -alpha=X sets
    args->alpha = 1/X, default 1/3000)."""
    k = crop_even_psf(kernel)
    grad = {None: REG_NONE_GRAD, "tv": REG_TV_GRAD, "fh": REG_FH_GRAD}[regularisation]
    regtype = {REG_TV_GRAD: REG_TV_MULT, REG_FH_GRAD: REG_FH_MULT}.get(grad, REG_NONE_MULT) \
        if multiplicative else grad
    # data->alpha = 1.f / alpha in float (command.c:2479-2488; -alpha=0 is
    # accepted there and gives inf), as the reference computes it
    if alpha is None:
        lam = ALPHA
    else:
        with np.errstate(divide="ignore"):
            lam = float(np.float32(1.0) / np.float32(alpha))
    fn = naive_richardson_lucy if k.shape[-1] < fft_cutoff else fft_richardson_lucy
    return fn(fdata, k, maxiter, regtype, stepsize, stopcriterion, stopcriterion_active, ctx, lam)


def set_memory_budget(nbytes: int, ctx=None) -> None:
    """Slice-geometry memory budget (get_available_memory() in the reference)."""
    from .stacking import default_context
    ctx = ctx or default_context()
    check(lib().sgpu_rl_set_memory(ctx.h, int(nbytes)), "sgpu_rl_set_memory")


def moffat_psf(ks: int, fwhm: float = 4.0, beta: float = 4.5, ellipticity: float = 1.0, angle: float = 0.0,
               offset=(0.0, 0.0)) -> np.ndarray:
    """Synthetic (optionally elliptical, off-centre) Moffat PSF, ks x ks float32."""
    r = ks // 2
    y, x = np.mgrid[-r:ks - r, -r:ks - r].astype(np.float64)
    x = x - offset[0]
    y = y - offset[1]
    ca, sa = np.cos(angle), np.sin(angle)
    xr, yr = ca * x + sa * y, (-sa * x + ca * y) * ellipticity
    alpha = fwhm / (2.0 * np.sqrt(2.0 ** (1.0 / beta) - 1.0))
    k = (1.0 + (xr * xr + yr * yr) / (alpha * alpha)) ** (-beta)
    return (k / k.sum()).astype(np.float32)
