"""Stack normalization: per-frame estimators on the GPU and the factors.

Mirrors the reference's normalization pass (stacking/normalization.c):
`do_normalization` / `compute_normalization` (:44-78, :249-294) gather the
per-frame estimators with `compute_all_channels_statistics_seqimage(...,
STATS_NORM or STATS_LITENORM)` (statistics_float.c:281-480), and
`compute_factors_from_estimators` (:150-185) turns them into the
coefficients the stack's gather applies (median_and_mean.c:1644-1686).

The statistics run as HIP kernels (siril_amd/csrc/norm_stats.hip) over frames
resident in HBM; the factor arithmetic is the C-ABI's `sgpu_norm_factors`.
Overlap normalization (`args->overlap_norm`) is not built.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import check, lib
from .stacking import Normalization


class NormalizationError(RuntimeError):
    """compute_normalization failed: the reference logs "Normalization failed.
    Check image %d first." and the stack returns ST_GENERIC_ERROR."""


@dataclass
class NormStats:
    """Per-frame estimators (imstats fields of one layer)."""
    median: np.ndarray
    mad: np.ndarray
    location: np.ndarray
    scale: np.ndarray
    ngood: np.ndarray
    status: np.ndarray

    def as_table(self) -> np.ndarray:
        return np.ascontiguousarray(np.stack([self.median, self.mad, self.location, self.scale], 1))


def _ptr(a):
    return C.c_void_p(a.ctypes.data)


def _unpack(tab, ng, st):
    return NormStats(tab[:, 0].copy(), tab[:, 1].copy(), tab[:, 2].copy(), tab[:, 3].copy(), ng, st)


def norm_stats(ctx, frames: np.ndarray, lite: bool = False) -> NormStats:
    """Estimators of every plane of `frames` (N, H, W), host memory: float32
    (DATA_FLOAT) or uint16 (DATA_USHORT, estimators in 16-bit units)."""
    u16 = np.asarray(frames).dtype == np.uint16
    fr = np.ascontiguousarray(frames, np.uint16 if u16 else np.float32)
    n = fr.shape[0]
    npix = int(np.prod(fr.shape[1:]))
    tab = np.zeros((n, 4), np.float64)
    ng = np.zeros(n, np.int64)
    st = np.zeros(n, np.int32)
    fn = lib().sgpu_norm_stats_u16 if u16 else lib().sgpu_norm_stats
    check(fn(ctx.h, _ptr(fr), n, npix, npix, int(bool(lite)), _ptr(tab), _ptr(ng), _ptr(st)), "sgpu_norm_stats")
    return _unpack(tab, ng, st)


def norm_stats_device(ctx, frames, lite: bool = False) -> NormStats:
    """Same for a torch tensor (N, H, W) on the context's device: float32, or
    int16/uint16 holding DATA_USHORT bits (runs on the context's stream,
    synchronises once)."""
    assert frames.is_contiguous() and frames.element_size() in (2, 4)
    u16 = frames.element_size() == 2
    n = int(frames.shape[0])
    npix = int(frames[0].numel())
    tab = np.zeros((n, 4), np.float64)
    ng = np.zeros(n, np.int64)
    st = np.zeros(n, np.int32)
    fn = lib().sgpu_norm_stats_u16_device if u16 else lib().sgpu_norm_stats_device
    check(fn(ctx.h, C.c_void_p(frames.data_ptr()), n, npix, npix, int(bool(lite)), _ptr(tab), _ptr(ng), _ptr(st)),
          "sgpu_norm_stats_device")
    return _unpack(tab, ng, st)


def factors(normalize: Normalization, stats: NormStats, ref_index: int = 0, lite: bool = False,
            ref_stats: NormStats | None = None):
    """compute_factors_from_estimators for one layer -> (offset, mul, scale),
    i.e. coeff.poffset / pmul / pscale.  Raises NormalizationError when a
    frame's statistics failed, as compute_normalization does."""
    bad = np.nonzero(stats.status)[0]
    if bad.size:
        raise NormalizationError(f"Normalization failed. Check image {int(bad[0]) + 1} first.")
    n = stats.median.size
    tab = stats.as_table()
    rtab = ref_stats.as_table() if ref_stats is not None else None
    off = np.zeros(n, np.float64)
    mul = np.ones(n, np.float64)
    scl = np.ones(n, np.float64)
    check(lib().sgpu_norm_factors(int(normalize), int(bool(lite)), n, int(ref_index), _ptr(tab),
                                  _ptr(rtab) if rtab is not None else None, _ptr(off), _ptr(mul), _ptr(scl)),
          "sgpu_norm_factors")
    return off, mul, scl


def compute_normalization(ctx, frames, normalize: Normalization, ref_index: int = 0, lite: bool = False):
    """do_normalization for a single-layer stack held in host memory
    (numpy) or HBM (torch tensor): returns (offset, mul, scale, stats)."""
    if int(normalize) == int(Normalization.NO_NORM):
        n = int(frames.shape[0])
        return np.zeros(n), np.ones(n), np.ones(n), None
    if isinstance(frames, np.ndarray):
        st = norm_stats(ctx, frames, lite)
    else:
        st = norm_stats_device(ctx, frames, lite)
    off, mul, scl = factors(normalize, st, ref_index, lite)
    return off, mul, scl, st
