"""Stack normalization: per-frame estimators on the GPU and the factors.

Mirrors the reference's normalization pass (stacking/normalization.c):
`do_normalization` / `compute_normalization` (:44-78, :249-294) gather the
per-frame estimators with `compute_all_channels_statistics_seqimage(...,
STATS_NORM or STATS_LITENORM)` (statistics_float.c:281-480), and
`compute_factors_from_estimators` (:150-185) turns them into the
coefficients the stack's gather applies (median_and_mean.c:1644-1686).

The statistics run as HIP kernels (siril_amd/csrc/norm_stats.hip) over frames
resident in HBM; the factor arithmetic is the C-ABI's `sgpu_norm_factors`.
Overlap normalization (`args->overlap_norm`, compute_normalization_overlaps
:666-906) runs the same estimator kernels on the pairwise overlaps
(siril_amd/csrc/overlap_norm.hip) and solves the reference's linear systems
(`compute_normalization_overlaps` below).
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


def bgnoise(ctx, frames) -> np.ndarray:
    """Background noise (imstats bgnoise, FnNoise1_float / _ushort) of every
    plane of `frames` (N, H, W): numpy (host) or a torch tensor on the
    context's device; float32, or uint16 / int16 holding DATA_USHORT bits
    (ADU).  The estimator -weight=noise divides by."""
    n, h, w = (int(x) for x in frames.shape)
    out = np.zeros(n, np.float64)
    if isinstance(frames, np.ndarray):
        u16 = frames.dtype == np.uint16
        fr = np.ascontiguousarray(frames, np.uint16 if u16 else np.float32)
        fn = lib().sgpu_bgnoise_u16 if u16 else lib().sgpu_bgnoise
        check(fn(ctx.h, _ptr(fr), n, w, h, h * w, _ptr(out)), "sgpu_bgnoise")
        return out
    assert frames.is_contiguous() and frames.element_size() in (2, 4)
    fn = lib().sgpu_bgnoise_u16_device if frames.element_size() == 2 else lib().sgpu_bgnoise_device
    check(fn(ctx.h, C.c_void_p(frames.data_ptr()), n, w, h, h * w, _ptr(out)), "sgpu_bgnoise_device")
    return out


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


@dataclass
class OverlapStats:
    """Per-pair overlap estimators (seq->ostats of one layer, normalization.c
    :567-589), pair p = get_ijth_pair_index(n, i, j): nij[p] samples,
    table[p] = medij, medji, madij, madji, locij, locji, scaij, scaji."""
    nij: np.ndarray
    table: np.ndarray


def pair_index(n: int, i: int, j: int) -> int:
    """get_ijth_pair_index (normalization.c:412-414)."""
    return i * (2 * n - i - 1) // 2 + j - i - 1


def overlap_rect(width: int, height: int, dxi: float, dyi: float, dxj: float, dyj: float):
    """compute_overlap (normalization.c:420-456) from translation_from_H shifts
    -> ((x, y, w, h) on frame i, (x, y, w, h) on frame j, npix)."""
    ai = (C.c_int * 4)()
    aj = (C.c_int * 4)()
    npx = C.c_long(0)
    check(lib().sgpu_overlap_rect(int(width), int(height), float(dxi), float(dyi), float(dxj), float(dyj),
                                  C.cast(ai, C.c_void_p), C.cast(aj, C.c_void_p), C.cast(C.pointer(npx), C.c_void_p)),
          "sgpu_overlap_rect")
    return tuple(ai), tuple(aj), int(npx.value)


def overlap_stats_device(ctx, frames, h02, h12, lite: bool = False) -> OverlapStats:
    """_compute_estimators_for_images over every pair of the frames (torch
    tensor [N, H, W] on the context's device, float32 or 16-bit), with the
    per-frame registration h02 / h12 of the registration layer."""
    assert frames.dim() == 3 and frames.is_contiguous() and frames.element_size() in (2, 4)
    n, h, w = (int(x) for x in frames.shape)
    if n < 2:
        raise ValueError("overlap normalization needs at least 2 frames")
    h02 = np.ascontiguousarray(h02, np.float64)
    h12 = np.ascontiguousarray(h12, np.float64)
    if h02.size != n or h12.size != n:
        raise ValueError("one h02 / h12 per frame")
    npairs = n * (n - 1) // 2
    nij = np.zeros(npairs, np.int64)
    tab = np.zeros((npairs, 8), np.float64)
    fn = lib().sgpu_overlap_stats_u16_device if frames.element_size() == 2 else lib().sgpu_overlap_stats_device
    check(fn(ctx.h, C.c_void_p(frames.data_ptr()), n, w, h, w * h, _ptr(h02), _ptr(h12), int(bool(lite)),
             _ptr(nij), _ptr(tab)), "sgpu_overlap_stats_device")
    return OverlapStats(nij, tab)


def overlap_factors(normalize: Normalization, ost: OverlapStats, ref_index: int = 0, lite: bool = False):
    """The coefficients of compute_normalization_overlaps (:804-906) ->
    (offset, mul, scale) = coeff.poffset / pmul / pscale of the layer."""
    npairs = ost.nij.size
    n = int(round((1 + (1 + 8 * npairs) ** 0.5) / 2))
    off = np.zeros(n, np.float64)
    mul = np.ones(n, np.float64)
    scl = np.ones(n, np.float64)
    nij = np.ascontiguousarray(ost.nij, np.int64)
    tab = np.ascontiguousarray(ost.table, np.float64)
    check(lib().sgpu_overlap_factors(int(normalize), int(bool(lite)), n, int(ref_index), _ptr(nij), _ptr(tab),
                                     _ptr(off), _ptr(mul), _ptr(scl)), "sgpu_overlap_factors")
    return off, mul, scl


def compute_normalization_overlaps(ctx, frames, normalize: Normalization, h02, h12, ref_index: int = 0,
                                   lite: bool = False):
    """do_normalization with args->overlap_norm for one layer held in HBM
    (torch tensor [N, H, W]) or host memory (numpy, uploaded once):
    returns (offset, mul, scale, OverlapStats)."""
    if int(normalize) == int(Normalization.NO_NORM):
        n = int(frames.shape[0])
        return np.zeros(n), np.ones(n), np.ones(n), None
    if isinstance(frames, np.ndarray):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(frames))
        if t.dtype == torch.uint16:
            t = t.view(torch.int16)
        frames = t.to(f"cuda:{ctx.device}")
    ost = overlap_stats_device(ctx, frames, h02, h12, lite)
    off, mul, scl = overlap_factors(normalize, ost, ref_index, lite)
    return off, mul, scl, ost
