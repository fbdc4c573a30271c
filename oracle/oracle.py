"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of the CPU restatement in
oracle/stack_ref.c (the parity checker and bench.py's cpu_baseline).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package (siril_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_stack.so")

# rejection enum, core/settings.h:43-52
NO_REJEC, PERCENTILE, SIGMA, MAD, SIGMEDIAN, WINSORIZED, LINEARFIT, GESDT = range(8)
# normalization enum, core/settings.h:34-40
NO_NORM, ADDITIVE, MULTIPLICATIVE, ADDITIVE_SCALING, MULTIPLICATIVE_SCALING = range(5)


class RejParams(C.Structure):
    _fields_ = [("type", C.c_int), ("sig", C.c_float * 2),
                ("crit", C.POINTER(C.c_float)), ("xf", C.POINTER(C.c_float)),
                ("m_x", C.c_float), ("m_dx2", C.c_float)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        fp, ip, dp = C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_double)
        L.or_quickmedian_f.restype = C.c_double
        L.or_quickmedian_f.argtypes = [fp, C.c_size_t]
        u16p = C.POINTER(C.c_uint16)
        L.or_quickmedian_u16.restype = C.c_double
        L.or_quickmedian_u16.argtypes = [u16p, C.c_size_t]
        L.or_histogram_median_u16.restype = C.c_double
        L.or_histogram_median_u16.argtypes = [u16p, C.c_size_t]
        L.or_quicksort_f.restype = None
        L.or_quicksort_f.argtypes = [fp, C.c_size_t]
        L.or_stats_float_sd.restype = C.c_float
        L.or_stats_float_sd.argtypes = [fp, C.c_int, fp]
        L.or_stats_float_mad.restype = C.c_double
        L.or_stats_float_mad.argtypes = [fp, C.c_size_t, C.c_double]
        L.or_norm_stats_f.restype = C.c_int
        L.or_norm_stats_f.argtypes = [fp, C.c_size_t, C.c_int, dp, C.POINTER(C.c_size_t)]
        L.or_norm_stats_u16.restype = C.c_int
        L.or_norm_stats_u16.argtypes = [C.POINTER(C.c_uint16), C.c_size_t, C.c_int, dp, C.POINTER(C.c_size_t)]
        L.or_linear_fit_setup.restype = None
        L.or_set_out16_mul.restype = None
        L.or_set_out16_mul.argtypes = [C.c_double]
        L.or_set_simd_lanes.restype = None
        L.or_set_simd_lanes.argtypes = [C.c_int]
        L.or_sum_f.restype = C.c_double
        L.or_sum_f.argtypes = [fp, C.c_int]
        L.or_linear_fit_setup.argtypes = [C.c_int, fp, fp, fp]
        L.or_stack_column_f.restype = C.c_double
        L.or_stack_column_f.argtypes = [fp, C.c_int, C.c_int, C.POINTER(RejParams), dp, ip, ip]
        L.or_stack_rows_f.restype = C.c_int
        L.or_stack_rows_f.argtypes = [fp, C.c_int, C.c_long, C.c_long, C.c_long, C.c_int,
                                      C.POINTER(RejParams), C.c_int, dp, dp, dp, dp, C.c_double,
                                      dp, C.c_int, fp, C.POINTER(C.c_uint16),
                                      C.POINTER(C.c_uint16), C.POINTER(C.c_uint64), C.c_int]
        L.or_stack_rows_planes_f.restype = C.c_int
        L.or_stack_rows_planes_f.argtypes = [fp, fp, fp] + L.or_stack_rows_f.argtypes[1:]
        u16p = C.POINTER(C.c_uint16)
        L.or_stack_rows_u16.restype = C.c_int
        L.or_stack_rows_u16.argtypes = [u16p, C.c_int, C.c_long, C.c_long, C.c_long, C.c_int,
                                        C.POINTER(RejParams), C.c_int, dp, dp, dp, dp, C.c_double,
                                        dp, C.c_int, fp, u16p, u16p, u16p, C.POINTER(C.c_uint64),
                                        C.c_int]
        L.or_stack_rows_u16_planes.restype = C.c_int
        L.or_stack_rows_u16_planes.argtypes = [u16p, fp, fp] + L.or_stack_rows_u16.argtypes[1:]
        _lib = L
    return _lib


def _fptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


def _dptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def gesd_critical_values(nb_frames: int, sig0: float, alpha: float) -> np.ndarray:
    """Critical values of median_and_mean.c:1477-1484 (gsl_cdf_tdist_Pinv there;
    scipy.stats.t.ppf here), evaluated in float like the reference."""
    from scipy.stats import t as tdist
    max_out = int(np.floor(nb_frames * np.float32(sig0)))
    out = np.zeros(max(max_out, 1), np.float32)
    size = nb_frames
    for j in range(max_out):
        td = np.float32(tdist.ppf(1.0 - np.float32(alpha) / (2 * size), size - 2))
        num = np.float32(size - 1) * td
        den = np.float32(np.sqrt(np.float32(size))) * np.float32(
            np.sqrt(np.float32(size - 2) + td * td))
        out[j] = np.float32(num / den)
        size -= 1
    return out


class Params:
    """Holds the ctypes RejParams plus the arrays it points to."""

    def __init__(self, rtype: int, sig=(3.0, 3.0), nb_frames: int = 0, crit=None):
        self.p = RejParams()
        self.p.type = rtype
        self.p.sig[0] = sig[0]
        self.p.sig[1] = sig[1]
        n = max(nb_frames, 1)
        self.xf = np.zeros(n, np.float32)
        mx, md = C.c_float(0), C.c_float(0)
        if nb_frames > 0:
            lib().or_linear_fit_setup(nb_frames, _fptr(self.xf), C.byref(mx), C.byref(md))
        self.p.xf = _fptr(self.xf)
        self.p.m_x, self.p.m_dx2 = mx.value, md.value
        if crit is None and rtype == GESDT and nb_frames > 0:
            crit = gesd_critical_values(nb_frames, sig[0], sig[1])
        self.crit = np.ascontiguousarray(crit if crit is not None else np.zeros(1), np.float32)
        self.p.crit = _fptr(self.crit)


def stack_column(col, rtype, sig=(3.0, 3.0), method=0, weights=None, crit=None):
    """mean_and_reject (method 0) or quickmedian_float (method 1) on one column.
    Returns (double result, rej_lo, rej_hi)."""
    col = np.ascontiguousarray(col, np.float32)
    P = Params(rtype, sig, len(col), crit)
    rej = (C.c_int * 2)()
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    r = lib().or_stack_column_f(_fptr(col), len(col), method, C.byref(P.p), _dptr(w), rej, None)
    return r, rej[0], rej[1]


def stack_rows(frames, rtype=WINSORIZED, sig=(3.0, 3.0), method=0, norm=NO_NORM, scale=None,
               offset=None, mul=None, shift_dx=None, shift_scale=1.0, weights=None,
               output_norm=False, nthreads=0, crit=None, drizz=None, mask=None):
    """Block driver: frames is a (N, rows, W) float32 array (frame-major).
    drizz / mask: per-sample drizzle weights / feather-mask planes of the same
    shape (args->drizzle, masking), or None.
    Returns (out[rows, W] float32, rej_lo, rej_hi uint16, counts[2])."""
    frames = np.ascontiguousarray(frames, np.float32)
    planes = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (drizz, mask)]
    n, rows, W = frames.shape
    P = Params(rtype, sig, n, crit)
    out = np.empty((rows, W), np.float32)
    rl = np.zeros((rows, W), np.uint16)
    rh = np.zeros((rows, W), np.uint16)
    counts = np.zeros(2, np.uint64)
    arr = lambda a: None if a is None else np.ascontiguousarray(a, np.float64)
    scale, offset, mul, shift_dx, weights = map(arr, (scale, offset, mul, shift_dx, weights))
    lib().or_stack_rows_planes_f(
        _fptr(frames), _fptr(planes[0]), _fptr(planes[1]), n, W, rows, rows * W, method, C.byref(P.p), norm,
        _dptr(scale),
        _dptr(offset), _dptr(mul), _dptr(shift_dx), shift_scale, _dptr(weights),
        int(bool(output_norm)), _fptr(out), rl.ctypes.data_as(C.POINTER(C.c_uint16)),
        rh.ctypes.data_as(C.POINTER(C.c_uint16)), counts.ctypes.data_as(C.POINTER(C.c_uint64)),
        nthreads)
    return out, rl, rh, counts


def norm_stats(frame, lite=False):
    """Per-frame normalization estimators of one DATA_FLOAT plane
    (statistics_internal_float STATS_NORM / STATS_LITENORM,
    algos/statistics_float.c:281-480).  Returns (status, median, mad,
    location, scale, ngood); status 1 where the reference returns NULL."""
    out = np.zeros(4, np.float64)
    ng = C.c_size_t(0)
    if np.asarray(frame).dtype == np.uint16:      # statistics_internal_ushort (statistics.c:231-449)
        a = np.ascontiguousarray(frame, np.uint16).ravel()
        st = lib().or_norm_stats_u16(a.ctypes.data_as(C.POINTER(C.c_uint16)), a.size, int(bool(lite)),
                                     _dptr(out), C.byref(ng))
    else:
        a = np.ascontiguousarray(frame, np.float32).ravel()
        st = lib().or_norm_stats_f(_fptr(a), a.size, int(bool(lite)), _dptr(out), C.byref(ng))
    return (int(st), float(out[0]), float(out[1]), float(out[2]), float(out[3]), int(ng.value))


def quickmedian(a):
    a = np.array(a, np.float32)
    return lib().or_quickmedian_f(_fptr(a), len(a))


def quickmedian_u16(a):
    """quickmedian (WORD), sorting.c:195-230 (sortnet_median below 9)."""
    a = np.array(a, np.uint16)
    return lib().or_quickmedian_u16(a.ctypes.data_as(C.POINTER(C.c_uint16)), len(a))


def histogram_median_u16(a):
    """histogram_median (WORD), sorting.c:577-642 (sortnet_median below 10)."""
    a = np.array(a, np.uint16)
    return lib().or_histogram_median_u16(a.ctypes.data_as(C.POINTER(C.c_uint16)), len(a))


def set_simd_lanes(lanes: int):
    """Summation order of the reference's `omp simd` reductions in later
    calls: 0 = sequential (default), 2 / 4 / 8 = the vectorised-reduction
    model of stack_ref.c (or_set_simd_lanes)."""
    lib().or_set_simd_lanes(int(lanes))


def stack_rows_u16(frames, rtype=WINSORIZED, sig=(3.0, 3.0), method=0, norm=NO_NORM, scale=None,
                   offset=None, mul=None, shift_dx=None, shift_scale=1.0, weights=None,
                   output_norm=False, use_32bit_output=True, nthreads=0, crit=None, drizz=None, mask=None,
                   bitpix8=False):
    """16-bit block driver (apply_rejection_ushort).  frames: (N, rows, W) uint16;
    drizz / mask: float32 weight planes of the same shape, or None; bitpix8:
    the samples come from BYTE_IMG files (normalize_to16bit with output_norm).
    Returns (out float32 or uint16, rej_lo, rej_hi, counts)."""
    frames = np.ascontiguousarray(frames, np.uint16)
    planes = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (drizz, mask)]
    n, rows, W = frames.shape
    P = Params(rtype, sig, n, crit)
    out_f = np.empty((rows, W), np.float32) if use_32bit_output else None
    out_u = None if use_32bit_output else np.empty((rows, W), np.uint16)
    rl = np.zeros((rows, W), np.uint16)
    rh = np.zeros((rows, W), np.uint16)
    counts = np.zeros(2, np.uint64)
    arr = lambda a: None if a is None else np.ascontiguousarray(a, np.float64)
    scale, offset, mul, shift_dx, weights = map(arr, (scale, offset, mul, shift_dx, weights))
    u16p = C.POINTER(C.c_uint16)
    lib().or_set_out16_mul(65535.0 / 255.0 if bitpix8 else 1.0)
    lib().or_stack_rows_u16_planes(
        frames.ctypes.data_as(u16p), _fptr(planes[0]), _fptr(planes[1]), n, W, rows, rows * W, method, C.byref(P.p), norm, _dptr(scale),
        _dptr(offset), _dptr(mul), _dptr(shift_dx), shift_scale, _dptr(weights),
        int(bool(output_norm)), None if out_f is None else _fptr(out_f),
        None if out_u is None else out_u.ctypes.data_as(u16p), rl.ctypes.data_as(u16p),
        rh.ctypes.data_as(u16p), counts.ctypes.data_as(C.POINTER(C.c_uint64)), nthreads)
    return (out_f if use_32bit_output else out_u), rl, rh, counts
