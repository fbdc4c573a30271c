"""Host-side mirror of Siril's stacking interface for the MI355X engine.

Names and argument meaning follow the reference:
  * `Rejection`, `Normalization`   -- core/settings.h:34-52
  * `StackingArgs`                 -- the fields of struct stacking_args
                                      (stacking/stacking.h:65-117) the
                                      per-pixel loop reads
  * `stack_mean_with_rejection`,
    `stack_median`                 -- stack_method entry points
                                      (stacking/median_and_mean.c:1103-1109)
  * `StackResult`                  -- args->result / rejmap_low / rejmap_high
                                      and the per-channel rejection totals
                                      (median_and_mean.c:1748-1773)
Return codes are Siril's ST_* values; errors raise `SgpuError` carrying them.

Frames are a frame-major float32 block `[nframes, rows, width]`: a numpy
array (host path, sgpu_stack_rows) or a torch tensor already on the GPU
(device path, sgpu_stack_rows_device, asynchronous on torch's current stream).
"""
from __future__ import annotations

import ctypes as C
import enum
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from ._lib import StackParams, check, lib

ST_OK, ST_GENERIC_ERROR, ST_SEQUENCE_ERROR, ST_CANCEL, ST_ALLOC_ERROR = 0, -1, -2, -9, -10


class Rejection(enum.IntEnum):            # core/settings.h:43-52
    NO_REJEC = 0
    PERCENTILE = 1
    SIGMA = 2
    MAD = 3
    SIGMEDIAN = 4
    WINSORIZED = 5
    LINEARFIT = 6
    GESDT = 7


class Normalization(enum.IntEnum):        # core/settings.h:34-40
    NO_NORM = 0
    ADDITIVE = 1
    MULTIPLICATIVE = 2
    ADDITIVE_SCALING = 3
    MULTIPLICATIVE_SCALING = 4


METHOD_MEAN, METHOD_MEDIAN = 0, 1


def round_to_int(x: float) -> int:
    """round_to_int, core/proto.h:208-213 (half away from zero, clamped)."""
    x = min(x, 2147483647 - 0.5)
    x = max(x, -2147483648 + 0.5)
    return int(x + (0.5 if x >= 0.0 else -0.5))


def shifts_from_registration(dx: Sequence[float], offset0: int = 0,
                             upscale_at_stacking: bool = False) -> np.ndarray:
    """Per-frame integer x shifts of median_and_mean.c:1615-1622:
    shiftx = round_to_int((dx - offset[0]) * scale), dx from translation_from_H."""
    scale = 2.0 if upscale_at_stacking else 1.0
    return np.array([round_to_int((d - offset0) * scale) for d in dx], np.int32)


def gesd_critical_values(nb_frames: int, sig0: float, alpha: float) -> np.ndarray:
    """GESD critical values, median_and_mean.c:1477-1484, in float as the
    reference (gsl_cdf_tdist_Pinv there, scipy.stats.t.ppf here)."""
    from scipy.stats import t as tdist
    # (int) floor(nb_frames * args->sig[0]): an int x float product, in float
    max_out = int(math.floor(np.float32(nb_frames) * np.float32(sig0)))
    out = np.zeros(max(max_out, 1), np.float32)
    size = nb_frames
    a = np.float32(alpha)
    for j in range(max_out):
        td = np.float32(tdist.ppf(np.float32(1.0 - a / np.float32(2 * size)), size - 2))
        num = np.float32(size - 1) * td
        den = np.float32(np.sqrt(np.float32(size))) * np.float32(np.sqrt(np.float32(size - 2) + td * td))
        out[j] = np.float32(num / den)
        size -= 1
    return out


@dataclass
class StackingArgs:
    """Per-pixel parameters of struct stacking_args (stacking.h:65-117)."""
    type_of_rejection: Rejection = Rejection.WINSORIZED
    sig: tuple = (3.0, 3.0)
    normalize: Normalization = Normalization.NO_NORM
    scale: Optional[np.ndarray] = None       # coeff.pscale[layer]
    offset: Optional[np.ndarray] = None      # coeff.poffset[layer]
    mul: Optional[np.ndarray] = None         # coeff.pmul[layer]
    shiftx: Optional[np.ndarray] = None      # per-frame integer x shifts
    weights: Optional[np.ndarray] = None     # weights[layer*N ...]
    critical_value: Optional[np.ndarray] = None
    output_norm: bool = False
    create_rejmaps: bool = True


@dataclass
class StackResult:
    result: np.ndarray                       # rows x width float32
    rejmap_low: Optional[np.ndarray] = None
    rejmap_high: Optional[np.ndarray] = None
    irej: tuple = (0, 0)                     # low / high rejection totals
    exact_pixels: int = 0                    # pixels resolved by the exact kernel
    retval: int = ST_OK


class _Keep:
    """Holds the ctypes arrays a StackParams points to."""

    def __init__(self):
        self.refs = []

    def d(self, a):
        if a is None:
            return None
        a = np.ascontiguousarray(a, np.float64)
        self.refs.append(a)
        return a.ctypes.data_as(C.POINTER(C.c_double))

    def f(self, a):
        if a is None:
            return None
        a = np.ascontiguousarray(a, np.float32)
        self.refs.append(a)
        return a.ctypes.data_as(C.POINTER(C.c_float))

    def i(self, a):
        if a is None:
            return None
        a = np.ascontiguousarray(a, np.int32)
        self.refs.append(a)
        return a.ctypes.data_as(C.POINTER(C.c_int))


def _params(args: StackingArgs, method: int, nframes: int, keep: _Keep) -> StackParams:
    p = StackParams()
    p.method = method
    p.type_of_rejection = int(args.type_of_rejection)
    p.sig[0], p.sig[1] = float(args.sig[0]), float(args.sig[1])
    p.normalize = int(args.normalize)
    p.scale = keep.d(args.scale)
    p.offset = keep.d(args.offset)
    p.mul = keep.d(args.mul)
    p.shiftx = keep.i(args.shiftx)
    p.weights = keep.d(args.weights)
    crit = args.critical_value
    if crit is None and method == METHOD_MEAN and args.type_of_rejection == Rejection.GESDT:
        crit = gesd_critical_values(nframes, args.sig[0], args.sig[1])
    p.critical_value = keep.f(crit)
    p.output_norm = int(bool(args.output_norm))
    return p


class Context:
    """One sgpu_context: a HIP device + stream + device workspace."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        check(L.sgpu_init(device, C.byref(h)), "sgpu_init")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().sgpu_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_exact_only(self, on):
        """True: every pixel through the sequential kernels; 2: through the
        one-wave-per-pixel kernel where it applies (float SIGMA, WINSORIZED,
        PERCENTILE and median columns of 33..1024 samples)."""
        check(lib().sgpu_set_exact_only(self.h, 2 if on == 2 else int(bool(on))), "sgpu_set_exact_only")

    def set_stream(self, stream_handle: int | None):
        """hipStream_t handle (torch's `cuda_stream`); 0 / None = the null stream."""
        check(lib().sgpu_set_stream(self.h, C.c_void_p(stream_handle or 0)), "sgpu_set_stream")

    def synchronize(self):
        check(lib().sgpu_synchronize(self.h), "sgpu_synchronize")

    def set_timing(self, on: bool):
        check(lib().sgpu_set_timing(self.h, int(on)), "sgpu_set_timing")

    def last_timing(self):
        """(main kernel ms, exact kernel ms) of the last stack call (HIP events)."""
        ms = (C.c_float * 2)()
        check(lib().sgpu_last_timing(self.h, ms), "sgpu_last_timing")
        return float(ms[0]), float(ms[1])

    def last_exact_pixels(self) -> int:
        return int(lib().sgpu_last_exact_pixels(self.h))

    def set_seq_readers(self, readers: int):
        """Host threads per block read of a sequence stack (0: OMP_NUM_THREADS, else 8)."""
        check(lib().sgpu_set_seq_readers(self.h, int(readers)), "sgpu_set_seq_readers")

    def release_seq_buffers(self):
        """Free the page-locked block / result buffers and the device block
        buffers a sequence stack keeps for the next one (sgpu_release_seq_buffers)."""
        check(lib().sgpu_release_seq_buffers(self.h), "sgpu_release_seq_buffers")

    def last_seq_stats(self) -> dict:
        """Measurements of the last sequence stack (sgpu_last_seq_stats)."""
        a = (C.c_double * 12)()
        check(lib().sgpu_last_seq_stats(self.h, a), "sgpu_last_seq_stats")
        return {"blocks": int(a[0]), "read_s": a[1], "h2d_ms": a[2], "h2d_bytes": a[3], "kernel_ms": a[4],
                "loop_s": a[5], "pinned": bool(a[6]), "readers": int(a[7]), "setup_s": a[8], "write_s": a[9],
                "call_s": a[10]}

    def last_order_sensitive(self, with_indices: bool = False):
        """Float NO_REJEC mean: pixels whose float mean the kernel could not
        prove independent of the summation order (sgpu_last_order_sensitive);
        with_indices: (count, launch-relative pixel indices)."""
        n = int(lib().sgpu_last_order_sensitive(self.h, None, 0))
        if n < 0:
            check(n, "sgpu_last_order_sensitive")
        if not with_indices:
            return n
        idx = np.zeros(max(n, 1), np.int32)
        check(min(0, int(lib().sgpu_last_order_sensitive(self.h, idx.ctypes.data_as(C.c_void_p), n))),
              "sgpu_last_order_sensitive")
        return n, np.sort(idx[:n])

    # ---- host buffers (sgpu_stack_rows / sgpu_stack_rows_u16) -------------
    def stack(self, frames: np.ndarray, args: StackingArgs, method: int = METHOD_MEAN,
              use_32bit_output: bool = True, drizzle: np.ndarray | None = None,
              mask: np.ndarray | None = None) -> StackResult:
        """frames: float32 (DATA_FLOAT) or uint16 (DATA_USHORT) [N, rows, W].
        16-bit input yields a float32 result when use_32bit_output, else uint16.
        drizzle / mask: per-sample drizzle weights (args->drizzle) / feather-mask
        weights (masking) of the block, float32 [N, rows, W] (DATA_FLOAT input;
        16-bit input takes them through stack_device)."""
        if np.asarray(frames).dtype == np.uint16:
            if drizzle is not None or mask is not None:
                raise ValueError("16-bit stacks take weight planes through stack_device")
            return self._stack_u16(frames, args, method, use_32bit_output)
        frames = np.ascontiguousarray(frames, np.float32)
        if frames.ndim != 3:
            raise ValueError("frames must be [nframes, rows, width]")
        n, rows, W = frames.shape
        planes = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (drizzle, mask)]
        for a in planes:
            if a is not None and a.shape != frames.shape:
                raise ValueError("weight planes must have the frames' shape")
        keep = _Keep()
        p = _params(args, method, n, keep)
        out = np.empty((rows, W), np.float32)
        want_maps = args.create_rejmaps and method == METHOD_MEAN
        rl = np.zeros((rows, W), np.uint16) if want_maps else None
        rh = np.zeros((rows, W), np.uint16) if want_maps else None
        counts = np.zeros(2, np.uint64)
        vp = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
        check(lib().sgpu_stack_rows_planes(self.h, vp(frames), vp(planes[0]), vp(planes[1]), n, W, rows, rows * W,
                                           C.byref(p), vp(out), vp(rl), vp(rh), vp(counts)), "sgpu_stack_rows")
        return StackResult(out, rl, rh, (int(counts[0]), int(counts[1])), self.last_exact_pixels())

    def _stack_u16(self, frames, args, method, use_32bit_output):
        frames = np.ascontiguousarray(frames, np.uint16)
        if frames.ndim != 3:
            raise ValueError("frames must be [nframes, rows, width]")
        n, rows, W = frames.shape
        keep = _Keep()
        p = _params(args, method, n, keep)
        out_f = np.empty((rows, W), np.float32) if use_32bit_output else None
        out_u = None if use_32bit_output else np.empty((rows, W), np.uint16)
        want_maps = args.create_rejmaps and method == METHOD_MEAN
        rl = np.zeros((rows, W), np.uint16) if want_maps else None
        rh = np.zeros((rows, W), np.uint16) if want_maps else None
        counts = np.zeros(2, np.uint64)
        vp = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
        check(lib().sgpu_stack_rows_u16(self.h, vp(frames), n, W, rows, rows * W, C.byref(p), vp(out_f),
                                        vp(out_u), vp(rl), vp(rh), vp(counts)), "sgpu_stack_rows_u16")
        res = out_f if use_32bit_output else out_u
        return StackResult(res, rl, rh, (int(counts[0]), int(counts[1])), self.last_exact_pixels())

    # ---- device tensors (sgpu_stack_rows_device) ------------------------
    def stack_device(self, frames, args: StackingArgs, method: int = METHOD_MEAN, out=None,
                     rej_lo=None, rej_hi=None, counts=None, stream=None, drizzle=None, mask=None):
        """frames: torch.cuda float32 tensor [N, rows, W] (contiguous rows), or
        a 16-bit one (int16 / uint16 storage holding DATA_USHORT samples: the
        sgpu_stack_rows_u16_device path, float output in [0,1] as with
        use_32bit_output).  Queues the stack on `stream` (default: torch's
        current stream) and returns (out, rej_lo, rej_hi, counts) device tensors."""
        import torch
        u16 = frames.dtype in (torch.int16, getattr(torch, "uint16", torch.int16))
        if (frames.dtype != torch.float32 and not u16) or not frames.is_cuda or frames.dim() != 3:
            raise ValueError("frames must be a float32 or 16-bit CUDA tensor [N, rows, W]")
        n, rows, W = frames.shape
        if frames.stride(2) != 1 or frames.stride(1) != W:
            raise ValueError("frames rows must be contiguous")
        dev = frames.device
        if out is None:
            out = torch.empty((rows, W), dtype=torch.float32, device=dev)
        if counts is None:
            counts = torch.zeros(2, dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        self.set_stream(s.cuda_stream)
        keep = _Keep()
        p = _params(args, method, n, keep)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        for a in (drizzle, mask):
            if a is not None and (a.dtype != torch.float32 or a.shape != frames.shape or a.stride() != frames.stride()):
                raise ValueError("weight planes must be float32 tensors laid out as the frames")
        if u16:
            check(lib().sgpu_stack_rows_u16_planes_device(self.h, ptr(frames), ptr(drizzle), ptr(mask), n, W, rows,
                                                          frames.stride(0), C.byref(p), ptr(out), None, ptr(rej_lo),
                                                          ptr(rej_hi), ptr(counts)), "sgpu_stack_rows_u16_device")
        else:
            check(lib().sgpu_stack_rows_planes_device(self.h, ptr(frames), ptr(drizzle), ptr(mask), n, W, rows,
                                                      frames.stride(0), C.byref(p), ptr(out), ptr(rej_lo),
                                                      ptr(rej_hi), ptr(counts)), "sgpu_stack_rows_device")
        return out, rej_lo, rej_hi, counts

    # ---- frame-sharded no-rejection mean (sgpu_mean_partial_device) -------
    def mean_partial_device(self, frames, args: StackingArgs, sum_=None, count=None, stream=None):
        """Accumulate into (sum_ f64 [rows, W], count int32 [rows, W]) the sums
        and counts of the present samples of `frames` ([n, rows, W] float32
        CUDA tensor, the shard's frames in order; args' per-frame arrays are
        the shard's).  The unweighted NO_REJEC mean only."""
        import torch
        if frames.dtype != torch.float32 or not frames.is_cuda or frames.dim() != 3:
            raise ValueError("frames must be a float32 CUDA tensor [N, rows, W]")
        n, rows, W = frames.shape
        if frames.stride(2) != 1 or frames.stride(1) != W:
            raise ValueError("frames rows must be contiguous")
        dev = frames.device
        if sum_ is None:
            sum_ = torch.zeros((rows, W), dtype=torch.float64, device=dev)
        if count is None:
            count = torch.zeros((rows, W), dtype=torch.int32, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        self.set_stream(s.cuda_stream)
        keep = _Keep()
        p = _params(args, METHOD_MEAN, n, keep)
        check(lib().sgpu_mean_partial_device(self.h, C.c_void_p(frames.data_ptr()), n, W, rows, frames.stride(0),
                                             C.byref(p), C.c_void_p(sum_.data_ptr()),
                                             C.c_void_p(count.data_ptr())), "sgpu_mean_partial_device")
        return sum_, count

    def mean_partial_guard_device(self, frames, args: StackingArgs, sum_=None, count=None, amin=None, amax=None,
                                  stream=None):
        """mean_partial_device that also folds min |x| / max |x| of the present
        samples into (amin, amax) float32 [rows, W] (the exactness guard of
        the partial sums, sgpu_mean_partial_guard_device)."""
        import torch
        if frames.dtype != torch.float32 or not frames.is_cuda or frames.dim() != 3:
            raise ValueError("frames must be a float32 CUDA tensor [N, rows, W]")
        n, rows, W = frames.shape
        if frames.stride(2) != 1 or frames.stride(1) != W:
            raise ValueError("frames rows must be contiguous")
        dev = frames.device
        sum_ = torch.zeros((rows, W), dtype=torch.float64, device=dev) if sum_ is None else sum_
        count = torch.zeros((rows, W), dtype=torch.int32, device=dev) if count is None else count
        amin = torch.full((rows, W), float("inf"), dtype=torch.float32, device=dev) if amin is None else amin
        amax = torch.zeros((rows, W), dtype=torch.float32, device=dev) if amax is None else amax
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        self.set_stream(s.cuda_stream)
        keep = _Keep()
        p = _params(args, METHOD_MEAN, n, keep)
        vp = lambda t: C.c_void_p(t.data_ptr())
        check(lib().sgpu_mean_partial_guard_device(self.h, vp(frames), n, W, rows, frames.stride(0), C.byref(p),
                                                   vp(sum_), vp(count), vp(amin), vp(amax)),
              "sgpu_mean_partial_guard_device")
        return sum_, count, amin, amax

    def mean_finish_guard_device(self, sum_, count, amin, amax, out=None, output_norm: bool = False, stream=None):
        """(out, flag): the mean as mean_finish_device, flag uint8 = 1 where the
        f64 sums are not provably exact in every summation order."""
        import torch
        out = torch.empty(sum_.shape, dtype=torch.float32, device=sum_.device) if out is None else out
        flag = torch.empty(sum_.shape, dtype=torch.uint8, device=sum_.device)
        s = stream if stream is not None else torch.cuda.current_stream(sum_.device)
        self.set_stream(s.cuda_stream)
        vp = lambda t: C.c_void_p(t.data_ptr())
        check(lib().sgpu_mean_finish_guard_device(self.h, vp(sum_), vp(count), vp(amin), vp(amax), sum_.numel(),
                                                  vp(out), int(bool(output_norm)), vp(flag)),
              "sgpu_mean_finish_guard_device")
        return out, flag

    def gather_columns_device(self, frames, args: StackingArgs, idx):
        """[n, k] float32: the shifted, normalized samples of the pixels idx
        (int64 CUDA tensor of flat indices) of frames [n, rows, W]."""
        import torch
        n, rows, W = frames.shape
        k = int(idx.numel())
        out = torch.empty((n, k), dtype=torch.float32, device=frames.device)
        self.set_stream(torch.cuda.current_stream(frames.device).cuda_stream)
        keep = _Keep()
        p = _params(args, METHOD_MEAN, n, keep)
        idx = idx.to(torch.int64).contiguous()
        check(lib().sgpu_gather_columns_device(self.h, C.c_void_p(frames.data_ptr()), n, W, rows, frames.stride(0),
                                               C.byref(p), C.c_void_p(idx.data_ptr()), k, C.c_void_p(out.data_ptr())),
              "sgpu_gather_columns_device")
        return out

    def mean_finish_device(self, sum_, count, out=None, output_norm: bool = False, stream=None):
        """out = sum/count of the present samples (0 where none), clamped to
        [0, 1] unless output_norm."""
        import torch
        if out is None:
            out = torch.empty(sum_.shape, dtype=torch.float32, device=sum_.device)
        s = stream if stream is not None else torch.cuda.current_stream(sum_.device)
        self.set_stream(s.cuda_stream)
        check(lib().sgpu_mean_finish_device(self.h, C.c_void_p(sum_.data_ptr()), C.c_void_p(count.data_ptr()),
                                            sum_.numel(), C.c_void_p(out.data_ptr()), int(bool(output_norm))),
              "sgpu_mean_finish_device")
        return out

    def norm_to_0_1_range_device(self, img, stream=None):
        """norm_to_0_1_range (median_and_mean.c:557-582) in place on a float32
        CUDA tensor (all layers together): the post-pass of a 32-bit stack
        with args->output_norm (:1774-1775)."""
        import torch
        if img.dtype != torch.float32 or not img.is_cuda or not img.is_contiguous():
            raise ValueError("img must be a contiguous float32 CUDA tensor")
        s = stream if stream is not None else torch.cuda.current_stream(img.device)
        self.set_stream(s.cuda_stream)
        check(lib().sgpu_norm_to_0_1_range_device(self.h, C.c_void_p(img.data_ptr()), img.numel()),
              "sgpu_norm_to_0_1_range_device")
        return img


class MultiContext:
    """sgpu_multi: contexts on several devices of one node (devices may
    repeat).  `stack` splits the rows of a host block into balanced bands, one
    per device, stacks them concurrently and gathers them on the host
    (sgpu_multi_stack_rows[_u16]); results equal Context.stack's."""

    def __init__(self, devices):
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(lib().sgpu_multi_init(devs, len(devices), C.byref(h)), "sgpu_multi_init")
        self.h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "h", None):
            lib().sgpu_multi_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stack(self, frames: np.ndarray, args: StackingArgs, method: int = METHOD_MEAN,
              use_32bit_output: bool = True) -> StackResult:
        u16 = np.asarray(frames).dtype == np.uint16
        frames = np.ascontiguousarray(frames, np.uint16 if u16 else np.float32)
        if frames.ndim != 3:
            raise ValueError("frames must be [nframes, rows, width]")
        n, rows, W = frames.shape
        keep = _Keep()
        p = _params(args, method, n, keep)
        want_maps = args.create_rejmaps and method == METHOD_MEAN
        rl = np.zeros((rows, W), np.uint16) if want_maps else None
        rh = np.zeros((rows, W), np.uint16) if want_maps else None
        counts = np.zeros(2, np.uint64)
        vp = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
        if u16:
            out_f = np.empty((rows, W), np.float32) if use_32bit_output else None
            out_u = None if use_32bit_output else np.empty((rows, W), np.uint16)
            check(lib().sgpu_multi_stack_rows_u16(self.h, vp(frames), n, W, rows, rows * W, C.byref(p),
                                                  vp(out_f), vp(out_u), vp(rl), vp(rh), vp(counts)),
                  "sgpu_multi_stack_rows_u16")
            out = out_f if use_32bit_output else out_u
        else:
            out = np.empty((rows, W), np.float32)
            check(lib().sgpu_multi_stack_rows(self.h, vp(frames), n, W, rows, rows * W, C.byref(p), vp(out),
                                              vp(rl), vp(rh), vp(counts)), "sgpu_multi_stack_rows")
        return StackResult(out, rl, rh, (int(counts[0]), int(counts[1])), -1)


def row_bands_c(rows: int, nparts: int):
    """sgpu_row_bands: [(y0, y1)] of the C-ABI's multi-device partition."""
    st = (C.c_long * (nparts + 1))()
    check(lib().sgpu_row_bands(rows, nparts, st), "sgpu_row_bands")
    return [(int(st[i]), int(st[i + 1])) for i in range(nparts)]


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def stack_mean_with_rejection(frames, args: StackingArgs, ctx: Optional[Context] = None) -> StackResult:
    """stack_mean_with_rejection (median_and_mean.c:1103-1105) on one block."""
    return (ctx or default_context()).stack(frames, args, METHOD_MEAN)


def stack_median(frames, args: Optional[StackingArgs] = None, ctx: Optional[Context] = None) -> StackResult:
    """stack_median (median_and_mean.c:1107-1109) on one block."""
    return (ctx or default_context()).stack(frames, args or StackingArgs(), METHOD_MEDIAN)
