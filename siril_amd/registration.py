"""Host-side mirror of Siril's DFT registration entry (REG_DFT) over the
C-ABI.

  * `register_shift_dft`  -- registration/shift_methods.c:60-321: shifts of
                              every frame against the reference frame on a
                              square selection, as Siril computes them
  * `set_shifts` / `translation_from_H` / `H_from_translation`
                            -- io/sequence.c:1863-1868, registration.c:301-313
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import check, lib


def H_from_translation(dx: float, dy: float) -> np.ndarray:
    """registration.c:306-313: identity with h02 = dx, h12 = -dy."""
    H = np.eye(3)
    H[0, 2] = dx
    H[1, 2] = -dy
    return H


def translation_from_H(H) -> tuple:
    """registration.c:301-304: dx = h02, dy = -h12."""
    return float(H[0][2]), float(-H[1][2])


def set_shifts(shiftx: float, shifty: float, top_down: bool = False) -> np.ndarray:
    """io/sequence.c:1863-1868: H of a (shiftx, shifty) registration."""
    return H_from_translation(shiftx, -shifty if top_down else shifty)


# filter_pattern strings (algos/demosaicing.c:54-73) for the 2x2 Bayer cases
BAYER_PATTERNS = {"RGGB": 0, "BGGR": 1, "GBRG": 2, "GRBG": 3}


def compiled_pattern(pattern: str) -> np.ndarray:
    """get_compiled_pattern (algos/demosaicing.c:327-341) of a 2x2 Bayer
    string (or a 36-letter X-Trans string): R 0, G 1, B 2."""
    m = {"R": 0, "G": 1, "B": 2}
    if len(pattern) not in (4, 36):
        raise ValueError("CFA pattern must have 4 (Bayer) or 36 (X-Trans) letters")
    return np.array([m.get(ch, 3) for ch in pattern.upper()], np.uint8)


def _cfa_args(cfa):
    if cfa is None:
        return None, 0
    pat = compiled_pattern(cfa) if isinstance(cfa, str) else np.ascontiguousarray(cfa, np.uint8).ravel()
    dim = {4: 2, 36: 6}.get(pat.size)
    if dim is None:
        raise ValueError("CFA pattern must have 4 or 36 entries")
    return pat, dim


def _is16(t):
    import torch
    return t.dtype in (torch.int16, getattr(torch, "uint16", torch.int16))


def interpolate_nongreen(img, cfa, ctx=None):
    """interpolate_nongreen (io/image_format_fits.c:4389-4401) in place on a
    torch.cuda 2-D tensor: float32 -> interpolate_nongreen_float (:4319-4349),
    16-bit WORD storage -> interpolate_nongreen_ushort (:4351-4381)."""
    import torch
    from .stacking import default_context
    ctx = ctx or default_context()
    pat, dim = _cfa_args(cfa)
    u16 = _is16(img)
    if (img.dtype != torch.float32 and not u16) or img.dim() != 2 or img.stride(1) != 1:
        raise TypeError("img must be a 2-D float32 or 16-bit tensor with unit column stride")
    ctx.set_stream(torch.cuda.current_stream(img.device).cuda_stream)
    name = "sgpu_interpolate_nongreen_u16_device" if u16 else "sgpu_interpolate_nongreen_device"
    check(getattr(lib(), name)(ctx.h, C.c_void_p(img.data_ptr()), img.shape[1], img.shape[0], img.stride(0),
                               pat.ctypes.data_as(C.c_void_p), dim), name)
    return img


def dft_shifts(ref: np.ndarray, frames: Sequence[np.ndarray], ctx=None, cfa=None) -> np.ndarray:
    """(nframes, 2) int array of (shiftx, shifty), host selections (S x S).
    `cfa`: Bayer string / compiled pattern of a CFA (one-layer) sequence."""
    from .stacking import default_context
    ctx = ctx or default_context()
    u16 = np.asarray(ref).dtype == np.uint16          # DATA_USHORT selections
    dt = np.uint16 if u16 else np.float32
    ref = np.ascontiguousarray(ref, dt)
    S = ref.shape[0]
    if ref.shape != (S, S):
        raise ValueError("DFT registration needs a square selection (shift_methods.c:75)")
    fr = [np.ascontiguousarray(f, dt) for f in frames]
    for f in fr:
        if f.shape != (S, S):
            raise ValueError("all selections must be S x S")
    ptrs = (C.c_void_p * len(fr))(*[f.ctypes.data for f in fr])
    sx = np.zeros(len(fr), np.int32)
    sy = np.zeros(len(fr), np.int32)
    pat, dim = _cfa_args(cfa)
    name = "sgpu_dft_shifts_u16" if u16 else "sgpu_dft_shifts_cfa"
    check(getattr(lib(), name)(ctx.h, ref.ctypes.data_as(C.c_void_p), ptrs, len(fr), S,
                               pat.ctypes.data_as(C.c_void_p) if pat is not None else None, dim,
                               sx.ctypes.data_as(C.c_void_p), sy.ctypes.data_as(C.c_void_p)), name)
    return np.stack([sx, sy], 1)


def register_shift_dft(frames, ref_index: int, selection, ctx=None, peaks: bool = False, cfa=None):
    """Device path: frames is a torch.cuda tensor [N, H, W] (one layer; float32,
    or int16 / uint16 storage of DATA_USHORT WORD samples),
    selection = (x, y, w, h) with w == h.  Returns a (N, 2) int tensor of
    (shiftx, shifty); the reference frame gets (0, 0) like set_shifts(ref, 0, 0)
    (shift_methods.c:182)."""
    import torch
    from .stacking import default_context
    ctx = ctx or default_context()
    x, y, w, h = selection
    if w != h:
        raise ValueError("DFT registration needs a square selection (shift_methods.c:75)")
    n, H, W = frames.shape
    if x < 0 or y < 0 or x + w > W or y + h > H:
        raise ValueError("selection outside the frames")
    base = frames[:, y:y + h, x:x + w]
    shifts = torch.zeros((n, 2), dtype=torch.int32, device=frames.device)
    pk = torch.zeros(n, dtype=torch.float32, device=frames.device) if peaks else None
    ctx.set_stream(torch.cuda.current_stream(frames.device).cuda_stream)
    ref = base[ref_index]
    pat, dim = _cfa_args(cfa)
    # float32 frames, or 16-bit WORD storage (DATA_USHORT sequences)
    name = "sgpu_dft_register_u16_device" if _is16(frames) else "sgpu_dft_register_cfa_device"
    check(getattr(lib(), name)(ctx.h, C.c_void_p(ref.data_ptr()), W, C.c_void_p(base.data_ptr()), W,
                               frames.stride(0), n, w,
                               pat.ctypes.data_as(C.c_void_p) if pat is not None else None, dim,
                               C.c_void_p(shifts.data_ptr()), C.c_void_p(pk.data_ptr()) if peaks else None), name)
    shifts[ref_index] = 0
    return (shifts, pk) if peaks else shifts


def quality_estimate(frames, ctx=None) -> np.ndarray:
    """QualityEstimate (algos/quality.c:39-45) of every image of `frames`
    [N, h, w]: float32 -> QualityEstimate_float (algos/quality_float.c:41-147),
    uint16 (DATA_USHORT) -> QualityEstimate_ushort (algos/quality.c:49-276).
    numpy, or a torch.cuda tensor (float32, or int16 / uint16 storage of WORD
    samples) whose rows may be a window of larger frames.  Unnormalised
    qualities, f64."""
    from .stacking import default_context
    ctx = ctx or default_context()
    if isinstance(frames, np.ndarray):
        u16 = frames.dtype == np.uint16
        fr = np.ascontiguousarray(frames, np.uint16 if u16 else np.float32)
        n, h, w = fr.shape
        q = np.zeros(n, np.float64)
        name = "sgpu_quality_estimate_u16" if u16 else "sgpu_quality_estimate"
        check(getattr(lib(), name)(ctx.h, fr.ctypes.data_as(C.c_void_p), n, w, h,
                                   q.ctypes.data_as(C.c_void_p)), name)
        return q
    import torch
    n, h, w = frames.shape
    u16 = frames.dtype in (torch.int16, getattr(torch, "uint16", torch.int16))
    assert (frames.dtype == torch.float32 or u16) and frames.stride(2) == 1
    ctx.set_stream(torch.cuda.current_stream(frames.device).cuda_stream)
    q = np.zeros(n, np.float64)
    name = "sgpu_quality_estimate_u16_device" if u16 else "sgpu_quality_estimate_device"
    check(getattr(lib(), name)(ctx.h, C.c_void_p(frames.data_ptr()), n, w, h, frames.stride(1),
                               frames.stride(0), q.ctypes.data_as(C.c_void_p)), name)
    return q


def normalize_quality(quality, ref_index: int):
    """register_shift_dft's q_min / q_max / best-frame tracking (seeded with
    the reference frame, shift_methods.c:184,241-246) and normalizeQualityData
    (:36-54).  Returns (normalised qualities, best frame index)."""
    q = np.array(quality, np.float64)
    q_min = q_max = q[ref_index]
    q_index = ref_index
    for i, v in enumerate(q):
        if i == ref_index:
            continue
        if v > q_max:
            q_max, q_index = v, i
        q_min = q_min if q_min < v else v      # the C min() macro (NaN propagates like it)
    lib().sgpu_normalize_quality(q.ctypes.data_as(C.c_void_p), len(q), q_min, q_max)
    return q, q_index


def register_shift_dft_full(frames, ref_index: int, selection, ctx=None, cfa=None):
    """register_shift_dft (registration/shift_methods.c:60-321) with its
    per-frame outputs: integer shifts (as register_shift_dft above), the
    normalised quality of every frame (QualityEstimate on the selection --
    after interpolate_nongreen for CFA frames, as the reference reads them --
    then normalizeQualityData) and the best frame index.
    Returns (shifts [N, 2] int32 tensor, quality [N] f64, best index)."""
    import torch
    from .stacking import default_context
    ctx = ctx or default_context()
    shifts = register_shift_dft(frames, ref_index, selection, ctx=ctx, cfa=cfa)
    x, y, w, h = selection
    win = frames[:, y:y + h, x:x + w]
    if cfa is not None:
        # a private copy (seq_read_frame_part reads one): contiguous() would
        # alias the caller's frames when the window is the whole block
        win = win.clone(memory_format=torch.contiguous_format)
        for i in range(win.shape[0]):
            interpolate_nongreen(win[i], cfa, ctx)
    q, best = normalize_quality(quality_estimate(win, ctx), ref_index)
    return shifts, q, best


# ---- applying the registration (apply_reg, interpolation "none") ----------
def apply_reg_shifts(Hs, ref_index: int):
    """Integer shifts of apply_reg with interpolation none: H = Href^-1 * Himg
    (cvTransfH) then shift_fit_from_reg's round_to_int(dx), round_to_int(dy)
    (registration.c:322-370).  Hs: per-frame 3x3 homographies (translations).
    Returns (shiftx, shifty) int32 arrays."""
    Hs = np.asarray(Hs, np.float64)
    n = Hs.shape[0]
    h02 = np.ascontiguousarray(Hs[:, 0, 2])
    h12 = np.ascontiguousarray(Hs[:, 1, 2])
    sx = np.zeros(n, np.int32)
    sy = np.zeros(n, np.int32)
    dp = lambda a: a.ctypes.data_as(C.c_void_p)
    check(lib().sgpu_apply_reg_shifts(n, dp(h02), dp(h12), ref_index, dp(sx), dp(sy)), "sgpu_apply_reg_shifts")
    return sx, sy


def shift_frames(frames, shiftx, shifty, out=None, ctx=None):
    """shift_fit_from_reg on every frame of a CUDA tensor [N, H, W] (float32,
    or 16-bit WORD samples): out[f, y + sy, x + sx] = frames[f, y, x], zero
    elsewhere (rows in FITS / Siril memory order).  Returns `out`."""
    import torch
    from .stacking import Context
    ctx = ctx or Context(frames.device.index or 0)
    if frames.dim() != 3 or not frames.is_cuda or not frames.is_contiguous():
        raise ValueError("frames must be a contiguous CUDA tensor [N, H, W]")
    es = frames.element_size()
    n, h, w = frames.shape
    if out is None:
        out = torch.empty_like(frames)
    sx = np.ascontiguousarray(shiftx, np.int32)
    sy = np.ascontiguousarray(shifty, np.int32)
    ctx.set_stream(torch.cuda.current_stream(frames.device).cuda_stream)
    check(lib().sgpu_shift_frames_device(ctx.h, C.c_void_p(frames.data_ptr()), C.c_void_p(out.data_ptr()), es, n, w, h,
                                         h * w, sx.ctypes.data_as(C.c_void_p), sy.ctypes.data_as(C.c_void_p)),
          "sgpu_shift_frames_device")
    return out


# interpolation enum (core/siril.h:333-340)
OPENCV_NEAREST, OPENCV_LINEAR, OPENCV_CUBIC, OPENCV_AREA, OPENCV_LANCZOS4, OPENCV_NONE = range(6)


def apply_reg(frames, Hs, ref_index: int, interpolation: int = OPENCV_LANCZOS4, out=None, ctx=None):
    """apply_reg (registration/applyreg.c:388-660) of translation
    registrations (REG_DFT's) at scale 1, FRAMING_CURRENT, with any
    interpolation: frames [N, H, W] CUDA tensor (float32 or 16-bit WORD
    storage), Hs [N, 3, 3] homographies.  Integer translations are exact
    shifts under every OpenCV kernel (sgpu_apply_reg_device); sub-pixel ones
    are refused except with OPENCV_NONE (rounded, shift_fit_from_reg)."""
    import torch
    from .stacking import Context
    ctx = ctx or Context(frames.device.index or 0)
    if frames.dim() != 3 or not frames.is_cuda or not frames.is_contiguous():
        raise ValueError("frames must be a contiguous CUDA tensor [N, H, W]")
    n, h, w = frames.shape
    H = np.ascontiguousarray(np.asarray(Hs, np.float64).reshape(n, 9))
    out = torch.empty_like(frames) if out is None else out
    ctx.set_stream(torch.cuda.current_stream(frames.device).cuda_stream)
    check(lib().sgpu_apply_reg_device(ctx.h, C.c_void_p(frames.data_ptr()), C.c_void_p(out.data_ptr()),
                                      frames.element_size(), n, w, h, h * w, H.ctypes.data_as(C.c_void_p), ref_index,
                                      int(interpolation)), "sgpu_apply_reg_device")
    return out
