"""Host-side mirror of Siril's debayer entry points over the C-ABI.

  * `debayer_buffer_new_float`        -- algos/demosaicing_rtp.cpp:228-390
  * `debayer_buffer_new_ushort`       -- algos/demosaicing_rtp.cpp:74-224
  * `debayer_buffer_superpixel_float` -- algos/demosaicing_siril.c:806-820
  * `debayer`                          -- device (torch) variant

Enums as core/settings.h:54-80 (sensor_pattern, interpolation_method).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ._lib import check, lib

BAYER_FILTER_RGGB, BAYER_FILTER_BGGR, BAYER_FILTER_GBRG, BAYER_FILTER_GRBG = range(4)
(BAYER_BILINEAR, BAYER_VNG, BAYER_AHD, BAYER_AMAZE, BAYER_DCB, BAYER_HPHD, BAYER_IGV, BAYER_LMMSE, BAYER_RCD,
 XTRANS) = range(10)
PATTERNS = {"RGGB": 0, "BGGR": 1, "GBRG": 2, "GRBG": 3}


def _pattern(p) -> int:
    return PATTERNS[p.upper()] if isinstance(p, str) else int(p)


def debayer_buffer_new_float(buf: np.ndarray, interpolation: int = BAYER_RCD, pattern=BAYER_FILTER_RGGB
                             ) -> Optional[np.ndarray]:
    """(h, w) float32 CFA -> (3, h, w) planar RGB, or None (the reference's NULL)."""
    buf = np.ascontiguousarray(buf, np.float32)
    h, w = buf.shape
    wi, hi = C.c_int(w), C.c_int(h)
    ptr = lib().sgpu_debayer_buffer_new_float(buf.ctypes.data_as(C.c_void_p), C.byref(wi), C.byref(hi),
                                              int(interpolation), _pattern(pattern), None)
    if not ptr:
        return None
    try:
        return np.ctypeslib.as_array(ptr, shape=(3, h, w)).copy()
    finally:
        lib().sgpu_free(C.cast(ptr, C.c_void_p))


def debayer_buffer_new_ushort(buf: np.ndarray, interpolation: int = BAYER_RCD, pattern=BAYER_FILTER_RGGB,
                              bit_depth: int = 16) -> Optional[np.ndarray]:
    """(h, w) uint16 CFA (raw WORD samples) -> (3, h, w) planar uint16 RGB, or
    None (the reference's NULL); bit_depth 8 (BYTE_IMG) rounds to [0, 255]."""
    buf = np.ascontiguousarray(buf, np.uint16)
    h, w = buf.shape
    wi, hi = C.c_int(w), C.c_int(h)
    ptr = lib().sgpu_debayer_buffer_new_ushort(buf.ctypes.data_as(C.c_void_p), C.byref(wi), C.byref(hi),
                                               int(interpolation), _pattern(pattern), None, int(bit_depth))
    if not ptr:
        return None
    try:
        return np.ctypeslib.as_array(ptr, shape=(3, h, w)).copy()
    finally:
        lib().sgpu_free(C.cast(ptr, C.c_void_p))


def debayer_buffer_siril_ushort(buf: np.ndarray, interpolation: int = BAYER_BILINEAR, pattern=BAYER_FILTER_RGGB,
                               bit_depth: int = 16) -> Optional[np.ndarray]:
    """Siril's own bilinear decoder (bayer_Bilinear, algos/demosaicing_siril.c
    :203-288; the tree's only bilinear, librtprocess's bayerfast being
    absent): (h, w) uint16 CFA -> (3, h, w) planar uint16, or None."""
    buf = np.ascontiguousarray(buf, np.uint16)
    h, w = buf.shape
    wi, hi = C.c_int(w), C.c_int(h)
    ptr = lib().sgpu_debayer_buffer_siril_ushort(buf.ctypes.data_as(C.c_void_p), C.byref(wi), C.byref(hi),
                                                 int(interpolation), _pattern(pattern), int(bit_depth))
    if not ptr:
        return None
    try:
        return np.ctypeslib.as_array(ptr, shape=(3, h, w)).copy()
    finally:
        lib().sgpu_free(C.cast(ptr, C.c_void_p))


def debayer_buffer_superpixel_float(buf: np.ndarray, pattern=BAYER_FILTER_RGGB) -> Optional[np.ndarray]:
    """(h, w) float32 CFA -> (h/2 + h%2, w/2 + w%2, 3) interleaved RGB."""
    buf = np.ascontiguousarray(buf, np.float32)
    h, w = buf.shape
    wi, hi = C.c_int(w), C.c_int(h)
    ptr = lib().sgpu_debayer_buffer_superpixel_float(buf.ctypes.data_as(C.c_void_p), C.byref(wi), C.byref(hi),
                                                     _pattern(pattern))
    if not ptr:
        return None
    try:
        return np.ctypeslib.as_array(ptr, shape=(hi.value, wi.value, 3)).copy()
    finally:
        lib().sgpu_free(C.cast(ptr, C.c_void_p))


def debayer(frame, pattern=BAYER_FILTER_RGGB, interpolation: int = BAYER_RCD, out=None, ctx=None,
            bit_depth: int = 16):
    """Device path: (h, w) float32 torch.cuda tensor -> (3, h, w) float32
    tensor (debayer_buffer_new_float); an int16 / uint16 tensor holding WORD
    samples -> (3, h, w) tensor of the same dtype (debayer_buffer_new_ushort)."""
    import torch
    from .stacking import default_context
    ctx = ctx or default_context()
    u16 = frame.dtype in (torch.int16, getattr(torch, "uint16", torch.int16))
    if (frame.dtype != torch.float32 and not u16) or frame.dim() != 2 or not frame.is_contiguous():
        raise TypeError("frame must be a contiguous 2-D float32 or 16-bit tensor")
    h, w = frame.shape
    if out is None:
        out = torch.empty((3, h, w), dtype=frame.dtype, device=frame.device)
    ctx.set_stream(torch.cuda.current_stream(frame.device).cuda_stream)
    if u16:
        check(lib().sgpu_debayer_u16_device(ctx.h, C.c_void_p(frame.data_ptr()), w, h, int(interpolation),
                                            _pattern(pattern), int(bit_depth), C.c_void_p(out.data_ptr())),
              "sgpu_debayer_u16_device")
        return out
    check(lib().sgpu_debayer_device(ctx.h, C.c_void_p(frame.data_ptr()), w, h, int(interpolation),
                                    _pattern(pattern), C.c_void_p(out.data_ptr())), "sgpu_debayer_device")
    return out


# ---- CFA helpers (extract_CFA_buffer_float, split_cfa, merge_cfa) ---------
def cfa_count(width: int, height: int, pattern, layer: int) -> int:
    from .registration import _cfa_args
    pat, dim = _cfa_args(pattern)
    return int(lib().sgpu_cfa_count(width, height, pat.ctypes.data_as(C.c_void_p), dim, layer))


def extract_cfa(frame, pattern, layer: int, ctx=None):
    """extract_CFA_buffer_float / _ushort (algos/demosaicing.c:936-975) of a
    CUDA image [H, W]: the samples of colour `layer` (0 R, 1 G, 2 B) of the
    compiled pattern (a 4- or 36-letter string or array), in raster order."""
    import torch
    from .registration import _cfa_args
    from .stacking import Context
    ctx = ctx or Context(frame.device.index or 0)
    pat, dim = _cfa_args(pattern)
    h, w = frame.shape
    n = cfa_count(w, h, pat, layer)
    out = torch.empty(max(n, 1), dtype=frame.dtype, device=frame.device)
    ctx.set_stream(torch.cuda.current_stream(frame.device).cuda_stream)
    ns = C.c_long()
    check(lib().sgpu_extract_cfa_device(ctx.h, C.c_void_p(frame.data_ptr()), frame.element_size(), w, h,
                                        pat.ctypes.data_as(C.c_void_p), dim, layer, C.c_void_p(out.data_ptr()),
                                        C.byref(ns)), "sgpu_extract_cfa_device")
    return out[:n]


def split_cfa(frame, ctx=None):
    """split_cfa_float / _ushort (algos/extraction.c:914-1050): the four
    (W/2) x (H/2) sub-planes of a CUDA image [H, W], as a [4, H/2, W/2] tensor."""
    import torch
    from .stacking import Context
    ctx = ctx or Context(frame.device.index or 0)
    h, w = frame.shape
    out = torch.empty((4, h // 2, w // 2), dtype=frame.dtype, device=frame.device)
    ctx.set_stream(torch.cuda.current_stream(frame.device).cuda_stream)
    p = [C.c_void_p(out[i].data_ptr()) for i in range(4)]
    check(lib().sgpu_split_cfa_device(ctx.h, C.c_void_p(frame.data_ptr()), frame.element_size(), w, h, *p),
          "sgpu_split_cfa_device")
    return out


def merge_cfa(planes, ctx=None):
    """merge_cfa (algos/demosaicing.c:757-840): [4, h, w] CUDA sub-planes ->
    the [2h, 2w] mosaic."""
    import torch
    from .stacking import Context
    ctx = ctx or Context(planes.device.index or 0)
    _, h, w = planes.shape
    planes = planes.contiguous()
    out = torch.empty((2 * h, 2 * w), dtype=planes.dtype, device=planes.device)
    ctx.set_stream(torch.cuda.current_stream(planes.device).cuda_stream)
    p = [C.c_void_p(planes[i].data_ptr()) for i in range(4)]
    check(lib().sgpu_merge_cfa_device(ctx.h, *p, planes.element_size(), w, h, C.c_void_p(out.data_ptr())),
          "sgpu_merge_cfa_device")
    return out
