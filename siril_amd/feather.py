"""Feathering masks of `stack ... -feather=<dist>`.

The producer is compute_masks (stacking/blending.c:131-224): per frame, the
distance to black of a 7x7-closed, 10x-downscaled 0/255 image of the
reference layer (cvDownscaleBlendMask, opencv/opencv.cpp:587-609), cached by
Siril as `<seq>_<n>.msk` FITS files.  The consumer is stack_read_block_data
(stacking/median_and_mean.c:483-525): per row block and frame, the block's
mask rows upscaled back (cvUpscaleBlendMask, opencv.cpp:611-616) and ramped
against the feather distance; the ramped values weight the samples of the
mean (n *= mstack[frame], :1060-1066), through the `mask` plane of
stacking.Context.stack / stack_device.

Here the masks stay in HBM (siril_amd/csrc/feather.hip); the headless
sequence engine (sequence.stack_seq with feather > 0) runs the whole pipeline.
The upscale of a frame's rows depends on the row blocks Siril's planner chose
(stack_compute_parallel_blocks, :295-356), restated by stack_blocks.
"""
import ctypes as C
from typing import List, Optional, Tuple

import numpy as np

from ._lib import check, lib


def stack_blocks(max_rows: int, height: int, channels: int, nb_threads: int) -> List[Tuple[int, int, int]]:
    """Siril's row blocks: [(channel, start_row, height)] in the reference's
    internal row order (row s is FITS row height - 1 - s)."""
    n = C.c_int(0)
    rc = lib().sgpu_stack_blocks(max_rows, height, channels, nb_threads, 0, None, None, None, C.byref(n), None)
    if n.value < 1:
        check(rc, "sgpu_stack_blocks")
    s = np.zeros(n.value, np.int64)
    h = np.zeros(n.value, np.int64)
    ch = np.zeros(n.value, np.int32)
    big = C.c_long(0)
    dp = lambda a: a.ctypes.data_as(C.c_void_p)
    check(lib().sgpu_stack_blocks(max_rows, height, channels, nb_threads, n.value, dp(s), dp(h), dp(ch), C.byref(n),
                                  C.byref(big)), "sgpu_stack_blocks")
    return [(int(ch[j]), int(s[j]), int(h[j])) for j in range(n.value)]


def mask_size(width: int, height: int) -> Tuple[int, int]:
    """(mask width, mask height) = ((int)(0.1 w), (int)(0.1 h))."""
    w, h = C.c_long(0), C.c_long(0)
    lib().sgpu_feather_mask_size(width, height, C.byref(w), C.byref(h))
    return w.value, h.value


def block_area(width: int, height: int, start_row: int, block_height: int, shifty: Optional[int] = None):
    """stack_read_block_data's area for one frame and block: (first block row
    written, area rows, first downscaled row, downscaled rows); shifty None =
    no registration data."""
    v = [C.c_int(0) for _ in range(4)]
    check(lib().sgpu_feather_block_area(width, height, start_row, block_height, int(shifty or 0),
                                        int(shifty is not None), *[C.byref(x) for x in v]), "sgpu_feather_block_area")
    return tuple(x.value for x in v)


def _ctx(t, ctx):
    import torch
    from .stacking import Context
    ctx = ctx or Context(t.device.index or 0)
    ctx.set_stream(torch.cuda.current_stream(t.device).cuda_stream)
    return ctx


def compute_masks(frames, ctx=None):
    """Downscaled distance masks [N, mh, mw] float32 of a CUDA tensor
    [N, H, W] of one layer, float32 or 16-bit WORD storage, FITS row order."""
    import torch
    if frames.dim() != 3 or not frames.is_cuda or not frames.is_contiguous():
        raise ValueError("frames must be a contiguous CUDA tensor [N, H, W]")
    n, h, w = frames.shape
    mw, mh = mask_size(w, h)
    out = torch.empty((n, mh, mw), dtype=torch.float32, device=frames.device)
    ctx = _ctx(frames, ctx)
    check(lib().sgpu_feather_masks_device(ctx.h, C.c_void_p(frames.data_ptr()), frames.element_size(), n, w, h, h * w,
                                          C.c_void_p(out.data_ptr())), "sgpu_feather_masks_device")
    return out


def block_planes(masks, width: int, height: int, start_row: int, block_height: int, feather: float,
                 shifty=None, placex=None, canvas_width: Optional[int] = None, fits_order: bool = True, ctx=None):
    """The ramped mask planes [N, block_height, canvas_width] of one block
    (data->mask of stack_read_block_data) from compute_masks' output."""
    import torch
    n = masks.shape[0]
    cw = canvas_width or width
    out = torch.empty((n, block_height, cw), dtype=torch.float32, device=masks.device)
    sy = None if shifty is None else np.ascontiguousarray(shifty, np.int32)
    px = None if placex is None else np.ascontiguousarray(placex, np.int32)
    ctx = _ctx(masks, ctx)
    dp = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    check(lib().sgpu_feather_block_device(ctx.h, C.c_void_p(masks.data_ptr()), n, width, height, start_row,
                                          block_height, dp(sy), dp(px), cw, float(feather), int(bool(fits_order)),
                                          C.c_void_p(out.data_ptr()), block_height * cw), "sgpu_feather_block_device")
    return out
