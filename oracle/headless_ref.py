"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the host-side rules of
Siril's headless `stack` path that sit around the per-pixel stack: how float
FITS data is brought to [0, 1] when read, and the output normalization
post-pass.  Only tests/ import this module.

* norm_to_0_1_range: stacking/median_and_mean.c:557-582 (called at :1774-1775
  when args->use_32bit_output && args->output_norm).
* convert_floats: io/image_format_fits.c:648-672 (FLOAT_IMG falls through to
  the USHORT case: data[i] * INV_USHRT_MAX_SINGLE, float product).
* partial_read_rescale: internal_read_partial_fits, image_format_fits.c:994-1007.
* whole_read_rescale: read_fits_with_convert :906-910 with keywords.data_max
  as io/fits_keywords.c:1281-1288 sets it.
"""
from __future__ import annotations

import numpy as np

INV_USHRT_MAX_SINGLE = np.float32(0.000015259022)     # core/siril.h (1/65535 as float)
FLT_MAX = np.float32(3.40282347e+38)


def norm_to_0_1_range(img: np.ndarray) -> np.ndarray:
    a = np.asarray(img, np.float32).ravel()
    mini, maxi = FLT_MAX, np.float32(-1.0) * FLT_MAX
    for t in a[1:]:                      # the reference's loop starts at i = 1
        if t == 0.0:
            continue
        if t < mini:
            mini = t
        if t > maxi:
            maxi = t
    out = np.where(a == 0.0, np.float32(0.0), (a - mini) / np.float32(maxi - mini)).astype(np.float32)
    return out.reshape(np.shape(img))


def norm_to_0_1_range_fast(img: np.ndarray) -> np.ndarray:
    """Vectorised form of norm_to_0_1_range (min/max are order-independent)."""
    a = np.asarray(img, np.float32).ravel()
    tail = a[1:]
    nz = tail[(tail != 0.0) & ~np.isnan(tail)]
    mini = min(FLT_MAX, nz.min()) if nz.size else FLT_MAX
    maxi = max(np.float32(-1.0) * FLT_MAX, nz.max()) if nz.size else np.float32(-1.0) * FLT_MAX
    with np.errstate(divide="ignore", invalid="ignore"):
        out = np.where(a == 0.0, np.float32(0.0), (a - np.float32(mini)) / np.float32(maxi - mini))
    return out.astype(np.float32).reshape(np.shape(img))


def convert_floats(a: np.ndarray) -> np.ndarray:
    return (np.asarray(a, np.float32) * INV_USHRT_MAX_SINGLE).astype(np.float32)


def partial_read_rescale(region: np.ndarray, datamax=None) -> np.ndarray:
    """Rows read by the block reader (inside the image): DATAMAX when the card
    exists, else max(0, dest[0], dest[n/3], ...) over the region; > 10 rescales."""
    flat = np.asarray(region, np.float32).ravel()
    n = flat.size
    if datamax is not None:
        dm = float(datamax)
    elif n > 3:
        dm = 0.0
        i = 0
        while i < n:
            dm = max(dm, float(flat[i]))
            i += n // 3
    else:
        return np.array(region, np.float32)
    return convert_floats(region) if dm > 10.0 else np.array(region, np.float32)


def whole_read_rescale(frame: np.ndarray, datamax=None, from_siril: bool = False) -> np.ndarray:
    """readfits of a whole float frame: data_max = the file's true max unless
    PROGRAM says Siril (then DATAMAX, default 0); > 10 rescales."""
    dm = float(np.max(frame)) if not from_siril else (float(datamax) if datamax is not None else 0.0)
    return convert_floats(frame) if dm > 10.0 else np.array(frame, np.float32)
