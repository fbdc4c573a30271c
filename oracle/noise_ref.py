"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the background-noise
estimator of Siril's image statistics (imstats bgnoise), the input of
-weight=noise (stacking/median_and_mean.c:1111-1135).  Only tests/ import it;
the product computes it in siril_amd/csrc/bgnoise.hip.

siril_fits_img_stats_float / _ushort (algos/quantize.c:139-205, 71-137) ->
FnNoise1_float (:1343-1488) / FnNoise1_ushort (:1202-1341): per row, the
first-order differences of consecutive valid pixels (float: != 0 and not
NaN, differences in float; 16-bit: != 0, differences in int), their mean /
RMS from double sums in array order (FnDiffMeanSigma_float / _int,
:327-422; np.cumsum keeps that sequential order), up to NITER = 3 rounds of
SIGMA_CLIP = 5 clipping (survivors keep their order); rows with fewer than
two differences are skipped; the median of the rows' RMS values x 0.70710678.
Float statistics are in the frame's own units (normValue 1,
statistics_float.c:389-400), 16-bit ones in ADU (statistics.c:325-341).
"""
from __future__ import annotations

import numpy as np

NITER = 3
SIGMA_CLIP = 5.0
f32 = np.float32


def _mean_sigma(d64: np.ndarray):
    """FnDiffMeanSigma_*: (mean, sigma) from sequential double sums."""
    n = d64.size
    if n == 0:
        return 0.0, 0.0
    s = float(np.cumsum(d64)[-1])
    if n == 1:
        return s, 0.0
    s2 = float(np.cumsum(d64 * d64)[-1])
    mean = s / n
    with np.errstate(invalid="ignore"):
        return mean, float(np.sqrt(s2 / n - mean * mean))


def _row_noise(row: np.ndarray, is_float: bool):
    if is_float:
        v = row[(row != 0) & ~np.isnan(row)].astype(f32)
        d = (v[:-1] - v[1:]).astype(f32)                    # differences in float
    else:
        v = row[row != 0].astype(np.int64)
        d = v[:-1] - v[1:]                                  # differences in int
    if d.size < 2:
        return None
    good = ~np.isnan(d) if is_float else np.ones(d.size, bool)
    mean, sd = _mean_sigma(d[good].astype(np.float64))
    if sd > 0.0:
        for _ in range(NITER):
            if is_float:
                keep = np.abs((d - f32(mean)).astype(f32)).astype(np.float64) < SIGMA_CLIP * sd
            else:
                keep = np.abs(d.astype(np.float64) - mean) < SIGMA_CLIP * sd
            if keep.all():
                break
            d = d[keep]
            good = ~np.isnan(d) if is_float else np.ones(d.size, bool)
            mean, sd = _mean_sigma(d[good].astype(np.float64))
    return sd


def bgnoise(frame: np.ndarray) -> float:
    """bgnoise of one plane (float32 or uint16)."""
    frame = np.asarray(frame)
    is_float = frame.dtype != np.uint16
    h, w = frame.shape
    if w < 3:
        return 0.0
    vals = [x for x in (_row_noise(frame[r], is_float) for r in range(h)) if x is not None]
    if not vals:
        return 0.0
    if len(vals) == 1:
        xn = vals[0]
    else:
        vals.sort()
        n = len(vals)
        xn = (vals[(n - 1) // 2] + vals[n // 2]) / 2.0
    return 0.70710678 * xn


def noise_weights(bgnoise_values, pscale) -> np.ndarray:
    """compute_noise_weights (median_and_mean.c:1111-1135), one layer:
    1 / (pscale^2 bgnoise^2), normalised to a mean of 1."""
    b = np.asarray(bgnoise_values, np.float64)
    s = np.asarray(pscale, np.float64)
    w = np.array([1.0 / (si * si * bi * bi) for si, bi in zip(s, b)])
    norm = 0.0
    for x in w:
        norm += x
    norm /= float(len(w))
    return w / norm
