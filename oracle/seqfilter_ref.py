"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the frame selection
and frame weighting of Siril's headless `stack` command.  Only tests/ import
this module; the product computes the same in siril_amd/csrc/sgpu_seq.cpp.

* registration data per frame (regdata, core/siril.h): fwhm, weighted_fwhm,
  roundness, background_lvl as float, quality as double, number_of_stars as
  int -- the types the .seq reader scans them into (io/seqfile.c:403-420);
* the filter predicates and their parameters: core/sequence_filtering.c:45-121
  (seq_filter_*: note the background and star-count filters test roundness > 0),
  :219-302 (convert_parsed_filter_to_filter: literal or percent / k-sigma
  values), :305-355 (setup_filtered_data / stack_fill_list_of_unfiltered_images:
  at least two images, reference image replaced by the first selected one),
  :364-470 (generic_compute_accepted_value[_with_rejection]);
* weights: stacking/median_and_mean.c:1137-1230 (compute_wfwhm_weights,
  compute_nbstars_weights) and :85-159 (NBSTACK_WEIGHT from the frames'
  STACKCNT / NCOMBINE keyword, io/image_format_fits.c:1086-1095);
* equalizeRGB: stacking/normalization.c:150-185 (every layer's factors taken
  against the reference image's registration-layer estimators).

The k-sigma threshold calls GSL (gsl_stats_median_from_sorted_data,
gsl_stats_sd), which is not vendored: restated from GSL 2.x's published
algorithm (running means in long double, variance * n / (n - 1)); parity at
the last bit of that threshold is unpinned.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

DBL_MAX = np.finfo(np.float64).max
DBL_MIN = np.finfo(np.float64).tiny      # C's DBL_MIN: the smallest positive normal


@dataclass
class RegData:
    fwhm: float = 0.0
    wfwhm: float = 0.0
    roundness: float = 0.0
    quality: float = 0.0
    bkg: float = 0.0
    nstars: int = 0

    def __post_init__(self):
        f32 = lambda v: float(np.float32(v))
        self.fwhm, self.wfwhm, self.roundness, self.bkg = map(f32, (self.fwhm, self.wfwhm, self.roundness, self.bkg))
        self.quality = float(self.quality)
        self.nstars = int(self.nstars)


@dataclass
class FilterConfig:
    """struct seq_filter_config (core/sequence_filtering.h:36-40)."""
    f_fwhm: float = 0.0
    f_fwhm_p: float = 0.0
    f_fwhm_k: bool = False
    f_wfwhm: float = 0.0
    f_wfwhm_p: float = 0.0
    f_wfwhm_k: bool = False
    f_round: float = 0.0
    f_round_p: float = 0.0
    f_round_k: bool = False
    f_quality: float = 0.0
    f_quality_p: float = 0.0
    f_quality_k: bool = False
    f_bkg: float = 0.0
    f_bkg_p: float = 0.0
    f_bkg_k: bool = False
    f_nbstars: float = 0.0
    f_nbstars_p: float = 0.0
    f_nbstars_k: bool = False
    filter_included: bool = False


# regdata selectors (sequence_filtering.c:357-362) and filter predicates (:45-121)
SEL = {"fwhm": lambda r: r.fwhm, "wfwhm": lambda r: r.wfwhm, "round": lambda r: r.roundness,
       "quality": lambda r: r.quality, "bkg": lambda r: r.bkg, "nbstars": lambda r: float(r.nstars)}


def _pred(kind, r: RegData, p: float) -> bool:
    if kind == "fwhm":
        return r.fwhm > 0.0 and r.fwhm <= p
    if kind == "wfwhm":
        return r.wfwhm > 0.0 and r.wfwhm <= p
    if kind == "round":
        return r.roundness > 0.0 and r.roundness >= p
    if kind == "bkg":
        return r.roundness > 0.0 and r.bkg <= p           # (sic) roundness tested
    if kind == "nbstars":
        return r.roundness > 0.0 and r.nstars >= int(p)   # (sic)
    if kind == "quality":
        return r.quality > 0.0 and r.quality >= p
    raise ValueError(kind)


def accepted_value(reg: List[RegData], percent: float, lower_is_better: bool, kind: str) -> float:
    """generic_compute_accepted_value (sequence_filtering.c:366-404)."""
    extreme = DBL_MAX if lower_is_better else DBL_MIN
    val = sorted(extreme if SEL[kind](r) <= 0.0 else SEL[kind](r) for r in reg)
    n = len(val)
    if val[n - 1] != extreme:
        nwd = n
    else:
        nwd = next(i for i in range(n) if val[i] == extreme)
    images_number = float(nwd - 1)
    if lower_is_better:
        t = val[int(percent * images_number / 100.0)]
        return 0.0 if t == extreme else t
    return val[int((100.0 - percent) * images_number / 100.0)]


def _gsl_median_sorted(v):
    n = len(v)
    if n == 0:
        return 0.0
    lhs, rhs = (n - 1) // 2, n // 2
    return v[lhs] if lhs == rhs else (v[lhs] + v[rhs]) / 2.0


def _gsl_sd(v):
    n = len(v)
    mean = np.longdouble(0)
    for i, x in enumerate(v):
        mean += (np.longdouble(x) - mean) / (i + 1)
    mean = float(mean)                                   # gsl_stats_mean returns double
    var = np.longdouble(0)
    for i, x in enumerate(v):
        d = np.longdouble(x - mean)
        var += (d * d - var) / (i + 1)
    with np.errstate(divide="ignore", invalid="ignore"):   # n == 1: C's 0 * inf = NaN
        return float(np.sqrt(np.float64(var) * (np.float64(n) / np.float64(n - 1.0))))


def accepted_value_ksigma(reg: List[RegData], k: float, lower_is_better: bool, kind: str) -> float:
    """generic_compute_accepted_value_with_rejection (sequence_filtering.c:408-452)."""
    factor = 1.0 if lower_is_better else -1.0
    val = [SEL[kind](r) * factor for r in reg if SEL[kind](r) > 0.0]
    if not val:
        return 0.0
    val.sort()
    n = len(val)
    while True:
        m = _gsl_median_sorted(val[:n])
        s = _gsl_sd(val[:n])
        t = m + k * s
        j = 0
        for i in range(n, 0, -1):
            if val[i - 1] > t:
                j += 1
            else:
                break
        n -= j
        if j <= 0:
            break
    if n < 0:
        return 0.0
    return factor * val[n - 1]


_KINDS = [("fwhm", True), ("wfwhm", True), ("round", False), ("bkg", True), ("nbstars", False), ("quality", False)]


def build_filters(cfg: FilterConfig, reg: Optional[List[RegData]]):
    """convert_parsed_filter_to_filter (:219-302): list of (kind, param); None
    on the literal-and-percent conflict."""
    for k in ("fwhm", "wfwhm", "round", "quality"):
        if getattr(cfg, f"f_{k}_p") > 0 and getattr(cfg, f"f_{k}") > 0:
            return None
    out = []
    if cfg.filter_included:
        out.append(("included", 0.0))
    for kind, lower in _KINDS:
        lit, pct, isk = getattr(cfg, f"f_{kind}"), getattr(cfg, f"f_{kind}_p"), getattr(cfg, f"f_{kind}_k")
        if pct > 0 or lit > 0:
            if lit > 0:
                p = float(np.float32(lit))
            elif reg is None:
                p = 0.0
            elif isk:
                p = accepted_value_ksigma(reg, float(np.float32(pct)), lower, kind)
            else:
                p = accepted_value(reg, float(np.float32(pct)), lower, kind)
            out.append((kind, p))
    return out


def select_frames(cfg: FilterConfig, reg: Optional[List[RegData]], incl: List[bool], ref_image: int):
    """Frame indices the stack uses and its (possibly replaced) reference
    image; None when fewer than two frames pass (setup_filtered_data)."""
    flt = build_filters(cfg, reg)
    if flt is None:
        return None
    n = len(incl)
    keep = []
    for i in range(n):
        ok = True
        for kind, p in flt:
            if kind == "included":
                ok = ok and bool(incl[i])
            else:
                ok = ok and reg is not None and _pred(kind, reg[i], p)
        if ok:
            keep.append(i)
    if len(keep) < 2:
        return None
    if ref_image not in keep:
        ref_image = keep[0]
    return keep, ref_image


def wfwhm_weights(reg: List[RegData], idx: List[int]) -> np.ndarray:
    """compute_wfwhm_weights (median_and_mean.c:1137-1180), one layer."""
    fmin, fmax = DBL_MAX, -DBL_MAX
    for i in idx:
        w = reg[i].wfwhm
        if w < fmin and w > 0:
            fmin = w
        if w > fmax:
            fmax = w
    invdenom = 1. / (1. / (fmin * fmin) - 1. / (fmax * fmax))
    invfwhmax2 = 1. / (fmax * fmax)
    out = np.zeros(len(idx))
    norm = 0.0
    for k, i in enumerate(idx):
        w = reg[i].wfwhm
        if w > 0:
            out[k] = (1. / (w * w) - invfwhmax2) * invdenom
            norm += out[k]
    norm /= float(len(idx))
    if not norm:
        raise ValueError("wFWHM weights: null norm")
    return out / norm


def nbstars_weights(reg: List[RegData], idx: List[int]) -> np.ndarray:
    """compute_nbstars_weights (median_and_mean.c:1182-1230), one layer."""
    smin, smax = 2147483647, 0
    for i in idx:
        s = reg[i].nstars
        if s < smin:
            smin = s
        if s > smax:
            smax = s
    invdenom = 1.0 if smax == smin else 1. / float(smax - smin)
    out = np.zeros(len(idx))
    norm = 0.0
    for k, i in enumerate(idx):
        out[k] = 1. if smax == smin else float(reg[i].nstars - smin) * float(reg[i].nstars - smin) * invdenom * invdenom
        norm += out[k]
    norm /= float(len(idx))
    return out / norm


def equalized_factors(normalize: int, stats_by_layer, ref_index: int, reglayer: int):
    """compute_factors_from_estimators with equalizeRGB (normalization.c:150-185):
    stats_by_layer[l] = (offset, mul, scale) estimator arrays of layer l;
    returns per-layer (poffset, pmul, pscale)."""
    rl = reglayer if reglayer > -1 else 1
    off0 = [s[0][ref_index] for s in stats_by_layer]
    mul0 = [s[1][ref_index] for s in stats_by_layer]
    sc0 = [s[2][ref_index] for s in stats_by_layer]
    out = []
    for layer, (po, pm, ps) in enumerate(stats_by_layer):
        po, pm, ps = np.array(po, float), np.array(pm, float), np.array(ps, float)
        for i in range(len(po)):
            if normalize in (3, 1):                 # ADDITIVE_SCALING falls through to ADDITIVE
                if normalize == 3:
                    ps[i] = 1 if ps[i] == 0 else sc0[rl] / ps[i]
                po[i] = ps[i] * po[i] - off0[rl]
            elif normalize in (4, 2):
                if normalize == 4:
                    ps[i] = 1 if ps[i] == 0 else sc0[rl] / ps[i]
                pm[i] = 1 if pm[i] == 0 else mul0[rl] / pm[i]
        out.append((po, pm, ps))
    return out
