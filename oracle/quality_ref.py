"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the DFT registration's
frame quality, the parity checker for siril_amd/csrc/quality.hip.  Never
imported by the product.

QualityEstimate_float (algos/quality_float.c:41-147) with SubSample
(:153-164), _smooth_image_float (:222-250) and Gradient (:166-219);
normalizeQualityData (registration/shift_methods.c:36-54).  Float steps are
evaluated in float32 in the reference's order; the gradient's f64 sum is
sequential in row-major order (np.cumsum), as the reference loop is.
Parity unpinned beyond this restatement: no reference test covers it.
"""
import numpy as np

THRESHOLD_FLOAT = np.float32(0.156863)
QMARGIN = 0.1
QSUBSAMPLE_MIN, QSUBSAMPLE_MAX, QSUBSAMPLE_INC = 3, 5, 1


def _subsample(img, s, xs, ys):
    """SubSample at every grid point: rows then columns, float accumulation."""
    v = np.zeros((ys, xs), np.float32)
    for r in range(s):
        for c in range(s):
            v = (v + img[r:r + ys * s:s, c:c + xs * s:s][:ys, :xs]).astype(np.float32)
    return (v / np.float32(s * s)).astype(np.float32)


def _smooth(b):
    out = b.copy()
    if b.shape[0] < 3 or b.shape[1] < 3:
        return out
    p, c, n = b[:-2], b[1:-1], b[2:]
    f = np.float32
    v = (p[:, :-2] + p[:, 1:-1]).astype(f)
    v = (v + (p[:, 2:] + c[:, :-2]).astype(f)).astype(f)
    v = (v + (c[:, 1:-1] + c[:, 2:]).astype(f)).astype(f)
    v = (v + (n[:, :-2] + n[:, 1:-1]).astype(f)).astype(f)
    v = (v + n[:, 2:]).astype(f)
    out[1:-1, 1:-1] = (v * (np.float32(1.0) / np.float32(9.0))).astype(f)
    return out


def _gradient(b):
    h, w = b.shape
    yb = int(h * QMARGIN) + 1
    xb = int(w * QMARGIN) + 1
    region = np.zeros_like(b, bool)
    region[yb:h - yb, xb:w - xb] = True
    above = region & (b >= THRESHOLD_FLOAT)
    if not above.any():
        return -1.0
    m = np.zeros_like(b, bool)
    ys, xs = np.nonzero(above)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            m[ys + dy, xs + dx] = True
    m &= region
    if not m.any():
        return -1.0
    yy, xx = np.nonzero(m)                      # row-major order
    d1 = (b[yy, xx] - b[yy, xx + 1]).astype(np.float32).astype(np.float64)
    d2 = (b[yy, xx] - b[yy + 1, xx]).astype(np.float32).astype(np.float64)
    terms = d1 * d1 + d2 * d2
    val = float(np.cumsum(terms)[-1])
    return val / float(len(terms)) / 10.0


def quality_estimate_float(img):
    img = np.ascontiguousarray(img, np.float32)
    height, width = img.shape
    region_w, region_h = width - 1, height - 1
    dval = 0.0
    s = QSUBSAMPLE_MIN
    while s <= QSUBSAMPLE_MAX:
        xs, ys = region_w // s, region_h // s
        if xs < 2 or ys < 2:
            break
        buf = _smooth(_subsample(img, s, xs, ys))
        q = _gradient(buf)
        dval += q * (float(QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (s * s))
        while True:
            s += QSUBSAMPLE_INC
            if not (width // s == xs and height // s == ys):
                break
    return float(np.sqrt(dval)) if dval >= 0 else float("nan")


def normalize_quality(q, q_min, q_max):
    q = np.array(q, np.float64)
    diff = q_max - q_min
    if diff == 0:
        q_min = 0.0
        diff = 1.0 if q_max == 0.0 else q_max
    q = (q - q_min) / diff
    q[(q < 0) | np.isnan(q)] = -1.0
    return q


# ---------------------------------------------------------------- 16-bit
# QualityEstimate_ushort (algos/quality.c:49-175) with SubSample (:180-190),
# Gradient (:192-247) and _smooth_image_16 (:250-276): WORD subsample
# rounded with round_to_WORD, the MAXP histogram stretch over the interior
# rows (:97-146), integer 3x3 smoothing, THRESHOLD_USHRT.
THRESHOLD_USHRT = 10240
MAXP = 6


def _subsample16(img, s, xs, ys):
    v = np.zeros((ys, xs), np.int64)
    for r in range(s):
        for c in range(s):
            v += img[r:r + ys * s:s, c:c + xs * s:s][:ys, :xs].astype(np.int64)
    x = v.astype(np.float64) / float(s * s) + 0.5          # round_to_WORD
    return np.clip(x, 0.0, 65535.0).astype(np.uint16)


def _maxp_level(buf):
    """The reference's running top list over rows 1 .. ys-2 in scan order."""
    maxp = [0] * MAXP
    for v in buf[1:-1].ravel().tolist():
        if v > maxp[2] and v < 65530:
            slot = 0 if v > maxp[0] else (1 if v > maxp[1] else 2)
            for j in range(MAXP - 1, slot, -1):
                maxp[j] = maxp[j - 1]
            maxp[slot] = v
    return sum(maxp[MAXP // 2:]) // (MAXP - MAXP // 2)


def _stretch16(buf, mx):
    if mx <= 0:
        return buf.copy()
    mult = 60000.0 / float(mx)
    v = np.floor(buf.astype(np.float64) * mult)            # (unsigned int)(double)
    return np.minimum(v, 65535.0).astype(np.uint16)


def _smooth16(b):
    out = b.copy()
    if b.shape[0] < 3 or b.shape[1] < 3:
        return out
    s = np.zeros((b.shape[0] - 2, b.shape[1] - 2), np.int64)
    for dy in range(3):
        for dx in range(3):
            s += b[dy:dy + s.shape[0], dx:dx + s.shape[1]].astype(np.int64)
    out[1:-1, 1:-1] = (s // 9).astype(np.uint16)
    return out


def _gradient16(b):
    h, w = b.shape
    yb = int(h * QMARGIN) + 1
    xb = int(w * QMARGIN) + 1
    region = np.zeros_like(b, bool)
    region[yb:h - yb, xb:w - xb] = True
    above = region & (b >= THRESHOLD_USHRT)
    if not above.any():
        return -1.0
    m = np.zeros_like(b, bool)
    ys, xs = np.nonzero(above)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            m[ys + dy, xs + dx] = True
    m &= region
    if not m.any():
        return -1.0
    yy, xx = np.nonzero(m)
    bi = b.astype(np.int64)
    d1 = bi[yy, xx] - bi[yy, xx + 1]
    d2 = bi[yy, xx] - bi[yy + 1, xx]
    val = float(np.sum(d1 * d1 + d2 * d2))                 # exact integer sum
    return val / float(len(yy)) / 10.0


def quality_estimate_ushort(img):
    img = np.ascontiguousarray(img, np.uint16)
    height, width = img.shape
    region_w, region_h = width - 1, height - 1
    dval = 0.0
    s = QSUBSAMPLE_MIN
    while s <= QSUBSAMPLE_MAX:
        xs, ys = region_w // s, region_h // s
        if xs < 2 or ys < 2:
            break
        buf = _subsample16(img, s, xs, ys)
        buf = _smooth16(_stretch16(buf, _maxp_level(buf)))
        q = _gradient16(buf)
        dval += q * (float(QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (s * s))
        while True:
            s += QSUBSAMPLE_INC
            if not (width // s == xs and height // s == ys):
                break
    return float(np.sqrt(dval)) if dval >= 0 else float("nan")
