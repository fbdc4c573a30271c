"""TEST INFRASTRUCTURE ONLY -- numpy restatement of Siril's Richardson-Lucy
deconvolution (the checker of the GPU path):

  fft_richardson_lucy    filters/deconvolution/deconvolve.cpp:56-84
  naive_richardson_lucy  filters/deconvolution/deconvolve.cpp:86-114
  rl_deconvolve_fft      filters/deconvolution/deconvolve.hpp:78-178
  rl_deconvolve_naive    filters/deconvolution/deconvolve.hpp:181-261
  edgetaper              filters/deconvolution/edgetaper.hpp
  add/remove_padding     filters/deconvolution/utils.hpp:71-124
  process_in_slices      algos/img_t/image.hpp:353-492 (+ slice-size strategies)
  padcirc / flip / ifft  algos/img_t/image.hpp:1233-1293, 717-730, 1088-1114
  conv2 (naive)          algos/img_t/image.hpp:498-600

  TV / FH regularisers   deconvolve.hpp:104-126 (FFT path: the lazy
                         gradient/divergence expressions of
                         algos/img_t/image_expr.hpp:780-1020) and :199-222
                         (naive path: img_t::gradient* / divergence,
                         image.hpp:804-1060), weights applied at :140-156 and
                         :233-249; lambda as deconvolve.cpp:72,102 pass it
                         (2 / lambda, then reallambda = 1 / that)

FFTW3f is not available here; the FFT path is restated with numpy FFTs in
complex128 (default) or complex64, so parity with the reference is a
relative tolerance, not bitwise.  The regularisers are
evaluated in float32 as the reference does (on real(est) for the FFT path).
"""
from __future__ import annotations

import numpy as np

# FFT backend (numpy's pocketfft; bench.py's CPU baseline swaps in a
# multi-threaded one with the same interface)
FFT = np.fft

REG_TV_GRAD, REG_FH_GRAD, REG_NONE_GRAD, REG_TV_MULT, REG_FH_MULT, REG_NONE_MULT = range(6)
GOOD_SIZES = [256, 320, 384, 400, 512, 640, 768, 800, 1024, 1280, 1536, 1600, 1920, 2048, 2560, 3072,
              3200, 3840, 4096, 5120, 6144, 6400, 7680, 8192]
AMPLE_MEMORY = 1 << 40


# ------------------------------------------------------------ slice geometry
def _slice_mem(w, h, K, N):
    return N * (w + 2 * K) * (h + 2 * K) * 4


def _smallest(W, H, M, K, N):
    w, h = W, H
    while _slice_mem(w, h, K, N) > M:
        if w > h:
            w = (w + 1) // 2
        else:
            h = (h + 1) // 2
    return w, h


def _fastest(W, H, M, K, N):
    best, area = (0, 0), 0
    for w in GOOD_SIZES:
        for h in GOOD_SIZES:
            if _slice_mem(w, h, K, N) <= M and w * h > area:
                best, area = (w, h), w * h
    return best if best[0] else _smallest(W, H, M, K, N)


def _next_good(s):
    for g in GOOD_SIZES:
        if g >= s:
            return g
    return GOOD_SIZES[-1]


def best_compromise(W, H, M, K, N, max_slice_size=32769):
    """image.hpp:353-401"""
    sm = _smallest(W, H, M, K, N)
    fa = _fastest(W, H, M, K, N)
    if fa[0] * fa[1] < 0.8 * sm[0] * sm[1]:
        best, best_score = sm, 0.0
        for w in GOOD_SIZES:
            for h in GOOD_SIZES:
                if _slice_mem(w, h, K, N) <= M:
                    score = min(w * h / (sm[0] * sm[1]), 1.0)
                    if score > best_score:
                        best, best_score = (w, h), score
    else:
        best = fa
    bw, bh = best
    if 511 < max_slice_size < 32769:
        bw, bh = min(bw, max_slice_size), min(bh, max_slice_size)
    if bw <= W and bh <= H:
        return bw, bh
    nw, nh = _next_good(W), _next_good(H)
    bw = nw if np.float32(nw) / np.float32(W) < np.float32(1.1) else W
    bh = nh if np.float32(nh) / np.float32(H) < np.float32(1.1) else H
    return bw, bh


def slices(W, H, M, overlap, N):
    """process_in_slices (image.hpp:404-492): list of
    (start_x, start_y, actual_w, actual_h, pad_left, pad_right, pad_top, pad_bottom)."""
    sw, sh = best_compromise(W, H, M, overlap, N)
    sw, sh = sw - 2 * overlap, sh - 2 * overlap
    out = []
    for sy in range((H + sh - 1) // sh):
        for sx in range((W + sw - 1) // sw):
            x0, y0 = sx * sw, sy * sh
            x1, y1 = min(x0 + sw, W), min(y0 + sh, H)
            out.append((x0, y0, x1 - x0, y1 - y0, min(overlap, x0), min(overlap, W - x1),
                        min(overlap, y0), min(overlap, H - y1)))
    return out


def _reflect(p, size):
    p = np.where(p < 0, -p, p)
    return np.where(p >= size, 2 * size - p - 2, p)


def extract_slice(img, s):
    x0, y0, aw, ah, pl, pr, pt, pb = s
    H, W = img.shape
    ys = _reflect(np.arange(y0 - pt, y0 + ah + pb), H)
    xs = _reflect(np.arange(x0 - pl, x0 + aw + pr), W)
    return img[np.ix_(ys, xs)].copy()


# ----------------------------------------------------------------- helpers
def add_padding(f, hw, hh):
    """utils.hpp:71-112 (rows first, then columns, mirrored about the edge)."""
    H, W = f.shape
    g = np.zeros((H + 2 * hh, W + 2 * hw), f.dtype)
    g[hh:hh + H, hw:hw + W] = f
    Hp, Wp = g.shape
    for y in range(hh):
        g[y, :] = g[2 * hh - y, :]
        g[Hp - 1 - y, :] = g[Hp - 1 - 2 * hh + y, :]
    for x in range(hw):
        g[:, x] = g[:, 2 * hw - x]
        g[:, Wp - 1 - x] = g[:, Wp - 1 - 2 * hw + x]
    return g


def remove_padding(f, hw, hh):
    return f[hh:f.shape[0] - hh, hw:f.shape[1] - hw].copy()


def flip_inplace(K):
    """img_t::flip() (image.hpp:717-730): swaps (x,y) <-> (w-1-x, h-1-y) for
    x < w/2 only, so the middle column of an odd kernel is left as is."""
    K = K.copy()
    h, w = K.shape
    for y in range(h):
        for x in range(w // 2):
            K[y, x], K[h - 1 - y, w - 1 - x] = K[h - 1 - y, w - 1 - x], K[y, x]
    return K


def padcirc(K, H, W, dtype):
    """image.hpp:1233-1293: kernel centre at the origin, wrapped."""
    out = np.zeros((H, W), dtype)
    kh, kw = K.shape
    hh, ww = kh // 2, kw // 2
    for y in range(kh):
        for x in range(kw):
            out[(y - hh) % H, (x - ww) % W] = K[y, x]
    return out


def fsum(a):
    """img_t::sum: sequential float fold."""
    s = np.float32(0)
    for v in np.asarray(a, np.float32).ravel():
        s = np.float32(s + v)
    return s


def ifft2n(X):
    """img_t::ifft: divide by w*h before the (unnormalised) backward FFT."""
    H, W = X.shape
    return FFT.ifft2(X / np.float32(W * H)) * (W * H)


def edgetaper(img, K, iterations, cdt):
    """edgetaper.hpp: Tukey-like weights, blend with the FFT blur."""
    H, W = img.shape
    kh, kw = K.shape
    y = np.arange(H)
    x = np.arange(W)
    wy = np.ones(H)
    m = y < kh
    wy[m] = np.sin(y[m] * np.pi / (kh * 2 - 1)) ** 2
    m = (y > H - kh) & (y >= kh)          # else-if (edgetaper.hpp:46-50)
    wy[m] = np.sin((H - 1 - y[m]) * np.pi / (kh * 2 - 1)) ** 2
    wx = np.ones(W)
    m = x < kw
    wx[m] = np.sin(x[m] * np.pi / (kw * 2 - 1)) ** 2
    m = (x > W - kw) & (x >= kw)
    wx[m] = np.sin((W - 1 - x[m]) * np.pi / (kw * 2 - 1)) ** 2
    weights = (wy.astype(np.float32)[:, None] * wx.astype(np.float32)[None, :])
    kft = FFT.fft2(padcirc(K, H, W, cdt))
    out = img.astype(np.float32)
    w64 = weights.astype(np.float64)
    for _ in range(iterations):
        blurred = ifft2n(FFT.fft2(out.astype(cdt)) * kft).real
        # out = w * out (float) + (1. - w) * blurred (double), stored as float
        out = ((weights * out).astype(np.float64) + (1.0 - w64) * blurred).astype(np.float32)
    return out


F32 = np.float32


def _sanitize(a):
    """img_t::sanitize (image.hpp:1337-1346): NaN or 0 -> 1e-9."""
    a = a.copy()
    a[np.isnan(a) | (a == 0)] = F32(1e-9)
    return a


def reg_fft_tv(w):
    """w <- divergence(dx / mag, dy / mag), mag = hypot(dx, dy) + FLT_EPSILON
    (deconvolve.hpp:106-112) with the expression classes' edge rules,
    including the (0, h-1) corner's flat indices (image_expr.hpp:882-884)."""
    w = np.asarray(w, F32)
    H, W = w.shape
    dx = np.zeros_like(w)
    dx[:, :-1] = w[:, 1:] - w[:, :-1]
    dy = np.zeros_like(w)
    dy[:-1, :] = w[1:, :] - w[:-1, :]
    mag = (np.hypot(dx, dy) + np.finfo(F32).eps).astype(F32)
    gx, gy = (dx / mag).astype(F32), (dy / mag).astype(F32)
    fx, fy = gx.ravel(), gy.ravel()
    out = np.zeros_like(w)
    out[1:-1, 1:-1] = ((gx[1:-1, 1:-1] - gx[1:-1, :-2]) + gy[1:-1, 1:-1]) - gy[:-2, 1:-1]
    out[1:-1, 0] = (gx[1:-1, 0] + gy[1:-1, 0]) - gy[:-2, 0]                      # x == 0
    out[0, 1:-1] = (gx[0, 1:-1] - gx[0, :-2]) + gy[0, 1:-1]                      # y == 0
    out[1:-1, -1] = (-gx[1:-1, W - 2] + gy[1:-1, -1]) - gy[:-2, -1]              # x == w-1
    out[-1, 1:-1] = (gx[-1, 1:-1] - gx[-1, :-2]) - gy[H - 2, 1:-1]               # y == h-1
    out[0, 0] = fx[0] + fy[0]
    out[0, W - 1] = -fx[W - 2] + fy[W - 1]
    out[H - 1, 0] = fx[H - 1] - fy[H - 2]
    out[H - 1, W - 1] = -fx[W - 2 + W * (H - 1)] - fy[W - 1 + W * (H - 2)]
    return out.astype(F32)


def _fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(F32)


def reg_fft_fh(w):
    """sqrt(gxx^2 + gyy^2 + 2 gxy^2) (fma), sanitized (deconvolve.hpp:115-125;
    gradientxx / yy / xy expressions, image_expr.hpp:910-1020)."""
    w = np.asarray(w, F32)
    gxx = np.zeros_like(w)
    gxx[:, 1:-1] = (w[:, 2:] - F32(2) * w[:, 1:-1]) + w[:, :-2]
    gyy = np.zeros_like(w)
    gyy[1:-1, :] = (w[2:, :] - F32(2) * w[1:-1, :]) + w[:-2, :]
    gxy = np.zeros_like(w)
    gxy[:-1, :-1] = ((w[1:, 1:] - w[:-1, 1:]) - w[1:, :-1]) + w[:-1, :-1]
    sumsq = (gxx * gxx + gyy * gyy).astype(F32)
    return _sanitize(np.sqrt(_fma32(F32(2), gxy * gxy, sumsq)).astype(F32))


def reg_naive_tv(w):
    """img_t path (deconvolve.hpp:201-211): sanitized forward differences,
    normalised by their hypot, then img_t::divergence (image.hpp:992-1060)."""
    w = np.asarray(w, F32)
    gx = np.zeros_like(w)
    gx[:, :-1] = w[:, 1:] - w[:, :-1]
    gx = _sanitize(gx)
    gy = np.zeros_like(w)
    gy[:-1, :] = w[1:, :] - w[:-1, :]
    gy = _sanitize(gy)
    m = np.hypot(gx, gy).astype(F32)
    gx, gy = (gx / m).astype(F32), (gy / m).astype(F32)
    out = np.zeros_like(w)
    out[1:-1, 1:-1] = ((gx[1:-1, 1:-1] - gx[1:-1, :-2]) + gy[1:-1, 1:-1]) - gy[:-2, 1:-1]
    out[0, 0] = gx[0, 0] + gy[0, 0]
    out[0, -1] = -gx[0, -2] + gy[0, -1]
    out[-1, 0] = gx[-1, 0] - gy[-2, 0]
    out[-1, -1] = -gx[-1, -2] - gy[-2, -1]
    out[1:-1, 0] = (gx[1:-1, 0] + gy[1:-1, 0]) - gy[:-2, 0]
    out[0, 1:-1] = (gx[0, 1:-1] - gx[0, :-2]) + gy[0, 1:-1]
    out[1:-1, -1] = (-gx[1:-1, -2] + gy[1:-1, -1]) - gy[:-2, -1]
    out[-1, 1:-1] = (gx[-1, 1:-1] - gx[-1, :-2]) - gy[-2, 1:-1]
    return out.astype(F32)


def reg_naive_fh(w):
    """(deconvolve.hpp:212-222) with img_t::gradientxx / yy / xy: returns
    (weight, gxy); max(1e-9, g) before squaring, pow(sum, 0.5)."""
    w = np.asarray(w, F32)
    gxx = np.zeros_like(w)
    gxx[:, 1:-1] = (w[:, 2:] + w[:, :-2]) - F32(2) * w[:, 1:-1]
    gyy = np.zeros_like(w)
    gyy[1:-1, :] = (w[2:, :] + w[:-2, :]) - F32(2) * w[1:-1, :]
    gxy = np.zeros_like(w)
    gxy[:-1, :-1] = ((w[1:, 1:] - w[:-1, 1:]) - w[1:, :-1]) + w[:-1, :-1]
    xx = np.maximum(F32(1e-9), gxx) ** 2
    xy2 = F32(2) * np.maximum(F32(1e-9), gxy) ** 2
    yy = np.maximum(F32(1e-9), gyy) ** 2
    s = (xx + (xy2 + yy)).astype(F32)
    return np.sqrt(s).astype(F32), gxy


def real_lambda(lam):
    """reallambda of rl_deconvolve_* for the entry points' lambda:
    deconvolve.cpp passes 2.f / lambda, deconvolve.hpp:100,194 take 1.f / that."""
    return F32(1.0) / (F32(2.0) / F32(lam))


def rl_fft_slice(f, K, maxiter, regtype, stepsize, cdt, stop_active=False, stopcrit=0.0, lam=1.0 / 3000):
    """rl_deconvolve_fft (deconvolve.hpp:78-178).  Returns (x, K_after):
    K is flipped in place (as the reference does) and stays flipped."""
    H, W = f.shape
    s = fsum(K)
    k_otf = FFT.fft2(padcirc(K, H, W, cdt) * (np.float32(1.0) / s))
    K = flip_inplace(K)
    s = fsum(K)
    kflip_otf = FFT.fft2(padcirc(K, H, W, cdt) * (np.float32(1.0) / s))
    est = f.astype(cdt)
    fc = f.astype(cdt)
    dt = stepsize
    rl = real_lambda(lam)
    for _ in range(maxiter):
        if regtype in (REG_TV_GRAD, REG_TV_MULT):
            w = reg_fft_tv(est.real.astype(F32))
        elif regtype in (REG_FH_GRAD, REG_FH_MULT):
            w = reg_fft_fh(est.real.astype(F32))
        ratio = ifft2n(FFT.fft2(est) * k_otf)
        bad = np.isnan(ratio) | (ratio == 0)
        ratio[bad] = 1e-9
        ratio = fc / ratio
        ratio = ifft2n(FFT.fft2(ratio) * kflip_otf)
        prev = est.real.copy()
        if regtype == REG_NONE_MULT:
            est = ratio * est
        elif regtype == REG_NONE_GRAD:
            est = est + dt * (-1.0 + ratio)
        elif regtype in (REG_TV_MULT, REG_FH_MULT):
            est = ratio * est * (F32(1) / (F32(1) - rl * w))
        else:
            est = est + dt * ((F32(-1) + rl * w) + ratio)
        if stop_active:
            meas = np.abs(est.real - prev) / np.abs(prev)
            if meas.sum() / meas.size < stopcrit:
                break
    return est.real, K


def fft_richardson_lucy(fdata, kernel, maxiter=50, regtype=REG_NONE_MULT, stepsize=0.0003,
                        mem=AMPLE_MEMORY, cdt=np.complex128, stop_active=False, stopcrit=0.002, lam=1.0 / 3000):
    """fdata: (nchans, ry, rx) float32; kernel: (kchans, ks, ks).  Returns a new array."""
    fdata = np.array(fdata, np.float32)
    nch = fdata.shape[0]
    ks = kernel.shape[-1]
    ncopies = 12 if regtype in (0, 3) else 10
    for c in range(nch):
        K = np.array(kernel[c if c < kernel.shape[0] else 0], np.float32)
        K = (K / fsum(K)).astype(np.float32)
        f = fdata[c].copy()
        mx = np.float32(f.max())
        if mx == 0:
            return None
        if mx != 1:
            f = (f / mx).astype(np.float32)
        fp = add_padding(f, ks // 2, ks // 2)
        u = np.zeros_like(fp, dtype=np.float64)
        for s in slices(fp.shape[1], fp.shape[0], mem, ks // 2, ncopies):
            sl = extract_slice(fp, s)
            sl = edgetaper(sl, K, 3, cdt).astype(np.float32)
            x, K = rl_fft_slice(sl, K, maxiter, regtype, stepsize, cdt, stop_active, stopcrit, lam)
            x0, y0, aw, ah, pl, pr, pt, pb = s
            u[y0:y0 + ah, x0:x0 + aw] = x[pt:pt + ah, pl:pl + aw]
        u = remove_padding(u, ks // 2, ks // 2)
        if mx != 1:
            u = u * mx
        fdata[c] = u.astype(np.float32)
    return fdata


def conv2_zero(x, k):
    """img_t::conv2 (image.hpp:498-600): correlation with zero borders."""
    H, W = x.shape
    ix = (k.shape[0] - 1) // 2
    xp = np.zeros((H + 2 * ix, W + 2 * ix), np.float64)
    xp[ix:ix + H, ix:ix + W] = x
    out = np.zeros((H, W), np.float64)
    for n in range(-ix, ix + 1):          # y offset
        for m in range(-ix, ix + 1):      # x offset
            out += xp[ix + n:ix + n + H, ix + m:ix + m + W] * float(k[n + ix, m + ix])
    return out


def rl_naive_slice(f, K, maxiter, regtype, stepsize, lam=1.0 / 3000, stop_active=False, stopcrit=0.0):
    """rl_deconvolve_naive (deconvolve.hpp:181-261).  The stop measure reads
    gxy (:250-251), written only by the FH regulariser: with TV or none it is
    a division by the zero-initialised image and never fires."""
    Kf = K[::-1, ::-1].copy()                 # flip(o): full flip
    x = f.astype(np.float64)
    rl = real_lambda(lam)
    for _ in range(maxiter):
        gxy = None
        if regtype in (REG_TV_GRAD, REG_TV_MULT):
            w = reg_naive_tv(x.astype(F32))
        elif regtype in (REG_FH_GRAD, REG_FH_MULT):
            w, gxy = reg_naive_fh(x.astype(F32))
        ratio = conv2_zero(x, K)
        # the caller passes the slice as both x and f (deconvolve.cpp:103), so
        # the numerator is the CURRENT estimate, not the observed slice
        ratio = x / ratio
        ratio = np.maximum(1e-9, ratio)
        ratio = conv2_zero(ratio, Kf)
        if regtype == REG_NONE_MULT:
            x = ratio * x
        elif regtype == REG_NONE_GRAD:
            x = x + stepsize * (-1.0 + ratio)
        elif regtype in (REG_TV_MULT, REG_FH_MULT):
            x = ratio * x * (F32(1) / (F32(1) - rl * w))
        else:
            x = x + stepsize * ((F32(-1) + rl * w) + ratio)
        if stop_active and gxy is not None:
            with np.errstate(divide="ignore", invalid="ignore"):
                meas = np.abs(x - gxy) / np.abs(gxy)
            if meas.sum() / meas.size < stopcrit:
                break
    return x


def naive_richardson_lucy(fdata, kernel, maxiter=10, regtype=REG_NONE_MULT, stepsize=0.0003,
                          mem=AMPLE_MEMORY, lam=1.0 / 3000, stop_active=False, stopcrit=0.002):
    fdata = np.array(fdata, np.float32)
    ks = kernel.shape[-1]
    for c in range(fdata.shape[0]):
        K = np.array(kernel[c if c < kernel.shape[0] else 0], np.float32)
        K = (K / fsum(K)).astype(np.float32)
        f = fdata[c].copy()
        mx = np.float32(f.max())
        if mx == 0:
            return None
        if mx != 1:
            f = (f / mx).astype(np.float32)
        fp = add_padding(f, 2 * ks, 2 * ks)
        u = np.zeros_like(fp, dtype=np.float64)
        for s in slices(fp.shape[1], fp.shape[0], mem, ks // 2, 7):
            sl = extract_slice(fp, s)
            sl = edgetaper(sl, K, 3, np.complex128).astype(np.float32)
            x = rl_naive_slice(sl, K, maxiter, regtype, stepsize, lam, stop_active, stopcrit)
            x0, y0, aw, ah, pl, pr, pt, pb = s
            u[y0:y0 + ah, x0:x0 + aw] = x[pt:pt + ah, pl:pl + aw]
        u = remove_padding(u, 2 * ks, 2 * ks)
        if mx != 1:
            u = u * mx
        fdata[c] = u.astype(np.float32)
    return fdata
