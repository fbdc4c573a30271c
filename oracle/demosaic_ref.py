"""TEST INFRASTRUCTURE ONLY -- numpy restatement of Siril's float debayer
entry (the checker of the GPU path).

  debayer_buffer_new_float     algos/demosaicing_rtp.cpp:228-390 (min/max
                               normalisation to [0, 65535], dispatch, the
                               inverse mapping `v * invfactor + min`)
  debayer_superpixel_float     algos/demosaicing_siril.c:128-176, 806-820
  pattern_to_cfarray           algos/demosaicing_rtp.cpp:20-41

BAYER_BILINEAR goes to librtprocess `bayerfast_demosaic` (demosaicing_rtp.cpp:
147-151, 318-323; forced for every colour SER frame, io/ser.c:1177-1182),
restated below (`bayerfast`) from the published RawTherapee fast_demosaic
(Emil Martinec, rtengine/fast_demo.cc, the source of librtprocess
bayerfast.cc): 5-pixel border by the 3x3 same-colour mean, green at red /
blue sites by the gradient-weighted mean of its four neighbours (weights
1 / (1 + |x - x2| + |x1 - x-1|)^2 per direction), red at blue / blue at red
sites by the colour difference of the four diagonals (the raw sum capped at
clip_pt = 4 * 65535 * initGain, initGain = 1.0 in Siril), red / blue at green
sites by the colour difference of the four cardinal neighbours, negatives
clipped to 0.  Parity with librtprocess is UNPINNED (the library is not in
the image): the summation order inside each expression is a stated choice
(left to right as written below), and the GPU kernel follows it operation
for operation, so GPU vs this oracle is bit-exact.

The default interpolation, librtprocess `rcd_demosaic`, is NOT in the
reference tree (empty submodule): it is restated here from the
published RCD 2.3 algorithm (Luis Sanz Rodriguez; the tiled RawTherapee /
librtprocess form): directional discrimination from squared 1-D high-pass
filters, a low-pass-ratio green estimate, diagonal P/Q red/blue at red/blue
sites, cardinal red/blue at green sites, a 6-pixel border filled by the
3x3 same-colour mean (border_interpolate).  Parity with librtprocess is
UNPINNED; buffers the tiled code leaves uninitialised are defined as 0 and
the PQ_Dir buffer keeps the low-pass values where step 4.1 does not write
(it is the same buffer in the tiled code).  The GPU kernel follows this
restatement operation for operation (f32, no contraction), so GPU vs this
oracle is bit-exact.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
RGGB, BGGR, GBRG, GRBG = range(4)
BAYER_BILINEAR = 0
BAYER_RCD = 8
EPS = f32(1e-5)
EPSSQ = f32(1e-10)
SCALE = f32(65536.0)
# outer pixels filled by border_interpolate: the RCD steps run on [4, -4) but
# read uninitialised neighbours there; 6 is the smallest margin whose output
# does not depend on them (a flat field comes back exact) -- unpinned choice
BORDER = 6

CFARRAY = {RGGB: ((0, 1), (1, 2)), BGGR: ((2, 1), (1, 0)), GBRG: ((1, 2), (0, 1)), GRBG: ((1, 0), (2, 1))}


def colour_map(h, w, pattern):
    ca = np.array(CFARRAY[pattern], np.int8)
    yy, xx = np.mgrid[0:h, 0:w]
    return ca[yy & 1, xx & 1]


class _P:
    """Zero-padded view helper: s(a, dy, dx)[y, x] == a[y + dy, x + dx]."""
    PAD = 8

    def __init__(self, h, w):
        self.h, self.w = h, w

    def pad(self, a):
        return np.pad(a, self.PAD)

    def s(self, ap, dy, dx):
        P = self.PAD
        return ap[P + dy:P + dy + self.h, P + dx:P + dx + self.w]


def _region(h, w, m):
    yy, xx = np.mgrid[0:h, 0:w]
    return (yy >= m) & (yy < h - m) & (xx >= m) & (xx < w - m)


def _hpf(c, d1, d2, d3):
    """SQR((c[-3] - c[-1] - c[+1] + c[+3]) - 3 (c[-2] + c[+2]) + 6 c[0])."""
    t = ((d3[0] - d1[0]) - d1[1]) + d3[1]
    t = t - f32(3.0) * (d2[0] + d2[1])
    t = t + f32(6.0) * c
    return t * t


def rcd(raw: np.ndarray, pattern: int):
    """rcd_demosaic on the normalised [0, 65535] CFA image -> (R, G, B)."""
    raw = np.asarray(raw, f32)
    h, w = raw.shape
    H = _P(h, w)
    col = colour_map(h, w, pattern)
    ng = col != 1
    cfa = np.clip(raw / SCALE, f32(0), f32(1)).astype(f32)
    cp = H.pad(cfa)
    s = H.s
    # step 1.1: squared vertical / horizontal high-pass
    v = _hpf(cfa, (s(cp, -1, 0), s(cp, 1, 0)), (s(cp, -2, 0), s(cp, 2, 0)), (s(cp, -3, 0), s(cp, 3, 0)))
    hh = _hpf(cfa, (s(cp, 0, -1), s(cp, 0, 1)), (s(cp, 0, -2), s(cp, 0, 2)), (s(cp, 0, -3), s(cp, 0, 3)))
    yy, xx = np.mgrid[0:h, 0:w]
    v = np.where((yy >= 3) & (yy < h - 3) & (xx >= 4) & (xx < w - 4), v, f32(0)).astype(f32)
    hh = np.where((yy >= 4) & (yy < h - 4) & (xx >= 3) & (xx < w - 3), hh, f32(0)).astype(f32)
    vp, hp = H.pad(v), H.pad(hh)
    # step 1.2: VH_Dir
    vs = np.maximum(EPSSQ, (s(vp, -1, 0) + v) + s(vp, 1, 0))
    hs = np.maximum(EPSSQ, (s(hp, 0, -1) + hh) + s(hp, 0, 1))
    r4 = _region(h, w, 4)
    vh = np.where(r4, vs / (vs + hs), f32(0)).astype(f32)
    # step 2: low pass at red/blue sites (rows/cols [2, -2))
    lp = cfa + f32(0.5) * (((s(cp, -1, 0) + s(cp, 1, 0)) + s(cp, 0, -1)) + s(cp, 0, 1)) \
        + f32(0.25) * (((s(cp, -1, -1) + s(cp, -1, 1)) + s(cp, 1, -1)) + s(cp, 1, 1))
    lpf = np.where(ng & _region(h, w, 2), lp, f32(0)).astype(f32)
    lpp = H.pad(lpf)
    # step 3: green at red/blue sites
    a = np.abs
    cN1, cS1, cW1, cE1 = s(cp, -1, 0), s(cp, 1, 0), s(cp, 0, -1), s(cp, 0, 1)
    # eps + (|.| + |.|) + (|.| + |.|), evaluated left to right
    N_Grad = (EPS + (a(cN1 - cS1) + a(cfa - s(cp, -2, 0)))) + (a(cN1 - s(cp, -3, 0)) + a(s(cp, -2, 0) - s(cp, -4, 0)))
    S_Grad = (EPS + (a(cN1 - cS1) + a(cfa - s(cp, 2, 0)))) + (a(cS1 - s(cp, 3, 0)) + a(s(cp, 2, 0) - s(cp, 4, 0)))
    W_Grad = (EPS + (a(cW1 - cE1) + a(cfa - s(cp, 0, -2)))) + (a(cW1 - s(cp, 0, -3)) + a(s(cp, 0, -2) - s(cp, 0, -4)))
    E_Grad = (EPS + (a(cW1 - cE1) + a(cfa - s(cp, 0, 2)))) + (a(cE1 - s(cp, 0, 3)) + a(s(cp, 0, 2) - s(cp, 0, 4)))
    l2 = lpf + lpf
    N_Est = cN1 * l2 / ((EPS + lpf) + s(lpp, -2, 0))
    S_Est = cS1 * l2 / ((EPS + lpf) + s(lpp, 2, 0))
    W_Est = cW1 * l2 / ((EPS + lpf) + s(lpp, 0, -2))
    E_Est = cE1 * l2 / ((EPS + lpf) + s(lpp, 0, 2))
    V_Est = (S_Grad * N_Est + N_Grad * S_Est) / (N_Grad + S_Grad)
    H_Est = (W_Grad * E_Est + E_Grad * W_Est) / (E_Grad + W_Grad)
    vhp = H.pad(vh)
    vh_nb = f32(0.25) * ((s(vhp, -1, -1) + s(vhp, -1, 1)) + (s(vhp, 1, -1) + s(vhp, 1, 1)))
    vh_disc = np.where(a(f32(0.5) - vh) < a(f32(0.5) - vh_nb), vh_nb, vh)
    g_est = vh_disc * (H_Est - V_Est) + V_Est
    G = np.where(~ng, cfa, np.where(ng & r4, g_est, f32(0))).astype(f32)
    Gp = H.pad(G)
    # step 4.0: squared diagonal high-pass at red/blue sites (rows/cols [3, -3))
    P = _hpf(cfa, (s(cp, -1, -1), s(cp, 1, 1)), (s(cp, -2, -2), s(cp, 2, 2)), (s(cp, -3, -3), s(cp, 3, 3)))
    Q = _hpf(cfa, (s(cp, -1, 1), s(cp, 1, -1)), (s(cp, -2, 2), s(cp, 2, -2)), (s(cp, -3, 3), s(cp, 3, -3)))
    r3 = _region(h, w, 3)
    P = np.where(ng & r3, P, f32(0)).astype(f32)
    Q = np.where(ng & r3, Q, f32(0)).astype(f32)
    Pp, Qp = H.pad(P), H.pad(Q)
    # step 4.1: PQ_Dir (shares the low-pass buffer)
    ps = np.maximum(EPSSQ, (s(Pp, -1, -1) + P) + s(Pp, 1, 1))
    qs = np.maximum(EPSSQ, (s(Qp, -1, 1) + Q) + s(Qp, 1, -1))
    pq = np.where(ng & r4, ps / (ps + qs), lpf).astype(f32)
    pqp = H.pad(pq)
    # step 4.2: red at blue sites and blue at red sites
    R = np.where(col == 0, cfa, f32(0)).astype(f32)
    B = np.where(col == 2, cfa, f32(0)).astype(f32)
    pq_nb = f32(0.25) * (((s(pqp, -1, -1) + s(pqp, -1, 1)) + s(pqp, 1, -1)) + s(pqp, 1, 1))
    pq_disc = np.where(a(f32(0.5) - pq) < a(f32(0.5) - pq_nb), pq_nb, pq)
    out42 = {}
    for c, plane in ((0, R), (2, B)):
        rp = H.pad(plane)
        NW, NE, SW, SE = s(rp, -1, -1), s(rp, -1, 1), s(rp, 1, -1), s(rp, 1, 1)
        NW_Grad = ((EPS + a(NW - SE)) + a(NW - s(rp, -3, -3))) + a(G - s(Gp, -2, -2))
        NE_Grad = ((EPS + a(NE - SW)) + a(NE - s(rp, -3, 3))) + a(G - s(Gp, -2, 2))
        SW_Grad = ((EPS + a(NE - SW)) + a(SW - s(rp, 3, -3))) + a(G - s(Gp, 2, -2))
        SE_Grad = ((EPS + a(NW - SE)) + a(SE - s(rp, 3, 3))) + a(G - s(Gp, 2, 2))
        NW_Est = NW - s(Gp, -1, -1)
        NE_Est = NE - s(Gp, -1, 1)
        SW_Est = SW - s(Gp, 1, -1)
        SE_Est = SE - s(Gp, 1, 1)
        P_Est = (NW_Grad * SE_Est + SE_Grad * NW_Est) / (NW_Grad + SE_Grad)
        Q_Est = (NE_Grad * SW_Est + SW_Grad * NE_Est) / (NE_Grad + SW_Grad)
        out42[c] = G + (pq_disc * (Q_Est - P_Est) + P_Est)
    R = np.where((col == 2) & r4, out42[0], R).astype(f32)
    B = np.where((col == 0) & r4, out42[2], B).astype(f32)
    # step 4.3: red and blue at green sites
    N1 = EPS + a(G - s(Gp, -2, 0))
    S1 = EPS + a(G - s(Gp, 2, 0))
    W1 = EPS + a(G - s(Gp, 0, -2))
    E1 = EPS + a(G - s(Gp, 0, 2))
    res = {}
    for c, plane in ((0, R), (2, B)):
        rp = H.pad(plane)
        SNabs = a(s(rp, -1, 0) - s(rp, 1, 0))
        EWabs = a(s(rp, 0, -1) - s(rp, 0, 1))
        N_Grad = (N1 + SNabs) + a(s(rp, -1, 0) - s(rp, -3, 0))
        S_Grad = (S1 + SNabs) + a(s(rp, 1, 0) - s(rp, 3, 0))
        W_Grad = (W1 + EWabs) + a(s(rp, 0, -1) - s(rp, 0, -3))
        E_Grad = (E1 + EWabs) + a(s(rp, 0, 1) - s(rp, 0, 3))
        N_Est = s(rp, -1, 0) - s(Gp, -1, 0)
        S_Est = s(rp, 1, 0) - s(Gp, 1, 0)
        W_Est = s(rp, 0, -1) - s(Gp, 0, -1)
        E_Est = s(rp, 0, 1) - s(Gp, 0, 1)
        V_Est = (N_Grad * S_Est + S_Grad * N_Est) / (N_Grad + S_Grad)
        H_Est = (E_Grad * W_Est + W_Grad * E_Est) / (E_Grad + W_Grad)
        res[c] = G + (vh_disc * (H_Est - V_Est) + V_Est)
    R = np.where((col == 1) & r4, res[0], R).astype(f32)
    B = np.where((col == 1) & r4, res[2], B).astype(f32)
    out = [np.maximum(f32(0), X * SCALE).astype(f32) for X in (R, G, B)]
    _border_interpolate(raw, col, BORDER, out)
    return out


def _border_interpolate(raw, col, bord, out):
    """border_interpolate: 3x3 same-colour mean in the `bord` outer pixels."""
    h, w = raw.shape
    R, G, B = out
    for i in range(h):
        for j in range(w):
            if bord <= i < h - bord and bord <= j < w - bord:
                continue
            sm = [f32(0)] * 6
            for i1 in range(i - 1, i + 2):
                for j1 in range(j - 1, j + 2):
                    if 0 <= i1 < h and 0 <= j1 < w:
                        c = int(col[i1, j1])
                        sm[c] = f32(sm[c] + raw[i1, j1])
                        sm[c + 3] = f32(sm[c + 3] + f32(1))
            c = int(col[i, j])
            if c == 1:
                R[i, j] = f32(sm[0] / sm[3])
                G[i, j] = raw[i, j]
                B[i, j] = f32(sm[2] / sm[5])
            else:
                G[i, j] = f32(sm[1] / sm[4])
                if c == 0:
                    R[i, j] = raw[i, j]
                    B[i, j] = f32(sm[2] / sm[5])
                else:
                    R[i, j] = f32(sm[0] / sm[3])
                    B[i, j] = raw[i, j]


BF_BORDER = 5                          # bayerfast: bord
BF_CLIP = f32(4 * 65535 * 1.0)         # clip_pt = 4 * 65535 * initGain (initGain = 1.0, demosaicing_rtp.cpp:151)


def bayerfast(raw: np.ndarray, pattern: int):
    """bayerfast_demosaic on the (normalised) CFA image -> (R, G, B) float32."""
    raw = np.asarray(raw, f32)
    h, w = raw.shape
    H = _P(h, w)
    col = colour_map(h, w, pattern)
    rp = H.pad(raw)
    s = H.s
    a = np.abs
    c = raw
    n1, s1, w1, e1 = s(rp, -1, 0), s(rp, 1, 0), s(rp, 0, -1), s(rp, 0, 1)
    one = f32(1)
    sq = lambda t: (t * t).astype(f32)
    # green at red / blue sites: directional weights from the image gradients
    wtu = one / sq((one + a(c - s(rp, -2, 0))) + a(n1 - s1))
    wtd = one / sq((one + a(c - s(rp, 2, 0))) + a(s1 - n1))
    wtl = one / sq((one + a(c - s(rp, 0, -2))) + a(w1 - e1))
    wtr = one / sq((one + a(c - s(rp, 0, 2))) + a(e1 - w1))
    gi = (((wtu * n1 + wtd * s1) + wtl * w1) + wtr * e1) / (((wtu + wtd) + wtl) + wtr)
    G = np.where(col == 1, c, gi).astype(f32)
    Gp = H.pad(G)
    # red at blue sites, blue at red sites: colour difference of the diagonals
    gd = ((s(Gp, -1, -1) + s(Gp, -1, 1)) + s(Gp, 1, 1)) + s(Gp, 1, -1)
    rd = ((s(rp, -1, -1) + s(rp, -1, 1)) + s(rp, 1, 1)) + s(rp, 1, -1)
    other = (G - f32(0.25) * (gd - np.where(rd < BF_CLIP, rd, BF_CLIP))).astype(f32)
    R = np.where(col == 0, c, np.where(col == 2, other, f32(0))).astype(f32)
    B = np.where(col == 2, c, np.where(col == 0, other, f32(0))).astype(f32)
    # red / blue at green sites: colour difference of the four cardinal neighbours
    gc = ((s(Gp, -1, 0) + s(Gp, 0, -1)) + s(Gp, 0, 1)) + s(Gp, 1, 0)
    out = []
    for X in (R, B):
        xp = H.pad(X)
        xc = ((s(xp, -1, 0) + s(xp, 0, -1)) + s(xp, 0, 1)) + s(xp, 1, 0)
        out.append(np.where(col == 1, (G - f32(0.25) * (gc - np.where(xc < BF_CLIP, xc, BF_CLIP))).astype(f32), X))
    rgb = [np.maximum(f32(0), X).astype(f32) for X in (out[0], G, out[1])]
    _border_interpolate(raw, col, BF_BORDER, rgb)
    return rgb


def _interpolate(raw, interpolation, pattern):
    """the librtprocess switch of demosaicing_rtp.cpp:141-160, 312-330
    (unknown values fall to RCD: `default: case BAYER_RCD`)"""
    if interpolation == BAYER_BILINEAR:
        return bayerfast(raw, pattern)
    if interpolation == BAYER_RCD or interpolation < 0 or interpolation > 9:
        return rcd(raw, pattern)
    raise NotImplementedError("only RCD and bayerfast are restated")


def debayer_buffer_new_float(buf: np.ndarray, interpolation: int, pattern: int):
    """demosaicing_rtp.cpp:228-390 -> planar (3, h, w) float32, or None when
    min == max.  RCD and BAYER_BILINEAR (bayerfast) are restated."""
    buf = np.asarray(buf, f32)
    mn, mx = f32(buf.min()), f32(buf.max())
    rng = f32(mx - mn)
    if rng == 0:
        return None
    factor = f32(f32(65535.0) / rng)
    invfactor = f32(1.0 / float(factor))
    norm = ((buf - mn) * factor).astype(f32)
    rgb = _interpolate(norm, interpolation, pattern)
    return np.stack([(p * invfactor + mn).astype(f32) for p in rgb])


def _round_to(v, top):
    """roundf_to_WORD / roundf_to_BYTE (core/proto.h:256-261, 341-346)."""
    f = (np.asarray(v, f32) + f32(0.5)).astype(f32)
    f = np.where(f > f32(top), f32(top), f)
    f = np.where(f < f32(0), f32(0), f)
    return f.astype(np.uint16)


def debayer_buffer_new_ushort(buf: np.ndarray, interpolation: int, pattern: int, bit_depth: int = 16):
    """demosaicing_rtp.cpp:74-224 -> planar (3, h, w) uint16: the WORD samples
    go to RCD as float, unnormalised (:95-96), the result is rounded per
    sample (:202-213; BYTE range when bit_depth == BYTE_IMG == 8)."""
    raw = np.asarray(buf, np.uint16).astype(f32)
    rgb = _interpolate(raw, interpolation, pattern)
    top = 255.0 if bit_depth == 8 else 65535.0
    return np.stack([_round_to(p, top) for p in rgb])


def superpixel(buf: np.ndarray, pattern: int):
    """super_pixel_float + debayer_buffer_superpixel_float: interleaved RGB of
    size (w/2 + w%2) x (h/2 + h%2); cells of an odd last row / column are not
    written by the reference (malloc) and are 0 here."""
    buf = np.asarray(buf, f32)
    h, w = buf.shape
    nw, nh = w // 2 + w % 2, h // 2 + h % 2
    out = np.zeros((nh, nw, 3), f32)
    a = buf[0:h - 1:2, 0:w - 1:2][: (h // 2), : (w // 2)]
    b = buf[0:h - 1:2, 1:w:2][: (h // 2), : (w // 2)]
    c = buf[1:h:2, 0:w - 1:2][: (h // 2), : (w // 2)]
    d = buf[1:h:2, 1:w:2][: (h // 2), : (w // 2)]
    hh, ww = a.shape
    o = out[:hh, :ww]
    if pattern == RGGB:
        o[..., 0], o[..., 1], o[..., 2] = a, (b + c) * f32(0.5), d
    elif pattern == BGGR:
        o[..., 2], o[..., 1], o[..., 0] = a, (b + c) * f32(0.5), d
    elif pattern == GBRG:
        o[..., 2], o[..., 0], o[..., 1] = b, c, (a + d) * f32(0.5)
    elif pattern == GRBG:
        o[..., 0], o[..., 2], o[..., 1] = b, c, (a + d) * f32(0.5)
    return out


# ---------------------------------------------------------------------------
# Siril's own bilinear decoder (algos/demosaicing_siril.c:179-288: ClearBorders
# + bayer_Bilinear, "OpenCV's Bayer decoding"), restated LITERALLY as its
# pointer walk over flat buffers (rgb interleaved RGBRGB), then debayer_ushort's
# RGBRGB -> RRGGBB loop with truncate_to_BYTE for 8-bit (:846-855).
def _clear_borders(rgb, sx, sy, w):
    i = 3 * sx * w - 1
    j = 3 * sx * sy - 1
    while i >= 0:
        rgb[i] = 0
        rgb[j] = 0
        i -= 1
        j -= 1
    low = sx * (w - 1) * 3 - 1 + w * 3
    i = low + sx * (sy - w * 2 + 1) * 3
    while i > low:
        j = 6 * w
        while j > 0:
            rgb[i] = 0
            i -= 1
            j -= 1
        i -= (sx - 2 * w) * 3


def bayer_bilinear_siril(bayer_img: np.ndarray, tile: int) -> np.ndarray:
    """(h, w) uint16 -> (h*w*3,) interleaved WORD RGB, literal walk."""
    sy, sx = bayer_img.shape
    bayer = [int(v) for v in np.asarray(bayer_img, np.uint16).ravel()]
    rgb = [0] * (3 * sx * sy)
    step, rgb_step = sx, 3 * sx
    width, height = sx, sy
    blue = -1 if tile in (1, 2) else 1                 # BGGR, GBRG
    start_with_green = tile in (2, 3)                  # GBRG, GRBG
    _clear_borders(rgb, sx, sy, 1)
    b = 0                                              # index into bayer
    r = rgb_step + 3 + 1                               # index into rgb
    height -= 2
    width -= 2
    rnd = lambda t: min(max(int(t + 0.5), 0), 65535)   # round_to_WORD of an int
    while height > 0:
        height -= 1
        bayer_end = b + width
        if start_with_green:
            t0 = (bayer[b + 1] + bayer[b + step * 2 + 1] + 1) >> 1
            t1 = (bayer[b + step] + bayer[b + step + 2] + 1) >> 1
            rgb[r - blue] = rnd(t0)
            rgb[r] = bayer[b + step + 1]
            rgb[r + blue] = rnd(t1)
            b += 1
            r += 3
        if blue > 0:
            while b <= bayer_end - 2:
                t0 = (bayer[b] + bayer[b + 2] + bayer[b + step * 2] + bayer[b + step * 2 + 2] + 2) >> 2
                t1 = (bayer[b + 1] + bayer[b + step] + bayer[b + step + 2] + bayer[b + step * 2 + 1] + 2) >> 2
                rgb[r - 1] = rnd(t0)
                rgb[r] = rnd(t1)
                rgb[r + 1] = bayer[b + step + 1]
                t0 = (bayer[b + 2] + bayer[b + step * 2 + 2] + 1) >> 1
                t1 = (bayer[b + step + 1] + bayer[b + step + 3] + 1) >> 1
                rgb[r + 2] = rnd(t0)
                rgb[r + 3] = bayer[b + step + 2]
                rgb[r + 4] = rnd(t1)
                b += 2
                r += 6
        else:
            while b <= bayer_end - 2:
                t0 = (bayer[b] + bayer[b + 2] + bayer[b + step * 2] + bayer[b + step * 2 + 2] + 2) >> 2
                t1 = (bayer[b + 1] + bayer[b + step] + bayer[b + step + 2] + bayer[b + step * 2 + 1] + 2) >> 2
                rgb[r + 1] = rnd(t0)
                rgb[r] = rnd(t1)
                rgb[r - 1] = bayer[b + step + 1]
                t0 = (bayer[b + 2] + bayer[b + step * 2 + 2] + 1) >> 1
                t1 = (bayer[b + step + 1] + bayer[b + step + 3] + 1) >> 1
                rgb[r + 4] = rnd(t0)
                rgb[r + 3] = bayer[b + step + 2]
                rgb[r + 2] = rnd(t1)
                b += 2
                r += 6
        if b < bayer_end:
            t0 = (bayer[b] + bayer[b + 2] + bayer[b + step * 2] + bayer[b + step * 2 + 2] + 2) >> 2
            t1 = (bayer[b + 1] + bayer[b + step] + bayer[b + step + 2] + bayer[b + step * 2 + 1] + 2) >> 2
            rgb[r - blue] = rnd(t0)
            rgb[r] = rnd(t1)
            rgb[r + blue] = bayer[b + step + 1]
            b += 1
            r += 3
        b -= width
        r -= width * 3
        blue = -blue
        start_with_green = not start_with_green
        b += step                                      # the loop increment
        r += rgb_step
    return np.array(rgb, np.uint16)


def debayer_buffer_siril_ushort(buf: np.ndarray, pattern: int, bit_depth: int = 16) -> np.ndarray:
    """debayer_ushort's USE_SIRIL_DEBAYER branch with BAYER_BILINEAR:
    (3, h, w) planar uint16."""
    h, w = buf.shape
    inter = bayer_bilinear_siril(buf, pattern).reshape(h * w, 3)
    out = np.ascontiguousarray(inter.T.reshape(3, h, w))
    if bit_depth == 8:
        out = np.minimum(out, 255).astype(np.uint16)
    return out
