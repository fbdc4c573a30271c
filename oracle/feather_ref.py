"""TEST INFRASTRUCTURE (oracle): restatement of Siril's feathering masks for
`stack ... -feather=<dist>` and of the row-block planner they depend on.
Only tests/ may import this file.

  * stack_blocks: stack_compute_parallel_blocks + refine_blocks_candidate
    (stacking/median_and_mean.c:255-356, round_to_ceiling_multiple
    core/proto.h:295-299), checked against the cases of the reference's own
    src/tests/stacking_blocks_test.c (tests/golden/stacking_blocks.json);
  * downscale_blend_mask: compute_mask_image_hook (blending.c:131-191) +
    cvDownscaleBlendMask (opencv/opencv.cpp:587-609): the reference layer as
    0/255 (float: != 0, WORD: > 0), dilate then erode with a 7x7 rectangle
    (OpenCV's constant border never wins the max / min), resize INTER_LINEAR
    to (int)(0.1 rx) x (int)(0.1 ry) into the interior of a zero image one
    pixel larger on every side, distanceTransform(DIST_L2, 3), cropped back;
  * block_area / block_planes: stack_read_block_data's area logic and mask
    branch (median_and_mean.c:406-446, 483-525): the block's downscaled rows
    read as read_mask_fits_area does (image_format_fits.c:4113-4123),
    cvUpscaleBlendMask (opencv.cpp:611-616: INTER_LINEAR float, then a
    vertical flip) and `1 if d > feather else ramp(d / feather)` for d != 0
    with init_ramp's table (blending.c:34-50).

OpenCV is not in this image, so the resize and distance-transform arithmetic
restates OpenCV 4.x's generic code as published (modules/imgproc resize.cpp,
distransform.cpp; no IPP):
  * coordinates: fx = (float)((d + 0.5) * scale - 0.5), scale = 1 /
    ((double)dst / src), sx = cvFloor(fx), fx -= sx; horizontally sx < 0 ->
    (0, 0) and sx >= src - 1 -> (src - 1, 0); vertically the fraction is kept
    and the two rows are fetched clipped to [0, h);
  * 8-bit: coefficients saturate_cast<short>(w * 2048); horizontal sums in
    int; vertical (b0 S0 + b1 S1 + 2^21) >> 22 in scalar code, and for the
    columns the baseline SSE2 VResizeLinearVec_32s8u covers (16-wide steps,
    then 8-wide while x < width - 8) ((S0 >> 4) b0 >> 16) + ((S1 >> 4) b1 >>
    16), + 2, >> 2;
  * float: S0 a0 + S1 a1 and R0 b0 + R1 b1 without FMA (x86-64 baseline);
  * distance transform: the 3x3 chamfer (0.955f, 1.3693f) as
    cvRound(x * 65536), two raster passes over a frame of INT_MAX, output
    (float)min(t, INT_MAX >> 2) / 65536.
Parity with Siril's binary is therefore unpinned (the system OpenCV may also
be built with other SIMD baselines or IPP)."""
import numpy as np

MASK_SCALE = 0.1
RAMP_PACE = 1000
COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS
DIST_SHIFT = 16
INIT_DIST0 = 0x7FFFFFFF
DIST_MAX = INIT_DIST0 >> 2
HV_DIST = int(np.rint(np.float32(0.955) * np.float32(1 << DIST_SHIFT)))
DIAG_DIST = int(np.rint(np.float32(1.3693) * np.float32(1 << DIST_SHIFT)))


# ---------------------------------------------------------------------------
# block planner
# ---------------------------------------------------------------------------
def _ceil_multiple(x, factor):
    r = x % factor
    return x + (factor - r) * (r != 0)


def _refine(nb_threads, nb_channels, minimum):
    factor = nb_channels
    if nb_threads < 4:
        if factor != 1 and nb_threads % factor == 0:
            factor = nb_threads
        else:
            factor *= nb_threads
        return _ceil_multiple(minimum, factor)
    minus = 1 if nb_threads < 8 else 3
    cand = _ceil_multiple(minimum, factor)
    while True:
        rem = cand % nb_threads
        if rem == 0 or rem >= nb_threads - minus:
            return cand
        cand += factor


def _cdiv(a, b):
    """C integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def stack_blocks(max_rows, naxes, nb_threads):
    """[(channel, start_row, height)] of stack_compute_parallel_blocks; naxes =
    (width, height, channels)."""
    h, ch = naxes[1], naxes[2]
    cand = nb_threads
    while _cdiv(max_rows * cand, nb_threads) < h * ch:
        cand += 1
    cand = _refine(nb_threads, 3 if ch == 3 else 1, cand)
    hb = h * ch // cand
    rem = h % (cand // ch)
    blocks = []
    c = row = 0
    while True:
        if len(blocks) >= cand:
            raise RuntimeError("rows left after the last block")
        start, chan = row, c
        end = row + hb - 1
        if rem > 0:
            end += 1
            rem -= 1
        if end >= h - 1 or h - end < hb // 10:
            end = h - 1
            row = 0
            c += 1
            rem = h - (cand // ch * hb)
        else:
            row = end + 1
        blocks.append((chan, start, end - start + 1))
        if c >= ch:
            break
    if len(blocks) != cand:
        raise RuntimeError("fewer blocks than planned")
    return blocks


# ---------------------------------------------------------------------------
# downscaled masks
# ---------------------------------------------------------------------------
def ramp_array():
    """init_ramp (blending.c:34-45): r * r * r * (6 r r - 15 r + 10) in float."""
    f = np.float32
    norm = f(1.0) / f(RAMP_PACE)
    out = np.empty(RAMP_PACE + 1, np.float32)
    for i in range(RAMP_PACE + 1):
        r = f(f(i) * norm)
        out[i] = f(f(f(r * r) * r) * f(f(f(f(6) * r) * r - f(f(15) * r)) + f(10)))
    return out


def mask_size(rx, ry):
    """compute_downscaled_mask_size (blending.c:52-59): (rx_out, ry_out, fx, fy)."""
    rxo, ryo = int(rx * MASK_SCALE), int(ry * MASK_SCALE)
    return rxo, ryo, rxo / rx, ryo / ry


def _morph(img, op, border):
    h, w = img.shape
    pad = np.pad(img, 3, mode="constant", constant_values=border)
    out = pad[3:3 + h, 3:3 + w].copy()
    for dy in range(-3, 4):
        for dx in range(-3, 4):
            out = op(out, pad[3 + dy:3 + dy + h, 3 + dx:3 + dx + w])
    return out


def _cv_floor(f):
    i = int(f)
    return i - (i > f)


def linear_table(src, dst, clamp):
    """Source index and fraction (float32) per destination index."""
    scale = 1.0 / (dst / src)
    ofs = np.empty(dst, np.int64)
    frac = np.empty(dst, np.float32)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = _cv_floor(float(f))
        f = np.float32(f - np.float32(s))
        if clamp:
            if s < 0:
                f, s = np.float32(0), 0
            if s + 1 >= src and s >= src - 1:
                f, s = np.float32(0), src - 1
        ofs[d], frac[d] = s, f
    return ofs, frac


def _sat_short(v):
    return int(np.clip(np.rint(np.float64(v)), -32768, 32767))


def simd_end(width):
    """First column of VResizeLinearVec_32s8u's scalar tail."""
    x = 0
    while x <= width - 16:
        x += 16
    while x < width - 8:
        x += 8
    return x


def resize_linear_u8(img, out_w, out_h):
    """cv::resize INTER_LINEAR of a CV_8U image (see the module docstring)."""
    h, w = img.shape
    sx, fx = linear_table(w, out_w, True)
    sy, fy = linear_table(h, out_h, False)
    one = np.float32(1)
    a0 = np.array([_sat_short(np.float32(one - f) * np.float32(COEF_SCALE)) for f in fx], np.int64)
    a1 = np.array([_sat_short(f * np.float32(COEF_SCALE)) for f in fx], np.int64)
    b0 = np.array([_sat_short(np.float32(one - f) * np.float32(COEF_SCALE)) for f in fy], np.int64)
    b1 = np.array([_sat_short(f * np.float32(COEF_SCALE)) for f in fy], np.int64)
    a = img.astype(np.int64)
    rows = a[:, sx] * a0[None, :] + a[:, np.minimum(sx + 1, w - 1)] * a1[None, :]
    S0 = rows[np.clip(sy, 0, h - 1)]
    S1 = rows[np.clip(sy + 1, 0, h - 1)]
    B0, B1 = b0[:, None], b1[:, None]
    scalar = (S0 * B0 + S1 * B1 + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS)
    vec = np.clip(((S0 >> 4) * B0 >> 16) + ((S1 >> 4) * B1 >> 16), -32768, 32767)
    vec = (vec + 2) >> 2
    xv = simd_end(out_w)
    out = scalar.copy()
    out[:, :xv] = vec[:, :xv]
    return np.clip(out, 0, 255).astype(np.uint8)


def resize_linear_f32(img, out_w, out_h):
    """cv::resize INTER_LINEAR of a CV_32F image."""
    h, w = img.shape
    sx, fx = linear_table(w, out_w, True)
    sy, fy = linear_table(h, out_h, False)
    a1 = fx.astype(np.float32)
    a0 = (np.float32(1) - a1).astype(np.float32)
    b1 = fy.astype(np.float32)
    b0 = (np.float32(1) - b1).astype(np.float32)
    f = img.astype(np.float32)
    rows = (f[:, sx] * a0[None, :]).astype(np.float32) + (f[:, np.minimum(sx + 1, w - 1)] * a1[None, :]).astype(np.float32)
    r0 = rows[np.clip(sy, 0, h - 1)]
    r1 = rows[np.clip(sy + 1, 0, h - 1)]
    return ((r0 * b0[:, None]).astype(np.float32) + (r1 * b1[:, None]).astype(np.float32)).astype(np.float32)


def distance_transform_3x3(src):
    """distanceTransform(DIST_L2, 3, CV_32F): the two raster passes of
    distanceTransform_3x3 in unsigned 32-bit fixed point."""
    h, w = src.shape
    t = np.full((h + 2, w + 2), INIT_DIST0, np.int64)
    for i in range(h):
        r = i + 1
        row_u, row_s = t[r - 1], src[i]
        cur = t[r]
        for j in range(w):
            c = j + 1
            if not row_s[j]:
                cur[c] = 0
            else:
                cur[c] = min(row_u[c - 1] + DIAG_DIST, row_u[c] + HV_DIST, row_u[c + 1] + DIAG_DIST,
                             cur[c - 1] + HV_DIST)
    out = np.empty((h, w), np.float32)
    for i in range(h - 1, -1, -1):
        r = i + 1
        row_d = t[r + 1]
        cur = t[r]
        for j in range(w - 1, -1, -1):
            c = j + 1
            t0 = cur[c]
            if t0 > HV_DIST:
                t0 = min(t0, row_d[c + 1] + DIAG_DIST, row_d[c] + HV_DIST, row_d[c - 1] + DIAG_DIST, cur[c + 1] + HV_DIST)
                cur[c] = t0
            out[i, j] = np.float32(np.float32(min(t0, DIST_MAX)) * np.float32(1.0 / (1 << DIST_SHIFT)))
    return out


def chamfer_closed_form(src):
    """The 3x3 chamfer distance as a global minimum over black pixels
    (b min(|dx|,|dy|) + a (max - min)), the property the GPU's scan
    formulation relies on; for checking distance_transform_3x3."""
    h, w = src.shape
    zy, zx = np.nonzero(src == 0)
    yy, xx = np.mgrid[0:h, 0:w]
    best = np.full((h, w), DIST_MAX, np.int64)
    for y, x in zip(zy, zx):
        dy, dx = np.abs(yy - y), np.abs(xx - x)
        mn, mx = np.minimum(dx, dy), np.maximum(dx, dy)
        best = np.minimum(best, DIAG_DIST * mn + HV_DIST * (mx - mn))
    return (np.minimum(best, DIST_MAX).astype(np.float32) * np.float32(1.0 / (1 << DIST_SHIFT))).astype(np.float32)


def downscale_blend_mask(layer, dt=distance_transform_3x3):
    """compute_mask_image_hook + cvDownscaleBlendMask for one frame's layer
    (float32 or uint16 [ry, rx], FITS row order): the (ry_o, rx_o) mask."""
    ry, rx = layer.shape
    rxo, ryo, _, _ = mask_size(rx, ry)
    nz = layer > 0 if layer.dtype == np.uint16 else layer != 0
    m8 = np.where(nz, 255, 0).astype(np.uint8)
    m8 = _morph(_morph(m8, np.maximum, 0), np.minimum, 255)
    big = np.zeros((ryo + 2, rxo + 2), np.uint8)
    big[1:1 + ryo, 1:1 + rxo] = resize_linear_u8(m8, rxo, ryo)
    return dt(big)[1:1 + ryo, 1:1 + rxo].copy()


# ---------------------------------------------------------------------------
# per-block planes
# ---------------------------------------------------------------------------
def block_area(rx, ry, start_row, block_height, shifty=None):
    """(first block row written, area rows, first downscaled row, downscaled
    rows) of stack_read_block_data for one frame; shifty None = no
    registration data."""
    ay, ah, off, read = start_row, block_height, 0, True
    if shifty is not None:
        if ay + ah + shifty <= 0 or ay + shifty >= ry:
            read = False
        elif ay + shifty < 0:
            ah += ay + shifty
            ah = min(ah, ry)
            off = -(ay + shifty)
            ay = 0
        elif ay + ah + shifty >= ry:
            ay += shifty
            ah += ry - (ay + ah)
        else:
            ay += shifty
        if ah <= 0:
            read = False
    rxo, ryo, _, fy = mask_size(rx, ry)
    ys, hs = int(fy * ay), int(fy * ah)
    if not read or ah == 0 or hs == 0 or rxo == 0:
        return off, 0, 0, 0
    if ryo - ys - hs < 0:          # read_mask_fits_area fails: ST_SEQUENCE_ERROR
        raise ValueError("mask area outside the mask")
    return off, ah, ryo - ys - hs, hs


def block_planes(masks, rx, ry, start_row, block_height, feather, shifty=None, placex=None, canvas_width=None,
                 fits_order=True):
    """data->mask of one block: [N, block_height, canvas_width] float32."""
    n = masks.shape[0]
    cw = canvas_width or rx
    out = np.zeros((n, block_height, cw), np.float32)
    ramp = ramp_array()
    distf = np.float32(feather)
    inv = np.float32(np.float32(1) / distf)
    for f in range(n):
        off, ah, base, hs = block_area(rx, ry, start_row, block_height, None if shifty is None else int(shifty[f]))
        if ah == 0:
            continue
        up = resize_linear_f32(masks[f, base:base + hs], rx, ah)          # ascending FITS rows
        v = up.copy()
        nz = up != 0
        over = up > distf
        idx = ((up * inv).astype(np.float32) * np.float32(RAMP_PACE)).astype(np.float32)
        idx = np.clip(np.trunc(idx).astype(np.int64), 0, RAMP_PACE)
        v[nz & over] = 1.0
        r = nz & ~over
        v[r] = ramp[idx[r]]
        rows = v if fits_order else v[::-1]
        y0 = block_height - off - ah if fits_order else off
        px = 0 if placex is None else int(placex[f])
        x0, x1 = max(0, px), min(cw, px + rx)
        if x1 > x0:
            out[f, y0:y0 + ah, x0:x1] = rows[:, x0 - px:x1 - px]
    return out
