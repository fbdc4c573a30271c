"""Float debayer (debayer_buffer_new_float, demosaicing_rtp.cpp:228-390;
super-pixel, demosaicing_siril.c:128-176, 806-820).

Parity: the super-pixel path and Siril's normalisation wrapper are exact
restatements of reference code; RCD (librtprocess, not vendored) is restated
from the published algorithm -- parity with librtprocess UNPINNED
(SURVEY.md §8c).  The GPU path must equal the restatement bitwise.
"""
import numpy as np
import pytest

from oracle import demosaic_ref as D


def _mosaic(h, w, pattern, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    L = 0.3 + 0.2 * np.cos(yy / 5.0) * np.sin(xx / 6.0) + 0.05 * rng.random((h, w))
    R, G, B = 1.2 * L, L, 0.7 * L
    col = D.colour_map(h, w, pattern)
    return (np.where(col == 0, R, np.where(col == 1, G, B)) * 1000.0 + 17.0).astype(np.float32)


def test_oracle_flat_field_is_exact():
    h, w = 40, 52
    col = D.colour_map(h, w, D.RGGB)
    mos = np.where(col == 0, 0.5, np.where(col == 1, 0.4, 0.3)).astype(np.float32)
    out = D.debayer_buffer_new_float(mos, D.BAYER_RCD, D.RGGB)
    for i, v in enumerate((0.5, 0.4, 0.3)):
        assert np.abs(out[i] - v).max() < 1e-6


def test_oracle_correlated_colour_reconstruction():
    h, w = 64, 80
    yy, xx = np.mgrid[0:h, 0:w]
    L = 0.4 + 0.2 * np.cos(yy / 5.0) * np.sin(xx / 6.0)
    col = D.colour_map(h, w, D.GRBG)
    mos = np.where(col == 0, 1.2 * L, np.where(col == 1, L, 0.7 * L)).astype(np.float32)
    out = D.debayer_buffer_new_float(mos, D.BAYER_RCD, D.GRBG)
    for i, k in enumerate((1.2, 1.0, 0.7)):
        assert np.abs(out[i] - k * L)[9:-9, 9:-9].max() < 6e-3


def test_oracle_min_equals_max_is_null():
    assert D.debayer_buffer_new_float(np.full((16, 16), 3.0, np.float32), D.BAYER_RCD, D.RGGB) is None


def test_superpixel_known_answer():
    buf = np.arange(1, 21, dtype=np.float32).reshape(4, 5)
    out = D.superpixel(buf, D.RGGB)
    assert out.shape == (2, 3, 3)
    assert out[0, 0].tolist() == [1.0, (2.0 + 6.0) * 0.5, 7.0]
    assert out[1, 1].tolist() == [13.0, (14.0 + 18.0) * 0.5, 19.0]
    assert out[0, 2].tolist() == [0.0, 0.0, 0.0]       # odd tail column is not written
    g = D.superpixel(buf, D.GBRG)
    assert g[0, 0].tolist() == [6.0, (1.0 + 7.0) * 0.5, 2.0]


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 80), (37, 53), (9, 11)])
def test_rcd_gpu_bit_exact(pattern, shape):
    from siril_amd import demosaic
    mos = _mosaic(*shape, pattern, seed=pattern)
    want = D.debayer_buffer_new_float(mos, D.BAYER_RCD, pattern)
    got = demosaic.debayer_buffer_new_float(mos, demosaic.BAYER_RCD, pattern)
    assert got is not None
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_rcd_device_api_and_unknown_method_is_rcd():
    import torch
    from siril_amd import demosaic
    mos = _mosaic(48, 64, 3, seed=9)
    want = D.debayer_buffer_new_float(mos, D.BAYER_RCD, 3)
    out = demosaic.debayer(torch.from_numpy(mos).cuda(), pattern="GRBG")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    # the reference's switch falls through `default:` to RCD
    got = demosaic.debayer_buffer_new_float(mos, 42, 3)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_rcd_null_cases():
    from siril_amd import demosaic
    assert demosaic.debayer_buffer_new_float(np.full((16, 16), 2.0, np.float32)) is None   # min == max
    assert demosaic.debayer_buffer_new_float(_mosaic(16, 16, 0), demosaic.BAYER_VNG, 0) is None  # not implemented


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(40, 60), (41, 61), (7, 3)])
@pytest.mark.parametrize("pattern", [0, 1, 2, 3])
def test_superpixel_gpu_exact(shape, pattern):
    from siril_amd import demosaic
    buf = np.random.default_rng(shape[0]).random(shape).astype(np.float32)
    got = demosaic.debayer_buffer_superpixel_float(buf, pattern)
    assert np.array_equal(got, D.superpixel(buf, pattern))


@pytest.mark.gpu
def test_rcd_full_frame_properties():
    """6000 x 4000 (BASELINE frame size): a flat CFA field comes back flat in
    every channel, and the output keeps the input range mapping."""
    import torch
    from siril_amd import demosaic
    h, w = 4000, 6000
    col = torch.from_numpy(D.colour_map(h, w, 0)).cuda()
    mos = torch.where(col == 0, 0.5, torch.where(col == 1, 0.4, 0.3)).float().contiguous()
    out = demosaic.debayer(mos, pattern=0)
    for i, v in enumerate((0.5, 0.4, 0.3)):
        assert float((out[i] - v).abs().max()) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["1", "2", "0", "3"])
@pytest.mark.parametrize("shape", [(131, 517), (96, 128), (33, 70)])
def test_rcd_tiles_and_multipass_bit_exact(mode, shape):
    """The fused LDS-tiled kernel (64x32 and 32x32 tiles, tile edges inside
    the image and at its border), the step-per-kernel pipeline and the
    two-kernel split (the default) all equal the restatement bitwise
    (SGPU_RCD_FUSED selects the variant)."""
    import os
    from siril_amd import demosaic
    old = os.environ.get("SGPU_RCD_FUSED")
    os.environ["SGPU_RCD_FUSED"] = mode
    try:
        for pattern in (0, 3):
            mos = _mosaic(*shape, pattern, seed=7 + pattern)
            want = D.debayer_buffer_new_float(mos, D.BAYER_RCD, pattern)
            got = demosaic.debayer_buffer_new_float(mos, demosaic.BAYER_RCD, pattern)
            assert np.array_equal(got, want), (mode, shape, pattern)
    finally:
        if old is None:
            os.environ.pop("SGPU_RCD_FUSED", None)
        else:
            os.environ["SGPU_RCD_FUSED"] = old


# ---- debayer_buffer_new_ushort (demosaicing_rtp.cpp:74-224) -----------------
def _mosaic16(h, w, pattern, seed=0, top=65535.0):
    m = _mosaic(h, w, pattern, seed)
    m = (m - m.min()) / (m.max() - m.min())
    return np.round(m * top * 0.98 + top * 0.01).astype(np.uint16)


def test_oracle_ushort_flat_field_and_rounding():
    """A flat 16-bit field comes back flat; values are rounded and clamped
    the roundf_to_WORD / roundf_to_BYTE way (+0.5, clamp, truncate)."""
    h, w = 40, 52
    col = D.colour_map(h, w, D.RGGB)
    mos = np.where(col == 0, 50000, np.where(col == 1, 40000, 30000)).astype(np.uint16)
    out = D.debayer_buffer_new_ushort(mos, D.BAYER_RCD, D.RGGB)
    assert out.dtype == np.uint16
    for i, v in enumerate((50000, 40000, 30000)):
        assert np.abs(out[i].astype(int) - v).max() <= 1
    assert D._round_to(np.array([-3.0, 0.49, 0.5, 1.5, 65534.6, 70000.0], np.float32), 65535.0).tolist() == \
        [0, 0, 1, 2, 65535, 65535]
    assert D._round_to(np.array([254.4, 254.5, 300.0], np.float32), 255.0).tolist() == [254, 255, 255]


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 80), (37, 53), (9, 11)])
def test_rcd_ushort_gpu_bit_exact(pattern, shape):
    from siril_amd import demosaic
    mos = _mosaic16(*shape, pattern, seed=pattern)
    want = D.debayer_buffer_new_ushort(mos, D.BAYER_RCD, pattern)
    got = demosaic.debayer_buffer_new_ushort(mos, demosaic.BAYER_RCD, pattern)
    assert got is not None and got.dtype == np.uint16
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["1", "2", "0", "3"])
def test_rcd_ushort_variants_byte_depth_and_device(mode):
    """Every RCD variant on 16-bit data, the BYTE_IMG rounding (bit_depth 8,
    8-bit samples) and the device entry point on an int16 tensor; a constant
    16-bit frame is not an error (the 16-bit wrapper does not normalise)."""
    import os
    import torch
    from siril_amd import demosaic
    old = os.environ.get("SGPU_RCD_FUSED")
    os.environ["SGPU_RCD_FUSED"] = mode
    try:
        mos = _mosaic16(131, 517, 2, seed=3)
        assert np.array_equal(demosaic.debayer_buffer_new_ushort(mos, demosaic.BAYER_RCD, 2),
                              D.debayer_buffer_new_ushort(mos, D.BAYER_RCD, 2))
        m8 = _mosaic16(96, 128, 0, seed=4, top=255.0)
        assert np.array_equal(demosaic.debayer_buffer_new_ushort(m8, demosaic.BAYER_RCD, 0, bit_depth=8),
                              D.debayer_buffer_new_ushort(m8, D.BAYER_RCD, 0, bit_depth=8))
        dev = torch.from_numpy(mos.view(np.int16)).cuda()
        out = demosaic.debayer(dev, pattern=2)
        torch.cuda.synchronize()
        assert out.dtype == torch.int16
        assert np.array_equal(out.cpu().numpy().view(np.uint16), D.debayer_buffer_new_ushort(mos, D.BAYER_RCD, 2))
        flat = np.full((16, 16), 1234, np.uint16)
        got = demosaic.debayer_buffer_new_ushort(flat)
        assert got is not None and (got == 1234).all()
    finally:
        if old is None:
            os.environ.pop("SGPU_RCD_FUSED", None)
        else:
            os.environ["SGPU_RCD_FUSED"] = old


# ---- Siril's own bilinear decoder (demosaicing_siril.c:203-288) ----------

def _bilinear_closed_form(buf, tile, byte=False):
    """The per-pixel closed form the kernel computes (demosaic.hip
    k_bilinear_siril), in numpy: checked here against the literal walk."""
    h, w = buf.shape
    a = buf.astype(np.int64)
    out = np.zeros((3, h, w), np.int64)
    blue0 = -1 if tile in (1, 2) else 1
    swg0 = 1 if tile in (2, 3) else 0
    for y in range(1, h - 1):
        odd = (y - 1) & 1
        blue_row = (-blue0 if odd else blue0) > 0
        for x in range(1, w - 1):
            green = ((x - 1) & 1) == (0 if (swg0 ^ odd) else 1)
            c = a[y, x]
            if green:
                vert = (a[y - 1, x] + a[y + 1, x] + 1) >> 1
                horz = (a[y, x - 1] + a[y, x + 1] + 1) >> 1
                r, g, b = (vert, c, horz) if blue_row else (horz, c, vert)
            else:
                diag = (a[y - 1, x - 1] + a[y - 1, x + 1] + a[y + 1, x - 1] + a[y + 1, x + 1] + 2) >> 2
                cross = (a[y - 1, x] + a[y, x - 1] + a[y, x + 1] + a[y + 1, x] + 2) >> 2
                r, g, b = (diag, cross, c) if blue_row else (c, cross, diag)
            out[:, y, x] = (r, g, b)
    if byte:
        out = np.minimum(out, 255)
    return out.astype(np.uint16)


@pytest.mark.parametrize("tile", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(7, 9), (8, 10), (11, 6), (3, 3)])
def test_siril_bilinear_closed_form_equals_walk(tile, shape):
    rng = np.random.default_rng(tile * 10 + shape[0])
    buf = rng.integers(0, 65536, shape).astype(np.uint16)
    want = D.debayer_buffer_siril_ushort(buf, tile)
    assert np.array_equal(_bilinear_closed_form(buf, tile), want)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [0, 1, 2, 3])
@pytest.mark.parametrize("shape,depth", [((37, 53), 16), ((64, 80), 16), ((9, 11), 8), ((4, 5), 16)])
def test_siril_bilinear_gpu_bit_exact(tile, shape, depth):
    from siril_amd import demosaic
    rng = np.random.default_rng(tile + 7 * shape[1])
    buf = rng.integers(0, 65536 if depth == 16 else 300, shape).astype(np.uint16)
    want = D.debayer_buffer_siril_ushort(buf, tile, depth)
    got = demosaic.debayer_buffer_siril_ushort(buf, demosaic.BAYER_BILINEAR, tile, depth)
    assert got is not None and np.array_equal(got, want)
    assert demosaic.debayer_buffer_siril_ushort(buf, 8, tile, depth) is None     # only BAYER_BILINEAR


# ---- BAYER_BILINEAR: librtprocess bayerfast_demosaic (restated, unpinned) ----

def test_oracle_bayerfast_uniform_colours_exact():
    """A scene of one colour per CFA channel comes back exact in every plane
    (interior and 5-pixel border), every pattern, float and 16-bit wrappers."""
    for pattern in range(4):
        col = D.colour_map(30, 34, pattern)
        mos = np.array([300.0, 1000.0, 500.0], np.float32)[col]
        out = D.debayer_buffer_new_float(mos, D.BAYER_BILINEAR, pattern)
        for i, v in enumerate((300.0, 1000.0, 500.0)):
            assert np.abs(out[i] - v).max() < 1e-3, (pattern, i)
        o16 = D.debayer_buffer_new_ushort(mos.astype(np.uint16), D.BAYER_BILINEAR, pattern)
        for i, v in enumerate((300, 1000, 500)):
            assert (o16[i] == v).all(), (pattern, i)


def test_oracle_bayerfast_correlated_colour_reconstruction():
    """Smooth correlated colours: the colour-difference interpolation tracks
    them inside the border (a sanity property of the restatement)."""
    h, w = 64, 80
    yy, xx = np.mgrid[0:h, 0:w]
    L = 0.4 + 0.2 * np.cos(yy / 7.0) * np.sin(xx / 8.0)
    col = D.colour_map(h, w, D.GBRG)
    mos = np.where(col == 0, 1.2 * L, np.where(col == 1, L, 0.7 * L)).astype(np.float32)
    out = D.debayer_buffer_new_float(mos, D.BAYER_BILINEAR, D.GBRG)
    for i, k in enumerate((1.2, 1.0, 0.7)):
        assert np.abs(out[i] - k * L)[6:-6, 6:-6].max() < 1.5e-2


def test_oracle_bayerfast_native_samples_kept():
    """Inside the border every native sample passes through unchanged (up to
    the wrapper's normalisation round trip; exact in the 16-bit wrapper)."""
    rng = np.random.default_rng(2)
    mos = rng.integers(100, 60000, (33, 41)).astype(np.uint16)
    for pattern in range(4):
        out = D.debayer_buffer_new_ushort(mos, D.BAYER_BILINEAR, pattern)
        col = D.colour_map(*mos.shape, pattern)
        for c in range(3):
            m = col == c
            assert np.array_equal(out[c][m], mos[m]), (pattern, c)


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 80), (37, 53), (11, 12), (9, 7), (97, 131), (70, 130)])
def test_bayerfast_gpu_bit_exact(pattern, shape):
    """BAYER_BILINEAR through the reference-signature entry points (float and
    16-bit wrappers, 8- and 16-bit depth) == the restatement, bit for bit."""
    from siril_amd import demosaic
    mos = _mosaic(*shape, pattern, seed=10 + pattern)
    want = D.debayer_buffer_new_float(mos, D.BAYER_BILINEAR, pattern)
    got = demosaic.debayer_buffer_new_float(mos, demosaic.BAYER_BILINEAR, pattern)
    assert got is not None
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    m16 = np.clip(mos * 40.0, 0, 65535).astype(np.uint16)
    assert np.array_equal(demosaic.debayer_buffer_new_ushort(m16, demosaic.BAYER_BILINEAR, pattern),
                          D.debayer_buffer_new_ushort(m16, D.BAYER_BILINEAR, pattern))
    m8 = (mos % 256).astype(np.uint16)
    assert np.array_equal(demosaic.debayer_buffer_new_ushort(m8, demosaic.BAYER_BILINEAR, pattern, bit_depth=8),
                          D.debayer_buffer_new_ushort(m8, D.BAYER_BILINEAR, pattern, bit_depth=8))


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [0, 2])
def test_bayerfast_gpu_unaligned_output(pattern):
    """The site-pair kernel's per-pixel stores (k_bf_pairs, vec = 0): an even
    width with an output 4 bytes off the 8-byte pair alignment, float and
    16-bit (2 bytes off the 4-byte pair word), bit-exact vs the restatement."""
    import torch
    from siril_amd import demosaic
    h, w = 70, 130
    mos = _mosaic(h, w, pattern, seed=21) * 2.0
    want = D.debayer_buffer_new_float(mos, D.BAYER_BILINEAR, pattern)
    store = torch.empty(3 * h * w + 1, dtype=torch.float32, device="cuda")
    out = store[1:].view(3, h, w)
    assert out.data_ptr() % 8 == 4
    demosaic.debayer(torch.from_numpy(mos).cuda(), pattern=pattern, out=out,
                     interpolation=demosaic.BAYER_BILINEAR)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    m16 = np.clip(mos * 40.0, 0, 65535).astype(np.uint16)
    want16 = D.debayer_buffer_new_ushort(m16, D.BAYER_BILINEAR, pattern)
    store16 = torch.empty(3 * h * w + 1, dtype=torch.int16, device="cuda")
    out16 = store16[1:].view(3, h, w)
    assert out16.data_ptr() % 4 == 2
    demosaic.debayer(torch.from_numpy(m16.view(np.int16)).cuda(), pattern=pattern, out=out16,
                     interpolation=demosaic.BAYER_BILINEAR)
    torch.cuda.synchronize()
    assert np.array_equal(out16.cpu().numpy().view(np.uint16), want16)


@pytest.mark.gpu
def test_bayerfast_gpu_full_frame_and_device_api():
    """A 400 x 600 RGGB frame through the device entry (torch tensors, the
    path a colour SER sequence takes): bit-exact vs the restatement."""
    import torch
    from siril_amd import demosaic
    mos = _mosaic(600, 400, 0, seed=3) * 3.0
    want = D.debayer_buffer_new_float(mos, D.BAYER_BILINEAR, 0)
    out = demosaic.debayer(torch.from_numpy(mos).cuda(), pattern=0, interpolation=demosaic.BAYER_BILINEAR)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
