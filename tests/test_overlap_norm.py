"""Overlap normalization (stack ... -overlap_norm, stacking/normalization.c
:296-938): the overlap rectangles, the per-pair estimators on the GPU, and the
least-squares coefficients, against oracle/overlap_ref.py.

Parity: the rectangles and sample counts are integer work (exact); median,
MAD and IKSS location are histogram order statistics (bit-exact, as for the
per-frame estimators in test_normalization.py); the IKSS scale is the sqrt
of a bwmv whose f64 sums the reference reduces in an OpenMP-order of its own,
so the float-cast scale is compared to relative 1e-6 (one float ulp).  The
coefficients come from the same LU algorithm in C++ and in the oracle
(relative 1e-12).  No reference test or fixture covers overlap normalization:
parity is pinned by the restatement only (GSL's LU is not vendored).
"""
import numpy as np
import pytest

from oracle import overlap_ref as OV
from siril_amd import normalization as N
from siril_amd.stacking import Normalization as NZ

SHIFTS = [(0.0, 0.0), (3.4, -2.6), (-7.5, 4.49), (12.0, 9.0), (-1.51, -11.2), (40.0, 0.0)]


def _frames(n, h, w, seed, u16=False, shifts=SHIFTS):
    """Registered-looking frames: a common sky shifted by integer offsets with
    zero fill outside, per-frame gain and pedestal, noise."""
    rng = np.random.default_rng(seed)
    my = 1 + max(abs(int(round(s[1]))) for s in shifts)
    mx = 1 + max(abs(int(round(s[0]))) for s in shifts)
    sky = 0.05 + 0.02 * rng.random((h + 2 * my, w + 2 * mx))
    out = np.zeros((n, h, w), np.float32)
    for f in range(n):
        dx, dy = (int(round(v)) for v in shifts[f % len(shifts)])
        img = sky[my + dy:my + dy + h, mx + dx:mx + dx + w] * (0.8 + 0.1 * f) + 0.01 * f
        img = img + rng.normal(0, 0.002, img.shape)
        # zero borders where the frame was shifted in (apply_reg's fill)
        if dx > 0:
            img[:, :dx] = 0
        elif dx < 0:
            img[:, dx:] = 0
        if dy > 0:
            img[:dy] = 0
        elif dy < 0:
            img[dy:] = 0
        out[f] = np.clip(img, 0, 1)
    if u16:
        return np.round(out * 65535.0).astype(np.uint16)
    return out


def _h(shifts, n):
    h02 = np.array([shifts[f % len(shifts)][0] for f in range(n)], np.float64)
    h12 = np.array([-shifts[f % len(shifts)][1] for f in range(n)], np.float64)
    return h02, h12


@pytest.mark.parametrize("dxi,dyi,dxj,dyj", [(0, 0, 0, 0), (0.4, 0.6, 3.5, -2.5), (-3.5, 2.5, 0, 0),
                                             (100.0, 0, 0, 0), (0, 0, -99.6, 48.5), (-0.5, -0.5, 0.5, 0.5),
                                             (2.49999, -7.50001, -1e9, 3e9)])
def test_overlap_rect_matches_reference_rule(dxi, dyi, dxj, dyj):
    """compute_overlap (normalization.c:420-456) through the C-ABI (host
    code, no GPU) vs the restatement."""
    got = N.overlap_rect(100, 50, dxi, dyi, dxj, dyj)
    exp = OV.compute_overlap(100, 50, dxi, dyi, dxj, dyj)
    assert got[2] == exp[2]
    if exp[2]:
        assert got[0] == exp[0] and got[1] == exp[1]


@pytest.mark.parametrize("normalize", [NZ.ADDITIVE, NZ.MULTIPLICATIVE, NZ.ADDITIVE_SCALING,
                                       NZ.MULTIPLICATIVE_SCALING, NZ.NO_NORM])
@pytest.mark.parametrize("lite", [False, True])
@pytest.mark.parametrize("ref", [0, 3])
def test_overlap_factors_match_oracle(normalize, lite, ref):
    """solve_overlap_coeffs + coefficient assembly (:296-355, :875-906) in the
    C-ABI (host code) vs the oracle, on a synthetic pair table with some pairs
    missing (Nij = 0)."""
    rng = np.random.default_rng(5 + ref)
    n = 6
    npairs = n * (n - 1) // 2
    nij = rng.integers(4, 50000, npairs).astype(np.int64)
    nij[[2, 7]] = 0
    tab = np.zeros((npairs, 8))
    tab[:, 0:2] = 0.05 + 0.02 * rng.random((npairs, 2))
    tab[:, 2:4] = 0.003 + 0.001 * rng.random((npairs, 2))
    tab[:, 4:6] = tab[:, 0:2] + 1e-4 * rng.random((npairs, 2))
    tab[:, 6:8] = tab[:, 2:4] * 1.48
    tab = tab.astype(np.float32).astype(np.float64)
    off, mul, scl = N.overlap_factors(normalize, N.OverlapStats(nij, tab), ref, lite)
    e_off, e_mul, e_scl = OV.overlap_factors(int(normalize), lite, nij, tab, ref)
    np.testing.assert_allclose(off, e_off, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(mul, e_mul, rtol=1e-12)
    np.testing.assert_allclose(scl, e_scl, rtol=1e-12)
    assert off[ref] == 0 and mul[ref] == 1 and scl[ref] == 1


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking as S
    c = S.Context(0)
    yield c
    c.close()


def _check_stats(got, exp_nij, exp_tab, lite):
    assert np.array_equal(got.nij, exp_nij)
    m = exp_nij > 0
    # median, MAD, location: bit-exact
    cols = [0, 1, 2, 3] if lite else [0, 1, 2, 3, 4, 5]
    assert np.array_equal(got.table[:, cols].view(np.uint64), exp_tab[:, cols].view(np.uint64))
    if not lite:
        np.testing.assert_allclose(got.table[m][:, 6:8], exp_tab[m][:, 6:8], rtol=1e-6)
    assert not got.table[~m].any()


@pytest.mark.gpu
@pytest.mark.parametrize("u16", [False, True])
@pytest.mark.parametrize("lite", [False, True])
def test_overlap_stats_gpu_matches_oracle(ctx, u16, lite):
    """_compute_estimators_for_images for every pair (k_overlap_pack + the
    STATS_NORM kernels) vs the restatement."""
    import torch
    n, h, w = 6, 72, 120
    fr = _frames(n, h, w, seed=3, u16=u16)
    h02, h12 = _h(SHIFTS, n)
    t = torch.from_numpy(fr.view(np.int16) if u16 else fr).cuda()
    got = N.overlap_stats_device(ctx, t, h02, h12, lite)
    exp_nij, exp_tab = OV.overlap_stats(fr, h02, h12, lite)
    _check_stats(got, exp_nij, exp_tab, lite)
    assert (got.nij > 0).sum() >= 10


@pytest.mark.gpu
def test_overlap_stats_gpu_sparse_pairs(ctx):
    """Pairs without overlap, with <= 3 common non-zero samples, and frames
    that are mostly zero."""
    import torch
    n, h, w = 5, 40, 64
    shifts = [(0.0, 0.0), (10.0, -3.0), (0.0, 4.0), (60.0, 0.0), (-70.0, 0.0)]
    rng = np.random.default_rng(9)
    fr = (0.05 + 0.01 * rng.random((n, h, w))).astype(np.float32)
    fr[1, 10:30, :] = 0           # a zero band: masked on both sides
    fr[2] = 0
    fr[2, 0, 0:3] = 0.1           # three samples: below the "> 3" bar
    # frame 3 overlaps the others on 4 columns, frame 4 on none
    h02, h12 = _h(shifts, n)
    got = N.overlap_stats_device(ctx, torch.from_numpy(fr).cuda(), h02, h12, False)
    exp_nij, exp_tab = OV.overlap_stats(fr, h02, h12, False)
    _check_stats(got, exp_nij, exp_tab, False)


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [NZ.ADDITIVE, NZ.MULTIPLICATIVE, NZ.ADDITIVE_SCALING,
                                       NZ.MULTIPLICATIVE_SCALING])
def test_overlap_normalization_end_to_end(ctx, normalize):
    """compute_normalization_overlaps on host frames: GPU estimators + C-ABI
    solve vs the oracle's estimators + restated solve."""
    n, h, w = 6, 64, 100
    fr = _frames(n, h, w, seed=21)
    h02, h12 = _h(SHIFTS, n)
    off, mul, scl, ost = N.compute_normalization_overlaps(ctx, fr, normalize, h02, h12, ref_index=1)
    exp_nij, exp_tab = OV.overlap_stats(fr, h02, h12, False)
    e_off, e_mul, e_scl = OV.overlap_factors(int(normalize), False, exp_nij, exp_tab, 1)
    np.testing.assert_allclose(off, e_off, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(mul, e_mul, rtol=1e-6)
    np.testing.assert_allclose(scl, e_scl, rtol=1e-6)
    # and the solve itself on the GPU's own table
    g_off, g_mul, g_scl = OV.overlap_factors(int(normalize), False, ost.nij, ost.table, 1)
    np.testing.assert_allclose(off, g_off, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(mul, g_mul, rtol=1e-12)
    np.testing.assert_allclose(scl, g_scl, rtol=1e-12)
