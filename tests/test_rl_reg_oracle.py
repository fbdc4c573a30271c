"""CPU checks of the RL regularisers restated in oracle/rl_ref.py
(deconvolve.hpp:104-126, 199-222) on images whose derivatives are known in
closed form.  Parity with the reference's own code is unpinned (Siril has no
test or vector for the regularisers); these pin the stencils' geometry."""
import numpy as np

from oracle import rl_ref as R


def _ramp(H, W, a=0.01, b=0.02):
    y, x = np.mgrid[0:H, 0:W]
    return (0.1 + a * x + b * y).astype(np.float32)


def test_tv_of_a_plane_is_zero_inside():
    w = _ramp(9, 11)
    for f in (R.reg_fft_tv, R.reg_naive_tv):
        out = f(w)
        # the unit gradient field is constant away from the last row/column
        assert np.allclose(out[1:-2, 1:-2], 0, atol=1e-5), f.__name__


def test_fft_tv_corner_uses_flat_indices():
    """divergence_img_expr_t (image_expr.hpp:882-884): (0, h-1) reads the
    unit field at flat indices h-1 and h-2, i.e. in row 0 when h <= w."""
    rng = np.random.default_rng(1)
    w = rng.random((5, 8)).astype(np.float32)
    H, W = w.shape
    dx = np.zeros_like(w)
    dx[:, :-1] = w[:, 1:] - w[:, :-1]
    dy = np.zeros_like(w)
    dy[:-1] = w[1:] - w[:-1]
    mag = np.hypot(dx, dy) + np.finfo(np.float32).eps
    gx, gy = (dx / mag).ravel(), (dy / mag).ravel()
    assert R.reg_fft_tv(w)[H - 1, 0] == np.float32(gx[H - 1] - gy[H - 2])
    # the img_t version reads the real column-0 neighbours
    assert R.reg_naive_tv(w)[H - 1, 0] != R.reg_fft_tv(w)[H - 1, 0]


def test_fh_of_a_quadratic():
    """w = c x^2 + d y^2 + e x y: gxx = 2c, gyy = 2d, gxy = e inside."""
    H, W = 10, 12
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    c, d, e = 0.002, 0.003, 0.001
    w = (c * x * x + d * y * y + e * x * y + 0.5).astype(np.float32)
    expect = np.sqrt((2 * c) ** 2 + (2 * d) ** 2 + 2 * e ** 2)
    fft = R.reg_fft_fh(w)
    naive, gxy = R.reg_naive_fh(w)
    assert np.allclose(fft[1:-1, 1:-1], expect, rtol=2e-3)
    assert np.allclose(naive[1:-1, 1:-1], expect, rtol=2e-3)
    assert np.allclose(gxy[:-1, :-1], e, rtol=2e-2)
    assert (gxy[-1] == 0).all() and (gxy[:, -1] == 0).all()


def test_naive_fh_clamps_negative_curvature():
    """max(1e-9f, g) before squaring (deconvolve.hpp:215-219): a concave
    surface has zero weight (up to 1e-9 terms), a convex one does not."""
    H, W = 8, 8
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    concave = (1 - 0.01 * (x * x + y * y)).astype(np.float32)
    w, _ = R.reg_naive_fh(concave)
    assert w[1:-1, 1:-1].max() < 1e-6        # only float rounding of gxy survives
    assert R.reg_fft_fh(concave)[1:-1, 1:-1].min() > 1e-3


def test_real_lambda():
    assert R.real_lambda(1.0 / 3000) == np.float32(1) / (np.float32(2) / np.float32(1.0 / 3000))
    assert abs(float(R.real_lambda(1.0 / 3000)) - 1.0 / 6000) < 1e-9
