"""GPU parity of the NO_REJEC mean stack (stack_mean.hip) against the oracle.

Reference: mean_and_reject with NO_REJEC (stacking/median_and_mean.c:1083-1097,
float; :1020-1034, DATA_USHORT) after the null-sample compaction of
apply_rejection_float / _ushort (rejection_float.c:128-142,
median_and_mean.c:717-736).

Bar: bit-exact float32 / WORD output.  The float sums for kept >= 16 use
`#pragma omp simd reduction` in the reference, an order fixed by its build;
the kernel proves per pixel that the float result is the same in every order
or lists the pixel (sgpu_last_order_sensitive).  test_mean_order_guard checks
that proof against the oracle's L-lane model of the SIMD order
(oracle/stack_ref.c simd_sum_f, L = 2, 4, 8): every pixel whose float mean
differs between the orders must be listed.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking
    c = stacking.Context(0)
    yield c
    c.close()


def _args(**kw):
    from siril_amd import stacking as S
    return S.StackingArgs(S.Rejection(0), (3.0, 3.0), **kw)


def _frames(rng, n, h, w, zeros=0.02):
    fr = (0.05 + 0.005 * rng.standard_normal((n, h, w))).astype(np.float32)
    m = rng.random(fr.shape) < 0.03
    fr[m] += rng.uniform(0.2, 0.6, int(m.sum())).astype(np.float32)
    fr = np.clip(fr, 1e-6, 1).astype(np.float32)
    fr[rng.random(fr.shape) < zeros] = 0
    return fr


def _frames16(rng, n, h, w, zeros=0.02):
    fr = 1500 + 40 * rng.standard_normal((n, h, w))
    m = rng.random(fr.shape) < 0.03
    fr[m] += rng.uniform(3000, 20000, int(m.sum()))
    fr = np.clip(np.round(fr), 1, 65535).astype(np.uint16)
    fr[rng.random(fr.shape) < zeros] = 0
    return fr


def _eq(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32 if a.dtype == np.float32 else np.uint16),
                          np.asarray(b).view(np.uint32 if b.dtype == np.float32 else np.uint16))


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 15, 16, 17, 33, 100, 257])
@pytest.mark.parametrize("shape", [(24, 40), (7, 33)], ids=["vec", "ragged"])
def test_mean_block_parity(ctx, oracle, n, shape):
    """16-byte path (npix % 4 == 0) and the per-pixel path (ragged sizes),
    every unroll remainder, all-zero columns (exact kernel), kept < 16 and
    >= 16; with and without -output_norm."""
    rng = np.random.default_rng(500 + n + shape[0])
    h, w = shape
    fr = _frames(rng, n, h, w, zeros=0.3 if n < 4 else 0.02)
    fr[:, 1, 3] = 0.0                                    # kept == 0
    for onorm in (False, True):
        res = ctx.stack(fr, _args(output_norm=onorm))
        ref = oracle.stack_rows(fr, 0, (3.0, 3.0), output_norm=onorm, nthreads=8)[0]
        assert _eq(res.result, ref), (n, shape, onorm)


@pytest.mark.parametrize("norm", [1, 2, 3, 4])
@pytest.mark.parametrize("n", [9, 40, 100])
def test_mean_norm_weights_shift(ctx, oracle, norm, n):
    """-norm= affines (vec path), frame weights (weighted branch
    :1043-1082) and registration shifts (per-pixel path)."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(800 + 10 * norm + n)
    fr = _frames(rng, n, 16, 48)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.01 * rng.standard_normal(n)
    mul = 1.0 + 0.03 * rng.standard_normal(n)
    weights = rng.uniform(0.5, 1.5, n)
    dx = rng.uniform(-3, 3, n)
    for use_w, shift in ((False, False), (True, False), (False, True), (True, True)):
        kw = dict(shiftx=S.shifts_from_registration(dx)) if shift else {}
        args = _args(normalize=S.Normalization(norm), scale=scale, offset=offset, mul=mul,
                     weights=weights if use_w else None, **kw)
        res = ctx.stack(fr, args)
        ref = oracle.stack_rows(fr, 0, (3.0, 3.0), norm=norm, scale=scale, offset=offset, mul=mul,
                                weights=weights if use_w else None, shift_dx=dx if shift else None, nthreads=8)[0]
        assert _eq(res.result, ref), (norm, n, use_w, shift)


def _stress(rng, n, cols):
    """Columns whose f64 sums are not exact in f64: negatives (an additive
    offset past the level), 1e-20 and 1e6 scales in one column, near-mean
    ties, zeros."""
    kind = rng.integers(0, 4, cols)
    lvl = np.where(kind == 0, 1e-3, np.where(kind == 1, 0.05, np.where(kind == 2, 1e-20, 3.0)))
    x = lvl[None, :] + 0.1 * lvl[None, :] * rng.standard_normal((n, cols))
    x -= np.where(kind == 0, 1.1e-3, 0.0)[None, :]
    big = rng.random(x.shape) < 0.01
    x[big] *= 1e7
    tiny = rng.random(x.shape) < 0.01
    x[tiny] *= 1e-12
    x = x.astype(np.float32)
    x[rng.random(x.shape) < 0.01] = 0
    return x


@pytest.mark.parametrize("n", [16, 24, 100])
def test_mean_order_guard(ctx, oracle, n):
    """Sum-order guard of the streaming mean: on 256 K stress columns the GPU
    equals the sequential oracle everywhere, and every pixel whose float mean
    differs between the sequential order and an L-lane SIMD order (L = 2, 4,
    8) is in the kernel's order-sensitive list; unlisted pixels equal every
    model order."""
    rng = np.random.default_rng(9100 + n)
    w = 4096
    fr = _stress(rng, n, 64 * w).reshape(n, 64, w)
    res = ctx.stack(fr, _args(output_norm=True))
    cnt, idx = ctx.last_order_sensitive(with_indices=True)
    listed = np.zeros(fr[0].size, bool)
    listed[idx] = True
    seq = oracle.stack_rows(fr, 0, (3.0, 3.0), output_norm=True, nthreads=16)[0]
    assert _eq(res.result, seq)
    diff_total = 0
    try:
        for lanes in (2, 4, 8):
            oracle.set_simd_lanes(lanes)
            lan = oracle.stack_rows(fr, 0, (3.0, 3.0), output_norm=True, nthreads=16)[0]
            diff = (lan.view(np.uint32) != seq.view(np.uint32)).ravel()
            diff_total += int(diff.sum())
            assert not (diff & ~listed).any(), f"L={lanes}: {int((diff & ~listed).sum())} unlisted order-dependent"
    finally:
        oracle.set_simd_lanes(0)
    print(f"mean order guard N={n}: {cnt} listed of {fr[0].size}, {diff_total} order-dependent under L=2/4/8")
    assert cnt < fr[0].size // 4


def test_mean_guard_quiet_on_siril_range(ctx, oracle):
    """Data in Siril's [0, 1] float range with a few binades of spread: every
    f64 sum is exact, no pixel is listed."""
    rng = np.random.default_rng(3)
    fr = _frames(rng, 100, 64, 256)
    res = ctx.stack(fr, _args())
    assert ctx.last_order_sensitive() == 0
    assert _eq(res.result, oracle.stack_rows(fr, 0, (3.0, 3.0), nthreads=8)[0])


@pytest.mark.parametrize("n", [3, 8, 16, 100])
@pytest.mark.parametrize("shape", [(12, 40), (5, 27)], ids=["vec", "ragged"])
def test_mean_u16(ctx, oracle, n, shape):
    """DATA_USHORT mean on the streaming kernel (integer sums): float and
    16-bit output, -norm= (round_to_WORD in the gather), weights, shifts."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(700 + n + shape[1])
    fr = _frames16(rng, n, *shape)
    fr[:, 2, 3] = 0
    for out32 in (True, False):
        res = ctx.stack(fr, _args(), use_32bit_output=out32)
        ref = oracle.stack_rows_u16(fr, 0, (3.0, 3.0), use_32bit_output=out32, nthreads=8)[0]
        assert _eq(res.result, ref), (n, shape, out32)
        assert ctx.last_exact_pixels() <= 1
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 60 * rng.standard_normal(n)
    mul = 1.0 + 0.03 * rng.standard_normal(n)
    weights = rng.uniform(0.5, 1.5, n)
    dx = rng.uniform(-3, 3, n)
    for norm, use_w, shift in ((3, False, False), (1, True, False), (4, False, True), (2, True, True)):
        kw = dict(shiftx=S.shifts_from_registration(dx)) if shift else {}
        args = _args(normalize=S.Normalization(norm), scale=scale, offset=offset, mul=mul,
                     weights=weights if use_w else None, **kw)
        res = ctx.stack(fr, args, use_32bit_output=False)
        ref = oracle.stack_rows_u16(fr, 0, (3.0, 3.0), norm=norm, scale=scale, offset=offset, mul=mul,
                                    weights=weights if use_w else None, shift_dx=dx if shift else None,
                                    use_32bit_output=False, nthreads=8)[0]
        assert _eq(res.result, ref), (n, shape, norm, use_w, shift)


@pytest.mark.parametrize("u16", [False, True], ids=["f32", "u16"])
def test_mean100_full_frame(ctx, oracle, u16):
    """mean100 at its bench size (100 x 6000 x 4000, synthetic recipe in HBM):
    every pixel bit for bit against the oracle, and on this recipe no pixel is
    order-sensitive."""
    import torch
    from siril_amd import stacking as S, synth
    h, w = 4000, 6000
    fr = synth.frames_torch(100, h, w, "cuda", seed=78)
    if u16:
        fr = torch.round(fr * 65535.0).to(torch.int32).to(torch.int16)
    out, _, _, _ = ctx.stack_device(fr, _args(), S.METHOD_MEAN)
    torch.cuda.synchronize()
    if not u16:
        assert ctx.last_order_sensitive() == 0
    got = out.cpu().numpy()
    host = fr.cpu().numpy()
    del fr, out
    torch.cuda.empty_cache()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    if u16:
        ref = oracle.stack_rows_u16(host.view(np.uint16), 0, (3.0, 3.0), nthreads=threads)[0]
    else:
        ref = oracle.stack_rows(host, 0, (3.0, 3.0), nthreads=threads)[0]
    assert _eq(got, ref)
