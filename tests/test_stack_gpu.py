"""GPU parity: libsirilgpu.so (HIP, gfx950) against the CPU restatement of
Siril's per-pixel stack (oracle/), through the C-ABI.

Bar: bit-exact float32 output and identical per-pixel rejection counts for
every rejection type, the median and the plain mean.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TYPES = [0, 1, 2, 3, 4, 5, 6, 7]


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking
    c = stacking.Context(0)
    yield c
    c.close()


def _args(rt, sig, **kw):
    from siril_amd import stacking as S
    return S.StackingArgs(S.Rejection(rt), sig, **kw)


def _frames(rng, n, h, w, zeros=0.02, outliers=0.03, wild=0.0):
    fr = (0.05 + 0.005 * rng.standard_normal((n, h, w))).astype(np.float32)
    m = rng.random(fr.shape) < outliers
    fr[m] += rng.uniform(0.2, 0.6, int(m.sum())).astype(np.float32)
    if wild:
        m = rng.random(fr.shape) < wild
        fr[m] = rng.uniform(0, 1, int(m.sum())).astype(np.float32)
    fr = np.clip(fr, 1e-6, 1).astype(np.float32)
    fr[rng.random(fr.shape) < zeros] = 0
    return fr


def _check(res, ref, method=0):
    out, rl, rh, counts = ref
    assert np.array_equal(res.result.view(np.uint32), out.view(np.uint32)), \
        f"{int((res.result != out).sum())} pixels differ"
    if method == 0:
        assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)
        assert tuple(res.irej) == (int(counts[0]), int(counts[1]))


def test_golden_columns(ctx, oracle):
    """Every committed golden vector, as pixels of small frame blocks."""
    import os
    from siril_amd import stacking as S
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "columns.npz"))
    groups = {}
    for i in range(len(g["n"])):
        key = (int(g["rtype"][i]), tuple(float(s) for s in g["sig"][i]), int(g["n"][i]))
        groups.setdefault(key, []).append(i)
    for (rt, sig, n), idx in groups.items():
        cols = g["cols"][idx, :n]                         # [k, n]
        frames = np.ascontiguousarray(cols.T[:, None, :])  # [n, 1, k]
        method = 1 if rt == 16 else 0
        args = S.StackingArgs(S.Rejection(0 if rt == 16 else rt), sig)
        res = ctx.stack(frames, args, method)
        exp = np.clip(g["expect"][idx], 0, 1).astype(np.float32)
        assert np.array_equal(res.result[0].view(np.uint32), exp.view(np.uint32)), (rt, sig, n)
        if method == 0:
            assert np.array_equal(res.rejmap_low[0], g["rej"][idx, 0]), (rt, sig, n)
            assert np.array_equal(res.rejmap_high[0], g["rej"][idx, 1]), (rt, sig, n)


@pytest.mark.parametrize("exact", [False, True])
def test_rejection_kats_hip(ctx, oracle, exact):
    """The reference's own known answers (src/tests/rejection_test.c:96-230:
    GESDT and PERCENTILE on set1, LINEARFIT on set2) through the HIP path:
    every pixel of a 2x32 block holds the KAT column (frame f = sample f), the
    sorted kernels (exact=False) and the sequential kernel (exact=True) must
    give the published rejection counts and mean.  -output_norm keeps the
    set1 means (> 1) unclamped (median_and_mean.c:1725-1727)."""
    import json
    import os
    kats = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rejection_kats.json")))
    ctx.set_exact_only(exact)
    try:
        for case in kats["cases"]:
            col = np.array(kats[case["set"]], np.float32)
            fr = np.ascontiguousarray(np.broadcast_to(col[:, None, None], (len(col), 2, 32)))
            args = _args(case["rejection"], tuple(case["sig"]), output_norm=True)
            res = ctx.stack(fr, args)
            assert (res.rejmap_low == case["rej"][0]).all() and (res.rejmap_high == case["rej"][1]).all(), case["name"]
            m = np.float32(case["mean"])
            assert (np.abs(res.result - m) <= case["tol"] * max(1.0, abs(case["mean"]))).all(), case["name"]
            out, _, _, _ = oracle.stack_rows(fr, case["rejection"], tuple(case["sig"]), output_norm=True, nthreads=2)
            assert np.array_equal(res.result.view(np.uint32), out.view(np.uint32)), case["name"]
    finally:
        ctx.set_exact_only(False)


@pytest.mark.parametrize("n", [2, 3, 5, 8, 9, 10, 16, 17, 24, 33, 64, 65, 100, 128, 129, 256, 400])
@pytest.mark.parametrize("rt", TYPES)
def test_block_parity(ctx, oracle, rt, n):
    if rt == 7 and n < 3:
        pytest.skip("GESDT needs 3 frames (median_and_mean.c:1281)")
    rng = np.random.default_rng(1000 * rt + n)
    h, w = (24, 40) if n <= 128 else (8, 40)
    fr = _frames(rng, n, h, w, wild=0.05 if n < 20 else 0.0)
    sig = (0.32, 0.05) if rt == 7 else ((0.2, 0.1) if rt == 1 else (3.0, 3.0))
    res = ctx.stack(fr, _args(rt, sig))
    ref = oracle.stack_rows(fr, rt, sig, nthreads=8)
    _check(res, ref)


def _stress_frames(rng, n, cols):
    """Columns whose f64 sums are NOT exact: normalized-looking data with
    negative values (additive offset larger than the level), many samples
    within a few ulp of the mean (tiny d^2 next to large ones), tiny values
    (~1e-20) and wide binade spans, plus the usual outliers and zeros."""
    kind = rng.integers(0, 4, cols)
    lvl = np.where(kind == 0, 1e-3, np.where(kind == 1, 0.05, np.where(kind == 2, 1e-20, 3.0)))
    spread = np.where(kind == 3, 1e-6, 0.1) * lvl                       # kind 3: near-mean ties
    x = lvl[None, :] + spread[None, :] * rng.standard_normal((n, cols))
    x -= np.where(kind == 0, 1.1e-3, 0.0)[None, :]                      # negatives around 0
    m = rng.random(x.shape) < 0.04
    x[m] += (rng.uniform(2, 8, int(m.sum())) * np.broadcast_to(np.abs(lvl)[None, :], x.shape)[m])
    big = rng.random(x.shape) < 0.002
    x[big] *= 1e6                                                         # wide binade span
    x = x.astype(np.float32)
    x[rng.random(x.shape) < 0.01] = 0
    return x


@pytest.mark.parametrize("n,rt", [(12, 5), (24, 2), (100, 5), (100, 2), (400, 5), (200, 2), (400, 2)])
def test_sum_order_stress(ctx, oracle, n, rt):
    """Sum-order guard (stack_sorted_impl.h, SumGuard): on columns whose f64
    sums are inexact the sorted path must either prove the float results
    order-independent or defer the pixel to the sequential kernel: 0
    mismatches against the oracle on >= 1 M columns (256 K at N = 400), with
    -output_norm (no clamp, so negative and large means are compared too).
    The deferral rate is printed."""
    rng = np.random.default_rng(4242 + n + rt)
    total = 1 << 20 if n < 400 else 1 << 18
    w = 4096
    bad = 0
    deferred = 0
    for r0 in range(0, total // w, 64):
        fr = _stress_frames(rng, n, 64 * w).reshape(n, 64, w)
        args = _args(rt, (3.0, 3.0), output_norm=True)
        res = ctx.stack(fr, args)
        deferred += ctx.last_exact_pixels()
        out, rl, rh, _ = oracle.stack_rows(fr, rt, (3.0, 3.0), output_norm=True, nthreads=16)
        bad += int((res.result.view(np.uint32) != out.view(np.uint32)).sum())
        bad += int((res.rejmap_low != rl).sum() + (res.rejmap_high != rh).sum())
    print(f"sum-order stress N={n} rt={rt}: {total} columns, {deferred} deferred "
          f"({100.0 * deferred / total:.3f} %), {bad} mismatches")
    assert bad == 0


@pytest.mark.parametrize("rt", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("sig", [(1.0, 1.0), (2.0, 1.5), (0.5, 0.5)])
def test_aggressive_sigma_cutoff(ctx, oracle, rt, sig):
    """Low sigmas make the order-dependent `N - r <= 4` cutoff fire often:
    those pixels must come out of the exact kernel with Siril's result."""
    rng = np.random.default_rng(7)
    for n in (6, 12, 20, 100):
        fr = _frames(rng, n, 16, 32, wild=0.2)
        res = ctx.stack(fr, _args(rt, sig))
        _check(res, oracle.stack_rows(fr, rt, sig, nthreads=8))


@pytest.mark.parametrize("n", [5, 12, 33, 100, 300])
def test_mad_quantized_ties(ctx, oracle, n):
    """MAD on the sorted path: quantized samples (many equal |x - median|,
    columns whose deviations are all equal, constant columns) exercise the
    histogram-interpolated percentile's tie and hi == lo branches."""
    rng = np.random.default_rng(300 + n)
    h, w = (16, 48) if n <= 128 else (6, 40)
    fr = _frames(rng, n, h, w, wild=0.1)
    fr = (np.round(fr * 64) / 64).astype(np.float32)         # heavy ties
    fr[:, 0, :8] = np.float32(0.25)                           # constant columns
    fr[:, 1, :8] = np.where(np.arange(n)[:, None] % 2 == 0, 0.25, 0.5).astype(np.float32)
    for sig in ((3.0, 3.0), (1.0, 1.0), (0.5, 2.0)):
        res = ctx.stack(fr, _args(3, sig))
        _check(res, oracle.stack_rows(fr, 3, sig, nthreads=8))
    assert ctx.last_exact_pixels() < fr.shape[1] * fr.shape[2]   # not all deferred


@pytest.mark.parametrize("n", [4, 9, 10, 100, 257])
def test_median_stack(ctx, oracle, n):
    from siril_amd import stacking as S
    rng = np.random.default_rng(n)
    fr = _frames(rng, n, 20, 36, zeros=0.1)
    res = ctx.stack(fr, S.StackingArgs(), S.METHOD_MEDIAN)
    _check(res, oracle.stack_rows(fr, 0, (3, 3), method=1, nthreads=8), method=1)


def test_normalization_shift_weights(ctx, oracle):
    from siril_amd import stacking as S
    rng = np.random.default_rng(11)
    n = 30
    fr = _frames(rng, n, 20, 50)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.01 * rng.standard_normal(n)
    mul = 1.0 + 0.03 * rng.standard_normal(n)
    dx = rng.uniform(-6, 6, n)
    shiftx = S.shifts_from_registration(dx)
    weights = rng.uniform(0.5, 2.0, n)
    for norm in (1, 2, 3, 4):
        for rt in (0, 2, 5, 6):
            args = S.StackingArgs(S.Rejection(rt), (2.5, 2.5), S.Normalization(norm), scale=scale,
                                  offset=offset, mul=mul, shiftx=shiftx)
            res = ctx.stack(fr, args)
            ref = oracle.stack_rows(fr, rt, (2.5, 2.5), norm=norm, scale=scale, offset=offset, mul=mul,
                                    shift_dx=dx, nthreads=8)
            _check(res, ref)
    for rt in (0, 2, 5):
        args = S.StackingArgs(S.Rejection(rt), (2.5, 2.5), weights=weights)
        _check(ctx.stack(fr, args), oracle.stack_rows(fr, rt, (2.5, 2.5), weights=weights, nthreads=8))


def test_nan_inf_and_empty_columns(ctx, oracle):
    rng = np.random.default_rng(5)
    n = 20
    fr = _frames(rng, n, 8, 16)
    fr[:, 0, 0] = 0.0                 # all missing
    fr[3, 0, 1] = np.nan
    fr[4, 0, 2] = np.inf
    fr[:, 0, 3] = 0.25                # constant
    fr[:n - 1, 0, 4] = 0.0            # one survivor
    fr[:, 0, 5] = -0.0
    for rt in TYPES:
        sig = (0.32, 0.05) if rt == 7 else (3.0, 3.0)
        res = ctx.stack(fr, _args(rt, sig))
        out, rl, rh, counts = oracle.stack_rows(fr, rt, sig, nthreads=4)
        assert np.array_equal(res.result.view(np.uint32), out.view(np.uint32)), rt
        assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh), rt


def test_output_norm_keeps_range(ctx, oracle):
    rng = np.random.default_rng(9)
    fr = (1.5 + 0.1 * rng.standard_normal((12, 10, 10))).astype(np.float32)
    res = ctx.stack(fr, _args(5, (3, 3), output_norm=True))
    _check(res, oracle.stack_rows(fr, 5, (3, 3), output_norm=True, nthreads=4))
    res2 = ctx.stack(fr, _args(5, (3, 3)))
    assert float(res2.result.max()) == 1.0


def test_exact_only_mode_agrees(ctx, oracle):
    rng = np.random.default_rng(21)
    fr = _frames(rng, 40, 16, 24, wild=0.05)
    for rt in (2, 5):
        fast = ctx.stack(fr, _args(rt, (2.0, 2.0)))
        ctx.set_exact_only(True)
        try:
            exact = ctx.stack(fr, _args(rt, (2.0, 2.0)))
            assert exact.exact_pixels == 16 * 24
        finally:
            ctx.set_exact_only(False)
        assert np.array_equal(fast.result.view(np.uint32), exact.result.view(np.uint32))
        assert np.array_equal(fast.rejmap_low, exact.rejmap_low)


def test_device_api_matches_host_api(ctx):
    import torch
    from siril_amd import stacking as S
    rng = np.random.default_rng(2)
    fr = _frames(rng, 100, 32, 64)
    host = ctx.stack(fr, _args(5, (3, 3)))
    d = torch.from_numpy(fr).cuda()
    rl = torch.zeros((32, 64), dtype=torch.int16, device="cuda")
    rh = torch.zeros_like(rl)
    out, _, _, counts = ctx.stack_device(d, _args(5, (3, 3)), S.METHOD_MEAN, rej_lo=rl, rej_hi=rh)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), host.result.view(np.uint32))
    assert np.array_equal(rl.cpu().numpy().view(np.uint16), host.rejmap_low)
    assert tuple(counts.cpu().tolist()) == host.irej


def test_device_api_orders_with_the_null_stream(ctx):
    """torch's default stream is the null stream (handle 0): work queued there
    right before the call (the counters' zero-fill, a frame copy) must be
    ordered before the stack, and the counters must accumulate over calls."""
    import torch
    from siril_amd import stacking as S
    rng = np.random.default_rng(3)
    fr = _frames(rng, 100, 64, 256)
    host = ctx.stack(fr, _args(5, (3, 3)))
    src = torch.from_numpy(fr).cuda()
    d = torch.empty_like(src)
    assert torch.cuda.current_stream().cuda_stream == 0
    for _ in range(3):
        d.copy_(src)                                    # null-stream copy, no sync
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        for _ in range(4):
            ctx.stack_device(d, _args(5, (3, 3)), S.METHOD_MEAN, counts=counts)
        torch.cuda.synchronize()
        assert tuple(counts.cpu().tolist()) == tuple(4 * x for x in host.irej)


@pytest.mark.parametrize("n,rt", [(100, 5), (400, 2)], ids=["config2_winsorized100", "config4_sigma400"])
def test_full_frame_parity(ctx, oracle, n, rt):
    """BASELINE configs 2 and 4 at full size on one GPU (100 x 6000 x 4000
    Winsorized 3/3; 400 x 6000 x 4000 = 38.4 GB sigma 3/3, the NP = 512
    kernel at its real launch shape), synthetic in HBM: EVERY pixel of the
    GPU image, both rejection maps and the totals are compared bit for bit
    with the oracle's stack of the same frames (16 OpenMP threads on the
    box: about 5 s for config 2, 13 s for config 4)."""
    import torch
    from siril_amd import stacking as S, synth
    h, w = 4000, 6000
    fr = synth.frames_torch(n, h, w, "cuda", seed=77)
    rl = torch.zeros((h, w), dtype=torch.int16, device="cuda")
    rh = torch.zeros_like(rl)
    out, _, _, counts = ctx.stack_device(fr, _args(rt, (3, 3)), S.METHOD_MEAN, rej_lo=rl, rej_hi=rh)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    got_rl = rl.cpu().numpy().view(np.uint16)
    got_rh = rh.cpu().numpy().view(np.uint16)
    got_counts = tuple(counts.cpu().tolist())
    host = fr.cpu().numpy()
    del fr, out, rl, rh
    torch.cuda.empty_cache()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    ref_out, ref_rl, ref_rh, ref_counts = oracle.stack_rows(host, rt, (3, 3), nthreads=threads)
    del host
    bad = int(np.count_nonzero(got.view(np.uint32) != ref_out.view(np.uint32)))
    assert bad == 0, f"{bad} of {h * w} pixels differ"
    assert np.array_equal(got_rl, ref_rl) and np.array_equal(got_rh, ref_rh)
    assert got_counts == (int(ref_counts[0]), int(ref_counts[1]))


def _frames16(rng, n, h, w, zeros=0.02):
    fr = (1500 + 40 * rng.standard_normal((n, h, w)))
    m = rng.random(fr.shape) < 0.03
    fr[m] += rng.uniform(3000, 20000, int(m.sum()))
    fr = np.clip(np.round(fr), 1, 65535).astype(np.uint16)
    fr[rng.random(fr.shape) < zeros] = 0
    return fr


@pytest.mark.parametrize("n", [3, 8, 9, 10, 24, 100])
@pytest.mark.parametrize("rt", TYPES)
def test_u16_parity(ctx, oracle, rt, n):
    """DATA_USHORT path (apply_rejection_ushort) against the 16-bit oracle,
    both output modes."""
    rng = np.random.default_rng(77 * rt + n)
    fr = _frames16(rng, n, 12, 20)
    sig = (0.32, 0.05) if rt == 7 else ((0.2, 0.1) if rt == 1 else (2.5, 2.5))
    for out32 in (True, False):
        res = ctx.stack(fr, _args(rt, sig), use_32bit_output=out32)
        out, rl, rh, counts = oracle.stack_rows_u16(fr, rt, sig, use_32bit_output=out32, nthreads=8)
        assert res.result.dtype == out.dtype
        assert np.array_equal(res.result.view(np.uint16 if not out32 else np.uint32),
                              out.view(np.uint16 if not out32 else np.uint32)), (rt, n, out32)
        assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)
        assert tuple(res.irej) == (int(counts[0]), int(counts[1]))


def test_u16_median_norm_shift(ctx, oracle):
    from siril_amd import stacking as S
    rng = np.random.default_rng(4)
    n = 16
    fr = _frames16(rng, n, 10, 30)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 20 * rng.standard_normal(n)
    mul = 1.0 + 0.03 * rng.standard_normal(n)
    dx = rng.uniform(-4, 4, n)
    res = ctx.stack(fr, S.StackingArgs(), S.METHOD_MEDIAN)
    _check(res, oracle.stack_rows_u16(fr, 0, (3, 3), method=1, nthreads=4), method=1)
    for norm in (1, 4):
        args = S.StackingArgs(S.Rejection.SIGMA, (2.5, 2.5), S.Normalization(norm), scale=scale,
                              offset=offset, mul=mul, shiftx=S.shifts_from_registration(dx))
        _check(ctx.stack(fr, args), oracle.stack_rows_u16(fr, 2, (2.5, 2.5), norm=norm, scale=scale,
                                                          offset=offset, mul=mul, shift_dx=dx, nthreads=4))


def test_u16_median_sorting_pin(ctx, oracle):
    """The reference's Sorting/Median property (src/tests/sorting.c:45-98:
    quickmedian(WORD) == median of a quicksort, sizes 1..400, rand() %
    USHRT_MAX data) through the 16-bit HIP median stack: every pixel of a
    block is one such column; the result must be the sort median in both
    output modes (double_ushort_to_float_range for 32-bit, round_to_WORD for
    16-bit) and bit-equal to the oracle."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(59)
    for n in list(range(1, 41)) + list(range(41, 401, 7)) + [400]:
        fr = rng.integers(0, 65535, (n, 2, 64)).astype(np.uint16)
        if n % 3 == 0:   # ties: the histogram walk / Lomuto over repeated values
            fr[:, 1, :] = rng.choice(np.array([0, 1, 65534, 65535], np.uint16), (n, 64))
        s = np.sort(fr, axis=0).astype(np.int64)
        med = np.where(n % 2 == 1, s[(n - 1) // 2], (s[(n - 1) // 2] + s[n // 2]) / 2.0).astype(np.float64)
        for out32 in (True, False):
            res = ctx.stack(fr, S.StackingArgs(), S.METHOD_MEDIAN, use_32bit_output=out32)
            out, _, _, _ = oracle.stack_rows_u16(fr, 0, (3, 3), method=1, use_32bit_output=out32, nthreads=4)
            if out32:
                expect = np.clip(med.astype(np.float32) * np.float32(.000015259022), 0, 1).astype(np.float32)
                assert np.array_equal(res.result.view(np.uint32), expect.view(np.uint32)), n
                assert np.array_equal(res.result.view(np.uint32), out.view(np.uint32)), n
            else:
                assert np.array_equal(res.result, np.floor(med + 0.5).astype(np.uint16)), n
                assert np.array_equal(res.result, out), n


@pytest.mark.parametrize("n", [9, 40, 100, 300])
@pytest.mark.parametrize("rt", [1, 2, 3, 4, 5, 6, 7, 16])
def test_u16_normalized_weighted_sorted_path(ctx, oracle, rt, n):
    """16-bit stacks with -norm= (round_to_WORD of the affine in the 16-bit
    gather, median_and_mean.c:1665-1684), frame weights and registration
    shifts on the 16-bit sorted kernels: bit for bit against the oracle, and
    the sorted path (not the sequential kernel) must answer most pixels."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(3000 + 10 * rt + n)
    fr = _frames16(rng, n, 16, 48)
    sig = {1: (0.2, 0.1), 5: (3.0, 3.0), 7: (0.3, 0.05)}.get(rt, (2.5, 2.5))
    method = 1 if rt == 16 else 0
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 60 * rng.standard_normal(n)
    mul = 1.0 + 0.03 * rng.standard_normal(n)
    weights = rng.uniform(0.5, 1.5, n)
    dx = rng.uniform(-3, 3, n)
    for norm, use_w, shift in ((3, False, False), (1, True, False), (4, False, True), (2, True, True)):
        kw = dict(shiftx=S.shifts_from_registration(dx)) if shift else {}
        args = S.StackingArgs(S.Rejection(0 if rt == 16 else rt), sig, S.Normalization(norm), scale=scale,
                              offset=offset, mul=mul, weights=weights if use_w else None, **kw)
        res = ctx.stack(fr, args, method, use_32bit_output=False)
        deferred = ctx.last_exact_pixels()
        out, rl, rh, counts = oracle.stack_rows_u16(
            fr, 0 if rt == 16 else rt, sig, method=method, norm=norm, scale=scale, offset=offset, mul=mul,
            weights=weights if use_w and method == 0 else None, shift_dx=dx if shift else None,
            use_32bit_output=False, nthreads=8)
        assert np.array_equal(res.result, out), (rt, n, norm, use_w, shift)
        if method == 0:
            assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)
            assert tuple(res.irej) == (int(counts[0]), int(counts[1]))
        if n <= 128 or rt not in (6, 7):
            assert deferred < fr[0].size // 2, (rt, n, norm, deferred)


@pytest.mark.parametrize("n", [5, 33, 65, 100, 129, 300])
@pytest.mark.parametrize("rt", [1, 2, 3, 4, 5, 6, 7, 16])
def test_u16_sorted_path(ctx, oracle, rt, n):
    """16-bit rejection stacks and the median on the sorted path (no
    normalization; with and without registration shifts) against the 16-bit
    oracle, bit for bit, and most pixels must not have been deferred to the
    exact kernel (LINEARFIT / GESDT: sorted path up to N = 128)."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(1000 * rt + n)
    fr = _frames16(rng, n, 24, 40)
    sig = {1: (0.2, 0.1), 5: (3.0, 3.0), 7: (0.3, 0.05)}.get(rt, (2.5, 2.5))
    method = 1 if rt == 16 else 0
    dx = rng.uniform(-5, 5, n)
    for shift in (False, True):
        kw = dict(shiftx=S.shifts_from_registration(dx)) if shift else {}
        args = S.StackingArgs(S.Rejection(0 if rt == 16 else rt), sig, **kw)
        for out32 in (True, False):
            res = ctx.stack(fr, args, method, use_32bit_output=out32)
            ok = dict(shift_dx=dx) if shift else {}
            out, rl, rh, counts = oracle.stack_rows_u16(fr, 0 if rt == 16 else rt, sig, method=method,
                                                        use_32bit_output=out32, nthreads=8, **ok)
            assert np.array_equal(res.result.view(np.uint16 if not out32 else np.uint32),
                                  out.view(np.uint16 if not out32 else np.uint32)), (rt, n, shift, out32)
            if method == 0:
                assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)
                assert tuple(res.irej) == (int(counts[0]), int(counts[1]))
        if not (rt in (6, 7) and n > 128):
            assert ctx.last_exact_pixels() < fr.shape[1] * fr.shape[2] // 2, "16-bit sorted path not used"


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("rt", [2, 5])
def test_multi_device_entry(oracle, devices, rt):
    """sgpu_multi_stack_rows: the C-ABI multi-device entry (row bands, one
    host thread and context per device, host gather); on a one-GPU box the
    contexts share device 0, which still exercises the band split, the
    concurrent band stacks and the gather.  Bit-exact vs the oracle."""
    from siril_amd.stacking import MultiContext
    rng = np.random.default_rng(40 + rt + len(devices))
    fr = _frames(rng, 30, 37, 45)
    m = MultiContext(devices)
    res = m.stack(fr, _args(rt, (3.0, 3.0)))
    _check(res, oracle.stack_rows(fr, rt, (3.0, 3.0), nthreads=8))
    fr16 = np.clip(np.round(fr * 65535.0), 0, 65535).astype(np.uint16)
    res = m.stack(fr16, _args(rt, (3.0, 3.0)))
    _check(res, oracle.stack_rows_u16(fr16, rt, (3.0, 3.0), nthreads=8))
    m.close()


@pytest.mark.parametrize("norm", [0, 3, 2])
def test_frame_sharded_mean_partials(ctx, oracle, norm):
    """sgpu_mean_partial_device over frame shards (accumulated one shard after
    the other, as the ranks' partials are all-reduced) + sgpu_mean_finish_device
    == the single-device NO_REJEC mean, bit for bit (data in Siril's [0, 1])."""
    import torch
    from siril_amd import stacking as S
    from siril_amd.distributed import _shard_args, frame_shards
    rng = np.random.default_rng(90 + norm)
    n, h, w = 23, 30, 52
    fr = _frames(rng, n, h, w, zeros=0.05)
    fr[:, 4, 7] = 0.0
    kw = {}
    if norm:
        kw = dict(normalize=S.Normalization(norm), scale=rng.uniform(0.9, 1.1, n),
                  offset=rng.uniform(-0.01, 0.01, n), mul=rng.uniform(0.9, 1.1, n))
    args = _args(0, (3.0, 3.0), **kw)
    if norm == 3:
        args.shiftx = rng.integers(-3, 4, n).astype(np.int32)
    d = torch.from_numpy(fr).cuda()
    s = c = None
    for f0, f1 in frame_shards(n, 3):
        s, c = ctx.mean_partial_device(d[f0:f1], _shard_args(args, f0, f1), s, c)
    out = ctx.mean_finish_device(s, c)
    torch.cuda.synchronize()
    ref = oracle.stack_rows(fr, 0, (3.0, 3.0), norm=norm, scale=kw.get("scale"), offset=kw.get("offset"),
                            mul=kw.get("mul"), shift_dx=None if args.shiftx is None else args.shiftx.astype(float),
                            nthreads=8)[0]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("norm", [0, 3, 4])
def test_frame_sharded_mean_guard(ctx, oracle, norm):
    """The guarded partial sums (sgpu_mean_partial_guard_device /
    sgpu_mean_finish_guard_device): min / max |x| folded over the shards, the
    HIP flag equal to the Python condition (distributed.partial_sums_exact),
    flagged pixels recomputed from sgpu_gather_columns_device in frame order;
    the result equals the oracle bit for bit, on normalized data with
    negative values and columns whose f64 sums are inexact."""
    import torch
    from siril_amd import stacking as S
    from siril_amd.distributed import _sequential_means, _shard_args, frame_shards, partial_sums_exact
    rng = np.random.default_rng(190 + norm)
    n, h, w = 23, 30, 52
    fr = _frames(rng, n, h, w, zeros=0.05)
    kw = {}
    if norm:
        kw = dict(normalize=S.Normalization(norm), scale=rng.uniform(0.9, 1.1, n),
                  offset=rng.uniform(0.045, 0.055, n), mul=rng.uniform(0.9, 1.1, n))
    even = (np.arange(n) % 2 == 0)[:, None]
    tiny = ((kw["offset"] / kw["scale"]).astype(np.float32)[:, None] if norm in (1, 3)
            else np.full((n, 1), 3e-9, np.float32))
    fr[:, 5, 10:30] = np.where(even, tiny, np.float32(0.9))
    args = _args(0, (3.0, 3.0), output_norm=True, **kw)
    d = torch.from_numpy(fr).cuda()
    s = c = lo = hi = None
    for f0, f1 in frame_shards(n, 3):
        s, c, lo, hi = ctx.mean_partial_guard_device(d[f0:f1], _shard_args(args, f0, f1), s, c, lo, hi)
    out, flag = ctx.mean_finish_guard_device(s, c, lo, hi, output_norm=True)
    want_flag = (~partial_sums_exact(c, lo, hi)).to(torch.uint8)
    assert torch.equal(flag, want_flag)
    assert int(flag.sum()) >= 10
    idx = torch.nonzero(flag.reshape(-1)).reshape(-1)
    cols = ctx.gather_columns_device(d, args, idx)
    out.view(-1)[idx] = _sequential_means(cols, True)
    torch.cuda.synchronize()
    ref = oracle.stack_rows(fr, 0, (3.0, 3.0), norm=norm, scale=kw.get("scale"), offset=kw.get("offset"),
                            mul=kw.get("mul"), output_norm=True, nthreads=8)[0]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def _planes(rng, shape, dzero=0.1, mzero=0.05):
    """Drizzle weights (pixfrac coverage in (0, 1], some exact zeros) and
    feather-mask values (ramped distances in [0, 1], some zeros)."""
    d = rng.uniform(0.05, 1.0, shape).astype(np.float32)
    d[rng.random(shape) < dzero] = 0.0
    m = np.clip(rng.uniform(-0.2, 1.3, shape), 0, 1).astype(np.float32)
    m[rng.random(shape) < mzero] = 0.0
    return d, m


@pytest.mark.parametrize("n", [5, 12, 100])
@pytest.mark.parametrize("rt", TYPES)
def test_drizzle_and_feather_planes(ctx, oracle, rt, n):
    """Per-sample weight planes (data->drizz, data->mask): drizzle-null
    samples leave the rejection stack (rejection_float.c:117-126), the mean
    is weighted by drizzle x mask x frame weight (median_and_mean.c:1043-1082),
    with shifts, normalization and frame weights; each plane alone and both."""
    from siril_amd import stacking as S
    if rt == 7 and n < 3:
        pytest.skip("GESDT needs 3 frames")
    rng = np.random.default_rng(500 + 10 * rt + n)
    fr = _frames(rng, n, 16, 40, wild=0.05 if n < 20 else 0.0)
    d, m = _planes(rng, fr.shape)
    sig = (0.32, 0.05) if rt == 7 else ((0.2, 0.1) if rt == 1 else (3.0, 3.0))
    dx = rng.uniform(-4, 4, n)
    weights = rng.uniform(0.5, 2.0, n)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.01 * rng.standard_normal(n)
    for dz, mk, use_w, norm in ((d, None, False, 0), (None, m, False, 0), (d, m, True, 3), (d, m, False, 0)):
        args = S.StackingArgs(S.Rejection(rt), sig, S.Normalization(norm), scale=scale if norm else None,
                              offset=offset if norm else None, shiftx=S.shifts_from_registration(dx),
                              weights=weights if use_w else None)
        res = ctx.stack(fr, args, drizzle=dz, mask=mk)
        ref = oracle.stack_rows(fr, rt, sig, norm=norm, scale=scale if norm else None,
                                offset=offset if norm else None, shift_dx=dx,
                                weights=weights if use_w else None, nthreads=8, drizz=dz, mask=mk)
        _check(res, ref)


def test_planes_device_and_u16(ctx, oracle):
    """The device entry points with weight planes (float and 16-bit), and the
    median stack ignoring them."""
    import torch
    from siril_amd import stacking as S
    rng = np.random.default_rng(77)
    n = 24
    fr = _frames(rng, n, 12, 64)
    d, m = _planes(rng, fr.shape)
    args = S.StackingArgs(S.Rejection(5), (3.0, 3.0), create_rejmaps=False)
    t = torch.from_numpy(fr).cuda()
    out, _, _, counts = ctx.stack_device(t, args, drizzle=torch.from_numpy(d).cuda(), mask=torch.from_numpy(m).cuda())
    torch.cuda.synchronize()
    ref = oracle.stack_rows(fr, 5, (3.0, 3.0), nthreads=8, drizz=d, mask=m)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref[0].view(np.uint32))
    assert tuple(counts.cpu().numpy().tolist()) == (int(ref[3][0]), int(ref[3][1]))
    fr16 = np.round(fr * 65535).astype(np.uint16)
    t16 = torch.from_numpy(fr16.view(np.int16)).cuda()
    for rt in (0, 2, 5):
        out, _, _, _ = ctx.stack_device(t16, S.StackingArgs(S.Rejection(rt), (2.5, 2.5)),
                                        drizzle=torch.from_numpy(d).cuda(), mask=torch.from_numpy(m).cuda())
        torch.cuda.synchronize()
        ref16 = oracle.stack_rows_u16(fr16, rt, (2.5, 2.5), nthreads=8, drizz=d, mask=m)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref16[0].view(np.uint32)), rt
    med = ctx.stack(fr, S.StackingArgs(), S.METHOD_MEDIAN, drizzle=d, mask=m)
    assert np.array_equal(med.result.view(np.uint32),
                          oracle.stack_rows(fr, 0, (3, 3), method=1, nthreads=8)[0].view(np.uint32))


@pytest.mark.parametrize("n", [72, 100, 250])
def test_u16_winsorized_moment_path(ctx, oracle, n):
    """16-bit WINSORIZED on the moment path (round 5: prep + rounds kernels
    on the WORD samples, roundf_to_WORD clamp bounds) over a block large
    enough for several chunks' worth of waves, with and without -norm=:
    bit for bit against the 16-bit oracle, float and 16-bit output."""
    from siril_amd import stacking as S
    rng = np.random.default_rng(5150 + n)
    h, w = (96, 512) if n <= 128 else (32, 512)
    fr = _frames16(rng, n, h, w)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 60 * rng.standard_normal(n)
    for norm in (0, 3):
        kw = {} if not norm else dict(normalize=S.Normalization(norm), scale=scale, offset=offset)
        args = S.StackingArgs(S.Rejection.WINSORIZED, (3.0, 3.0), **kw)
        okw = {} if not norm else dict(norm=norm, scale=scale, offset=offset)
        for out32 in (True, False):
            res = ctx.stack(fr, args, use_32bit_output=out32)
            out, rl, rh, counts = oracle.stack_rows_u16(fr, 5, (3.0, 3.0), use_32bit_output=out32, nthreads=16,
                                                        **okw)
            assert np.array_equal(res.result.view(np.uint16 if not out32 else np.uint32),
                                  out.view(np.uint16 if not out32 else np.uint32)), (n, norm, out32)
            assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)
            assert tuple(res.irej) == (int(counts[0]), int(counts[1]))
            assert ctx.last_exact_pixels() < h * w // 20


@pytest.mark.parametrize("rt", [1, 2, 4, 5, 16])
@pytest.mark.parametrize("n", [33, 64, 100, 257, 400, 1000])
def test_exact_wave_kernel_all_pixels(ctx, oracle, rt, n):
    """The one-wave-per-pixel exact kernel (stack_exact_wave.hip: Lomuto
    partitions in closed form, ballot compactions, the `N - r <= 4` cutoff as
    a prefix count, sequential f64 sums on lane 0) on EVERY pixel of a block
    (set_exact_only(2)): bit-exact against the oracle, with the quickselect
    permutations, cutoffs and summation orders the reference's.  Data with
    ties, zeros, wild outliers, a mixed-sign block with -output_norm, and
    weights."""
    rng = np.random.default_rng(900 + 10 * rt + n)
    method = 1 if rt == 16 else 0
    r = 0 if rt == 16 else rt
    sig = (0.2, 0.1) if rt == 1 else (2.0, 2.5)
    ctx.set_exact_only(2)
    try:
        fr = _frames(rng, n, 3, 64, wild=0.1)
        fr[:, 0, :8] = np.round(fr[:, 0, :8] * 64) / 64              # ties
        fr[:, 1, 0] = 0.0                                              # all missing
        fr[: n - 1, 1, 1] = 0.0                                        # one survivor
        res = ctx.stack(fr, _args(r, sig), method)
        _check(res, oracle.stack_rows(fr, r, sig, method=method, nthreads=16), method)
        mixed = rng.normal(-0.1, 1.0, (n, 2, 64)).astype(np.float32)
        args = _args(r, sig, output_norm=True)
        _check(ctx.stack(mixed, args, method),
               oracle.stack_rows(mixed, r, sig, method=method, output_norm=True, nthreads=16), method)
        if method == 0:
            from siril_amd import stacking as S
            weights = rng.uniform(0.5, 2.0, n)
            args = S.StackingArgs(S.Rejection(r), sig, weights=weights)
            _check(ctx.stack(fr, args), oracle.stack_rows(fr, r, sig, weights=weights, nthreads=16))
    finally:
        ctx.set_exact_only(False)
