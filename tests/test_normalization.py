"""Stack normalization: per-frame estimators
(statistics_internal_float STATS_NORM / STATS_LITENORM,
algos/statistics_float.c:281-480) on the GPU vs the oracle restatement, the
factor arithmetic (compute_factors_from_estimators,
stacking/normalization.c:150-185), and normalized stacks end to end.

Parity: median, MAD and IKSS location are histogram order statistics with
float interpolation (rt/rt_algo.cc:38-172) and must be bit-exact.  The IKSS
scale is sqrt of a bwmv whose two f64 sums the reference reduces in an
OpenMP-thread-count-dependent order (statistics_float.c:113-123); the GPU
sums in a fixed order of its own, so scale is checked to relative 1e-12.
No reference test covers these estimators: beyond the restatement (whose
histogram percentile the MAD rejection KATs exercise) parity is unpinned.
"""
import numpy as np
import pytest

from siril_amd import synth
from siril_amd.stacking import Normalization as NZ


def np_percentile_half(x):
    """Independent numpy restatement of findMinMaxPercentile(0.5) for the
    oracle cross-check (rt_algo.cc:38-172), float32 arithmetic."""
    x = np.asarray(x, np.float32)
    n = x.size
    lo, hi = np.float32(x.min()), np.float32(x.max())
    if np.abs(hi - lo) == 0:
        return lo
    hs = min(65536, n)
    scale = np.float32(hs - 1) / np.float32(hi - lo)
    b = (scale * (x - lo)).astype(np.float32).astype(np.int64) & 0xFFFF
    h = np.bincount(b, minlength=hs)
    thr = np.float32(0.5) * np.float32(n)
    cum = np.cumsum(h)
    j = int(np.argmax(cum.astype(np.float32) >= thr))
    k = j + 1
    count, count_ = cum[j], cum[j] - h[j]
    c0 = np.float32(count) - thr
    c1 = thr - np.float32(count_)
    out = (c1 * np.float32(k) + c0 * np.float32(k - 1)) / (c0 + c1)
    out = np.float32(np.float32(out / scale) + lo)
    return np.float32(max(lo, min(out, hi)))


def frame_cases():
    rng = np.random.default_rng(77)
    cases = {}
    cases["gauss_small"] = rng.normal(0.1, 0.01, (40, 50)).astype(np.float32)          # n < 65536
    f = synth.frames_numpy(1, 300, 400, seed=3)[0]
    f[rng.random(f.shape) < 0.05] = 0.0                                                  # missing pixels
    f[0, :7] = np.nan
    cases["synth_zeros_nan"] = f
    cases["negative"] = rng.normal(-0.2, 0.05, (256, 512)).astype(np.float32)
    g = rng.normal(0.3, 0.02, (512, 700)).astype(np.float32)
    g[rng.random(g.shape) < 0.02] = rng.uniform(0.5, 1.0, 1).astype(np.float32)       # hot pixels
    cases["outliers"] = g
    cases["odd_size"] = rng.normal(0.15, 0.03, (301, 299)).astype(np.float32)   # scalar-load path
    nc = np.full((600, 500), 0.5, np.float32)                                     # > 65535 samples in one
    nc[rng.random(nc.shape) < 0.01] = np.float32(0.4)                               # bin of a histogram block:
    nc[rng.random(nc.shape) < 0.01] = np.float32(0.6)                               # packed-counter fallback
    cases["near_constant"] = nc
    cases["ties"] = (np.round(rng.normal(0.2, 0.01, (300, 300)) * 200) / 200).astype(np.float32)
    return cases


# ---------------------------------------------------------------- CPU tests

def test_oracle_percentile_matches_independent_restatement(oracle):
    for name, f in frame_cases().items():
        good = f[(f != 0) & ~np.isnan(f)]
        st, med, mad, loc, scl, ng = oracle.norm_stats(f, lite=True)
        assert st == 0 and ng == good.size, name
        assert np.float32(med) == np_percentile_half(good), name
        assert np.float32(mad) == np_percentile_half(np.abs(good - np.float32(med))), name


def test_oracle_estimators_are_robust(oracle):
    rng = np.random.default_rng(5)
    f = rng.normal(0.1, 0.01, (600, 800)).astype(np.float32)
    f[rng.random(f.shape) < 0.01] = np.float32(0.9)
    st, med, mad, loc, scl, ng = oracle.norm_stats(f)
    assert st == 0
    assert abs(med - 0.1) < 2e-4 and abs(loc - 0.1) < 2e-4
    assert abs(mad - 0.6745 * 0.01) < 2e-4
    assert abs(scl - 0.01) / 0.01 < 0.03           # IKSS scale ~ sigma for a Gaussian


def test_oracle_null_stats(oracle):
    assert oracle.norm_stats(np.zeros((8, 8), np.float32))[0] == 1          # no good pixel
    c = np.full((16, 16), 0.25, np.float32)
    assert oracle.norm_stats(c, lite=True)[0] == 0                           # lite: median, mad = 0 fine
    assert oracle.norm_stats(c)[0] == 1                                      # IKSS: MAD is null


def ref_factors(normalize, tab, ref, lite):
    """compute_factors_from_estimators restated in Python (normalization.c:150-185)."""
    n = tab.shape[0]
    off, mul, scl = np.zeros(n), np.ones(n), np.ones(n)
    locs = tab[:, 0] if lite else tab[:, 2]
    scls = 1.5 * tab[:, 1] if lite else tab[:, 3]
    if normalize in (NZ.ADDITIVE_SCALING, NZ.MULTIPLICATIVE_SCALING):
        scl = np.array([1.0 if s == 0 else scls[ref] / s for s in scls])
    if normalize in (NZ.ADDITIVE, NZ.ADDITIVE_SCALING):
        off = scl * locs - locs[ref]
    elif normalize in (NZ.MULTIPLICATIVE, NZ.MULTIPLICATIVE_SCALING):
        mul = np.array([1.0 if m == 0 else locs[ref] / m for m in locs])
    return off, mul, scl


@pytest.mark.parametrize("normalize", [NZ.ADDITIVE, NZ.MULTIPLICATIVE, NZ.ADDITIVE_SCALING,
                                       NZ.MULTIPLICATIVE_SCALING])
@pytest.mark.parametrize("lite", [False, True])
def test_factors_host_logic(normalize, lite):
    from siril_amd import normalization as N
    rng = np.random.default_rng(int(normalize) * 10 + lite)
    n = 7
    tab = np.stack([rng.uniform(0.05, 0.2, n), rng.uniform(0.001, 0.01, n),
                    rng.uniform(0.05, 0.2, n), rng.uniform(0.001, 0.01, n)], 1)
    tab[4, 3] = 0.0            # zero scale estimator -> factor 1
    tab[5, 2] = tab[5, 0] = 0  # zero location -> mul 1
    st = N.NormStats(tab[:, 0], tab[:, 1], tab[:, 2], tab[:, 3], np.ones(n, np.int64), np.zeros(n, np.int32))
    off, mul, scl = N.factors(normalize, st, ref_index=2, lite=lite)
    e_off, e_mul, e_scl = ref_factors(normalize, tab, 2, lite)
    assert np.array_equal(off, e_off) and np.array_equal(mul, e_mul) and np.array_equal(scl, e_scl)


def test_factors_reject_failed_frame():
    from siril_amd import normalization as N
    n = 3
    st = N.NormStats(np.ones(n), np.ones(n), np.ones(n), np.ones(n), np.ones(n, np.int64),
                     np.array([0, 1, 0], np.int32))
    with pytest.raises(N.NormalizationError, match="image 2"):
        N.factors(NZ.ADDITIVE_SCALING, st)


# ---------------------------------------------------------------- GPU tests

@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking as S
    c = S.Context(0)
    yield c
    c.close()


def check_stats(gs, i, ref, lite):
    st, med, mad, loc, scl, ng = ref
    assert gs.status[i] == st
    if st:
        return
    assert gs.ngood[i] == ng
    assert np.float32(gs.median[i]) == np.float32(med) and gs.median[i] == med
    assert gs.mad[i] == mad
    if not lite:
        assert gs.location[i] == loc
        assert abs(gs.scale[i] - scl) <= 1e-12 * abs(scl)


@pytest.mark.gpu
@pytest.mark.parametrize("lite", [False, True])
@pytest.mark.parametrize("name", list(frame_cases().keys()))
def test_gpu_stats_match_oracle(ctx, oracle, name, lite):
    from siril_amd import normalization as N
    f = frame_cases()[name]
    gs = N.norm_stats(ctx, f[None], lite)
    check_stats(gs, 0, oracle.norm_stats(f, lite), lite)


@pytest.mark.gpu
def test_gpu_stats_batch_and_null_frames(ctx, oracle):
    from siril_amd import normalization as N
    fr = synth.frames_numpy(6, 200, 333, seed=11)
    fr[2] = 0.0                                   # no good pixel -> status 1
    fr[4] = np.float32(0.3)                       # constant -> IKSS MAD null -> status 1
    fr[5, :, :100] = 0.0
    for lite in (False, True):
        gs = N.norm_stats(ctx, fr, lite)
        for i in range(fr.shape[0]):
            check_stats(gs, i, oracle.norm_stats(fr[i], lite), lite)


@pytest.mark.gpu
def test_gpu_stats_full_frame_device(ctx, oracle):
    """One 6000x4000 frame of the benchmark recipe, HBM-resident (hs = 65536)."""
    import torch
    from siril_amd import normalization as N
    fr = synth.frames_numpy(2, 4000, 6000, seed=21)
    d = torch.from_numpy(fr).cuda()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gs = N.norm_stats_device(ctx, d)
    for i in range(2):
        check_stats(gs, i, oracle.norm_stats(fr[i]), False)


@pytest.mark.gpu
@pytest.mark.parametrize("normalize,lite", [(NZ.ADDITIVE_SCALING, False), (NZ.ADDITIVE, False),
                                            (NZ.MULTIPLICATIVE_SCALING, False), (NZ.ADDITIVE_SCALING, True)])
def test_gpu_normalized_stack_matches_oracle(ctx, oracle, normalize, lite):
    """stack ... -norm=addscale (etc.) rej w 3 3: GPU estimators + factors,
    then the GPU stack vs the oracle stack driven by the oracle's own
    estimators restated through the same factor formula."""
    from siril_amd import normalization as N
    from siril_amd import stacking as S
    fr = synth.frames_numpy(12, 48, 160, seed=31)
    fr *= np.linspace(0.8, 1.2, 12, dtype=np.float32)[:, None, None]       # per-frame gain
    fr += np.linspace(-0.01, 0.02, 12, dtype=np.float32)[:, None, None]    # per-frame pedestal
    fr = np.clip(fr, 1e-6, 1.0)
    off, mul, scl, gs = N.compute_normalization(ctx, fr, normalize, ref_index=0, lite=lite)
    tab = np.array([oracle.norm_stats(f, lite)[1:5] for f in fr])
    e_off, e_mul, e_scl = ref_factors(normalize, tab, 0, lite)
    assert np.allclose(off, e_off, rtol=1e-12, atol=1e-15) and np.array_equal(mul, e_mul)
    assert np.allclose(scl, e_scl, rtol=1e-12, atol=0)
    args = S.StackingArgs(S.Rejection.WINSORIZED, (3.0, 3.0), normalize, scale=scl, offset=off, mul=mul)
    res = ctx.stack(fr, args)
    out, rl, rh, counts = oracle.stack_rows(fr, oracle.WINSORIZED, (3.0, 3.0), norm=int(normalize),
                                            scale=scl, offset=off, mul=mul, nthreads=4)
    assert np.array_equal(res.result.view(np.uint32), out.view(np.uint32))
    assert np.array_equal(res.rejmap_low, rl) and np.array_equal(res.rejmap_high, rh)


# ------------------------------------------------------------ DATA_USHORT

def u16_cases():
    rng = np.random.default_rng(91)
    c = {}
    c["u16_gauss"] = np.clip(np.round(rng.normal(3000, 80, (256, 300))), 0, 65535).astype(np.uint16)
    f = np.clip(np.round(rng.normal(1200, 40, (301, 299))), 0, 65535).astype(np.uint16)     # odd size
    f[rng.random(f.shape) < 0.03] = 0                                                       # missing
    f[rng.random(f.shape) < 0.01] = 60000                                                   # hot
    c["u16_zeros_hot"] = f
    u = np.full((600, 500), 1000, np.uint16)                                        # counter-overflow fallback
    u[rng.random(u.shape) < 0.01] = 900
    u[rng.random(u.shape) < 0.01] = 1100
    c["u16_near_constant"] = u
    c["u16_tiny_odd"] = np.array([[5, 9, 0, 7, 3, 11, 4]], np.uint16)                      # n < 10
    c["u16_tiny_even"] = np.array([[5, 9, 2, 7, 3, 11, 4, 8, 1, 6, 12, 10]], np.uint16)
    return c


def test_oracle_u16_estimators(oracle):
    for name, f in u16_cases().items():
        good = f[f > 0].astype(np.int64)
        st, med, mad, loc, scl, ng = oracle.norm_stats(f, lite=True)
        assert st == 0 and ng == good.size, name
        assert med == float(np.median(good)), name                  # exact order statistics
        mi = int(np.floor(med + 0.5))
        assert mad == float(np.median(np.abs(good - mi))), name


@pytest.mark.gpu
@pytest.mark.parametrize("lite", [False, True])
@pytest.mark.parametrize("name", list(u16_cases().keys()))
def test_gpu_u16_stats_match_oracle(ctx, oracle, name, lite):
    from siril_amd import normalization as N
    f = u16_cases()[name]
    gs = N.norm_stats(ctx, f[None], lite)
    check_stats(gs, 0, oracle.norm_stats(f, lite), lite)


@pytest.mark.gpu
def test_gpu_u16_normalized_stack_matches_oracle(ctx, oracle):
    """16-bit lights, -norm=addscale: GPU estimators (16-bit units) and the
    16-bit stack (apply_rejection_ushort, round_to_WORD normalization)."""
    from siril_amd import normalization as N
    from siril_amd import stacking as S
    fr = synth.frames_numpy(10, 40, 96, seed=41)
    fr = fr * np.linspace(0.8, 1.2, 10, dtype=np.float32)[:, None, None]
    fr16 = np.clip(np.round(fr * 65535.0), 0, 65535).astype(np.uint16)
    off, mul, scl, gs = N.compute_normalization(ctx, fr16, NZ.ADDITIVE_SCALING, ref_index=0)
    for i in range(fr16.shape[0]):
        check_stats(gs, i, oracle.norm_stats(fr16[i]), False)
    args = S.StackingArgs(S.Rejection.WINSORIZED, (3.0, 3.0), NZ.ADDITIVE_SCALING, scale=scl, offset=off, mul=mul)
    res = ctx.stack(fr16, args)
    out, rl, rh, counts = oracle.stack_rows_u16(fr16, oracle.WINSORIZED, (3.0, 3.0), norm=int(NZ.ADDITIVE_SCALING),
                                                scale=scl, offset=off, mul=mul, nthreads=4)
    assert np.array_equal(np.asarray(res.result).view(np.uint32), np.asarray(out).view(np.uint32))
