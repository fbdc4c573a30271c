"""Background noise (imstats bgnoise: FnNoise1_float / FnNoise1_ushort,
algos/quantize.c:1202-1488) and -weight=noise (median_and_mean.c:1111-1135).

The restatement (oracle/noise_ref.py) follows the reference line by line;
no reference fixture holds a bgnoise value, so parity with the reference is
pinned by the restatement only (the estimator's published definition is
checked on synthetic Gaussian noise below).  The GPU path must equal the
restatement bit for bit."""
import numpy as np
import pytest

from oracle import noise_ref as NR


def _frames(n, h, w, seed, u16=False):
    rng = np.random.default_rng(seed)
    sig = np.linspace(0.004, 0.02, n)
    x = 0.25 + rng.normal(0.0, 1.0, (n, h, w)) * sig[:, None, None]
    if w > 5:
        x[:, :, 5] += 0.3 * (rng.random((n, h)) < 0.1)     # hot columns: clipped outliers
    x[:, 3, :] = 0.0                                       # an empty row (skipped)
    x[:, 4, ::2] = 0.0                                     # a row with missing pixels
    if u16:
        return np.clip(np.round(x * 60000.0), 0, 65535).astype(np.uint16)
    x = x.astype(np.float32)
    x[:, 6, min(7, w - 1)] = np.nan                        # NaN pixels are skipped too
    return x


def test_oracle_gaussian_noise_estimate():
    """sigma of first differences / sqrt(2) recovers the noise sigma."""
    rng = np.random.default_rng(1)
    x = (0.3 + rng.normal(0, 0.01, (120, 400))).astype(np.float32)
    assert abs(NR.bgnoise(x) - 0.01) < 3e-4
    u = np.round(1000 + rng.normal(0, 20, (120, 400))).astype(np.uint16)
    assert abs(NR.bgnoise(u) - 20.0) < 0.6
    assert NR.bgnoise(np.zeros((8, 9), np.float32)) == 0.0          # no valid row
    assert NR.bgnoise(np.ones((8, 2), np.float32)) == 0.0           # rows of < 3 pixels


def test_oracle_noise_weights_normalised():
    w = NR.noise_weights([0.01, 0.02, 0.04], [1.0, 1.0, 0.5])
    assert abs(w.mean() - 1.0) < 1e-12
    assert w[0] > w[1] and abs(w[1] - w[2]) < 1e-12                # pscale 0.5 cancels noise 0.04


@pytest.mark.gpu
@pytest.mark.parametrize("u16", [False, True])
@pytest.mark.parametrize("shape", [(5, 40, 64), (3, 17, 3), (2, 9, 1000)])
def test_bgnoise_gpu_bit_exact(u16, shape):
    import torch
    from siril_amd import normalization as N
    from siril_amd.stacking import Context
    fr = _frames(*shape, seed=shape[1], u16=u16)
    ctx = Context(0)
    got = N.bgnoise(ctx, fr)
    want = np.array([NR.bgnoise(f) for f in fr])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), (got, want)
    dev = torch.from_numpy(fr.view(np.int16) if u16 else fr).cuda()
    got_d = N.bgnoise(ctx, dev)
    assert np.array_equal(got_d.view(np.uint64), want.view(np.uint64))


@pytest.mark.gpu
def test_bgnoise_full_frame():
    """6000 x 4000 (BASELINE frame size, one thread per row over 4000 rows):
    the estimate recovers the noise sigma, and a 300-row band of the same
    frame equals the restatement bit for bit."""
    import torch
    from siril_amd import normalization as N
    from siril_amd.stacking import Context
    g = torch.Generator(device="cuda").manual_seed(3)
    fr = (0.2 + 0.01 * torch.randn((1, 4000, 6000), device="cuda", generator=g)).float().contiguous()
    ctx = Context(0)
    got = N.bgnoise(ctx, fr)[0]
    assert abs(got - 0.01) < 2e-4
    band = fr[:, 1000:1300].contiguous()
    want = NR.bgnoise(band[0].cpu().numpy())
    assert N.bgnoise(ctx, band)[0] == want


@pytest.mark.gpu
def test_stack_weight_noise(tmp_path, oracle):
    """`stack ... -norm=addscale -weight=noise`: per-frame bgnoise and the
    normalization scale give the weights 1 / (pscale^2 bgnoise^2), normalised
    (median_and_mean.c:1111-1135); -nonorm ignores them (command.c)."""
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    n, h, w = 9, 30, 44
    fr = np.clip(_frames(n, h, w, seed=5), 1e-6, 1).astype(np.float32)
    fr[:, 3, :] = 0.3                                       # keep the stack free of empty rows
    fr = np.nan_to_num(fr, nan=0.3).astype(np.float32)
    seq = synth.write_sequence(str(tmp_path), fr, name="nz_", shifts=[(0, 0)] * n)
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -norm=addscale -weight=noise -32b -out={tmp_path}/nz.fit")
    ctx = Context(0)
    st = N.norm_stats(ctx, fr)
    off, mul, scl = N.factors(Normalization.ADDITIVE_SCALING, st, 0)
    wts = NR.noise_weights([NR.bgnoise(f) for f in fr], scl)
    ref, _, _, cnt = oracle.stack_rows(fr, 5, (3.0, 3.0), norm=int(Normalization.ADDITIVE_SCALING), scale=scl,
                                       offset=off, mul=mul, weights=wts, nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))
    out2, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -weight=noise -32b -out={tmp_path}/nz2.fit")
    ref2, _, _, _ = oracle.stack_rows(fr, 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(Q.read_fits(out2).view(np.uint32), ref2.view(np.uint32))
