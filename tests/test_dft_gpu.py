"""GPU DFT registration (register_shift_dft, shift_methods.c:60-321) against
the numpy restatement (oracle/dft_ref.py) and the injected shifts.
Parity bar: identical integer (shiftx, shifty) per frame (the quantity the
reference stores); spectra themselves are float FFTs with a different
rounding than FFTW (parity unpinned at that level)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking
    c = stacking.Context(0)
    yield c
    c.close()


def _case(S, nstars, shifts, seed=7):
    from siril_amd import synth
    base = synth.star_field(S, S, nstars=nstars, seed=seed)
    return synth.shifted_frames(base, [(0, 0)] + list(shifts), seed=seed + 1)


@pytest.mark.parametrize("S", [64, 100, 120, 128, 210, 256, 343, 500, 1000, 2048])
def test_dft_shifts_match_oracle(ctx, S):
    from oracle import dft_ref
    from siril_amd import registration as R
    rng = np.random.default_rng(S)
    half = S // 2
    shifts = [tuple(int(v) for v in rng.integers(-half + 1, half, 2)) for _ in range(6)]
    shifts += [(half, 0), (0, -half), (1, 1)]
    fr = _case(S, max(20, S * S // 400), shifts)
    got = R.dft_shifts(fr[0], list(fr[1:]), ctx)
    for i, (dx, dy) in enumerate(shifts):
        sx, sy, _ = dft_ref.dft_shift(fr[0], fr[i + 1])
        assert (got[i, 0], got[i, 1]) == (sx, sy), (S, i, (dx, dy))
        # the stored shift undoes the injected translation (modulo the wrap)
        assert (sx + dx) % S == 0 and (sy + dy) % S == 0


@pytest.mark.parametrize("S", [100, 210, 500, 1000, 2000, 4000])
def test_dft_peak_value_matches_oracle(ctx, S):
    """The correlation peak itself (the unnormalised backward transform at the
    argmax, shift_methods.c:257-265) against the complex128 restatement:
    checks the transforms, not only where their maximum falls.  The sizes
    run every plan shape (odd radix first, sgpu_dft.cpp factorize): 10 x 10
    (100), 3 x 10 x 7 through the generic prime pass (210), 5 x 10 x 10
    (500), 5 x 8 x 5 x 5 (1000), 5 x 8 x 10 x 5 (2000), 5 x 8 x 10 x 10
    (4000, BASELINE config 3).  Tolerance: 2e-5
    relative (float32 transforms of S^2 products; a wrong twiddle or
    butterfly is off by orders of magnitude more)."""
    import torch
    from oracle import dft_ref
    from siril_amd import registration as R
    rng = np.random.default_rng(S + 1)
    shifts = [tuple(int(v) for v in rng.integers(-S // 3, S // 3, 2)) for _ in range(2 if S >= 2000 else 4)]
    fr = _case(S, max(20, S * S // 400), shifts, seed=S)
    got, pk = R.register_shift_dft(torch.from_numpy(fr).cuda(), 0, (0, 0, S, S), ctx, peaks=True)
    got, pk = got.cpu().numpy(), pk.cpu().numpy()
    for i in range(1, len(fr)):
        sx, sy, peak = dft_ref.dft_shift(fr[0], fr[i])
        assert tuple(got[i]) == (sx, sy)
        assert abs(float(pk[i]) - peak) <= 2e-5 * abs(peak), (S, i, float(pk[i]), peak)


def test_dft_reference_frame_is_zero(ctx):
    from siril_amd import registration as R
    fr = _case(96, 40, [])
    assert R.dft_shifts(fr[0], [fr[0]], ctx).tolist() == [[0, 0]]


def test_dft_device_window_of_full_frames(ctx):
    """BASELINE config 3 shape at reduced size: centred square window of
    wider frames in HBM (no copy), reference frame 0."""
    import torch
    from oracle import dft_ref
    from siril_amd import registration as R, synth
    H, W, S = 600, 900, 512
    base = synth.star_field(H, W, nstars=400, seed=3)
    shifts = [(0, 0), (5, -3), (-40, 22), (61, -64), (-7, 0)]
    fr = synth.shifted_frames(base, shifts, seed=4)
    x0, y0 = (W - S) // 2, (H - S) // 2
    d = torch.from_numpy(fr).cuda()
    got = R.register_shift_dft(d, 0, (x0, y0, S, S), ctx).cpu().numpy()
    for i in range(1, len(shifts)):
        sel0 = fr[0, y0:y0 + S, x0:x0 + S]
        sel = fr[i, y0:y0 + S, x0:x0 + S]
        sx, sy, _ = dft_ref.dft_shift(sel0, sel)
        assert tuple(got[i]) == (sx, sy)
        assert (sx, sy) == (-shifts[i][0], -shifts[i][1])
    assert tuple(got[0]) == (0, 0)


def test_dft_full_size_config3(ctx):
    """S = 4000 = 2^5 * 5^3 (BASELINE config 3 selection) on 4 frames."""
    from oracle import dft_ref
    from siril_amd import registration as R, synth
    S = 4000
    base = synth.star_field(S, S, nstars=3000, seed=9)
    shifts = [(0, 0), (17, -29), (-64, 64), (3, 0)]
    fr = synth.shifted_frames(base, shifts, seed=10)
    got = R.dft_shifts(fr[0], list(fr[1:]), ctx)
    for i in range(1, len(shifts)):
        assert tuple(got[i - 1]) == (-shifts[i][0], -shifts[i][1])
    sx, sy, _ = dft_ref.dft_shift(fr[0], fr[1], np.complex64)
    assert (sx, sy) == tuple(got[0])


def test_dft_unfused_column_passes_subprocess():
    """SGPU_DFT_FUSED=0 selects the separate forward-column and
    cross-power/inverse-column kernels (A/B knob of the fused column pass):
    same shifts as the oracle and as the default build path."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {root!r})\n"
        "from tests.test_dft_gpu import _case\n"
        "from oracle import dft_ref\n"
        "from siril_amd import registration as R, stacking\n"
        "ctx = stacking.Context(0)\n"
        "bad = 0\n"
        "for S in (100, 343, 512):\n"
        "    rng = np.random.default_rng(S)\n"
        "    sh = [tuple(int(v) for v in rng.integers(-S // 2 + 1, S // 2, 2)) for _ in range(5)]\n"
        "    fr = _case(S, max(20, S * S // 400), sh)\n"
        "    got = R.dft_shifts(fr[0], list(fr[1:]), ctx)\n"
        "    for i in range(len(sh)):\n"
        "        sx, sy, _ = dft_ref.dft_shift(fr[0], fr[i + 1])\n"
        "        bad += (int(got[i, 0]), int(got[i, 1])) != (sx, sy)\n"
        "print('BAD', bad)\n")
    env = dict(os.environ, SGPU_DFT_FUSED="0", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert int(r.stdout.split("BAD")[1]) == 0
