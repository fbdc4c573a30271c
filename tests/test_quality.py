"""Frame quality of the DFT registration:
QualityEstimate_float (algos/quality_float.c:41-147) on the GPU vs the numpy
restatement (oracle/quality_ref.py), and normalizeQualityData /
best-frame selection (registration/shift_methods.c:36-54,184,241-246).
The f64 gradient sum is reduced in a different order on the GPU: relative
tolerance 1e-12.  Parity unpinned beyond the restatement (no reference test)."""
import numpy as np
import pytest

from oracle import quality_ref as Q
from siril_amd import synth


def cases():
    c = {}
    c["stars_256"] = (0.05 + 0.9 * synth.star_field(256, 256, nstars=120, seed=3)).astype(np.float32)
    c["stars_odd_301x257"] = (0.05 + 0.9 * synth.star_field(257, 301, nstars=90, seed=4)).astype(np.float32)
    c["tiny_9x10"] = np.random.default_rng(1).uniform(0, 1, (10, 9)).astype(np.float32)
    c["flat"] = np.full((64, 64), 0.05, np.float32)              # no pixel above threshold -> q = -1
    return c


def test_oracle_quality_ranks_sharpness():
    img = (0.05 + 0.9 * synth.star_field(256, 256, nstars=120, seed=3)).astype(np.float32)
    k = np.ones(5, np.float32) / 5
    blur = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, img)
    blur = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 0, blur).astype(np.float32)
    assert Q.quality_estimate_float(img) > Q.quality_estimate_float(blur) > 0
    assert np.isnan(Q.quality_estimate_float(cases()["flat"]))    # sqrt of a negative sum


def test_normalize_quality_host():
    from siril_amd import registration as R
    q = np.array([2.0, 3.0, 1.0, 5.0, 4.0])
    nq, best = R.normalize_quality(q, ref_index=0)
    assert best == 3
    assert np.array_equal(nq, Q.normalize_quality(q, 1.0, 5.0))
    nq, best = R.normalize_quality(np.array([2.0, np.nan, 2.0]), ref_index=0)
    assert best == 0 and nq[1] == -1.0
    nq, _ = R.normalize_quality(np.array([0.0]), ref_index=0)     # single frame: diff 0, q_max 0
    assert nq[0] == 0.0


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking as S
    c = S.Context(0)
    yield c
    c.close()


def close(a, b):
    if np.isnan(b):
        return np.isnan(a)
    return abs(a - b) <= 1e-12 * abs(b)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(cases().keys()))
def test_gpu_quality_matches_oracle(ctx, name):
    from siril_amd import registration as R
    img = cases()[name]
    q = R.quality_estimate(img[None], ctx)
    assert close(q[0], Q.quality_estimate_float(img)), (q[0], Q.quality_estimate_float(img))


@pytest.mark.gpu
def test_gpu_quality_batch_device_window(ctx):
    """Selection windows of HBM-resident frames (row stride = frame width)."""
    import torch
    from siril_amd import registration as R
    base = synth.star_field(300, 400, nstars=200, seed=9)
    fr = np.stack([np.roll(base, (i, 2 * i), (0, 1)) * (1 - 0.03 * i) + 0.05 for i in range(5)]).astype(np.float32)
    d = torch.from_numpy(fr).cuda()
    win = d[:, 20:276, 60:316]                                    # 256x256 centred-ish selection
    q = R.quality_estimate(win, ctx)
    for i in range(5):
        assert close(q[i], Q.quality_estimate_float(fr[i, 20:276, 60:316]))
    # a window that is not 16-byte aligned takes the scalar-load kernel
    q1 = R.quality_estimate(d[:, 20:276, 61:317], ctx)
    for i in range(5):
        assert close(q1[i], Q.quality_estimate_float(fr[i, 20:276, 61:317]))
    assert not np.isnan(q).any()
    nq, best = R.normalize_quality(q, 0)
    eq = Q.normalize_quality(q, q.min(), q.max())
    assert best == int(np.argmax(q)) and np.allclose(nq, eq, rtol=0, atol=1e-15)


@pytest.mark.gpu
def test_gpu_register_shift_dft_full(ctx):
    """Shifts + normalised quality + best frame of one registration call."""
    import torch
    from siril_amd import registration as R
    base = synth.star_field(256, 320, nstars=150, seed=12)
    sh = [(0, 0), (3, -2), (-5, 4), (7, 1)]
    fr = np.stack([np.roll(base, (dy, dx), (0, 1)) * g + 0.05
                   for (dx, dy), g in zip(sh, (1.0, 0.9, 1.1, 0.95))]).astype(np.float32)
    d = torch.from_numpy(fr).cuda()
    shifts, q, best = R.register_shift_dft_full(d, 0, (32, 0, 256, 256), ctx)
    raw = np.array([Q.quality_estimate_float(fr[i, 0:256, 32:288]) for i in range(4)])
    assert best == int(np.argmax(raw))
    assert np.allclose(q, Q.normalize_quality(raw, raw.min(), raw.max()), rtol=0, atol=1e-12)
    assert q.max() == 1.0 and q.min() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3])
def test_gpu_register_cfa_does_not_touch_frames(ctx, n):
    """The CFA quality pass interpolates a private copy of the selection
    (seq_read_frame_part), also when the selection is the whole block."""
    import torch
    from siril_amd import registration as R
    base = synth.star_field(128, 128, nstars=60, seed=21)
    fr = np.stack([np.roll(base, (i, -i), (0, 1)) + 0.05 for i in range(n)]).astype(np.float32)
    d = torch.from_numpy(fr).cuda()
    before = d.clone()
    R.register_shift_dft_full(d, 0, (0, 0, 128, 128), ctx, cfa="RGGB")
    torch.cuda.synchronize()
    assert torch.equal(d, before)


@pytest.mark.gpu
@pytest.mark.parametrize("knob,val", [("SGPU_QE_FUSED", "0"), ("SGPU_QE_VEC", "0"), ("SGPU_QE_SPLIT", "1")])
def test_gpu_quality_unfused_subsample_path(knob, val):
    """SGPU_QE_FUSED=0 selects the per-level subsample kernels, SGPU_QE_VEC=0
    the scalar-load fused kernel, SGPU_QE_SPLIT=1 separate smooth and
    gradient kernels; same results."""
    import os
    import subprocess
    import sys
    code = ("import numpy as np, torch\n"
            "from siril_amd import registration as R, synth\n"
            "from oracle import quality_ref as Q\n"
            "base = synth.star_field(300, 400, nstars=200, seed=9)\n"
            "fr = np.stack([np.roll(base, (i, 2 * i), (0, 1)) * (1 - 0.03 * i) + 0.05 for i in range(3)]).astype(np.float32)\n"
            "d = torch.from_numpy(fr).cuda()\n"
            "q = R.quality_estimate(d[:, 20:276, 60:316])\n"
            "for i in range(3):\n"
            "    e = Q.quality_estimate_float(fr[i, 20:276, 60:316])\n"
            "    assert abs(q[i] - e) <= 1e-12 * abs(e), (i, q[i], e)\n"
            "img = (0.05 + 0.9 * synth.star_field(257, 301, nstars=90, seed=4)).astype(np.float32)\n"
            "q = R.quality_estimate(img[None])\n"
            "e = Q.quality_estimate_float(img)\n"
            "assert abs(q[0] - e) <= 1e-12 * abs(e), (q[0], e)\n"
            "print('ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, **{knob: val})
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def _u16(img):
    return (np.clip(img, 0, 1) * 65535).astype(np.uint16)


def test_oracle_u16_maxp_is_the_sequential_list():
    """The stretch divisor replays the reference's running top list: a value
    enters only above the current third entry, so a descending scan keeps
    only its first three values (entries 4-6 stay 0) while an ascending one
    ends with the 4th-6th largest."""
    desc = np.arange(300, 200, -1, dtype=np.uint16).reshape(10, 10)
    asc = desc[::-1, ::-1].copy()
    assert Q._maxp_level(desc) == 0
    inner = np.sort(asc[1:-1].ravel())[::-1]
    assert Q._maxp_level(asc) == int(inner[3:6].astype(int).sum()) // 3


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(cases().keys()))
def test_gpu_quality_u16_matches_oracle(ctx, name):
    """QualityEstimate_ushort: exact (integer sums), so equal to the oracle."""
    from siril_amd import registration as R
    img = _u16(cases()[name])
    q = R.quality_estimate(img[None], ctx)
    e = Q.quality_estimate_ushort(img)
    assert (np.isnan(q[0]) and np.isnan(e)) or q[0] == e, (q[0], e)


@pytest.mark.gpu
def test_gpu_quality_u16_batch_window_and_orders():
    """HBM windows of 16-bit frames, including a descending-brightness frame
    (few list insertions) and a saturated one (values >= 65530 never enter)."""
    import torch
    from siril_amd import registration as R
    base = synth.star_field(300, 400, nstars=200, seed=9)
    fr = [np.roll(base, (i, 2 * i), (0, 1)) * (1 - 0.03 * i) + 0.05 for i in range(4)]
    y, x = np.mgrid[0:300, 0:400]
    fr.append(0.9 - 0.8 * (y * 400 + x) / (300 * 400) + 0.3 * base)          # descending scan
    fr.append(np.where(base > 0.5, 1.0, 0.2 + 0.5 * base))                     # saturated stars
    fr = np.stack([_u16(f) for f in fr])
    d = torch.from_numpy(fr.view(np.int16)).cuda()
    win = d[:, 20:276, 60:316]
    q = R.quality_estimate(win)
    for i in range(len(fr)):
        e = Q.quality_estimate_ushort(fr[i, 20:276, 60:316])
        assert (np.isnan(q[i]) and np.isnan(e)) or q[i] == e, (i, q[i], e)
