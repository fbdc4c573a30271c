"""Frame-level data movement either side of the stack:
apply_reg with interpolation none (shift_fit_from_reg), extract_CFA_buffer,
split_cfa / merge_cfa.  Host logic on the CPU; HIP kernels on the GPU vs the
literal restatements in oracle/cfa_ref.py (bit-exact: pure data movement)."""
import numpy as np
import pytest

XTRANS = "GGRGGBGGBGGRBRGRBGGGBGGRGGRGGBRBGBRG"   # a 6x6 X-Trans layout (36 letters)


def test_apply_reg_shifts_host():
    """sgpu_apply_reg_shifts == Href^-1 * Himg + round_to_int (cvTransfH)."""
    from oracle import cfa_ref as R
    from siril_amd import registration as Rg
    rng = np.random.default_rng(3)
    Hs = [Rg.H_from_translation(float(dx), float(dy)) for dx, dy in rng.uniform(-40, 40, (12, 2))]
    Hs += [Rg.H_from_translation(2.5, -2.5), Rg.H_from_translation(-3.5, 3.5), Rg.H_from_translation(0.49999, 0)]
    for ref in (0, 5, len(Hs) - 1):
        sx, sy = Rg.apply_reg_shifts(Hs, ref)
        ex, ey = R.apply_reg_shifts(Hs, ref)
        assert np.array_equal(sx, ex) and np.array_equal(sy, ey)
        assert sx[ref] == 0 and sy[ref] == 0


@pytest.mark.parametrize("w,h", [(8, 6), (13, 7), (37, 25), (36, 36)])
@pytest.mark.parametrize("pat", ["RGGB", "GBRG", XTRANS])
def test_cfa_count_host(w, h, pat):
    from oracle import cfa_ref as R
    from siril_amd import demosaic as Dm
    from siril_amd.registration import compiled_pattern
    cp = compiled_pattern(pat)
    ps = 2 if len(pat) == 4 else 6
    img = np.arange(w * h, dtype=np.float32).reshape(h, w)
    for layer in (0, 1, 2):
        assert Dm.cfa_count(w, h, pat, layer) == len(R.extract_CFA_buffer(img, cp, ps, layer))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
def test_shift_frames_gpu(dtype):
    import torch
    from oracle import cfa_ref as R
    from siril_amd import registration as Rg
    rng = np.random.default_rng(5)
    n, h, w = 6, 37, 71
    fr = (rng.random((n, h, w)) * 60000).astype(dtype)
    sx = np.array([0, 3, -5, 70, -71, 2], np.int32)
    sy = np.array([0, -2, 7, 1, 0, -37], np.int32)
    d = torch.from_numpy(fr.view(np.int16) if dtype == np.uint16 else fr).cuda()
    out = Rg.shift_frames(d, sx, sy).cpu().numpy()
    if dtype == np.uint16:
        out = out.view(np.uint16)
    for f in range(n):
        assert np.array_equal(out[f], R.shift_fit_from_reg(fr[f], int(sx[f]), int(sy[f]))), f


@pytest.mark.gpu
@pytest.mark.parametrize("interp", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
def test_apply_reg_dft_translations_gpu(interp, dtype):
    """apply_reg of REG_DFT registrations (integer translations from
    set_shifts) with every interpolation: the rounded shift of
    shift_fit_from_reg for NONE, the exact phase-0 OpenCV warp = the same
    shift for NEAREST..LANCZOS4 (sgpu_apply_reg_device); sub-pixel
    translations are refused under 0-4 and rounded under NONE;
    non-translation homographies are refused."""
    import torch
    from oracle import cfa_ref as R
    from siril_amd import registration as Rg
    from siril_amd._lib import SgpuError
    rng = np.random.default_rng(50 + interp)
    n, h, w = 5, 29, 43
    fr = (rng.random((n, h, w)) * 60000).astype(dtype)
    d = torch.from_numpy(fr.view(np.int16) if dtype == np.uint16 else fr).cuda()
    Hs = [Rg.set_shifts(int(a), int(b)) for a, b in rng.integers(-12, 13, (n, 2))]
    out = Rg.apply_reg(d, Hs, 2, interp).cpu().numpy()
    out = out.view(np.uint16) if dtype == np.uint16 else out
    sx, sy = R.apply_reg_shifts(Hs, 2)
    for f in range(n):
        assert np.array_equal(out[f], R.shift_fit_from_reg(fr[f], int(sx[f]), int(sy[f]))), f
    sub = [H.copy() for H in Hs]
    sub[1][0, 2] += 0.25
    if interp == 5:
        out = Rg.apply_reg(d, sub, 2, interp).cpu().numpy()
        out = out.view(np.uint16) if dtype == np.uint16 else out
        sx, sy = R.apply_reg_shifts(sub, 2)
        assert np.array_equal(out[1], R.shift_fit_from_reg(fr[1], int(sx[1]), int(sy[1])))
    else:
        with pytest.raises(SgpuError):
            Rg.apply_reg(d, sub, 2, interp)
    rot = [H.copy() for H in Hs]
    rot[3][0, 1] = 0.01
    with pytest.raises(SgpuError):
        Rg.apply_reg(d, rot, 2, interp)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(8, 6), (13, 7), (64, 33), (37, 25)])
@pytest.mark.parametrize("pat", ["RGGB", "BGGR", "GRBG", XTRANS])
@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
def test_extract_cfa_gpu(w, h, pat, dtype):
    import torch
    from oracle import cfa_ref as R
    from siril_amd import demosaic as Dm
    from siril_amd.registration import compiled_pattern
    rng = np.random.default_rng(w * h)
    img = (rng.random((h, w)) * 60000).astype(dtype)
    d = torch.from_numpy(img.view(np.int16) if dtype == np.uint16 else img).cuda()
    cp = compiled_pattern(pat)
    for layer in (0, 1, 2):
        got = Dm.extract_cfa(d, pat, layer).cpu().numpy()
        if dtype == np.uint16:
            got = got.view(np.uint16)
        assert np.array_equal(got, R.extract_CFA_buffer(img, cp, 2 if len(pat) == 4 else 6, layer)), layer


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(8, 6), (13, 7), (64, 33), (200, 150)])
@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
def test_split_merge_cfa_gpu(w, h, dtype):
    import torch
    from oracle import cfa_ref as R
    from siril_amd import demosaic as Dm
    rng = np.random.default_rng(w + h)
    img = (rng.random((h, w)) * 60000).astype(dtype)
    d = torch.from_numpy(img.view(np.int16) if dtype == np.uint16 else img).cuda()
    planes = Dm.split_cfa(d)
    got = planes.cpu().numpy()
    if dtype == np.uint16:
        got = got.view(np.uint16)
    ref = R.split_cfa(img)
    assert np.array_equal(got, ref)
    merged = Dm.merge_cfa(planes).cpu().numpy()
    if dtype == np.uint16:
        merged = merged.view(np.uint16)
    assert np.array_equal(merged, R.merge_cfa(ref))
    assert np.array_equal(merged, img[: 2 * (h // 2), : 2 * (w // 2)])
