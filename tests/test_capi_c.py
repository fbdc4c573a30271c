"""A compiled C caller of include/sirilgpu.h (tests/capi_c/capi_check.c).

Siril's host is C: it would include the header and link libsirilgpu.so
(stacking.h:16 stack_method, deconvolution.h:138, demosaicing.h,
registration.h:15).  Every other test reaches the library through ctypes with
a hand-mirrored struct layout (siril_amd/_lib.py); this one builds a C99
program with gcc -Werror against the header alone, checks the struct layout
it sees against the ctypes mirror (CPU), and on the GPU runs the four drop-in
entry points on small inputs and compares their outputs with the oracle:
  * sgpu_stack_rows (Winsorized 3/3, N = 24): bit-exact vs oracle/stack_ref.c;
  * sgpu_dft_shifts: the injected integer shifts and oracle/dft_ref.py;
  * sgpu_fft_richardson_lucy (the reference's 14-argument signature):
    rel L-inf <= 1e-4 vs oracle/rl_ref.py (complex128);
  * sgpu_debayer_buffer_new_float (RCD, RGGB): bit-exact vs
    oracle/demosaic_ref.py (RCD parity with librtprocess unpinned).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "capi_c", "capi_check.c")
LIBDIR = os.path.join(ROOT, "siril_amd")

ST_N, ST_ROWS, ST_W = 24, 16, 40
DFT_S, DFT_NF = 64, 3
RL_W, RL_H, RL_KS, RL_IT = 80, 64, 15, 4
DM_W, DM_H = 40, 32


def _build(tmp):
    exe = os.path.join(tmp, "capi_check")
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-O1",
           "-I" + os.path.join(ROOT, "include"), SRC, "-o", exe,
           "-L" + LIBDIR, "-lsirilgpu", "-Wl,-rpath," + LIBDIR]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    from siril_amd import build as B
    B.build(verbose=False)
    return _build(str(tmp_path_factory.mktemp("capi")))


def test_c_caller_builds_and_struct_layout_matches_ctypes(exe):
    """gcc -std=c99 -pedantic -Werror compiles the header and links every
    entry point the program uses; sizeof / offsetof of sgpu_stack_params and
    sgpu_stack_seq_options as C sees them equal the ctypes mirror's."""
    from siril_amd._lib import ABI_VERSION, StackParams, StackSeqOptions
    r = subprocess.run([exe, "layout"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    seen = dict(line.rsplit(" ", 1) for line in r.stdout.strip().splitlines())
    assert int(seen["abi"]) == ABI_VERSION
    assert int(seen["sgpu_stack_params.size"]) == C.sizeof(StackParams)
    for name, _ in StackParams._fields_:
        assert int(seen[f"sgpu_stack_params.{name}"]) == getattr(StackParams, name).offset, name
    assert int(seen["sgpu_stack_seq_options.size"]) == C.sizeof(StackSeqOptions)
    for name in ("filter_included", "max_block_bytes"):
        assert int(seen[f"sgpu_stack_seq_options.{name}"]) == getattr(StackSeqOptions, name).offset, name


def _inputs(d):
    from siril_amd import synth
    from siril_amd.deconvolution import moffat_psf
    from oracle import rl_ref as R
    rng = np.random.default_rng(11)
    fr = (0.05 + 0.005 * rng.standard_normal((ST_N, ST_ROWS, ST_W))).astype(np.float32)
    m = rng.random(fr.shape) < 0.04
    fr[m] += rng.uniform(0.2, 0.6, int(m.sum())).astype(np.float32)
    fr = np.clip(fr, 1e-6, 1).astype(np.float32)
    fr[rng.random(fr.shape) < 0.02] = 0
    fr.tofile(os.path.join(d, "stack_frames.in.bin"))
    base = synth.star_field(DFT_S, DFT_S, nstars=12, seed=5)
    shifts = [(3, -5), (-7, 2), (11, 9)]
    sel = synth.shifted_frames(base, [(0, 0)] + shifts, seed=6)
    sel[0].tofile(os.path.join(d, "dft_ref.in.bin"))
    np.ascontiguousarray(sel[1:]).tofile(os.path.join(d, "dft_frames.in.bin"))
    K = moffat_psf(RL_KS, fwhm=3.0).astype(np.float32)
    img = synth.star_field(RL_H, RL_W, nstars=40, sigma=1.2, seed=3)
    obs = R.ifft2n(np.fft.fft2(img) * np.fft.fft2(R.padcirc(K, RL_H, RL_W, np.complex128))).real
    obs = np.clip(obs + np.random.default_rng(3).normal(0, 0.002, obs.shape), 1e-4, None).astype(np.float32)
    obs.tofile(os.path.join(d, "rl_img.in.bin"))
    K.tofile(os.path.join(d, "rl_psf.in.bin"))
    cfa = (rng.random((DM_H, DM_W)) * 0.5 + 0.1).astype(np.float32)
    cfa.tofile(os.path.join(d, "dm_cfa.in.bin"))
    return fr, sel, shifts, obs, K, cfa


@pytest.mark.gpu
def test_c_caller_entry_points_match_oracle(exe, oracle, tmp_path):
    from oracle import demosaic_ref as Dm, dft_ref, rl_ref as R
    d = str(tmp_path)
    fr, sel, shifts, obs, K, cfa = _inputs(d)
    r = subprocess.run([exe, "run", d], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rd = lambda n, dt, shape: np.fromfile(os.path.join(d, n), dt).reshape(shape)
    # stack_method drop-in: bit-exact mean, both maps, the totals
    out, rl, rh, counts = oracle.stack_rows(fr, 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(rd("stack_out.out.bin", np.uint32, out.shape), out.view(np.uint32))
    assert np.array_equal(rd("stack_rl.out.bin", np.uint16, rl.shape), rl)
    assert np.array_equal(rd("stack_rh.out.bin", np.uint16, rh.shape), rh)
    assert rd("stack_counts.out.bin", np.uint64, (2,)).tolist() == [int(x) for x in counts]
    # REG_DFT: integer shifts, the quantity set_shifts stores
    got = rd("dft_shifts.out.bin", np.int32, (DFT_NF, 2))
    for f in range(DFT_NF):
        sx, sy, _ = dft_ref.dft_shift(sel[0], sel[f + 1])
        assert (int(got[f, 0]), int(got[f, 1])) == (sx, sy)
    # fft_richardson_lucy (deconvolution.h:138 argument list)
    want = R.fft_richardson_lucy(obs[None], K[None], maxiter=RL_IT, regtype=R.REG_NONE_GRAD)[0]
    got = rd("rl_img.out.bin", np.float32, (RL_H, RL_W))
    assert float(np.abs(got.astype(np.float64) - want).max() / np.abs(want).max()) <= 1e-4
    # debayer_buffer_new_float, RCD RGGB
    want = Dm.debayer_buffer_new_float(cfa, Dm.BAYER_RCD, Dm.RGGB)
    assert np.array_equal(rd("dm_rgb.out.bin", np.float32, want.shape), want)
