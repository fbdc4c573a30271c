"""Headless sequence path (siril_amd/sequence.py + csrc/sgpu_seq.cpp):
FITS / .seq host logic on the CPU, the `stack` command end to end on the GPU
(BASELINE config 1: mean of 10 synthetic 1024x1024 FITS frames), checked
against the oracle on the same data."""
import os

import numpy as np
import pytest


def test_fits_roundtrip(tmp_path):
    from siril_amd import sequence as Q
    rng = np.random.default_rng(3)
    a = rng.random((37, 53)).astype(np.float32)
    p = str(tmp_path / "a.fit")
    Q.write_fits(p, a)
    assert os.path.getsize(p) % 2880 == 0
    assert Q.fits_info(p) == (53, 37, -32)
    assert np.array_equal(Q.read_fits(p), a)
    part = Q.read_fits(p, -3, 10)                 # rows outside the image read as zero
    assert np.array_equal(part[3:], a[:7]) and not part[:3].any()
    u = rng.integers(0, 65536, (9, 11)).astype(np.uint16)
    q = str(tmp_path / "u.fit")
    Q.write_fits(q, u)
    assert Q.fits_info(q) == (11, 9, 16)
    assert np.array_equal(Q.read_fits(q), u)
    raw = open(q, "rb").read()
    assert b"BZERO   =                32768" in raw   # unsigned 16-bit convention


def _fits_bytes(cards, payload):
    hdr = b"".join(c.ljust(80).encode() for c in cards + ["END"])
    hdr += b" " * ((2880 - len(hdr) % 2880) % 2880)
    return hdr + payload + b"\0" * ((2880 - len(payload) % 2880) % 2880)


def test_fits_short_conventions(tmp_path):
    """src/tests/fits_scaling_test.c: BITPIX 16 with BZERO 2^15 and plain signed
    shorts both read as DATA_USHORT `stored + 32768` (:190-205, :317-332);
    physical BSCALE/BZERO float scaling is refused here (not the stack path)."""
    from siril_amd import sequence as Q
    from siril_amd._lib import SgpuError
    raw = np.array([-32768, -1, 0, 1, 1234, 32767], dtype=">i2")
    base = ["SIMPLE  =                    T", "BITPIX  =                   16", "NAXIS   =                    2",
            "NAXIS1  =                    3", "NAXIS2  =                    2"]
    want = (raw.astype(np.int32) + 32768).astype(np.uint16).reshape(2, 3)
    for extra in ([], ["BZERO   =                32768", "BSCALE  =                    1"]):
        p = tmp_path / f"s{len(extra)}.fit"
        p.write_bytes(_fits_bytes(base + extra, raw.tobytes()))
        assert np.array_equal(Q.read_fits(str(p)), want)
    p = tmp_path / "phys.fit"
    p.write_bytes(_fits_bytes(base + ["BZERO   =                  1.0", "BSCALE  =               0.0001"],
                              raw.tobytes()))
    with pytest.raises(SgpuError):
        Q.read_fits(str(p))


def test_stack_command_parse():
    from siril_amd import sequence as Q
    from siril_amd.stacking import METHOD_MEAN, METHOD_MEDIAN, Rejection
    c = Q.parse_stack_command("stack synth_ rej w 3 3 -nonorm -32b -out=r.fit".split())
    assert (c.seq, c.method, c.args.type_of_rejection, c.args.sig, c.force32b, c.out) == \
        ("synth_", METHOD_MEAN, Rejection.WINSORIZED, (3.0, 3.0), True, "r.fit")
    c = Q.parse_stack_command("stack s rej 2.5 2 -nonorm".split())   # number: default WINSORIZED
    assert c.args.type_of_rejection == Rejection.WINSORIZED and c.args.sig == (2.5, 2.0)
    c = Q.parse_stack_command("stack s mean sigma 1.5 4".split())
    assert c.args.type_of_rejection == Rejection.SIGMA and c.args.sig == (1.5, 4.0)
    c = Q.parse_stack_command("stack s mean n -32b".split())         # no sigmas needed for none
    assert c.args.type_of_rejection == Rejection.NO_REJEC and c.force32b
    # evaluate_stacking_should_output_32bits (stacking.c:48-73): mean/median
    # stacks are 32-bit by default, 16-bit only with com.pref.force_16bit
    assert c.use_32bit_output() and Q.parse_stack_command("stack s median".split()).use_32bit_output()
    assert not Q.parse_stack_command("stack s median".split()).use_32bit_output(Q.Preferences(force_16bit=True))
    assert Q.parse_stack_command("stack s median -32b".split()).use_32bit_output(Q.Preferences(force_16bit=True))
    assert Q.parse_stack_command("stack s median -noreg".split()).method == METHOD_MEDIAN
    from siril_amd.stacking import Normalization
    c = Q.parse_stack_command("stack s rej w 3 3 -norm=addscale -fastnorm".split())
    assert c.args.normalize == Normalization.ADDITIVE_SCALING and c.lite_norm
    c = Q.parse_stack_command("stack s rej w 3 3 -fastnorm -norm=mul".split())   # order matters
    assert c.args.normalize == Normalization.MULTIPLICATIVE and not c.lite_norm
    assert Q.parse_stack_command("stack s rej w 3 3 -norm=bogus".split()).args.normalize == 0
    for bad in ("stack s rej w 3", "stack s rej g 3 0.05", "stack s sum", "stack s rej w 3 3 -upscale",
                "stack s rej w 3 3 -bogus"):
        with pytest.raises(ValueError):
            Q.parse_stack_command(bad.split())
    assert Q.default_output("synth_") == "synth_stacked.fit"
    assert Q.default_output("dir/light.seq") == "dir/light_stacked.fit"


def test_seq_writer_layout(tmp_path):
    from siril_amd import sequence as Q
    p = str(tmp_path / "x.seq")
    Q.write_seq(p, "x_", 3, included=[True, False, True], shifts=[(0, 0), (2.0, -1.0), (-3.0, 4.0)])
    lines = [l for l in open(p).read().splitlines() if not l.startswith("#")]
    assert lines[0] == "S 'x_' 1 3 2 5 0 4 0 0 0" and lines[1] == "L 1"
    assert lines[2:5] == ["I 1 1", "I 2 0", "I 3 1"]
    h = lines[6].split()      # frame 2: h02 = dx = 2, h12 = -dy = 1
    assert h[0] == "R0" and float(h[10]) == 2.0 and float(h[13]) == 1.0


def _read_shifted(fr, dy):
    """The block reader's row map: output row R reads input row R - dy (zero outside)."""
    out = np.zeros_like(fr)
    h = fr.shape[0]
    for r in range(h):
        s = r - dy
        if 0 <= s < h:
            out[r] = fr[s]
    return out


@pytest.mark.gpu
def test_config1_mean_stack(tmp_path, oracle):
    """BASELINE config 1: `stack synth_ rej n -nonorm -32b` over 10 FITS frames
    1024x1024, bit-exact vs the oracle's no-rejection mean of the same arrays."""
    from siril_amd import sequence as Q, synth
    fr = synth.config1_frames(10, 1024, 1024)
    seq = synth.write_sequence(str(tmp_path), fr)
    out, _ = Q.run_command(f"stack {seq} rej n -nonorm -32b -out={tmp_path}/r.fit")
    res = Q.read_fits(out)
    ref, _, _, _ = oracle.stack_rows(fr, 0, (3, 3), nthreads=8)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_sequence_winsorized_registered_blocks(tmp_path, oracle):
    """Winsorized stack of a registered sequence, small row blocks (several
    reader/GPU pipeline steps), one excluded frame: x shift on the device,
    y shift in the reader, against the oracle on host-shifted frames."""
    from siril_amd import sequence as Q, synth
    from siril_amd.stacking import Rejection, StackingArgs
    rng = np.random.default_rng(8)
    n, h, w = 12, 96, 130
    fr = synth.frames_numpy(n, h, w, seed=5)
    shifts = [(0, 0)] + [(int(rng.integers(-6, 7)), int(rng.integers(-5, 6))) for _ in range(n - 1)]
    inc = [True] * n
    inc[4] = False
    seq = synth.write_sequence(str(tmp_path), fr, shifts=shifts, included=inc)
    out, counts = Q.stack_seq(seq, StackingArgs(Rejection.WINSORIZED, (3.0, 3.0)), out=str(tmp_path / "w.fit"),
                              use_32bit_output=True, max_block_bytes=n * w * 4 * 20,
                              filters=Q.SeqFilters(filter_included=True))
    res = Q.read_fits(out)
    keep = [i for i in range(n) if inc[i]]
    pre = np.stack([_read_shifted(fr[i], shifts[i][1]) for i in keep])
    ref, rl, rh, cnt = oracle.stack_rows(pre, 5, (3.0, 3.0), shift_dx=np.array([shifts[i][0] for i in keep], float),
                                         nthreads=8)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


@pytest.mark.gpu
def test_sequence_u16_median(tmp_path, oracle):
    """16-bit FITS sequence (BZERO 32768) median stack: 32-bit output by
    default (stacking.c:66-70), 16-bit output with com.pref.force_16bit."""
    from siril_amd import sequence as Q, synth
    rng = np.random.default_rng(9)
    fr = np.clip(np.round(1500 + 60 * rng.standard_normal((9, 40, 50))), 0, 65535).astype(np.uint16)
    seq = synth.write_sequence(str(tmp_path), fr, name="u_")
    out, _ = Q.run_command(f"stack {seq} median -nonorm", prefs=Q.Preferences(force_16bit=True))
    assert out.endswith("u_stacked.fit") and Q.fits_info(out)[2] == 16
    ref, _, _, _ = oracle.stack_rows_u16(fr, 0, (3, 3), method=1, use_32bit_output=False, nthreads=4)
    assert np.array_equal(Q.read_fits(out), ref)
    out, _ = Q.run_command(f"stack {seq} median -nonorm -out={tmp_path}/f.fit")
    assert Q.fits_info(out)[2] == -32
    ref, _, _, _ = oracle.stack_rows_u16(fr, 0, (3, 3), method=1, use_32bit_output=True, nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))


def test_force_16bit_refuses_float_sequence(tmp_path):
    """stacking.c:51-58: force_16bit with a 32-bit input sequence is an error."""
    from siril_amd import sequence as Q, synth
    seq = synth.write_sequence(str(tmp_path), synth.frames_numpy(3, 8, 8), name="f_")
    with pytest.raises(ValueError):
        Q.run_command(f"stack {seq} rej w 3 3", prefs=Q.Preferences(force_16bit=True))


def _float_fits(path, data, extra_cards=()):
    """Hand-written BITPIX -32 FITS (big-endian) with optional extra cards."""
    h, w = data.shape
    cards = ["SIMPLE  =                    T", "BITPIX  =                  -32", "NAXIS   =                    2",
             f"NAXIS1  = {w:20d}", f"NAXIS2  = {h:20d}"] + list(extra_cards)
    open(path, "wb").write(_fits_bytes(cards, np.ascontiguousarray(data, ">f4").tobytes()))


def test_float_read_rescale_rules(tmp_path):
    """Siril brings float FITS holding ADU values to [0, 1]:
    internal_read_partial_fits (image_format_fits.c:994-1007: DATAMAX, else a
    3-sample diagonal probe of the rows read, > 10 -> convert_floats) and
    readfits (:906-910: the file's max unless PROGRAM says Siril).  Host
    reader vs the numpy restatement (oracle/headless_ref.py), bit for bit."""
    from oracle import headless_ref as HR
    from siril_amd import sequence as Q
    rng = np.random.default_rng(4)
    adu = (100 + 2000 * rng.random((30, 17))).astype(np.float32)
    small = rng.random((30, 17)).astype(np.float32)
    mixed = small.copy()
    mixed[20:, :] *= 500.0            # only the upper rows are above 10
    cases = {
        "adu_nokey": (adu, [], None, False),
        "adu_key_small": (adu, ["DATAMAX =                  1.0"], 1.0, False),
        "small_key_big": (small, ["DATAMAX =              65535.0"], 65535.0, False),
        "small_nokey": (small, [], None, False),
        "mixed_nokey": (mixed, [], None, False),
        "siril_adu_nokey": (adu, ["PROGRAM = 'Siril 1.4.0'"], None, True),
        "siril_adu_key": (adu, ["PROGRAM = 'Siril 1.4.0'", "DATAMAX =              65535.0"], 65535.0, True),
    }
    for name, (a, cards, dm, siril) in cases.items():
        p = str(tmp_path / f"{name}.fit")
        _float_fits(p, a, cards)
        assert np.array_equal(Q.read_fits(p), a), name                               # raw
        for r0, n in ((0, 30), (5, 10), (18, 12), (-4, 9), (25, 10)):
            got = Q.read_fits(p, r0, n, mode=Q.READ_PARTIAL)
            a0, b0 = max(r0, 0), min(r0 + n, 30)
            want = np.zeros((n, 17), np.float32)
            want[a0 - r0:b0 - r0] = HR.partial_read_rescale(a[a0:b0], dm)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (name, r0, n)
        got = Q.read_fits(p, mode=Q.READ_WHOLE)
        want = HR.whole_read_rescale(a, dm, siril)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), name


def test_norm_to_0_1_range_restatement():
    """The vectorised oracle form equals the literal loop (index 0 excluded
    from min/max, zeros kept)."""
    from oracle import headless_ref as HR
    rng = np.random.default_rng(2)
    a = (rng.random((13, 11)) * 3 - 1).astype(np.float32)
    a[rng.random(a.shape) < 0.2] = 0.0
    a.flat[0] = 50.0                   # outside the min/max loop, still rescaled
    assert np.array_equal(HR.norm_to_0_1_range(a).view(np.uint32), HR.norm_to_0_1_range_fast(a).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("u16", [False, True])
def test_sequence_output_norm(tmp_path, oracle, u16):
    """`stack <seq> rej w 3 3 -nonorm -output_norm`: unclamped 32-bit result,
    then norm_to_0_1_range (median_and_mean.c:557-582, :1774-1775) on the
    device; bit-exact vs oracle stack + the restated post-pass."""
    from oracle import headless_ref as HR
    from siril_amd import sequence as Q, synth
    n, h, w = 10, 60, 90
    fr = synth.frames_numpy(n, h, w, seed=31)
    fr[2, 5:9, :] = 0.0                                   # missing samples
    fr[:, 0, 0] = fr[:, 0, 0] * 3.0                       # pixel 0 (outside the min/max loop) above 1
    if u16:
        fr16 = np.clip(np.round(fr * 40000.0), 0, 65535).astype(np.uint16)
        seq = synth.write_sequence(str(tmp_path), fr16, name="on16_")
        ref, _, _, _ = oracle.stack_rows_u16(fr16, 5, (3.0, 3.0), output_norm=True, use_32bit_output=True, nthreads=4)
    else:
        seq = synth.write_sequence(str(tmp_path), fr, name="on_")
        ref, _, _, _ = oracle.stack_rows(fr, 5, (3.0, 3.0), output_norm=True, nthreads=4)
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -output_norm -out={tmp_path}/o.fit")
    res = Q.read_fits(out)
    want = HR.norm_to_0_1_range(ref)
    assert np.array_equal(res.view(np.uint32), want.view(np.uint32))
    # pixel 0 is outside the reference's min/max loop: it may leave [0, 1]
    assert res.ravel()[1:].max() == 1.0 and res.ravel()[1:].min() >= 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("output_norm", [True, False])
def test_sequence_8bit_16bit_output(tmp_path, oracle, output_norm):
    """8-bit SER lights stacked to a 16-bit result (force_16bit): with
    -output_norm the mean is scaled by 65535/255 before round_to_WORD
    (normalize_to16bit, median_and_mean.c:547-555, 1729-1732); without it the
    result stays BYTE_IMG (:1326-1330) and is written as BITPIX 8."""
    from siril_amd import sequence as Q
    n, h, w = 9, 24, 40
    rng = np.random.default_rng(17)
    fr = np.clip(np.round(90 + 12 * rng.standard_normal((n, h, w))), 1, 255).astype(np.uint16)
    fr[4, 3, :7] = 250                                    # outliers to reject
    Q.write_ser(str(tmp_path / "b_.ser"), np.ascontiguousarray(fr[:, ::-1, :]), Q.SER_MONO, bit_depth=8)
    seq = str(tmp_path / "b_.seq")
    Q.write_seq(seq, "b_", n, kind="S")
    opt = "-output_norm" if output_norm else ""
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm {opt} -out={tmp_path}/b.fit",
                           prefs=Q.Preferences(force_16bit=True))
    hdr = open(out, "rb").read(2880).decode("ascii")
    bitpix = int(hdr[hdr.index("BITPIX  =") + 9:][:21])
    assert bitpix == (16 if output_norm else 8)
    ref, _, _, _ = oracle.stack_rows_u16(fr, 5, (3.0, 3.0), output_norm=output_norm, use_32bit_output=False,
                                         nthreads=4, bitpix8=True)
    res = Q.read_fits(out)
    assert np.array_equal(res, ref)
    if output_norm:
        assert res.max() > 255                            # scaled to the 16-bit range
    else:
        assert res.max() <= 255


@pytest.mark.gpu
@pytest.mark.parametrize("datamax", [True, False])
def test_sequence_float_adu(tmp_path, oracle, datamax):
    """Float FITS frames holding ADU values (DATAMAX > 10, or no DATAMAX and a
    probe above 10): Siril rescales every block by INV_USHRT_MAX_SINGLE on
    read, so the stack equals the oracle stack of the rescaled frames."""
    from oracle import headless_ref as HR
    from siril_amd import sequence as Q
    n, h, w = 8, 40, 56
    rng = np.random.default_rng(12)
    adu = np.clip(1200 + 80 * rng.standard_normal((n, h, w)), 1, 65535).astype(np.float32)
    adu[3, 10, 10] = 60000.0
    cards = ["DATAMAX =              65535.0"] if datamax else []
    for f in range(n):
        _float_fits(str(tmp_path / f"adu_{f + 1:05d}.fit"), adu[f], cards)
    seq = str(tmp_path / "adu_.seq")
    Q.write_seq(seq, "adu_", n)
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -out={tmp_path}/a.fit")
    res = Q.read_fits(out)
    scaled = HR.convert_floats(adu)
    ref, _, _, cnt = oracle.stack_rows(scaled, 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


@pytest.mark.gpu
@pytest.mark.parametrize("opts,lite", [("-norm=addscale", False), ("-norm=mul -fastnorm", True)])
def test_sequence_normalized_stack(tmp_path, oracle, opts, lite):
    """`stack <seq> rej w 3 3 -norm=... [-fastnorm] -32b`: the engine reads
    each included frame whole, computes the estimators on the GPU and the
    factors against the reference image (frame 0), then stacks.  Checked
    against the oracle stack driven by the same coefficients (recomputed
    from the in-memory frames) and the estimators against the oracle."""
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    n, h, w = 9, 80, 120
    fr = synth.frames_numpy(n, h, w, seed=17)
    fr = np.clip(fr * np.linspace(0.7, 1.3, n, dtype=np.float32)[:, None, None]
                 + np.linspace(0.0, 0.03, n, dtype=np.float32)[:, None, None], 1e-6, 1.0).astype(np.float32)
    inc = [True] * n
    inc[3] = False
    seq = synth.write_sequence(str(tmp_path), fr, included=inc)
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 {opts} -32b -filter-incl -out={tmp_path}/n.fit")
    res = Q.read_fits(out)
    keep = [i for i in range(n) if inc[i]]
    ctx = Context(0)
    norm = Normalization.ADDITIVE_SCALING if "addscale" in opts else Normalization.MULTIPLICATIVE
    off, mul, scl, st = N.compute_normalization(ctx, fr[keep], norm, ref_index=0, lite=lite)
    for j, i in enumerate(keep):
        o = oracle.norm_stats(fr[i], lite)
        assert st.median[j] == o[1] and st.mad[j] == o[2]
    ref, rl, rh, cnt = oracle.stack_rows(fr[keep], 5, (3.0, 3.0), norm=int(norm), scale=scl, offset=off, mul=mul,
                                         nthreads=8)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


@pytest.mark.gpu
def test_sequence_u16_normalized_stack(tmp_path, oracle):
    """16-bit FITS sequence, `rej w 3 3 -norm=addscale -32b`: 16-bit
    estimators (statistics_internal_ushort) on the GPU, then the 16-bit stack."""
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    fr = synth.frames_numpy(8, 50, 64, seed=23)
    fr = fr * np.linspace(0.8, 1.25, 8, dtype=np.float32)[:, None, None]
    fr16 = np.clip(np.round(fr * 65535.0), 0, 65535).astype(np.uint16)
    seq = synth.write_sequence(str(tmp_path), fr16, name="n16_")
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -norm=addscale -32b -out={tmp_path}/n16.fit")
    res = Q.read_fits(out)
    off, mul, scl, st = N.compute_normalization(Context(0), fr16, Normalization.ADDITIVE_SCALING, ref_index=0)
    for i in range(8):
        o = oracle.norm_stats(fr16[i])
        assert st.median[i] == o[1] and st.mad[i] == o[2] and st.location[i] == o[3]
    ref, _, _, cnt = oracle.stack_rows_u16(fr16, 5, (3.0, 3.0), norm=int(Normalization.ADDITIVE_SCALING),
                                           scale=scl, offset=off, mul=mul, nthreads=4)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


# ---------------------------------------------------------------- SER / FITSEQ
def test_ser_header_and_trailer(tmp_path):
    """The reference's SER tests (src/tests/ser_test.c) as fixtures of this
    reader: 3 frames 20x10 -> frame_count 3 (test_ser_image_number, :66-87);
    per-frame dates 100/200/300 s round-trip through the timestamp trailer
    (test_ser_dates, :128-155); a 40x20 RGB file keeps SER_RGB, its size, the
    observer string and date_utc (test_ser_create_from_copy, :244-282)."""
    from siril_amd import sequence as Q
    p = str(tmp_path / "a.ser")
    Q.write_ser(p, np.zeros((3, 10, 20), np.uint16))
    assert Q.ser_info(p)["frame_count"] == 3 and Q.ser_info(p)["timestamps"] == []
    Q.write_ser(p, np.zeros((3, 10, 20), np.uint16), unix_seconds=[100, 200, 300])
    inf = Q.ser_info(p)
    assert inf["frame_count"] == 3 and inf["timestamps"] == [100, 200, 300]
    Q.write_ser(p, np.zeros((3, 20, 40, 3), np.uint16), Q.SER_RGB, unix_seconds=[100, 200, 300],
                observer="super observer", date_utc=100)
    inf = Q.ser_info(p)
    assert (inf["color_id"], inf["width"], inf["height"], inf["frame_count"]) == (Q.SER_RGB, 40, 20, 3)
    assert inf["observer"] == "super observer" and inf["date_utc"] == 100
    assert inf["timestamps"][:2] == [100, 200]


def test_ser_header_frame_count_recomputed(tmp_path):
    """frame_count 0 in the header (a capture that crashed): recomputed from
    the file size (ser_recompute_frame_count, io/ser.c:179-200)."""
    from siril_amd import sequence as Q
    p = tmp_path / "b.ser"
    Q.write_ser(str(p), np.ones((4, 6, 8), np.uint16))
    raw = bytearray(p.read_bytes())
    raw[38:42] = b"\0\0\0\0"
    p.write_bytes(bytes(raw))
    assert Q.ser_info(str(p))["frame_count"] == 4


@pytest.mark.parametrize("depth,endian", [(8, 0), (12, 0), (16, 1), (16, 0)])
@pytest.mark.parametrize("color", [0, 100, 101])
def test_ser_block_rows(tmp_path, depth, endian, color):
    """The block reader's view of a SER frame (ser_read_opened_partial,
    io/ser.c:1054-1213 + the stack's row map): FITS-order row q is SER row
    H-1-q, samples widened / byte-swapped per the (inverted) endianness flag,
    RGB / BGR de-interleaved; rows outside the frame read as zero."""
    from siril_amd import sequence as Q
    rng = np.random.default_rng(depth + color + endian)
    h, w = 9, 13
    hi = 255 if depth <= 8 else (1 << depth) - 1
    shape = (3, h, w, 3) if color else (3, h, w)
    fr = rng.integers(0, hi + 1, shape).astype(np.uint16)
    p = str(tmp_path / "c.ser")
    Q.write_ser(p, fr, color, depth, endian)
    for f in range(3):
        for layer in (range(3) if color else [0]):
            plane = fr[f][..., layer if color != 101 else 2 - layer] if color else fr[f]
            want = plane[::-1]
            got = Q.read_frame_rows(p, f, layer)
            assert np.array_equal(got, want), (f, layer)
            part = Q.read_frame_rows(p, f, layer, row0=-2, nrows=5)
            assert not part[:2].any() and np.array_equal(part[2:], want[:3])


def test_fitseq_frames(tmp_path):
    """FITSEQ (io/fits_sequence.c:39-120): every image HDU is a frame."""
    from siril_amd import sequence as Q
    rng = np.random.default_rng(1)
    fr = rng.random((4, 7, 11)).astype(np.float32)
    p = str(tmp_path / "s.fit")
    Q.write_fitseq(p, fr)
    for f in range(4):
        assert np.array_equal(Q.read_frame_rows(p, f), fr[f])
    rgb = rng.integers(0, 65536, (3, 3, 5, 6)).astype(np.uint16)
    Q.write_fitseq(p, rgb)
    for f in range(3):
        for layer in range(3):
            assert np.array_equal(Q.read_frame_rows(p, f, layer), rgb[f, layer])


def test_rejmap_option_parse():
    from siril_amd import sequence as Q
    assert Q.parse_stack_command("stack s rej w 3 3 -rejmap".split()).rejmaps == 1
    assert Q.parse_stack_command("stack s rej w 3 3 -rejmaps".split()).rejmaps == 2
    assert Q.parse_stack_command("stack s rej n -rejmaps".split()).rejmaps == 0      # no rejection: ignored
    assert Q.parse_stack_command("stack s median -rejmap".split()).rejmaps == 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ser", "fitseq"])
def test_sequence_ser_fitseq_stack(tmp_path, oracle, kind):
    """Single-file sequences: a 16-bit SER (registered, one excluded frame)
    and a float FITSEQ, Winsorized, small row blocks; bit-exact vs the oracle
    on the frames as the block reader sees them."""
    from siril_amd import sequence as Q, synth
    from siril_amd.stacking import Rejection, StackingArgs
    rng = np.random.default_rng(77)
    n, h, w = 10, 40, 66
    fr = synth.frames_numpy(n, h, w, seed=41)
    if kind == "ser":
        fr = np.clip(np.round(fr * 50000), 0, 65535).astype(np.uint16)
    shifts = [(0, 0)] + [(int(rng.integers(-4, 5)), int(rng.integers(-4, 5))) for _ in range(n - 1)]
    inc = [True] * n
    inc[6] = False
    seq = synth.write_sequence(str(tmp_path), fr, name="k_", shifts=shifts, included=inc, kind=kind)
    es = 2 if kind == "ser" else 4
    out, counts = Q.stack_seq(seq, StackingArgs(Rejection.WINSORIZED, (3.0, 3.0)), out=str(tmp_path / "o.fit"),
                              use_32bit_output=True, max_block_bytes=n * w * es * 9,
                              filters=Q.SeqFilters(filter_included=True))
    res = Q.read_fits(out)
    keep = [i for i in range(n) if inc[i]]
    pre = np.stack([_read_shifted(fr[i], shifts[i][1]) for i in keep])
    dx = np.array([shifts[i][0] for i in keep], float)
    if kind == "ser":
        ref, _, _, cnt = oracle.stack_rows_u16(pre, 5, (3.0, 3.0), shift_dx=dx, nthreads=8)
    else:
        ref, _, _, cnt = oracle.stack_rows(pre, 5, (3.0, 3.0), shift_dx=dx, nthreads=8)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,rej", [("fits", "-rejmaps"), ("ser", "-rejmap")])
def test_sequence_rgb_with_rejmaps(tmp_path, oracle, kind, rej):
    """Three-layer sequences (RGB FITS planes / RGB SER): every layer stacked
    with the registration of the first layer that has data (R1 here), output
    NAXIS3 = 3; -rejmaps / -rejmap write the maps as count * (1/N) floats
    (command.c:11778-11803)."""
    import os
    from siril_amd import sequence as Q, synth
    rng = np.random.default_rng(5)
    n, h, w = 9, 30, 44
    fr = np.stack([synth.frames_numpy(n, h, w, seed=60 + c) for c in range(3)], axis=1)   # [N, 3, H, W]
    if kind == "ser":
        fr = np.clip(np.round(fr * 50000), 0, 65535).astype(np.uint16)
    shifts = [(0, 0)] + [(int(rng.integers(-3, 4)), int(rng.integers(-3, 4))) for _ in range(n - 1)]
    seq = synth.write_sequence(str(tmp_path), fr, name="rgb_", shifts=shifts, kind=kind, reg_layer=1)
    outp = str(tmp_path / "rgb.fit")
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b {rej} -out={outp}")
    res = Q.read_fits(out)
    assert res.shape == (3, h, w)
    tot = [0, 0]
    dx = np.array([s[0] for s in shifts], float)
    for c in range(3):
        pre = np.stack([_read_shifted(fr[i, c], shifts[i][1]) for i in range(n)])
        if kind == "ser":
            ref, rl, rh, cnt = oracle.stack_rows_u16(pre, 5, (3.0, 3.0), shift_dx=dx, nthreads=8)
        else:
            ref, rl, rh, cnt = oracle.stack_rows(pre, 5, (3.0, 3.0), shift_dx=dx, nthreads=8)
        assert np.array_equal(res[c].view(np.uint32), ref.view(np.uint32)), c
        tot[0] += int(cnt[0])
        tot[1] += int(cnt[1])
        op = np.float32(1.0) / np.float32(n)
        if rej == "-rejmaps":
            lo = Q.read_fits(outp.replace(".fit", "_low_rejmap.fit"), layer=c)
            hi = Q.read_fits(outp.replace(".fit", "_high_rejmap.fit"), layer=c)
            assert np.array_equal(lo, (rl.astype(np.float32) * op).astype(np.float32))
            assert np.array_equal(hi, (rh.astype(np.float32) * op).astype(np.float32))
        else:
            m = Q.read_fits(outp.replace(".fit", "_low+high_rejmap.fit"), layer=c)
            assert np.array_equal(m, ((rl.astype(np.int32) + rh).astype(np.float32) * op).astype(np.float32))
    assert counts == tuple(tot)
    assert not os.path.exists(outp.replace(".fit", "_high_rejmap.fit")) or rej == "-rejmaps"


@pytest.mark.gpu
def test_sequence_reference_image_from_registration(tmp_path, oracle):
    """reference_image -1 in the .seq: the normalization reference is the
    included frame with the best (lowest) FWHM of the registration data
    (sequence_find_refimage, io/sequence.c:1791-1846), not the first frame."""
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    n, h, w = 7, 40, 60
    fr = synth.frames_numpy(n, h, w, seed=19)
    fr = np.clip(fr * np.linspace(0.7, 1.3, n, dtype=np.float32)[:, None, None], 1e-6, 1.0).astype(np.float32)
    fwhm = [3.0, 2.9, 2.5, 3.3, 2.1, 2.8, 3.0]        # frame 4 is the best; frame 2 next
    inc = [True] * n
    seq = synth.write_sequence(str(tmp_path), fr, shifts=[(0, 0)] * n, included=inc, reference=-1, fwhm=fwhm)
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -norm=addscale -32b -out={tmp_path}/r.fit")
    res = Q.read_fits(out)
    off, mul, scl, st = N.compute_normalization(Context(0), fr, Normalization.ADDITIVE_SCALING, ref_index=4)
    ref, _, _, cnt = oracle.stack_rows(fr, 5, (3.0, 3.0), norm=int(Normalization.ADDITIVE_SCALING), scale=scl,
                                       offset=off, mul=mul, nthreads=8)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))


# ---------------------------------------------------------------- round 3:
# the rest of the `stack` command line (command.c:11493-11614)

def _regdata(n, seed):
    from oracle import seqfilter_ref as R
    rng = np.random.default_rng(seed)
    return [R.RegData(fwhm=rng.uniform(1.5, 4.5), wfwhm=rng.uniform(1.8, 5.0), roundness=rng.uniform(0.3, 0.95),
                      quality=rng.uniform(0.1, 1.0), bkg=rng.uniform(0.01, 0.2), nstars=int(rng.integers(5, 400)))
            for _ in range(n)]


def _regkw(reg):
    return {"wfwhm": [r.wfwhm for r in reg], "roundness": [r.roundness for r in reg],
            "bkg": [r.bkg for r in reg], "nstars": [r.nstars for r in reg]}


@pytest.mark.gpu
def test_stack_uses_every_frame_without_filter(tmp_path, oracle):
    """No filter option: seq_filter_all (sequence_filtering.c:283-286) -- the
    .seq's excluded frames are stacked too; -filter-incl leaves them out."""
    from siril_amd import sequence as Q, synth
    n, h, w = 8, 30, 40
    fr = synth.frames_numpy(n, h, w, seed=71)
    inc = [True] * n
    inc[2] = inc[5] = False
    seq = synth.write_sequence(str(tmp_path), fr, included=inc)
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -out={tmp_path}/all.fit")
    ref, _, _, cnt = oracle.stack_rows(fr, 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -filter-incl -out={tmp_path}/inc.fit")
    keep = [i for i in range(n) if inc[i]]
    ref, _, _, _ = oracle.stack_rows(fr[keep], 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("opts,weighting", [
    ("-filter-fwhm=80% -filter-round=0.4", None),
    ("-filter-wfwhm=1k -filter-nbstars=50", None),
    ("-filter-quality=60% -weight=wfwhm", "wfwhm"),
    ("-filter-bkg=90% -weight=nbstars", "nbstars"),
    ("-weight=nbstack", "nbstack"),
])
def test_stack_filters_and_weights(tmp_path, oracle, opts, weighting):
    """-filter-* frame selection (literal, percent and k-sigma thresholds on the
    registration data) and -weight=wfwhm / nbstars / nbstack, against the
    restatement (oracle/seqfilter_ref.py) driving the oracle stack."""
    from oracle import seqfilter_ref as R
    from siril_amd import sequence as Q, synth
    n, h, w = 14, 24, 36
    fr = synth.frames_numpy(n, h, w, seed=73)
    reg = _regdata(n, 74)
    stackcnt = [1 + (i * 7) % 5 for i in range(n)]
    seq = synth.write_sequence(str(tmp_path), fr, shifts=[(0, 0)] * n, reference=0,
                               fwhm=[r.fwhm for r in reg], quality=[r.quality for r in reg], regdata=_regkw(reg),
                               stackcnt=stackcnt)
    cmd = Q.parse_stack_command(f"stack {seq} rej w 3 3 -nonorm -32b {opts}".split())
    cfg = R.FilterConfig(**{k: getattr(cmd.filters, k) for k in R.FilterConfig.__dataclass_fields__})
    keep, _ = R.select_frames(cfg, reg, [True] * n, 0)
    assert Q.stack_frames(seq, cmd.filters)[0] == keep
    wts = None
    if weighting == "wfwhm":
        wts = R.wfwhm_weights(reg, keep)
    elif weighting == "nbstars":
        wts = R.nbstars_weights(reg, keep)
    elif weighting == "nbstack":
        wts = np.array([float(stackcnt[i]) for i in keep])
    out, counts = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b {opts} -out={tmp_path}/f.fit")
    ref, _, _, cnt = oracle.stack_rows(fr[keep], 5, (3.0, 3.0), weights=wts, nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))
    assert counts == (int(cnt[0]), int(cnt[1]))


@pytest.mark.gpu
def test_stack_rgb_equal(tmp_path, oracle):
    """`-norm=addscale -rgb_equal` (the reference's OSC script line): every
    layer's factors against the reference image's estimators of the
    registration layer (normalization.c:157-159)."""
    from oracle import seqfilter_ref as R
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    n, h, w = 7, 28, 36
    fr = np.stack([synth.frames_numpy(n, h, w, seed=80 + c) * np.float32(0.6 + 0.2 * c) for c in range(3)], axis=1)
    fr = np.clip(fr, 1e-6, 1).astype(np.float32)
    seq = synth.write_sequence(str(tmp_path), fr, name="eq_", shifts=[(0, 0)] * n, reg_layer=1)
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -norm=addscale -rgb_equal -32b -out={tmp_path}/eq.fit")
    res = Q.read_fits(out)
    ctx = Context(0)
    est = []
    for c in range(3):
        st = N.norm_stats(ctx, fr[:, c])
        est.append((st.location, np.ones(n), st.scale))        # ADDITIVE_SCALING: location, scale
    facs = R.equalized_factors(int(Normalization.ADDITIVE_SCALING), est, 0, 1)
    for c in range(3):
        off, mul, scl = facs[c]
        ref, _, _, _ = oracle.stack_rows(fr[:, c], 5, (3.0, 3.0), norm=int(Normalization.ADDITIVE_SCALING),
                                         scale=scl, offset=off, mul=mul, nthreads=4)
        assert np.array_equal(res[c].view(np.uint32), ref.view(np.uint32)), c
    out2, _ = Q.run_command(f"stack {seq} rej w 3 3 -norm=addscale -32b -out={tmp_path}/ne.fit")
    assert not np.array_equal(Q.read_fits(out2), res)      # equalization changed layers 0 and 2


@pytest.mark.gpu
def test_stack_reference_shift_offset(tmp_path, oracle):
    """Registration relative to a reference image that has its own shift:
    the stack subtracts the reference's shift truncated to int
    (args->offset, median_and_mean.c:190-194, :416-417, :1622)."""
    from siril_amd import sequence as Q, synth
    n, h, w = 6, 30, 44
    fr = synth.frames_numpy(n, h, w, seed=91)
    shifts = [(2.7, -1.6), (0.0, 0.0), (5.2, 3.4), (-3.6, 2.2), (1.4, -4.8), (7.1, 0.4)]
    seq = synth.write_sequence(str(tmp_path), fr, shifts=shifts, reference=0)
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -out={tmp_path}/o.fit")
    ox, oy = int(shifts[0][0]), int(shifts[0][1])                  # (int) truncation
    rnd = lambda v: int(np.floor(v + 0.5)) if v >= 0 else int(np.ceil(v - 0.5))
    dy = [rnd(s[1] - oy) for s in shifts]
    dx = np.array([rnd(s[0] - ox) for s in shifts], float)
    pre = np.stack([_read_shifted(fr[i], dy[i]) for i in range(n)])
    ref, _, _, _ = oracle.stack_rows(pre, 5, (3.0, 3.0), shift_dx=dx, nthreads=4)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_stack_maximize_framing(tmp_path, oracle):
    """-maximize: the output is the union of the shifted frames
    (stack_open_all_files, median_and_mean.c:160-190: size (int)xmax -
    (int)xmin + 1, origin ((int)xmin, -(int)ymin)); each frame sits on the
    canvas at its shift, zero (missing) elsewhere."""
    from siril_amd import sequence as Q, synth
    n, h, w = 6, 26, 34
    fr = synth.frames_numpy(n, h, w, seed=93)
    shifts = [(0.0, 0.0), (3.0, 2.0), (-2.0, 4.0), (5.0, -3.0), (1.0, 1.0), (-4.0, -2.0)]
    seq = synth.write_sequence(str(tmp_path), fr, shifts=shifts, reference=0)
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -nonorm -32b -maximize -out={tmp_path}/m.fit")
    res = Q.read_fits(out)
    h02 = [s[0] for s in shifts]
    h12 = [-s[1] for s in shifts]
    xmin, xmax = min(h02), max(x + w for x in h02)
    ymin, ymax = min(h12), max(y + h for y in h12)
    W, H = int(xmax) - int(xmin) + 1, int(ymax) - int(ymin) + 1
    assert res.shape == (H, W)
    offx, offy = int(xmin), -int(ymin)
    canvas = np.zeros((n, H, W), np.float32)
    for i, (dx, dy) in enumerate(shifts):
        sx, sy = int(round(dx - offx)), int(round(dy - offy)) + (H - h)
        for r in range(H):                       # FITS row R reads the frame's row R - sy
            q = r - sy
            if 0 <= q < h:
                for x in range(W):
                    if 0 <= x - sx < w:
                        canvas[i, r, x] = fr[i, q, x - sx]
    ref, _, _, _ = oracle.stack_rows(canvas, 5, (3.0, 3.0), nthreads=4)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("norm", ["addscale", "mul"])
def test_stack_maximize_overlap_norm(tmp_path, oracle, norm):
    """`-maximize -overlap_norm` (command.c:11696-11699, normalization.c:
    666-906): the coefficients come from every pair's overlap on the
    registration layer's translations, then the frames are stacked on the
    maximized canvas.  Expected: the library's own overlap coefficients
    (checked against the restatement in test_overlap_norm.py) driving the
    oracle stack of the canvas; -overlap_norm without -maximize is ignored."""
    from siril_amd import normalization as N, sequence as Q, synth
    from siril_amd.stacking import Context, Normalization
    n, h, w = 6, 30, 40
    base = synth.frames_numpy(1, h + 20, w + 20, seed=97)[0]
    shifts = [(0.0, 0.0), (3.0, 2.0), (-2.0, 4.0), (5.0, -3.0), (1.0, 1.0), (-4.0, -2.0)]
    fr = np.zeros((n, h, w), np.float32)
    for i, (dx, dy) in enumerate(shifts):
        sx, sy = 10 + int(dx), 10 - int(dy)
        fr[i] = base[sy:sy + h, sx:sx + w] * np.float32(0.8 + 0.1 * i) + np.float32(0.01 * i)
    seq = synth.write_sequence(str(tmp_path), fr, shifts=shifts, reference=0)
    out, _ = Q.run_command(f"stack {seq} rej w 3 3 -norm={norm} -32b -maximize -overlap_norm -out={tmp_path}/o.fit")
    res = Q.read_fits(out)
    h02 = np.array([s[0] for s in shifts])
    h12 = np.array([-s[1] for s in shifts])
    nz = Normalization.ADDITIVE_SCALING if norm == "addscale" else Normalization.MULTIPLICATIVE
    off, mul, scl, _ = N.compute_normalization_overlaps(Context(0), fr, nz, h02, h12, ref_index=0)
    xmin, xmax = h02.min(), max(x + w for x in h02)
    ymin, ymax = h12.min(), max(y + h for y in h12)
    W, H = int(xmax) - int(xmin) + 1, int(ymax) - int(ymin) + 1
    assert res.shape == (H, W)
    offx, offy = int(xmin), -int(ymin)
    canvas = np.zeros((n, H, W), np.float32)
    for i, (dx, dy) in enumerate(shifts):
        sx, sy = int(round(dx - offx)), int(round(dy - offy)) + (H - h)
        for r in range(H):
            q = r - sy
            if 0 <= q < h:
                lo, hi = max(0, sx), min(W, sx + w)
                canvas[i, r, lo:hi] = fr[i, q, lo - sx:hi - sx]
    ref, _, _, _ = oracle.stack_rows(canvas, 5, (3.0, 3.0), norm=int(nz), scale=scl, offset=off, mul=mul,
                                     nthreads=4)
    assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
    # without -maximize the overlap request is dropped: the whole-frame pass
    out2, _ = Q.run_command(f"stack {seq} rej w 3 3 -norm={norm} -32b -overlap_norm -out={tmp_path}/o2.fit")
    out3, _ = Q.run_command(f"stack {seq} rej w 3 3 -norm={norm} -32b -out={tmp_path}/o3.fit")
    assert np.array_equal(Q.read_fits(out2).view(np.uint32), Q.read_fits(out3).view(np.uint32))


@pytest.mark.gpu
def test_compat_seq_entry_stacks_included_frames(tmp_path, oracle):
    """sgpu_stack_seq_ex2 (the pre-options entry point) keeps its ABI-3
    behaviour: only the .seq's included frames are stacked, so a caller that
    sized the GESD critical values for them gets the stack of those frames."""
    import ctypes as C
    from siril_amd import stacking as S, synth
    from siril_amd._lib import lib, StackParams
    n, h, w = 10, 20, 32
    fr = synth.frames_numpy(n, h, w, seed=81)
    inc = [True] * n
    inc[1] = inc[6] = inc[7] = False
    seq = synth.write_sequence(str(tmp_path), fr, included=inc)
    keep = [i for i in range(n) if inc[i]]
    crit = S.gesd_critical_values(len(keep), 0.3, 0.05)           # sized for the included count
    p = StackParams()
    p.method, p.type_of_rejection = 0, 7
    p.sig[0], p.sig[1] = 0.3, 0.05
    p.critical_value = crit.ctypes.data_as(C.POINTER(C.c_float))
    counts = np.zeros(2, np.uint64)
    ctx = S.Context(0)
    out = str(tmp_path / "compat.fit")
    rc = lib().sgpu_stack_seq_ex2(ctx.h, seq.encode(), C.byref(p), 0, 1, out.encode(),
                                  counts.ctypes.data_as(C.c_void_p), 0, 0, 0)
    assert rc == 0
    from siril_amd import sequence as Q
    ref, _, _, cnt = oracle.stack_rows(fr[keep], 7, (0.3, 0.05), nthreads=4, crit=crit)
    assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32))
    assert counts.tolist() == [int(cnt[0]), int(cnt[1])]
    ctx.close()


@pytest.mark.gpu
def test_input_bitpix_restored_after_8bit_sequence(tmp_path, oracle):
    """An 8-bit SER stack with -output_norm scales its 16-bit result by
    65535/255 (normalize_to16bit); that source bit depth belongs to the call:
    a later 16-bit row stack with output_norm on the same context must not be
    scaled."""
    from siril_amd import sequence as Q, stacking as S
    n, h, w = 9, 16, 24
    rng = np.random.default_rng(5)
    fr8 = np.clip(np.round(90 + 12 * rng.standard_normal((n, h, w))), 1, 255).astype(np.uint16)
    Q.write_ser(str(tmp_path / "b_.ser"), np.ascontiguousarray(fr8[:, ::-1, :]), Q.SER_MONO, bit_depth=8)
    seq = str(tmp_path / "b_.seq")
    Q.write_seq(seq, "b_", n, kind="S")
    ctx = S.Context(0)
    Q.run_command(f"stack {seq} rej w 3 3 -nonorm -output_norm -out={tmp_path}/b.fit", ctx=ctx,
                  prefs=Q.Preferences(force_16bit=True))
    fr16 = np.clip(np.round(3000 + 200 * rng.standard_normal((n, h, w))), 1, 65535).astype(np.uint16)
    res = ctx.stack(fr16, S.StackingArgs(S.Rejection.WINSORIZED, (3.0, 3.0), output_norm=True),
                    use_32bit_output=False)
    ref, _, _, _ = oracle.stack_rows_u16(fr16, 5, (3.0, 3.0), output_norm=True, use_32bit_output=False,
                                         nthreads=4, bitpix8=False)
    assert np.array_equal(res.result, ref)
    ctx.close()


@pytest.mark.gpu
def test_sequence_failed_stack_keeps_result(tmp_path):
    """The result streams to a temporary file renamed over the path only when
    the last block is written: a stack that fails part-way leaves
    the earlier result at that path untouched and no partial file behind;
    sgpu_release_seq_buffers frees the kept buffers and the next stack is
    unchanged."""
    import glob
    import os
    from siril_amd import sequence as Q, synth
    from siril_amd.stacking import Context, Rejection, StackingArgs
    n, h, w = 10, 41, 52
    fr = synth.frames_numpy(n, h, w, seed=8)
    seq = synth.write_sequence(str(tmp_path), fr, name="f_", kind="fits")
    ctx = Context(0)
    try:
        args = StackingArgs(Rejection.WINSORIZED, (3.0, 3.0))
        out = str(tmp_path / "res.fit")
        Q.stack_seq(seq, args, out=out, use_32bit_output=True, ctx=ctx)
        before = open(out, "rb").read()
        ctx.release_seq_buffers()
        again, _ = Q.stack_seq(seq, args, out=str(tmp_path / "again.fit"), use_32bit_output=True, ctx=ctx,
                               max_block_bytes=n * w * 4 * 7)
        assert open(again, "rb").read()[2880:] == before[2880:]
        # a frame cut short: its later rows cannot be read
        frames = sorted(glob.glob(str(tmp_path / "f_*.fit")))
        victim = frames[3]
        size = os.path.getsize(victim)
        with open(victim, "r+b") as f:
            f.truncate(size - 2880 * 3)
        with pytest.raises(Exception):
            Q.stack_seq(seq, args, out=out, use_32bit_output=True, ctx=ctx, max_block_bytes=n * w * 4 * 7)
        assert open(out, "rb").read() == before
        assert not glob.glob(str(tmp_path / "*.sgpu-part"))
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["fits", "ser"])
def test_sequence_pinned_pipeline_blocks(tmp_path, oracle, kind):
    """The block pipeline (round 5: page-locked block buffers, H2D on a copy
    stream overlapping the next block's read, double-buffered device blocks):
    a many-block plan with every reader count gives the one-block result bit
    for bit, and the pipeline's own measurements are consistent (blocks, H2D
    bytes = every sample once, page-locked buffers, reader threads)."""
    from siril_amd import sequence as Q, synth
    from siril_amd.stacking import Context, Rejection, StackingArgs
    n, h, w = 12, 57, 70
    fr = synth.frames_numpy(n, h, w, seed=5)
    if kind == "ser":
        fr = np.clip(np.round(fr * 50000), 0, 65535).astype(np.uint16)
    es = 2 if kind == "ser" else 4
    seq = synth.write_sequence(str(tmp_path), fr, name="p_", kind=kind)
    ctx = Context(0)
    try:
        args = StackingArgs(Rejection.WINSORIZED, (3.0, 3.0))
        one, c1 = Q.stack_seq(seq, args, out=str(tmp_path / "one.fit"), use_32bit_output=True, ctx=ctx)
        ref = Q.read_fits(one)
        for readers, rows in ((1, 5), (3, 8), (16, 13)):
            ctx.set_seq_readers(readers)
            out, c = Q.stack_seq(seq, args, out=str(tmp_path / f"b{readers}.fit"), use_32bit_output=True,
                                 ctx=ctx, max_block_bytes=n * w * es * rows, rejmaps=2)
            assert np.array_equal(Q.read_fits(out).view(np.uint32), ref.view(np.uint32)), readers
            assert c == c1
            st = ctx.last_seq_stats()
            first = rows // 4 if h > rows and rows >= 4 else 0      # the quarter-size first block
            assert st["blocks"] == (1 if first else 0) + -(-(h - first) // rows), st
            assert st["h2d_bytes"] == n * h * w * es, st
            assert st["pinned"] and st["readers"] == min(readers, n), st
            assert st["h2d_ms"] > 0 and st["kernel_ms"] > 0
        pre = fr.astype(np.float32) if kind == "fits" else fr
        want = (oracle.stack_rows(pre, 5, (3.0, 3.0), nthreads=8)[0] if kind == "fits"
                else oracle.stack_rows_u16(pre, 5, (3.0, 3.0), nthreads=8)[0])
        assert np.array_equal(ref.view(np.uint32), want.view(np.uint32))
    finally:
        ctx.close()
