"""Headless sequence stacking: Siril's scripting path `stack <seq> ...`.

Mirrors the reference's command surface for the stacking methods this engine
runs (core/command.c:11985-12076 process_stackone and
parse_stack_command_line): `rej`/`mean` with a rejection letter or name
(p, s, a, m, l, w, g, n and their long forms; a number in that position means
the default WINSORIZED) and sigma low/high, or `med`/`median`; options
`-nonorm`, `-32b`, `-output_norm`, `-out=<file>`, `-noreg` (the reference
uses the sequence's registration when present).  The work happens in the
C-ABI (`sgpu_stack_seq`, siril_amd/csrc/sgpu_seq.cpp): .seq reader, FITS
block reader with the registration y-shift, GPU stack per block, FITS writer.
`-norm=add|addscale|mul|mulscale` and `-fastnorm` run the per-frame
normalization statistics on the GPU first (DATA_FLOAT sequences).
`sum`, `min`, `max`, overlap normalization and the frame filters are not
part of this engine and raise `SgpuError`-like ValueErrors.

Also the format helpers the tests and the synthetic config-1 generator use:
`write_fits` / `read_fits` (BITPIX -32, or 16 with BZERO 32768) and
`write_seq` (io/seqfile.c:730-910 layout for a regular FITS sequence).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from ._lib import check, lib
from .stacking import (METHOD_MEAN, METHOD_MEDIAN, Context, Normalization, Rejection, StackingArgs,
                       _Keep, _params)

REJ_WORDS = {
    "p": Rejection.PERCENTILE, "percentile": Rejection.PERCENTILE,
    "s": Rejection.SIGMA, "sigma": Rejection.SIGMA,
    "a": Rejection.MAD, "mad": Rejection.MAD,
    "m": Rejection.SIGMEDIAN, "median": Rejection.SIGMEDIAN,
    "l": Rejection.LINEARFIT, "linear": Rejection.LINEARFIT,
    "w": Rejection.WINSORIZED, "winsorized": Rejection.WINSORIZED,
    "g": Rejection.GESDT, "generalized": Rejection.GESDT,
    "n": Rejection.NO_REJEC, "none": Rejection.NO_REJEC,
}


# ------------------------------------------------------------------- formats
def write_fits(path: str, data: np.ndarray, stackcnt: Optional[int] = None):
    """FITS image: float32 -> BITPIX -32, uint16 -> BITPIX 16/BZERO 32768;
    [H, W] (one plane) or [3, H, W] (RGB planes).  Row 0 of a plane is the
    first FITS row (bottom of the image).  stackcnt: a STACKCNT card."""
    a = np.ascontiguousarray(data)
    if stackcnt is not None:
        with open(path, "wb") as f:
            f.write(_hdu_bytes(a, True, [f"STACKCNT= {int(stackcnt):20d}"]))
        return
    bitpix = {np.dtype(np.float32): -32, np.dtype(np.uint16): 16}.get(a.dtype)
    if bitpix is None or a.ndim not in (2, 3) or (a.ndim == 3 and a.shape[0] != 3):
        raise ValueError("write_fits takes a [H, W] or [3, H, W] float32 or uint16 array")
    nl = 1 if a.ndim == 2 else 3
    check(lib().sgpu_fits_write_planes(path.encode(), a.ctypes.data_as(C.c_void_p), a.shape[-1], a.shape[-2], nl,
                                       bitpix), "sgpu_fits_write_planes")


def _hdu_bytes(a: np.ndarray, primary: bool, extra=()) -> bytes:
    """One FITS HDU (header + big-endian data) of a [H, W] or [L, H, W] array."""
    bitpix = {np.dtype(np.float32): -32, np.dtype(np.uint16): 16}[a.dtype]
    cards = ["SIMPLE  =                    T" if primary else "XTENSION= 'IMAGE   '",
             f"BITPIX  = {bitpix:20d}", f"NAXIS   = {a.ndim:20d}", f"NAXIS1  = {a.shape[-1]:20d}",
             f"NAXIS2  = {a.shape[-2]:20d}"]
    if a.ndim == 3:
        cards.append(f"NAXIS3  = {a.shape[0]:20d}")
    if not primary:
        cards += ["PCOUNT  =                    0", "GCOUNT  =                    1"]
    if bitpix == 16:
        cards += ["BZERO   =                32768", "BSCALE  =                    1"]
        payload = (a.astype(np.int32) - 32768).astype(">i2").tobytes()
    else:
        payload = a.astype(">f4").tobytes()
    hdr = b"".join(c.ljust(80).encode() for c in cards + list(extra) + ["END"])
    hdr += b" " * ((2880 - len(hdr) % 2880) % 2880)
    return hdr + payload + b"\0" * ((2880 - len(payload) % 2880) % 2880)


def write_fitseq(path: str, frames: np.ndarray):
    """A FITS sequence file (io/fits_sequence.c): frame 0 in the primary HDU,
    the others in IMAGE extensions.  frames: [N, H, W] or [N, 3, H, W]."""
    with open(path, "wb") as f:
        for i in range(frames.shape[0]):
            f.write(_hdu_bytes(np.ascontiguousarray(frames[i]), i == 0))


SER_MONO, SER_RGB, SER_BGR = 0, 100, 101


def write_ser(path: str, frames: np.ndarray, color_id: int = SER_MONO, bit_depth: int = 16, endian_flag: int = 0,
              unix_seconds=None, observer: str = "", date_utc: int = 0):
    """SER file (io/ser.c layout): frames [N, H, W] (mono / CFA) or
    [N, H, W, 3] (RGB or BGR interleaved) uint16 in the file's top-down row
    order; endian_flag as Siril reads it (0 little-endian, 1 big-endian)."""
    a = np.ascontiguousarray(frames, np.uint16)
    n, h, w = a.shape[:3]
    ts = None if unix_seconds is None else np.ascontiguousarray(unix_seconds, np.int64)
    check(lib().sgpu_ser_write(path.encode(), a.ctypes.data_as(C.c_void_p), n, w, h, color_id, bit_depth,
                               endian_flag, None if ts is None else ts.ctypes.data_as(C.c_void_p),
                               observer.encode(), date_utc), "sgpu_ser_write")


def ser_info(path: str, max_ts: int = 4096) -> dict:
    w, h, n, col, bd, en = (C.c_int() for _ in range(6))
    obs = C.create_string_buffer(40)
    du = C.c_uint64()
    ts = np.zeros(max_ts, np.int64)
    r = lib().sgpu_ser_info(path.encode(), C.byref(w), C.byref(h), C.byref(n), C.byref(col), C.byref(bd),
                            C.byref(en), obs, C.byref(du), ts.ctypes.data_as(C.c_void_p), max_ts)
    if r < 0:
        check(r, "sgpu_ser_info")
    return {"width": w.value, "height": h.value, "frame_count": n.value, "color_id": col.value,
            "bit_depth": bd.value, "endian_flag": en.value, "observer": obs.value.decode(errors="replace"),
            "date_utc": du.value, "timestamps": ts[:r].tolist()}


def fits_info(path: str):
    w, h, b = C.c_long(), C.c_long(), C.c_int()
    check(lib().sgpu_fits_info(path.encode(), C.byref(w), C.byref(h), C.byref(b)), "sgpu_fits_info")
    return int(w.value), int(h.value), int(b.value)


READ_RAW, READ_PARTIAL, READ_WHOLE = 0, 1, 2


def fits_layers(path: str) -> int:
    n = lib().sgpu_fits_layers(path.encode())
    if n < 0:
        check(n, "sgpu_fits_layers")
    return n


def read_fits(path: str, row0: int = 0, nrows: Optional[int] = None, mode: int = READ_RAW,
              layer: Optional[int] = None) -> np.ndarray:
    """Rows [row0, row0+nrows) in FITS order (zero outside the image); all
    planes ([3, rows, W]) of an RGB image unless `layer` is given.
    mode: READ_RAW stored values; READ_PARTIAL / READ_WHOLE bring float data to
    [0, 1] as Siril's block reader (image_format_fits.c:994-1007) / readfits
    (:906-910) do (x * INV_USHRT_MAX_SINGLE when the data max is above 10)."""
    w, h, b = fits_info(path)
    nrows = h - row0 if nrows is None else nrows
    nl = fits_layers(path)
    layers = [layer] if layer is not None else list(range(nl))
    out = np.empty((len(layers), nrows, w), np.float32 if b == -32 else np.uint16)
    for j, l in enumerate(layers):
        check(lib().sgpu_image_read_rows(path.encode(), 0, l, row0, nrows, out[j].ctypes.data_as(C.c_void_p), mode),
              "sgpu_image_read_rows")
    return out[0] if len(layers) == 1 else out


def read_frame_rows(path: str, frame: int, layer: int = 0, row0: int = 0, nrows: Optional[int] = None,
                    mode: int = READ_RAW, width: Optional[int] = None, height: Optional[int] = None,
                    dtype=np.uint16) -> np.ndarray:
    """Rows of one frame of a FITSEQ / SER file as the stack's block reader
    sees them (FITS row order; SER rows are stored top-down)."""
    if width is None or height is None:
        if path.endswith(".ser"):
            inf = ser_info(path)
            width, height = inf["width"], inf["height"]
        else:
            width, height, b = fits_info(path)
            dtype = np.float32 if b == -32 else np.uint16
    nrows = height - row0 if nrows is None else nrows
    out = np.empty((nrows, width), dtype)
    check(lib().sgpu_image_read_rows(path.encode(), frame, layer, row0, nrows, out.ctypes.data_as(C.c_void_p), mode),
          "sgpu_image_read_rows")
    return out


def write_seq(path: str, name: str, number: int, beg: int = 1, fixed: int = 5, reference: int = 0,
              included: Optional[Sequence[bool]] = None, shifts: Optional[Sequence[tuple]] = None,
              kind: Optional[str] = None, nb_layers: int = 1, reg_layer: int = 0, fwhm=None, quality=None,
              wfwhm=None, roundness=None, bkg=None, nstars=None):
    """Sequence file, version 4 (io/seqfile.c:730-910): S, T (kind "S" SER,
    "F" FITSEQ; None regular FITS), L and I lines, and R<reg_layer> lines with
    the shift-only homography when `shifts` (dx, dy) is given (h02 = dx,
    h12 = -dy, registration.c:306-313) and optional per-frame registration
    values (fwhm, weighted fwhm, roundness, quality, background, stars;
    seqfile.c:814-829)."""
    inc = list(included) if included is not None else [True] * number
    lines = ["#Siril sequence file. Contains list of images, selection, registration data and statistics",
             "#S 'sequence_name' start_index nb_images nb_selected fixed_len reference_image version"
             " variable_size fz_flag drizzle_flag",
             f"S '{name}' {beg} {number} {sum(bool(x) for x in inc)} {fixed} {reference} 4 0 0 0"]
    if kind:
        lines.append(f"T{kind}")
    lines.append(f"L {nb_layers}")
    for i in range(number):
        lines.append(f"I {(beg + i) if not kind else i} {int(bool(inc[i]))}")
    if shifts is not None:
        for i, (dx, dy) in enumerate(shifts):
            v = [0 if a is None else a[i] for a in (fwhm, wfwhm, roundness, quality, bkg)]
            ns = 0 if nstars is None else int(nstars[i])
            lines.append(f"R{reg_layer} {v[0]:.9g} {v[1]:.9g} {v[2]:.9g} {v[3]:.17g} {v[4]:.9g} {ns} "
                         f"H 1 0 {dx:.17g} 0 1 {-dy:.17g} 0 0 1")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def frame_name(name: str, num: int, fixed: int = 5) -> str:
    return f"{name}{num:0{fixed}d}.fit"


# ------------------------------------------------------------------- stacking
@dataclass
class Preferences:
    """The com.pref fields the stack command reads (core/settings.c)."""
    force_16bit: bool = False        # settings.c:38
    # the block plan of -feather= stacks (stack_compute_parallel_blocks):
    # com.max_thread and the rows stack_get_max_number_of_rows allows
    # (0: one thread, the whole image)
    max_thread: int = 0
    stack_max_rows: int = 0


# weightingType (stacking/stacking.h:47-53)
NO_WEIGHT, NBSTARS_WEIGHT, WFWHM_WEIGHT, NOISE_WEIGHT, NBSTACK_WEIGHT = range(5)
WEIGHT_WORDS = {"noise": NOISE_WEIGHT, "nbstars": NBSTARS_WEIGHT, "nbstack": NBSTACK_WEIGHT, "wfwhm": WFWHM_WEIGHT}


@dataclass
class SeqFilters:
    """struct seq_filter_config (core/sequence_filtering.h:36-40): a literal
    value, or a percentage (`%`) / k-sigma (`k`) of the sequence's values."""
    f_fwhm: float = 0.0
    f_fwhm_p: float = 0.0
    f_fwhm_k: bool = False
    f_wfwhm: float = 0.0
    f_wfwhm_p: float = 0.0
    f_wfwhm_k: bool = False
    f_round: float = 0.0
    f_round_p: float = 0.0
    f_round_k: bool = False
    f_quality: float = 0.0
    f_quality_p: float = 0.0
    f_quality_k: bool = False
    f_bkg: float = 0.0
    f_bkg_p: float = 0.0
    f_bkg_k: bool = False
    f_nbstars: float = 0.0
    f_nbstars_p: float = 0.0
    f_nbstars_k: bool = False
    filter_included: bool = False


# -filter-<name>= prefixes (command.c:11075-11190) -> SeqFilters field stem
FILTER_WORDS = [("-filter-fwhm=", "fwhm"), ("-filter-wfwhm=", "wfwhm"), ("-filter-round=", "round"),
                ("-filter-roundness=", "round"), ("-filter-qual=", "quality"), ("-filter-quality=", "quality"),
                ("-filter-bkg=", "bkg"), ("-filter-background=", "bkg"), ("-filter-nbstars=", "nbstars")]


def _strtof(text: str):
    """strtof's longest float prefix: (value, rest) or (None, text)."""
    import re
    m = re.match(r"\s*[+-]?(?:(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?|inf(?:inity)?|nan)", text, re.I)
    if not m:
        return None, text
    return float(np.float32(float(m.group(0)))), text[m.end():]


def parse_filter_arg(word: str, f: SeqFilters) -> bool:
    """parse_filter_args (command.c:11073-11191): True when `word` is a filter
    option (ValueError on a bad value)."""
    if word.startswith("-filter-incl"):          # also -filter-included
        f.filter_included = True
        return True
    for prefix, stem in FILTER_WORDS:
        if word.startswith(prefix):
            value = word[len(prefix):]
            if value == "":
                raise ValueError(f"Missing argument to {word}, aborting.")
            v, rest = _strtof(value)
            if v is None:
                raise ValueError(f"Could not parse argument `{value}' to the filter `{word}', aborting.")
            if rest[:1] in ("%", "k"):
                setattr(f, f"f_{stem}_p", v)
                setattr(f, f"f_{stem}_k", rest[:1] == "k")
            else:
                setattr(f, f"f_{stem}", v)
            return True
    return False


@dataclass
class StackCommand:
    seq: str
    method: int
    args: StackingArgs
    force32b: bool = False           # -32b (command.c:11507)
    out: Optional[str] = None
    use_registration: bool = True
    lite_norm: bool = False
    rejmaps: int = 0                 # -rejmap 1 (merged low+high), -rejmaps 2 (command.c:11592-11602)
    equalize_rgb: bool = False       # -rgb_equal (command.c:11570-11577)
    weighting: int = NO_WEIGHT       # -weight= (command.c:11513-11530)
    filters: SeqFilters = field(default_factory=SeqFilters)
    maximize: bool = False           # -maximize (command.c:11603)
    overlap_norm: bool = False       # -overlap_norm (command.c:11507-11512)
    feather: int = 0                 # -feather= (command.c:11553-11569)

    def use_32bit_output(self, prefs: Optional[Preferences] = None) -> bool:
        """args.use_32bit_output = force32b || evaluate_stacking_should_output_32bits
        (command.c:11718; stacking.c:48-73): mean/median stacks are 32-bit unless
        com.pref.force_16bit, which refuses a 32-bit input sequence."""
        prefs = prefs or Preferences()
        return self.force32b or not prefs.force_16bit


def parse_stack_command(words: Sequence[str]) -> StackCommand:
    """`stack seqfilename { rej | mean } [type] sigma_low sigma_high [options]`
    or `stack seqfilename { med | median } [options]` (command.c:12000-12070)."""
    w = list(words)
    if w and w[0] == "stack":
        w = w[1:]
    if len(w) < 2:
        raise ValueError("usage: stack seqfilename {rej|mean|med|median} ...")
    seq, meth = w[0], w[1]
    args = StackingArgs()
    opts_at = 2
    if meth in ("med", "median"):
        method = METHOD_MEDIAN
    elif meth in ("rej", "mean"):
        method = METHOD_MEAN
        if len(w) < 3:
            raise ValueError("Missing arguments for rejection stacking.")
        shift = 1
        rt = REJ_WORDS.get(w[2])
        if rt is None:
            rt, shift = Rejection.WINSORIZED, 0
        args.type_of_rejection = rt

        def num(s):
            try:
                return float(s)
            except (TypeError, ValueError):
                return None
        lo = num(w[2 + shift]) if len(w) > 2 + shift else None
        hi = num(w[3 + shift]) if len(w) > 3 + shift else None
        if lo is None or hi is None or lo < 0 or hi < 0:
            if rt != Rejection.NO_REJEC:
                raise ValueError("The average stacking with rejection requires two extra arguments:"
                                 " sigma low and high.")
            opts_at = 2 + shift
        else:
            args.sig = (lo, hi)
            opts_at = 4 + shift
        if rt in (Rejection.GESDT, Rejection.PERCENTILE) and (args.sig[0] > 1.0 or args.sig[1] > 1.0):
            raise ValueError("Extra parameters of this rejection algorithm must be between 0 and 1.")
    elif meth in ("sum", "min", "max"):
        raise ValueError(f"stacking method '{meth}' is not part of the MI355X engine")
    else:
        raise ValueError(f"Stacking method type '{meth}' is invalid")
    cmd = StackCommand(seq, method, args)
    rej_ok = method == METHOD_MEAN           # allow_rej_options (command.c:12050-12062)
    force_no_norm = False
    for o in w[opts_at:]:
        if o in ("-nonorm", "-no_norm"):
            force_no_norm = True
        elif o == "-32b":
            cmd.force32b = True
        elif o == "-output_norm":
            args.output_norm = True
        elif o.startswith("-out="):
            cmd.out = o[5:]
        elif o == "-noreg":
            cmd.use_registration = False
        elif o.startswith("-rejmap"):
            # only with rejection stacking; ignored (with a message) otherwise
            if method == METHOD_MEAN and args.type_of_rejection != Rejection.NO_REJEC:
                cmd.rejmaps = 2 if o.endswith("s") else 1
        elif o == "-fastnorm":
            # order-dependent like the reference: ignored unless -norm= came first (command.c:11531-11538)
            if args.normalize != Normalization.NO_NORM:
                cmd.lite_norm = True
        elif o.startswith("-norm="):
            # unknown values are ignored, as command.c:11539-11551 does
            v = {"add": Normalization.ADDITIVE, "addscale": Normalization.ADDITIVE_SCALING,
                 "mul": Normalization.MULTIPLICATIVE, "mulscale": Normalization.MULTIPLICATIVE_SCALING}.get(o[6:])
            if v is not None:
                args.normalize = v
        elif o == "-rgb_equal":
            # order-dependent like -fastnorm: only after -norm= (command.c:11570-11577)
            if args.normalize != Normalization.NO_NORM:
                cmd.equalize_rgb = True
        elif o.startswith("-weight="):
            if rej_ok:
                if o[8:] not in WEIGHT_WORDS:
                    raise ValueError(f"Unknown argument to {o}, aborting.")
                cmd.weighting = WEIGHT_WORDS[o[8:]]
        elif o == "-overlap_norm":
            if rej_ok:
                cmd.overlap_norm = True
        elif o.startswith("-feather="):
            if rej_ok:
                v, rest = _strtof(o[9:])
                if v is None or v < 0 or v != int(v):
                    raise ValueError(f"Unknown argument to {o}, aborting.")
                cmd.feather = min(int(v), 2000)
        elif o == "-maximize":
            cmd.maximize = True
        elif o == "-upscale":
            raise ValueError("stack option '-upscale' (upscale at stacking) is not part of the MI355X engine")
        elif parse_filter_arg(o, cmd.filters):
            pass
        else:
            raise ValueError(f"Unexpected argument to stacking `{o}', aborting.")
    if force_no_norm:                        # stack_one_seq (command.c:11645-11648)
        args.normalize = Normalization.NO_NORM
    return cmd


def default_output(seq: str) -> str:
    """seqname + ("" if it ends with '_' or '-' else "_") + "stacked" + ".fit"
    (command.c:11744-11749)."""
    base = seq[:-4] if seq.endswith(".seq") else seq
    return base + ("" if base.endswith(("_", "-")) else "_") + "stacked.fit"


def _options(lite_norm=False, rejmaps=0, equalize_rgb=False, weighting=NO_WEIGHT, filters=None,
             maximize=False, overlap_norm=False, feather=0, max_block_bytes=0, block_threads=0, block_max_rows=0):
    from ._lib import StackSeqOptions
    o = StackSeqOptions()
    o.lite_norm, o.rejmaps, o.equalize_rgb, o.weighting = int(bool(lite_norm)), int(rejmaps), int(bool(equalize_rgb)), \
        int(weighting)
    f = filters or SeqFilters()
    for name, _ in StackSeqOptions._fields_:
        if name.startswith("f_") or name == "filter_included":
            setattr(o, name, getattr(f, name))
    o.maximize, o.overlap_norm, o.feather = int(bool(maximize)), int(bool(overlap_norm)), int(feather)
    o.max_block_bytes = int(max_block_bytes)
    o.block_threads, o.block_max_rows = int(block_threads), int(block_max_rows)
    return o


def stack_frames(seq: str, filters: Optional[SeqFilters] = None):
    """(sequence indices the stack uses, reference image) for these filters
    (sgpu_stack_seq_frames: setup_filtered_data / stack_fill_list_of_unfiltered_images)."""
    o = _options(filters=filters)
    n, ref = C.c_int(0), C.c_int(0)
    check(lib().sgpu_stack_seq_frames(seq.encode(), C.byref(o), None, 0, C.byref(n), C.byref(ref)),
          "sgpu_stack_seq_frames")
    idx = np.zeros(max(n.value, 1), np.int32)
    check(lib().sgpu_stack_seq_frames(seq.encode(), C.byref(o), idx.ctypes.data_as(C.c_void_p), n.value, C.byref(n),
                                      C.byref(ref)), "sgpu_stack_seq_frames")
    return [int(i) for i in idx[:n.value]], int(ref.value)


def stack_seq(seq: str, args: StackingArgs, method: int = METHOD_MEAN, out: Optional[str] = None,
              use_32bit_output: bool = False, use_registration: bool = True,
              ctx: Optional[Context] = None, max_block_bytes: int = 0, lite_norm: bool = False, rejmaps: int = 0,
              filters: Optional[SeqFilters] = None, equalize_rgb: bool = False, weighting: int = NO_WEIGHT,
              maximize: bool = False, overlap_norm: bool = False, feather: int = 0, block_threads: int = 0,
              block_max_rows: int = 0):
    """Stack a sequence (regular FITS, FITSEQ or SER) with the GPU engine as the
    headless `stack` command does; returns (output path, (rejected_low,
    rejected_high)).  Frames: all images of the sequence unless `filters`
    selects (SeqFilters.filter_included = -filter-incl).  With
    args.normalize set and no coefficient arrays, the engine computes the
    normalization first (per-frame estimators on the GPU; lite_norm =
    -fastnorm, equalize_rgb = -rgb_equal).  feather > 0: -feather= masks over
    Siril's block plan for block_threads / block_max_rows (see
    sgpu_stack_blocks)."""
    ctx = ctx or Context(0)
    out = out or default_output(seq)
    keep = _Keep()
    o = _options(lite_norm, rejmaps, equalize_rgb, weighting, filters, maximize, overlap_norm, feather,
                 max_block_bytes, block_threads, block_max_rows)
    # nframes only matters here for GESD critical values (the selected
    # frames: one more pass over every frame header, so only for GESDT)
    gesd = method == METHOD_MEAN and int(args.type_of_rejection) == int(Rejection.GESDT) and \
        args.critical_value is None
    n = len(stack_frames(seq, filters)[0]) if gesd and os.path.exists(seq if seq.endswith(".seq") else seq + ".seq") \
        else 1
    p = _params(args, method, n, keep)
    counts = np.zeros(2, np.uint64)
    check(lib().sgpu_stack_seq_opts(ctx.h, seq.encode(), C.byref(p), int(use_registration), int(use_32bit_output),
                                    out.encode(), counts.ctypes.data_as(C.c_void_p), C.byref(o)),
          "sgpu_stack_seq_opts")
    return out, (int(counts[0]), int(counts[1]))


def run_command(line: str, ctx: Optional[Context] = None, prefs: Optional[Preferences] = None):
    """Run one `stack` command line; prefs = com.pref (default: Siril's defaults)."""
    cmd = parse_stack_command(line.split())
    if cmd.feather and (prefs is None or not (prefs.max_thread and prefs.stack_max_rows)):
        # the masks are upscaled per block of Siril's plan
        # (stack_compute_parallel_blocks), which depends on com.max_thread
        # and the memory budget; the single-block default is exact only
        # against a one-thread, whole-image Siril run
        import warnings
        warnings.warn("-feather= without Preferences.max_thread / stack_max_rows: one block over the whole "
                      "image (Siril plans one block per thread; the mask upscale differs at its seams)",
                      stacklevel=2)
    prefs = prefs or Preferences()
    if prefs.force_16bit and not cmd.force32b and _sequence_is_float(cmd.seq):
        # evaluate_stacking_should_output_32bits (stacking.c:51-58)
        raise ValueError("Input sequence is in 32-bit format but preferences are set to 16-bit output format.")
    return stack_seq(cmd.seq, cmd.args, cmd.method, cmd.out, cmd.use_32bit_output(prefs), cmd.use_registration,
                     ctx, lite_norm=cmd.lite_norm, rejmaps=cmd.rejmaps, filters=cmd.filters,
                     equalize_rgb=cmd.equalize_rgb, weighting=cmd.weighting, maximize=cmd.maximize,
                     overlap_norm=cmd.overlap_norm, feather=cmd.feather, block_threads=prefs.max_thread,
                     block_max_rows=prefs.stack_max_rows)


def _sequence_is_float(seq: str) -> bool:
    """bitpix of the sequence's first included frame is -32."""
    path = seq if seq.endswith(".seq") else seq + ".seq"
    d = os.path.dirname(path)
    name, fixed, first = None, 5, None
    with open(path) as f:
        for line in f:
            if line.startswith("TS"):
                return False                     # SER: 8/16-bit data
            if line.startswith("TF"):
                base = path[:-4]
                for ext in (".fit", ".fits", ".fts"):
                    if os.path.exists(base + ext):
                        return fits_info(base + ext)[2] == -32
                return False
            if line.startswith("S "):
                parts = line[2:].strip()
                if parts.startswith("'"):
                    name, rest = parts[1:].split("'", 1)
                    rest = rest.split()
                else:
                    name, *rest = parts.split()
                fixed = int(rest[3])
            elif line.startswith("I ") and first is None:
                num, inc = line.split()[1:3]
                if inc != "0":
                    first = int(num)
    for ext in (".fit", ".fits", ".fts"):
        p = os.path.join(d, f"{name}{first:0{fixed}d}{ext}")
        if os.path.exists(p):
            return fits_info(p)[2] == -32
    return False
