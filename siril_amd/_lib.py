"""ctypes binding of the in-tree C-ABI library (include/sirilgpu.h).

The product path is the HIP library; there is no CPU fallback.  `lib()`
raises when libsirilgpu.so is missing, and every compute call raises when no
HIP device is present.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SGPU_LIB") or os.path.join(PKG, "libsirilgpu.so")

# exported symbols, in include/sirilgpu.h order
EXPORTS = (
    "sgpu_abi_version", "sgpu_device_count", "sgpu_init", "sgpu_release", "sgpu_set_stream", "sgpu_synchronize",
    "sgpu_last_error", "sgpu_stack_rows", "sgpu_stack_rows_device", "sgpu_last_exact_pixels", "sgpu_last_order_sensitive",
    "sgpu_set_exact_only", "sgpu_set_timing", "sgpu_last_timing", "sgpu_stack_rows_u16",
    "sgpu_stack_rows_u16_device", "sgpu_dft_shifts", "sgpu_dft_register_device",
    "sgpu_quality_estimate_device", "sgpu_quality_estimate", "sgpu_normalize_quality",
    "sgpu_quality_estimate_u16_device", "sgpu_quality_estimate_u16",
    "sgpu_fft_richardson_lucy", "sgpu_naive_richardson_lucy", "sgpu_rl_fft", "sgpu_rl_naive",
    "sgpu_rl_fft_device", "sgpu_rl_naive_device", "sgpu_rl_set_memory", "sgpu_rl_last_conv_launches",
    "sgpu_rl_last_iter_flops", "sgpu_dft_shifts_cfa", "sgpu_dft_register_cfa_device",
    "sgpu_interpolate_nongreen_device", "sgpu_debayer_buffer_new_float",
    "sgpu_debayer_buffer_superpixel_float", "sgpu_debayer_device", "sgpu_superpixel_device", "sgpu_free",
    "sgpu_debayer_buffer_new_ushort", "sgpu_debayer_u16_device",
    "sgpu_bgnoise_device", "sgpu_bgnoise_u16_device", "sgpu_bgnoise", "sgpu_bgnoise_u16",
    "sgpu_stack_seq", "sgpu_stack_seq_ex", "sgpu_norm_stats_device", "sgpu_norm_stats",
    "sgpu_norm_stats_u16_device", "sgpu_norm_stats_u16", "sgpu_norm_factors",
    "sgpu_fits_info", "sgpu_fits_read_rows", "sgpu_fits_read_rows_ex", "sgpu_fits_write",
    "sgpu_norm_to_0_1_range_device", "sgpu_multi_init", "sgpu_multi_release", "sgpu_multi_size",
    "sgpu_multi_context", "sgpu_multi_stack_rows", "sgpu_multi_stack_rows_u16", "sgpu_row_bands",
    "sgpu_mean_partial_device", "sgpu_mean_finish_device", "sgpu_mean_partial_guard_device",
    "sgpu_mean_finish_guard_device", "sgpu_gather_columns_device", "sgpu_dft_register_u16_device",
    "sgpu_dft_shifts_u16", "sgpu_interpolate_nongreen_u16_device", "sgpu_apply_reg_device",
    "sgpu_debayer_buffer_siril_ushort", "sgpu_debayer_siril_u16_device", "sgpu_apply_reg_shifts", "sgpu_shift_frames_device",
    "sgpu_extract_cfa_device", "sgpu_cfa_count", "sgpu_split_cfa_device", "sgpu_merge_cfa_device",
    "sgpu_stack_seq_ex2", "sgpu_fits_layers", "sgpu_image_read_rows", "sgpu_fits_write_planes", "sgpu_ser_write",
    "sgpu_ser_info", "sgpu_overlap_rect", "sgpu_overlap_stats_device", "sgpu_overlap_stats_u16_device",
    "sgpu_overlap_factors", "sgpu_rl_last_fft_convs", "sgpu_rl_last_iter_bytes",
    "sgpu_stack_rows_planes", "sgpu_stack_rows_planes_device", "sgpu_stack_rows_u16_planes_device",
    "sgpu_set_input_bitpix", "sgpu_stack_seq_opts", "sgpu_stack_seq_frames",
    "sgpu_stack_blocks", "sgpu_feather_mask_size", "sgpu_feather_masks_device", "sgpu_feather_block_area",
    "sgpu_feather_block_device", "sgpu_set_seq_readers", "sgpu_last_seq_stats", "sgpu_release_seq_buffers",
)

SGPU_OK = 0
SGPU_NO_DEVICE = -20
ABI_VERSION = 4          # SGPU_ABI_VERSION of include/sirilgpu.h this binding is written against


class StackParams(C.Structure):
    """sgpu_stack_params (include/sirilgpu.h)."""
    _fields_ = [
        ("method", C.c_int),
        ("type_of_rejection", C.c_int),
        ("sig", C.c_float * 2),
        ("normalize", C.c_int),
        ("scale", C.POINTER(C.c_double)),
        ("offset", C.POINTER(C.c_double)),
        ("mul", C.POINTER(C.c_double)),
        ("shiftx", C.POINTER(C.c_int)),
        ("weights", C.POINTER(C.c_double)),
        ("critical_value", C.POINTER(C.c_float)),
        ("output_norm", C.c_int),
    ]


class StackSeqOptions(C.Structure):
    """sgpu_stack_seq_options (include/sirilgpu.h)."""
    _fields_ = [("lite_norm", C.c_int), ("rejmaps", C.c_int), ("equalize_rgb", C.c_int), ("weighting", C.c_int)] + \
        [(f, C.c_float) for f in ("f_fwhm", "f_fwhm_p", "f_wfwhm", "f_wfwhm_p", "f_round", "f_round_p", "f_quality",
                                  "f_quality_p", "f_bkg", "f_bkg_p", "f_nbstars", "f_nbstars_p")] + \
        [(f, C.c_int) for f in ("f_fwhm_k", "f_wfwhm_k", "f_round_k", "f_quality_k", "f_bkg_k", "f_nbstars_k",
                                "filter_included", "maximize", "overlap_norm", "feather")] + \
        [("max_block_bytes", C.c_long), ("block_threads", C.c_int), ("block_max_rows", C.c_long)]


class SgpuError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib().sgpu_last_error().decode(errors="replace")
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles a libamdhip64.so.7 with
        # the same SONAME as /opt/rocm's.  Loading torch first makes our
        # library bind to torch's copy (so torch tensors and streams are valid
        # handles for it); loading ours first would make torch initialise on
        # the other runtime and fail.  Pure C users get /opt/rocm's runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (the MI355X engine has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        L.sgpu_abi_version.restype = C.c_int
        L.sgpu_abi_version.argtypes = []
        if L.sgpu_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: ABI version {L.sgpu_abi_version()}, binding expects {ABI_VERSION}"
                              " (rebuild the library)")
        vp = C.c_void_p
        L.sgpu_device_count.restype = C.c_int
        L.sgpu_device_count.argtypes = []
        L.sgpu_init.restype = C.c_int
        L.sgpu_init.argtypes = [C.c_int, C.POINTER(vp)]
        L.sgpu_release.restype = None
        L.sgpu_release.argtypes = [vp]
        L.sgpu_set_stream.restype = C.c_int
        L.sgpu_set_stream.argtypes = [vp, vp]
        L.sgpu_synchronize.restype = C.c_int
        L.sgpu_synchronize.argtypes = [vp]
        L.sgpu_last_error.restype = C.c_char_p
        L.sgpu_last_error.argtypes = []
        L.sgpu_stack_rows.restype = C.c_int
        L.sgpu_stack_rows.argtypes = [vp, vp, C.c_int, C.c_long, C.c_long, C.c_long,
                                      C.POINTER(StackParams), vp, vp, vp, vp]
        L.sgpu_stack_rows_device.restype = C.c_int
        L.sgpu_stack_rows_device.argtypes = [vp, vp, C.c_int, C.c_long, C.c_long, C.c_long,
                                             C.POINTER(StackParams), vp, vp, vp, vp]
        L.sgpu_stack_rows_u16.restype = C.c_int
        L.sgpu_stack_rows_u16.argtypes = [vp, vp, C.c_int, C.c_long, C.c_long, C.c_long,
                                          C.POINTER(StackParams), vp, vp, vp, vp, vp]
        L.sgpu_stack_rows_planes.restype = C.c_int
        L.sgpu_stack_rows_planes.argtypes = [vp, vp, vp, vp] + list(L.sgpu_stack_rows.argtypes[2:])
        L.sgpu_stack_rows_planes_device.restype = C.c_int
        L.sgpu_stack_rows_planes_device.argtypes = [vp, vp, vp, vp] + list(L.sgpu_stack_rows_device.argtypes[2:])
        L.sgpu_stack_rows_u16_device.restype = C.c_int
        L.sgpu_stack_rows_u16_device.argtypes = [vp, vp, C.c_int, C.c_long, C.c_long, C.c_long,
                                                 C.POINTER(StackParams), vp, vp, vp, vp, vp]
        L.sgpu_stack_rows_u16_planes_device.restype = C.c_int
        L.sgpu_stack_rows_u16_planes_device.argtypes = [vp, vp, vp, vp] + list(L.sgpu_stack_rows_u16_device.argtypes[2:])
        L.sgpu_dft_shifts.restype = C.c_int
        L.sgpu_dft_shifts.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp]
        L.sgpu_dft_register_device.restype = C.c_int
        L.sgpu_dft_register_device.argtypes = [vp, vp, C.c_long, vp, C.c_long, C.c_long, C.c_int,
                                               C.c_int, vp, vp]
        L.sgpu_last_exact_pixels.restype = C.c_long
        L.sgpu_last_exact_pixels.argtypes = [vp]
        L.sgpu_last_order_sensitive.restype = C.c_long
        L.sgpu_last_order_sensitive.argtypes = [vp, vp, C.c_long]
        L.sgpu_set_exact_only.restype = C.c_int
        L.sgpu_set_exact_only.argtypes = [vp, C.c_int]
        L.sgpu_set_input_bitpix.restype = C.c_int
        L.sgpu_set_input_bitpix.argtypes = [vp, C.c_int]
        L.sgpu_set_timing.restype = C.c_int
        L.sgpu_set_timing.argtypes = [vp, C.c_int]
        L.sgpu_last_timing.restype = C.c_int
        L.sgpu_last_timing.argtypes = [vp, C.POINTER(C.c_float)]
        u, i, f = C.c_uint, C.c_int, C.c_float
        for name in ("sgpu_fft_richardson_lucy", "sgpu_naive_richardson_lucy"):
            getattr(L, name).restype = i
            getattr(L, name).argtypes = [vp, u, u, u, vp, i, u, f, i, f, i, i, f, i]
        for name in ("sgpu_rl_fft", "sgpu_rl_naive", "sgpu_rl_fft_device", "sgpu_rl_naive_device"):
            getattr(L, name).restype = i
            getattr(L, name).argtypes = [vp, vp, u, u, u, vp, i, u, f, i, f, i, f, i]
        L.sgpu_dft_shifts_cfa.restype = i
        L.sgpu_dft_shifts_cfa.argtypes = [vp, vp, vp, i, i, vp, i, vp, vp]
        L.sgpu_dft_register_cfa_device.restype = i
        L.sgpu_dft_register_cfa_device.argtypes = [vp, vp, C.c_long, vp, C.c_long, C.c_long, i, i, vp, i, vp, vp]
        L.sgpu_interpolate_nongreen_device.restype = i
        L.sgpu_interpolate_nongreen_device.argtypes = [vp, vp, i, i, C.c_long, vp, i]
        pi = C.POINTER(C.c_int)
        L.sgpu_debayer_buffer_new_float.restype = C.POINTER(C.c_float)
        L.sgpu_debayer_buffer_new_float.argtypes = [vp, pi, pi, i, i, vp]
        L.sgpu_debayer_buffer_superpixel_float.restype = C.POINTER(C.c_float)
        L.sgpu_debayer_buffer_superpixel_float.argtypes = [vp, pi, pi, i]
        L.sgpu_debayer_device.restype = i
        L.sgpu_debayer_device.argtypes = [vp, vp, i, i, i, i, vp]
        L.sgpu_superpixel_device.restype = i
        L.sgpu_superpixel_device.argtypes = [vp, vp, i, i, i, vp]
        if hasattr(L, "sgpu_bgnoise"):
            for name in ("sgpu_bgnoise_device", "sgpu_bgnoise_u16_device", "sgpu_bgnoise", "sgpu_bgnoise_u16"):
                getattr(L, name).restype = i
                getattr(L, name).argtypes = [vp, vp, i, i, i, C.c_long, vp]
        if hasattr(L, "sgpu_debayer_u16_device"):
            L.sgpu_debayer_buffer_new_ushort.restype = C.POINTER(C.c_uint16)
            L.sgpu_debayer_buffer_new_ushort.argtypes = [vp, pi, pi, i, i, vp, i]
            L.sgpu_debayer_u16_device.restype = i
            L.sgpu_debayer_u16_device.argtypes = [vp, vp, i, i, i, i, i, vp]
        L.sgpu_free.restype = None
        L.sgpu_free.argtypes = [vp]
        for name in ("sgpu_norm_stats_device", "sgpu_norm_stats", "sgpu_norm_stats_u16_device", "sgpu_norm_stats_u16"):
            getattr(L, name).restype = i
            getattr(L, name).argtypes = [vp, vp, i, C.c_long, C.c_long, i, vp, vp, vp]
        L.sgpu_norm_factors.restype = i
        L.sgpu_norm_factors.argtypes = [i, i, i, i, vp, vp, vp, vp, vp]
        L.sgpu_overlap_rect.restype = i
        L.sgpu_overlap_rect.argtypes = [i, i, C.c_double, C.c_double, C.c_double, C.c_double, vp, vp, vp]
        for name in ("sgpu_overlap_stats_device", "sgpu_overlap_stats_u16_device"):
            getattr(L, name).restype = i
            getattr(L, name).argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long, vp, vp, i, vp, vp]
        L.sgpu_overlap_factors.restype = i
        L.sgpu_overlap_factors.argtypes = [i, i, i, i, vp, vp, vp, vp, vp]
        L.sgpu_quality_estimate_device.restype = i
        L.sgpu_quality_estimate_device.argtypes = [vp, vp, i, i, i, C.c_long, C.c_long, vp]
        L.sgpu_quality_estimate.restype = i
        L.sgpu_quality_estimate.argtypes = [vp, vp, i, i, i, vp]
        L.sgpu_quality_estimate_u16_device.restype = i
        L.sgpu_quality_estimate_u16_device.argtypes = [vp, vp, i, i, i, C.c_long, C.c_long, vp]
        L.sgpu_quality_estimate_u16.restype = i
        L.sgpu_quality_estimate_u16.argtypes = [vp, vp, i, i, i, vp]
        L.sgpu_normalize_quality.restype = None
        L.sgpu_normalize_quality.argtypes = [vp, i, C.c_double, C.c_double]
        L.sgpu_rl_set_memory.restype = i
        L.sgpu_rl_set_memory.argtypes = [vp, C.c_size_t]
        L.sgpu_stack_seq.restype = i
        L.sgpu_stack_seq.argtypes = [vp, C.c_char_p, C.POINTER(StackParams), i, i, C.c_char_p, vp, C.c_long]
        L.sgpu_stack_seq_ex.restype = i
        L.sgpu_stack_seq_ex.argtypes = [vp, C.c_char_p, C.POINTER(StackParams), i, i, C.c_char_p, vp, C.c_long, i]
        L.sgpu_stack_seq_ex2.restype = i
        L.sgpu_stack_seq_ex2.argtypes = [vp, C.c_char_p, C.POINTER(StackParams), i, i, C.c_char_p, vp, C.c_long, i,
                                         i]
        if hasattr(L, "sgpu_stack_seq_frames"):     # (tuning-variant libraries may predate them)
            L.sgpu_stack_seq_opts.restype = i
            L.sgpu_stack_seq_opts.argtypes = [vp, C.c_char_p, C.POINTER(StackParams), i, i, C.c_char_p, vp,
                                              C.POINTER(StackSeqOptions)]
            L.sgpu_stack_seq_frames.restype = i
            L.sgpu_stack_seq_frames.argtypes = [C.c_char_p, C.POINTER(StackSeqOptions), vp, i, C.POINTER(i),
                                                C.POINTER(i)]
        if hasattr(L, "sgpu_last_seq_stats"):
            L.sgpu_set_seq_readers.restype = i
            L.sgpu_set_seq_readers.argtypes = [vp, i]
            L.sgpu_release_seq_buffers.restype = i
            L.sgpu_release_seq_buffers.argtypes = [vp]
            L.sgpu_last_seq_stats.restype = i
            L.sgpu_last_seq_stats.argtypes = [vp, vp]
        L.sgpu_fits_layers.restype = i
        L.sgpu_fits_layers.argtypes = [C.c_char_p]
        L.sgpu_image_read_rows.restype = i
        L.sgpu_image_read_rows.argtypes = [C.c_char_p, i, i, C.c_long, C.c_long, vp, i]
        L.sgpu_fits_write_planes.restype = i
        L.sgpu_fits_write_planes.argtypes = [C.c_char_p, vp, C.c_long, C.c_long, i, i]
        L.sgpu_ser_write.restype = i
        L.sgpu_ser_write.argtypes = [C.c_char_p, vp, i, i, i, i, i, i, vp, C.c_char_p, C.c_uint64]
        L.sgpu_ser_info.restype = i
        L.sgpu_ser_info.argtypes = [C.c_char_p, pi, pi, pi, pi, pi, pi, C.c_char_p, C.POINTER(C.c_uint64), vp, i]
        L.sgpu_fits_info.restype = i
        L.sgpu_fits_info.argtypes = [C.c_char_p, C.POINTER(C.c_long), C.POINTER(C.c_long), pi]
        L.sgpu_fits_read_rows.restype = i
        L.sgpu_fits_read_rows.argtypes = [C.c_char_p, C.c_long, C.c_long, vp]
        L.sgpu_fits_read_rows_ex.restype = i
        L.sgpu_fits_read_rows_ex.argtypes = [C.c_char_p, C.c_long, C.c_long, vp, i]
        L.sgpu_norm_to_0_1_range_device.restype = i
        L.sgpu_norm_to_0_1_range_device.argtypes = [vp, vp, C.c_long]
        L.sgpu_multi_init.restype = i
        L.sgpu_multi_init.argtypes = [vp, i, C.POINTER(vp)]
        L.sgpu_multi_release.restype = None
        L.sgpu_multi_release.argtypes = [vp]
        L.sgpu_multi_size.restype = i
        L.sgpu_multi_size.argtypes = [vp]
        L.sgpu_multi_context.restype = vp
        L.sgpu_multi_context.argtypes = [vp, i]
        L.sgpu_multi_stack_rows.restype = i
        L.sgpu_multi_stack_rows.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long, C.POINTER(StackParams),
                                            vp, vp, vp, vp]
        L.sgpu_multi_stack_rows_u16.restype = i
        L.sgpu_multi_stack_rows_u16.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long,
                                                C.POINTER(StackParams), vp, vp, vp, vp, vp]
        L.sgpu_mean_partial_device.restype = i
        L.sgpu_mean_partial_device.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long, C.POINTER(StackParams),
                                               vp, vp]
        L.sgpu_mean_finish_device.restype = i
        L.sgpu_mean_finish_device.argtypes = [vp, vp, vp, C.c_long, vp, i]
        L.sgpu_mean_partial_guard_device.restype = i
        L.sgpu_mean_partial_guard_device.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long,
                                                     C.POINTER(StackParams), vp, vp, vp, vp]
        L.sgpu_mean_finish_guard_device.restype = i
        L.sgpu_mean_finish_guard_device.argtypes = [vp, vp, vp, vp, vp, C.c_long, vp, i, vp]
        L.sgpu_dft_register_u16_device.restype = i
        L.sgpu_dft_register_u16_device.argtypes = [vp, vp, C.c_long, vp, C.c_long, C.c_long, i, i, vp, i, vp, vp]
        L.sgpu_dft_shifts_u16.restype = i
        L.sgpu_dft_shifts_u16.argtypes = [vp, vp, vp, i, i, vp, i, vp, vp]
        L.sgpu_interpolate_nongreen_u16_device.restype = i
        L.sgpu_interpolate_nongreen_u16_device.argtypes = [vp, vp, i, i, C.c_long, vp, i]
        L.sgpu_debayer_buffer_siril_ushort.restype = C.POINTER(C.c_uint16)
        L.sgpu_debayer_buffer_siril_ushort.argtypes = [vp, C.POINTER(i), C.POINTER(i), i, i, i]
        L.sgpu_debayer_siril_u16_device.restype = i
        L.sgpu_debayer_siril_u16_device.argtypes = [vp, vp, i, i, i, i, i, vp]
        L.sgpu_apply_reg_device.restype = i
        L.sgpu_apply_reg_device.argtypes = [vp, vp, vp, i, i, i, i, C.c_long, vp, i, i]
        L.sgpu_stack_blocks.restype = i
        L.sgpu_stack_blocks.argtypes = [C.c_long, C.c_long, C.c_long, i, i, vp, vp, vp, C.POINTER(i),
                                        C.POINTER(C.c_long)]
        L.sgpu_feather_mask_size.restype = None
        L.sgpu_feather_mask_size.argtypes = [C.c_long, C.c_long, C.POINTER(C.c_long), C.POINTER(C.c_long)]
        L.sgpu_feather_masks_device.restype = i
        L.sgpu_feather_masks_device.argtypes = [vp, vp, i, i, C.c_long, C.c_long, C.c_long, vp]
        L.sgpu_feather_block_area.restype = i
        L.sgpu_feather_block_area.argtypes = [C.c_long, C.c_long, C.c_long, C.c_long, i, i] + [C.POINTER(i)] * 4
        L.sgpu_feather_block_device.restype = i
        L.sgpu_feather_block_device.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long, C.c_long, vp, vp,
                                                C.c_long, C.c_float, i, vp, C.c_long]
        L.sgpu_gather_columns_device.restype = i
        L.sgpu_gather_columns_device.argtypes = [vp, vp, i, C.c_long, C.c_long, C.c_long, C.POINTER(StackParams),
                                                 vp, C.c_longlong, vp]
        L.sgpu_apply_reg_shifts.restype = i
        L.sgpu_apply_reg_shifts.argtypes = [i, vp, vp, i, vp, vp]
        L.sgpu_shift_frames_device.restype = i
        L.sgpu_shift_frames_device.argtypes = [vp, vp, vp, i, i, i, i, C.c_long, vp, vp]
        L.sgpu_extract_cfa_device.restype = i
        L.sgpu_extract_cfa_device.argtypes = [vp, vp, i, i, i, vp, i, i, vp, C.POINTER(C.c_long)]
        L.sgpu_cfa_count.restype = C.c_long
        L.sgpu_cfa_count.argtypes = [i, i, vp, i, i]
        L.sgpu_split_cfa_device.restype = i
        L.sgpu_split_cfa_device.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp]
        L.sgpu_merge_cfa_device.restype = i
        L.sgpu_merge_cfa_device.argtypes = [vp, vp, vp, vp, vp, i, i, i, vp]
        L.sgpu_row_bands.restype = i
        L.sgpu_row_bands.argtypes = [C.c_long, i, vp]
        L.sgpu_fits_write.restype = i
        L.sgpu_fits_write.argtypes = [C.c_char_p, vp, C.c_long, C.c_long, i]
        L.sgpu_rl_last_conv_launches.restype = C.c_long
        L.sgpu_rl_last_conv_launches.argtypes = [vp]
        L.sgpu_rl_last_iter_flops.restype = C.c_double
        L.sgpu_rl_last_iter_flops.argtypes = [vp]
        L.sgpu_rl_last_fft_convs.restype = C.c_long
        L.sgpu_rl_last_fft_convs.argtypes = [vp]
        L.sgpu_rl_last_iter_bytes.restype = C.c_double
        L.sgpu_rl_last_iter_bytes.argtypes = [vp]
        _lib = L
    return _lib


def check(code: int, where: str) -> None:
    if code != SGPU_OK:
        raise SgpuError(code, where)
