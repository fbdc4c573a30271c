"""TEST INFRASTRUCTURE ONLY -- numpy restatement of Siril's DFT
cross-correlation registration (register_shift_dft,
registration/shift_methods.c:60-321), used as the checker of the GPU path.

FFTW3f (the reference's FFT, pinned 3.3.10 in build/flatpak/org.siril.Siril.json:364)
is not available here; numpy's pocketfft computes the same transforms with a
different rounding, so parity is pinned at the integer-shift level (the
quantity the reference stores), not bitwise -- "parity unpinned" for the
intermediate spectra.
"""
import numpy as np

# FFT backend (numpy's pocketfft; bench.py's CPU baseline swaps in a
# multi-threaded one with the same interface)
FFT = np.fft


def dft_shift(ref: np.ndarray, img: np.ndarray, dtype=np.complex128):
    """Returns (shiftx, shifty, peak) for one S x S selection."""
    S = ref.shape[0]
    assert ref.shape == (S, S) and img.shape == (S, S)
    fin = FFT.fft2(ref.astype(dtype))                    # :178 forward of the reference
    fout = FFT.fft2(img.astype(dtype))                   # :249
    conv = fin * np.conj(fout)                              # :253-255
    out = FFT.ifft2(conv) * (S * S)                      # :257 (FFTW backward is unnormalised)
    re = out.real.ravel()
    shift = int(np.argmax(re))                              # first maximum in row-major order (:259-265)
    sy, sx = shift // S, shift % S
    if sy > S // 2:                                         # :266-273
        sy -= S
    if sx > S // 2:
        sx -= S
    return sx, sy, float(re[shift])


def second_peak_margin(ref, img, dtype=np.complex128):
    """Relative gap between the largest and second-largest correlation value
    (to exclude near-ties from exact-shift comparisons)."""
    S = ref.shape[0]
    out = FFT.ifft2(FFT.fft2(ref.astype(dtype)) * np.conj(FFT.fft2(img.astype(dtype)))).real
    v = np.sort(out.ravel())
    return float((v[-1] - v[-2]) / max(abs(v[-1]), 1e-30))


XTRANS_1 = "GGRGGBGGBGGRBRGRBGGGBGGRGGRGGBRBGBRG"     # algos/demosaicing.c:44-50


def xtrans_in_place_safe(cfa):
    """True when no non-green site of a 6x6 pattern has a neighbour that the
    reference's transposed test FC_array(nx, ny) calls green while it is not:
    then interpolate_nongreen's in-place loop never reads a pixel it rewrote
    (see sgpu_dft.cpp make_cfa)."""
    c = [int(v) for v in cfa]
    for r in range(6):
        for q in range(6):
            if c[r * 6 + q] == 1:
                continue
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dx == 0 and dy == 0:
                        continue
                    ny, nx = (r + dy) % 6, (q + dx) % 6
                    if c[nx * 6 + ny] == 1 and c[ny * 6 + nx] != 1:
                        return False
    return True


def fc_array(row, col, cfa, dim):
    """FC_array (algos/demosaicing.c:363-370)."""
    if dim == 2:
        return int(cfa[((row & 1) << 1) | (col & 1)])
    return int(cfa[(row % dim) * dim + (col % dim)])


def interpolate_nongreen(img: np.ndarray, cfa, dim: int) -> np.ndarray:
    """interpolate_nongreen_float (io/image_format_fits.c:4319-4349), float32,
    returns a new array.  Non-green pixels except the last row/column become
    the weighted mean of their green 8-neighbours; the neighbour test uses
    FC_array(nx, ny) (column first) and the weight is 1 only when dx + dy == 1
    (right / lower neighbour), RECIPSQRT2 = 0.70710678f otherwise."""
    h, w = img.shape
    out = np.array(img, np.float32)
    src = out                      # in place, raster order, as the reference
    r2 = np.float32(0.70710678)
    for row in range(h - 1):
        for col in range(w - 1):
            if fc_array(row, col, cfa, dim) == 1:
                continue
            interp = np.float32(0)
            weight = np.float32(0)
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dx == 0 and dy == 0:
                        continue
                    nx, ny = col + dx, row + dy
                    if 0 <= nx < w and 0 <= ny < h and fc_array(nx, ny, cfa, dim) == 1:
                        wc = np.float32(1) if dx + dy == 1 else r2
                        interp = np.float32(interp + np.float32(wc * src[ny, nx]))
                        weight = np.float32(weight + wc)
            out[row, col] = np.float32(interp / weight)
    return out


def interpolate_nongreen_ushort(img: np.ndarray, cfa, dim: int) -> np.ndarray:
    """interpolate_nongreen_ushort (io/image_format_fits.c:4351-4381), uint16,
    returns a new array: the float weighted mean of the green neighbours of
    (float)WORD samples (bounds tested before FC_array(nx, ny)), stored back
    with roundf_to_WORD (core/proto.h:341-346: f + 0.5f, clamped, truncated)."""
    h, w = img.shape
    out = np.array(img, np.uint16)
    src = out                      # in place, raster order, as the reference
    r2 = np.float32(0.70710678)
    for row in range(h - 1):
        for col in range(w - 1):
            if fc_array(row, col, cfa, dim) == 1:
                continue
            interp = np.float32(0)
            weight = np.float32(0)
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dx == 0 and dy == 0:
                        continue
                    nx, ny = col + dx, row + dy
                    if 0 <= nx < w and 0 <= ny < h and fc_array(nx, ny, cfa, dim) == 1:
                        wc = np.float32(1) if dx + dy == 1 else r2
                        interp = np.float32(interp + np.float32(wc * np.float32(src[ny, nx])))
                        weight = np.float32(weight + wc)
            f = np.float32(np.float32(interp / weight) + np.float32(0.5))
            f = np.float32(65535.0) if f > np.float32(65535.0) else f
            f = np.float32(0.0) if f < np.float32(0.0) else f
            out[row, col] = np.uint16(int(f))
    return out
