// dft_register.hip -- DFT cross-correlation global alignment on the GPU
// (register_shift_dft, registration/shift_methods.c:60-321).
//
// Per frame, on the square S x S selection:
//   F = FFT2(img)                       (:249, real input as complex)
//   C = Fref . conj(F)                  (:253-255)
//   c = IFFT2(C), unnormalised           (:257)
//   shift = first strict argmax of Re c (:259-265), wrapped to +-S/2 (:266-273)
// The 2-D transforms are row FFTs in LDS on the half spectrum (real input
// and output, see k_rows_real2_fwd) whose results are stored straight into the
// column-major layout of the column pass (k_rows_real2_fwd_t /
// k_rows_c2r2_argmax_t; the tiled transpose kernel is the A/B form), batched
// over frames; the cross-power product is fused into the load of the first
// inverse pass and the argmax into the last one (the correlation surface is
// never written back).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fft_lds.h"

namespace sgpu {
namespace dft {

using fft::Plan;

// float -> uint32 with the same ordering (for packed argmax atomics)
__device__ __forceinline__ uint32_t ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// FC_array (algos/demosaicing.c:363-370)
__device__ __forceinline__ int fc_array(int row, int col, const fft::Cfa &p) {
    if (p.dim == 2) return p.c[(row & 1) << 1 | (col & 1)];
    return p.c[(row % p.dim) * p.dim + (col % p.dim)];
}

// interpolate_nongreen_float (io/image_format_fits.c:4319-4349) at (row, col)
// of a w x h selection: non-green pixels (except the last row and column)
// become a weighted mean of their green 8-neighbours.  Only green pixels are
// read, so the in-place loop of the reference has no order dependency.
// Quirks kept: the neighbour test calls FC_array(nx, ny) (column first),
// and `distance = dx + dy` gives weight 1 only to the right and lower
// neighbours (0.70710678f to all others).
__device__ __forceinline__ float nongreen(const float *img, long long stride, int w, int h, int row, int col,
                                          const fft::Cfa &p) {
    const float v = img[(long long)row * stride + col];
    if (p.dim == 0 || row >= h - 1 || col >= w - 1 || fc_array(row, col, p) == 1) return v;
    float interp = 0.f, weight = 0.f;
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int nx = col + dx, ny = row + dy;
            if (nx >= 0 && nx < w && ny >= 0 && ny < h && fc_array(nx, ny, p) == 1) {
                const float wc = (dx + dy == 1) ? 1.f : 0.70710678f;
                interp = interp + wc * img[(long long)ny * stride + nx];
                weight = weight + wc;
            }
        }
    return interp / weight;
}

// interpolate_nongreen_ushort (io/image_format_fits.c:4351-4381) at (row,
// col): the same weighted mean of the green neighbours, accumulated in float
// from (float)WORD samples (the bounds are tested before FC_array here --
// equivalent for Bayer), and the result stored back as roundf_to_WORD
// (core/proto.h:341-346); returned as the float the DFT then reads
// ((float)data, shift_methods.c:166-169).
__device__ __forceinline__ float nongreen16(const uint16_t *img, long long stride, int w, int h, int row, int col,
                                            const fft::Cfa &p) {
    const float v = (float)img[(long long)row * stride + col];
    if (p.dim == 0 || row >= h - 1 || col >= w - 1 || fc_array(row, col, p) == 1) return v;
    float interp = 0.f, weight = 0.f;
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int nx = col + dx, ny = row + dy;
            if (nx >= 0 && nx < w && ny >= 0 && ny < h && fc_array(nx, ny, p) == 1) {
                const float wc = (dx + dy == 1) ? 1.f : 0.70710678f;
                interp = interp + wc * (float)img[(long long)ny * stride + nx];
                weight = weight + wc;
            }
        }
    float f = interp / weight + 0.5f;
    f = (f > 65535.f) ? 65535.f : f;
    f = (f < 0.f) ? 0.f : f;
    return (float)(uint16_t)f;
}

__device__ __forceinline__ float sel_sample(const float *f, long long stride, int n, int row, int col,
                                            const fft::Cfa &cfa) {
    return cfa.dim == 0 ? f[(long long)row * stride + col] : nongreen(f, stride, n, n, row, col, cfa);
}
__device__ __forceinline__ float sel_sample(const uint16_t *f, long long stride, int n, int row, int col,
                                            const fft::Cfa &cfa) {
    return cfa.dim == 0 ? (float)f[(long long)row * stride + col] : nongreen16(f, stride, n, n, row, col, cfa);
}

// rows of the real selection -> complex row spectra.  grid (S, batch)
// `plane`: elements per batch plane (n*n full spectra, nh*n half spectra)
__global__ __launch_bounds__(fft::kThreads) void k_rows_fwd(Plan pl, float2 *data, long long plane) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n;
    float2 *a = lds, *b = lds + n;
    float2 *d = data + (long long)blockIdx.y * plane + (long long)blockIdx.x * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = d[i];
    __syncthreads();
    float2 *r = fft::run<-1, true>(a, b, pl);
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = r[i];
}

// cross power Fref . conj(F) then backward row transform, in place.
__global__ __launch_bounds__(fft::kThreads) void k_rows_xpow_bwd(Plan pl, const float2 *fref, float2 *data,
                                                                 long long plane) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n;
    float2 *a = lds, *b = lds + n;
    float2 *d = data + (long long)blockIdx.y * plane + (long long)blockIdx.x * n;
    const float2 *rr = fref + (long long)blockIdx.x * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float2 x = rr[i], y = d[i];
        // in[x] * conjf(out2[x])  (shift_methods.c:254)
        a[i] = make_float2(x.x * y.x + x.y * y.y, x.y * y.x - x.x * y.y);
    }
    __syncthreads();
    float2 *r = fft::run<+1, true>(a, b, pl);
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = r[i];
}

// column pass of a frame, fused: forward transform, cross power with the
// reference's (transposed) spectrum, backward transform -- the same values
// as k_rows_fwd followed by k_rows_xpow_bwd without the plane's HBM round
// trip between them.
// remap: the frames of one column run next to each other, on one XCD (the
// dispatcher deals consecutive workgroups round-robin over the 8 XCDs, each
// with its own L2), so the reference spectrum's column is read from HBM once
// per batch instead of once per frame (32 x 64 MB per batch at S = 4000).
__global__ __launch_bounds__(fft::kThreads) void k_cols_fwd_xpow_bwd(Plan pl, const float2 *fref, float2 *data,
                                                                     long long plane, int remap) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n;
    float2 *a = lds, *b = lds + n;
    int col = blockIdx.x, frame = blockIdx.y;
    if (remap) {
        const unsigned nbf = gridDim.y, total = gridDim.x * gridDim.y;
        const unsigned L = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned w = (total % 8u == 0u) ? (L % 8u) * (total / 8u) + L / 8u : L;   // XCD-contiguous ranges
        col = (int)(w / nbf);
        frame = (int)(w % nbf);
    }
    float2 *d = data + (long long)frame * plane + (long long)col * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = d[i];
    __syncthreads();
    float2 *r = fft::run<-1, true>(a, b, pl);
    float2 *o = fft::plan_inplace(pl) ? r : ((r == a) ? b : a);   // product in place when it can
    const float2 *rr = fref + (long long)col * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float2 x = rr[i], y = r[i];
        o[i] = make_float2(x.x * y.x + x.y * y.y, x.y * y.x - x.x * y.y);   // shift_methods.c:254
    }
    __syncthreads();
    r = fft::run<+1, true>(o, (o == a) ? b : a, pl);
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = r[i];
}

// last backward row transform + first-max argmax of the real part.
// best[frame] = (ord(value) << 32) | ~index: atomicMax keeps the largest
// value and, among equal values, the smallest row-major index.
// ---------------------------------------------------------------- half spectrum
// The image and the correlation surface are real, so only the half spectrum
// kx in [0, n/2] is carried through the column passes (nh = n/2 + 1 columns):
// two real rows are transformed as one complex row (z = x + i y, X[k] =
// (Z[k] + conj Z[n-k]) / 2, Y[k] = (Z[k] - conj Z[n-k]) / 2i), and the
// inverse row pass rebuilds Z = X + i Y from two half spectra (Hermitian
// extension) so one complex inverse yields both real correlation rows.  Half
// the column work and traffic of the full complex pipeline; the integer
// argmax is what parity is pinned on (FFT bitwise parity unpinned).

// rows 2j, 2j+1 of a frame -> half spectra rows 2j, 2j+1 (nh each, row pitch nh)
// T: float selections, or WORD ones (DATA_USHORT sequences: (float)data,
// after interpolate_nongreen_ushort for CFA frames)
template <class T>
__global__ __launch_bounds__(fft::kThreads) void k_rows_real2_fwd(Plan pl, const T *src,
                                                                  long long row_stride,
                                                                  long long frame_stride, float2 *dst,
                                                                  fft::Cfa cfa) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    const T *f = src + blockIdx.y * frame_stride;
    const int r0 = 2 * blockIdx.x, r1 = r0 + 1;
    const bool has1 = r1 < n;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        a[i] = make_float2(sel_sample(f, row_stride, n, r0, i, cfa),
                           has1 ? sel_sample(f, row_stride, n, r1, i, cfa) : 0.f);
    __syncthreads();
    const float2 *r = fft::run<-1, true>(a, b, pl);
    float2 *d0 = dst + ((long long)blockIdx.y * n + r0) * nh;
    float2 *d1 = d0 + nh;
    for (int k = threadIdx.x; k < nh; k += blockDim.x) {
        const float2 z = r[k], zc = r[k == 0 ? 0 : n - k];
        d0[k] = make_float2(0.5f * (z.x + zc.x), 0.5f * (z.y - zc.y));     // X[k]
        if (has1) d1[k] = make_float2(0.5f * (z.y + zc.y), 0.5f * (zc.x - z.x));   // Y[k]
    }
}

// XCD-aware order of the row-pair workgroups of the transposed-layout kernels
// below: the dispatcher deals consecutive workgroups round-robin over the 8
// XCDs (each with its own L2), so logical row pairs are numbered to put 8
// consecutive pairs -- the 16 rows that share every 128-byte line of a
// column in the [nh][n] layout -- on one XCD, where their partial-line
// writes (reads) merge in that XCD's L2 instead of reaching HBM separately.
__device__ __forceinline__ void pair_frame(int &pair, int &frame) {
    const unsigned np = gridDim.x, total = gridDim.x * gridDim.y;
    const unsigned L = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned w = (total % 8u == 0u) ? (L % 8u) * (total / 8u) + L / 8u : L;
    pair = (int)(w % np);
    frame = (int)(w / np);
}

// k_rows_real2_fwd writing the half spectra straight into the column-major
// layout the column pass reads ([nh][n] per frame: column k's n values
// contiguous), replacing the rectangular transpose kernel: rows r0, r0 + 1
// of column k are adjacent, so each k is one 16-byte store.
template <class T>
__global__ __launch_bounds__(fft::kThreads) void k_rows_real2_fwd_t(Plan pl, const T *src, long long row_stride,
                                                                    long long frame_stride, float2 *dst,
                                                                    fft::Cfa cfa) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    int pair, frame;
    pair_frame(pair, frame);
    const T *f = src + frame * frame_stride;
    const int r0 = 2 * pair, r1 = r0 + 1;
    const bool has1 = r1 < n;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        a[i] = make_float2(sel_sample(f, row_stride, n, r0, i, cfa),
                           has1 ? sel_sample(f, row_stride, n, r1, i, cfa) : 0.f);
    __syncthreads();
    const float2 *r = fft::run<-1, true>(a, b, pl);
    float2 *d = dst + (long long)frame * nh * n + r0;
    for (int k = threadIdx.x; k < nh; k += blockDim.x) {
        const float2 z = r[k], zc = r[k == 0 ? 0 : n - k];
        const float2 x = make_float2(0.5f * (z.x + zc.x), 0.5f * (z.y - zc.y));      // X[k]
        const float2 y = make_float2(0.5f * (z.y + zc.y), 0.5f * (zc.x - z.x));      // Y[k]
        float2 *dk = d + (long long)k * n;
        if (has1 && (n & 1) == 0) {              // 16-byte aligned (n, r0 even)
            *reinterpret_cast<float4 *>(dk) = make_float4(x.x, x.y, y.x, y.y);
        } else {
            dk[0] = x;
            if (has1) dk[1] = y;
        }
    }
}
template __global__ void k_rows_real2_fwd_t<float>(Plan, const float *, long long, long long, float2 *, fft::Cfa);
template __global__ void k_rows_real2_fwd_t<uint16_t>(Plan, const uint16_t *, long long, long long, float2 *,
                                                      fft::Cfa);

// k_rows_c2r2_argmax reading the column-major half spectra directly (X[q],
// Y[q] of rows r0, r0 + 1: one 16-byte load per q)
__global__ __launch_bounds__(fft::kThreads) void k_rows_c2r2_argmax_t(Plan pl, const float2 *data,
                                                                      unsigned long long *best) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ unsigned long long wbest[fft::kThreads / 64];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    int pair, frame;
    pair_frame(pair, frame);
    const int r0 = 2 * pair, r1 = r0 + 1;
    const bool has1 = r1 < n;
    const float2 *D = data + (long long)frame * nh * n + r0;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const bool lo = k < nh;
        const int q = lo ? k : n - k;
        float2 x, y;
        const float2 *Dq = D + (long long)q * n;
        if (has1 && (n & 1) == 0) {              // 16-byte aligned (n, r0 even)
            const float4 v = *reinterpret_cast<const float4 *>(Dq);
            x = make_float2(v.x, v.y);
            y = make_float2(v.z, v.w);
        } else {
            x = Dq[0];
            y = has1 ? Dq[1] : make_float2(0.f, 0.f);
        }
        if (!lo) { x.y = -x.y; y.y = -y.y; }                    // Hermitian extension
        a[k] = make_float2(x.x - y.y, x.y + y.x);               // Z = X + i Y
    }
    __syncthreads();
    const float2 *r = fft::run<+1, true>(a, b, pl);
    unsigned long long m = 0;
    const uint32_t base0 = (uint32_t)r0 * (uint32_t)n, base1 = (uint32_t)r1 * (uint32_t)n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long k0 = ((unsigned long long)ord(r[i].x) << 32) | (uint32_t)~(base0 + (uint32_t)i);
        m = k0 > m ? k0 : m;
        if (has1) {
            const unsigned long long k1 = ((unsigned long long)ord(r[i].y) << 32) | (uint32_t)~(base1 + (uint32_t)i);
            m = k1 > m ? k1 : m;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = wbest[w] > m ? wbest[w] : m;
        atomicMax(best + frame, m);
    }
}

// inverse row pass on half spectra rows 2j, 2j+1 (pitch nh) + argmax of both
// real rows (first strict maximum in row-major order, packed u64 atomicMax:
// ordered float value, then the complement of the row-major index)
__global__ __launch_bounds__(fft::kThreads) void k_rows_c2r2_argmax(Plan pl, const float2 *data,
                                                                    unsigned long long *best) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ unsigned long long wbest[fft::kThreads / 64];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    const int r0 = 2 * blockIdx.x, r1 = r0 + 1;
    const bool has1 = r1 < n;
    const float2 *X = data + ((long long)blockIdx.y * n + r0) * nh;
    const float2 *Y = X + nh;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const bool lo = k < nh;
        const int q = lo ? k : n - k;
        float2 x = X[q], y = has1 ? Y[q] : make_float2(0.f, 0.f);
        if (!lo) { x.y = -x.y; y.y = -y.y; }                    // Hermitian extension
        a[k] = make_float2(x.x - y.y, x.y + y.x);               // Z = X + i Y
    }
    __syncthreads();
    const float2 *r = fft::run<+1, true>(a, b, pl);
    unsigned long long m = 0;
    const uint32_t base0 = (uint32_t)r0 * (uint32_t)n, base1 = (uint32_t)r1 * (uint32_t)n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long k0 = ((unsigned long long)ord(r[i].x) << 32) | (uint32_t)~(base0 + (uint32_t)i);
        m = k0 > m ? k0 : m;
        if (has1) {
            const unsigned long long k1 = ((unsigned long long)ord(r[i].y) << 32) | (uint32_t)~(base1 + (uint32_t)i);
            m = k1 > m ? k1 : m;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = wbest[w] > m ? wbest[w] : m;
        atomicMax(best + blockIdx.y, m);
    }
}

// rectangular transpose of `batch` planes: in [rows][cols] -> out [cols][rows]
__global__ __launch_bounds__(256) void k_transpose_rect(const float2 *in, float2 *out, int rows, int cols) {
    __shared__ float2 tile[32][33];
    const long long off = (long long)blockIdx.z * rows * cols;
    const int bx = blockIdx.x * 32, by = blockIdx.y * 32;    // bx: column block, by: row block
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
        const int x = bx + tx, y = by + ty + k;
        if (x < cols && y < rows) tile[ty + k][tx] = in[off + (long long)y * cols + x];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
        const int x = by + tx, y = bx + ty + k;              // out row y = in column, out col x = in row
        if (x < rows && y < cols) out[off + (long long)y * rows + x] = tile[tx][ty + k];
    }
}

__global__ void k_finalize(const unsigned long long *best, int nframes, int n, int *shifts,
                           float *peak) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    const unsigned long long m = best[f];
    const uint32_t idx = ~(uint32_t)(m & 0xffffffffu);
    int sy = (int)(idx / (uint32_t)n), sx = (int)(idx % (uint32_t)n);
    if (sy > n / 2) sy -= n;
    if (sx > n / 2) sx -= n;
    shifts[2 * f] = sx;
    shifts[2 * f + 1] = sy;
    if (peak) peak[f] = unord((uint32_t)(m >> 32));
}

// standalone in-place pass (interpolate_nongreen on a device image)
__global__ __launch_bounds__(256) void k_nongreen(float *img, long long stride, int w, int h, fft::Cfa cfa) {
    const int col = blockIdx.x * 64 + (threadIdx.x & 63);
    const int row = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (col >= w - 1 || row >= h - 1) return;
    if (fc_array(row, col, cfa) == 1) return;
    // reads only green pixels, writes only non-green ones: safe in place
    img[(long long)row * stride + col] = nongreen(img, stride, w, h, row, col, cfa);
}

template __global__ void k_rows_real2_fwd<float>(Plan, const float *, long long, long long, float2 *, fft::Cfa);
template __global__ void k_rows_real2_fwd<uint16_t>(Plan, const uint16_t *, long long, long long, float2 *,
                                                    fft::Cfa);

// interpolate_nongreen_ushort in place on a device image (reads only green
// pixels, writes only non-green ones)
__global__ __launch_bounds__(256) void k_nongreen16(uint16_t *img, long long stride, int w, int h, fft::Cfa cfa) {
    const int col = blockIdx.x * 64 + (threadIdx.x & 63);
    const int row = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (col >= w - 1 || row >= h - 1) return;
    if (fc_array(row, col, cfa) == 1) return;
    img[(long long)row * stride + col] = (uint16_t)nongreen16(img, stride, w, h, row, col, cfa);
}

// X-Trans patterns whose transposed green test selects non-green neighbours
// (sgpu_dft.cpp make_cfa): the reference's in-place raster loop reads the
// already rewritten value of such a neighbour when it comes earlier in raster
// order (and was itself rewritten: not in the last row / column), the
// original one otherwise.  The chains of such reads are short (depth 2 for
// XTRANS_1 at any origin, checked on the 6x6 torus by the host), so the
// sequential result is reached by depth + 1 Jacobi passes: pass k reads the
// rewritten neighbours from pass k - 1 (the original image for k = 1) and
// everything else from the original image.  out / prev are w x h, contiguous.
__device__ __forceinline__ float ng_in(const float *o, long long so, int y, int x) { return o[(long long)y * so + x]; }
__device__ __forceinline__ float ng_in(const uint16_t *o, long long so, int y, int x) {
    return (float)o[(long long)y * so + x];
}
template <class T>
__global__ __launch_bounds__(256) void k_nongreen_pass(const T *orig, long long so, const T *prev, T *out, int w,
                                                       int h, fft::Cfa cfa) {
    const int col = blockIdx.x * 64 + (threadIdx.x & 63);
    const int row = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (col >= w || row >= h) return;
    const long long o = (long long)row * w + col;
    if (row >= h - 1 || col >= w - 1 || fc_array(row, col, cfa) == 1) {
        out[o] = orig[(long long)row * so + col];
        return;
    }
    float interp = 0.f, weight = 0.f;
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int nx = col + dx, ny = row + dy;
            if (nx >= 0 && nx < w && ny >= 0 && ny < h && fc_array(nx, ny, cfa) == 1) {
                // rewritten before (row, col): earlier in raster order, non-green, processed
                const bool rew = prev && (dy < 0 || (dy == 0 && dx < 0)) && fc_array(ny, nx, cfa) != 1 &&
                                 ny < h - 1 && nx < w - 1;
                const float v = rew ? ng_in(prev, w, ny, nx) : ng_in(orig, so, ny, nx);
                const float wc = (dx + dy == 1) ? 1.f : 0.70710678f;
                interp = interp + wc * v;
                weight = weight + wc;
            }
        }
    if constexpr (sizeof(T) == 4) {
        out[o] = interp / weight;
    } else {
        float f = interp / weight + 0.5f;
        f = (f > 65535.f) ? 65535.f : f;
        f = (f < 0.f) ? 0.f : f;
        out[o] = (T)(uint16_t)f;
    }
}
template __global__ void k_nongreen_pass<float>(const float *, long long, const float *, float *, int, int, fft::Cfa);
template __global__ void k_nongreen_pass<uint16_t>(const uint16_t *, long long, const uint16_t *, uint16_t *, int,
                                                   int, fft::Cfa);

}  // namespace dft
}  // namespace sgpu
