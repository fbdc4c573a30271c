// rl_fft.hip -- FFT convolution for the Richardson-Lucy FFT path
// (filters/deconvolution/deconvolve.hpp:78-178).
//
// The reference convolves a slice through FFTW: IFFT(FFT(x) . FFT(padcirc(K)))
// = the circular convolution over the slice (W x H, any size -- the
// geometry of process_in_slices rarely gives FFT-friendly lengths, e.g.
// 6062 = 2 x 3031).  Here the same circular convolution is computed as a
// linear convolution of the slice's periodic extension: rows / columns
// extended by h = ks/2 on both sides (x_ext[r][c] = x[(r-h) mod H][(c-h) mod W])
// and zero-padded to 2-3-5-smooth lengths n1 >= W + 3h, n2 >= H + 3h, so the
// length-n circular transform of the extension has no wrap-around in the
// output window [h, h+W) x [h, h+H).
//
// Passes per convolution (half spectra: two real rows per complex row FFT,
// as in dft_register.hip):
//   k_rlf_rows_fwd   rows of x_ext -> half spectra [n2][nh1]   (zero rows skipped)
//   transpose        -> [nh1][n2]   (or stored there directly: SGPU_RL_TRANSPOSE=0)
//   k_rlf_cols       per column: forward FFT, x Khat, inverse FFT (in LDS)
//   transpose        -> [n2][nh1]
//   k_rlf_rows_inv   inverse rows of the output window, fused RL epilogue
// Khat (the taps' spectrum, / (n1 n2)) comes from the same passes on the
// wrapped taps.  Row FFTs in LDS (fft_lds.h, Stockham mixed radix).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include <cmath>
#include <cstdlib>
#include <vector>

#include "fft_lds.h"
#include "rl_conv.h"

namespace sgpu {
namespace dft {
__global__ void k_transpose_rect(const float2 *in, float2 *out, int rows, int cols);
}

namespace rl {

using fft::Plan;

// value of the source image at (r, c) of the n2 x n1 transform input:
// mode 0: periodic extension of the W x H slice `in`; mode 1: the ks x ks taps
// wrapped around (0, 0) (K[(ky-h) mod n2][(kx-h) mod n1] = taps[ky][kx])
struct SrcDesc {
    const float *in;
    int W, H, h, ks, mode, n1, n2;
};

__device__ __forceinline__ bool row_nonzero(const SrcDesc &d, int r) {
    if (d.mode == 0) return r < d.H + 2 * d.h;
    const int dy = (r <= d.h) ? r : r - d.n2;
    return dy >= -d.h && dy <= d.h;
}
__device__ __forceinline__ float src_at(const SrcDesc &d, int r, int c) {
    if (d.mode == 0) {
        if (r >= d.H + 2 * d.h || c >= d.W + 2 * d.h) return 0.f;
        int y = r - d.h, x = c - d.h;
        y = y < 0 ? y + d.H : (y >= d.H ? y - d.H : y);
        x = x < 0 ? x + d.W : (x >= d.W ? x - d.W : x);
        return d.in[(long long)y * d.W + x];
    }
    const int dy = (r <= d.h) ? r : r - d.n2, dx = (c <= d.h) ? c : c - d.n1;
    if (dy < -d.h || dy > d.h || dx < -d.h || dx > d.h) return 0.f;
    return d.in[(dy + d.h) * d.ks + dx + d.h];
}

// Element (row r, frequency k) of the half-spectrum plane: row-major [n2][nh1]
// (pitch nh1, for the rectangular transpose kernel; the default) or
// column-major [nh1][n2] (pitch n2: tr = 1, A/B), which the column pass reads
// directly -- the row kernels store / load there with rows r, r + 1 of a
// column adjacent, instead of two transposes per convolution.
struct HPlane {
    float2 *p;
    int nh, n2, tr;
    __device__ __forceinline__ long long at(int r, int k) const {
        return tr ? (long long)k * n2 + r : (long long)r * nh + k;
    }
};

// Row-pair index of a block.  Column-major plane: 8 consecutive pairs (the
// 16 rows sharing each 128-byte line of a column) on one XCD, where their
// partial-line stores / loads merge in that XCD's L2 (the dispatcher deals
// consecutive blocks round-robin over the 8 XCDs).
__device__ __forceinline__ int row_pair(const HPlane &t) {
    const unsigned total = gridDim.x, L = blockIdx.x;
    if (!t.tr || total % 8u) return (int)L;
    return (int)((L % 8u) * (total / 8u) + L / 8u);
}

// rows 2j, 2j+1 -> half spectra rows of the plane
__global__ __launch_bounds__(fft::kThreads) void k_rlf_rows_fwd(Plan pl, SrcDesc d, HPlane t) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n, nh = n / 2 + 1;
    const int r0 = 2 * row_pair(t), r1 = r0 + 1;
    const bool has1 = r1 < d.n2;
    const bool nz0 = row_nonzero(d, r0), nz1 = has1 && row_nonzero(d, r1);
    if (!nz0 && !nz1) {                          // block-uniform
        for (int k = threadIdx.x; k < nh; k += blockDim.x) {
            t.p[t.at(r0, k)] = make_float2(0.f, 0.f);
            if (has1) t.p[t.at(r1, k)] = make_float2(0.f, 0.f);
        }
        return;
    }
    float2 *a = lds, *b = lds + n;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        a[i] = make_float2(nz0 ? src_at(d, r0, i) : 0.f, nz1 ? src_at(d, r1, i) : 0.f);
    __syncthreads();
    const float2 *r = fft::run<-1>(a, b, pl);
    for (int k = threadIdx.x; k < nh; k += blockDim.x) {
        const float2 z = r[k], zc = r[k == 0 ? 0 : n - k];
        const float2 x = make_float2(0.5f * (z.x + zc.x), 0.5f * (z.y - zc.y));      // X[k]
        const float2 y = make_float2(0.5f * (z.y + zc.y), 0.5f * (zc.x - z.x));      // Y[k]
        if (t.tr && has1) {                      // r0 and n2 even: one aligned 16-byte store
            *reinterpret_cast<float4 *>(t.p + t.at(r0, k)) = make_float4(x.x, x.y, y.x, y.y);
        } else {
            t.p[t.at(r0, k)] = x;
            if (has1) t.p[t.at(r1, k)] = y;
        }
    }
}

// one column (row of the transposed plane, length n2) per block.
// mode 1: forward transform scaled by `scale` (the taps' spectrum);
// mode 2: forward, times khat, inverse
__global__ __launch_bounds__(fft::kThreads) void k_rlf_cols(Plan pl, float2 *t2, const float2 *khat, int mode,
                                                            float scale) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = pl.n;
    float2 *a = lds, *b = lds + n;
    float2 *row = t2 + (long long)blockIdx.x * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = row[i];
    __syncthreads();
    float2 *r = fft::run<-1>(a, b, pl);
    if (mode == 1) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) row[i] = fft::cscale(r[i], scale);
        return;
    }
    const float2 *kr = khat + (long long)blockIdx.x * n;
    float2 *o = fft::plan_inplace(pl) ? r : ((r == a) ? b : a);   // product in place when it can
    for (int i = threadIdx.x; i < n; i += blockDim.x) o[i] = fft::cmul(r[i], kr[i]);
    __syncthreads();
    r = fft::run<+1>(o, (o == a) ? b : a, pl);
    for (int i = threadIdx.x; i < n; i += blockDim.x) row[i] = r[i];
}

// inverse rows h+2j, h+2j+1 (half spectra, pitch nh1) -> output rows 2j, 2j+1
// of the W x H window, RL epilogue fused
__global__ __launch_bounds__(fft::kThreads) void k_rlf_rows_inv(Plan pl, HPlane t, int h, ConvArgs ca, int epi) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ double wsum[fft::kThreads / 64];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    const int y0 = 2 * row_pair(t), y1 = y0 + 1;
    const bool has1 = y1 < ca.H;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const bool lo = k < nh;
        const int q = lo ? k : n - k;
        float2 x = t.p[t.at(h + y0, q)], y = has1 ? t.p[t.at(h + y1, q)] : make_float2(0.f, 0.f);
        if (!lo) { x.y = -x.y; y.y = -y.y; }                    // Hermitian extension
        a[k] = make_float2(x.x - y.y, x.y + y.x);               // Z = X + i Y
    }
    __syncthreads();
    const float2 *r = fft::run<+1>(a, b, pl);
    double stop_part = 0.0;
    for (int x = threadIdx.x; x < ca.W; x += blockDim.x) {
        const float2 z = r[h + x];
        rl_epilogue(ca, epi, (long long)y0 * ca.W + x, x, y0, z.x, stop_part);
        if (has1) rl_epilogue(ca, epi, (long long)y1 * ca.W + x, x, y1, z.y, stop_part);
    }
    if (ca.stop_acc) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) stop_part += __shfl_xor(stop_part, off, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = stop_part;
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int w = 0; w < (int)(blockDim.x >> 6); w++) s += wsum[w];
            atomicAdd(ca.stop_acc, s);
        }
    }
}

// k_rlf_rows_inv followed, in the same block, by the forward transform of
// the two output rows as rows of the next convolution's periodic extension
// (ext row y + h, plus its wrap copy y + h + H for y < h or y + h - H for
// y >= H - h), written back into t1.  The rows the block reads (h + y0,
// h + y1) are the ones it rewrites; wrap copies land outside [h, h + H), which
// no block reads.  Rows >= H + 2h are zeroed by the host.
constexpr int kMaxPer = (fft::kMaxLen + fft::kThreads - 1) / fft::kThreads;
__global__ __launch_bounds__(fft::kThreads) void k_rlf_rows_inv_fwd(Plan pl, HPlane t, int h, ConvArgs ca,
                                                                    int epi) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ double wsum[fft::kThreads / 64];
    const int n = pl.n, nh = n / 2 + 1;
    float2 *a = lds, *b = lds + n;
    const int W = ca.W, H = ca.H;
    const int y0 = 2 * row_pair(t), y1 = y0 + 1;
    const bool has1 = y1 < H;
    {
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const bool lo = k < nh;
            const int q = lo ? k : n - k;
            float2 x = t.p[t.at(h + y0, q)], y = has1 ? t.p[t.at(h + y1, q)] : make_float2(0.f, 0.f);
            if (!lo) { x.y = -x.y; y.y = -y.y; }
            a[k] = make_float2(x.x - y.y, x.y + y.x);
        }
    }
    __syncthreads();
    float2 *r = fft::run<+1>(a, b, pl);
    double stop_part = 0.0;
    float v0[kMaxPer], v1[kMaxPer];
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const int x = threadIdx.x + k * fft::kThreads;
        v0[k] = v1[k] = 0.f;
        if (x < W) {
            const float2 z = r[h + x];
            v0[k] = rl_epilogue(ca, epi, (long long)y0 * W + x, x, y0, z.x, stop_part);
            if (has1) v1[k] = rl_epilogue(ca, epi, (long long)y1 * W + x, x, y1, z.y, stop_part);
        }
    }
    __syncthreads();                                   // r (== a) fully read
    for (int c = W + 2 * h + threadIdx.x; c < n; c += blockDim.x) a[c] = make_float2(0.f, 0.f);
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const int x = threadIdx.x + k * fft::kThreads;
        if (x < W) {
            const float2 v = make_float2(v0[k], v1[k]);
            a[x + h] = v;
            if (x < h) a[x + W + h] = v;
            if (x >= W - h) a[x - W + h] = v;
        }
    }
    __syncthreads();
    const float2 *f = fft::run<-1>(a, b, pl);
    const int ry0 = y0 + h, ry1 = y1 + h;
    const int wy0 = y0 < h ? y0 + h + H : (y0 >= H - h ? y0 + h - H : -1);
    const int wy1 = !has1 ? -1 : (y1 < h ? y1 + h + H : (y1 >= H - h ? y1 + h - H : -1));
    for (int k = threadIdx.x; k < nh; k += blockDim.x) {
        const float2 z = f[k], zc = f[k == 0 ? 0 : n - k];
        const float2 X = make_float2(0.5f * (z.x + zc.x), 0.5f * (z.y - zc.y));
        const float2 Y = make_float2(0.5f * (z.y + zc.y), 0.5f * (zc.x - z.x));
        t.p[t.at(ry0, k)] = X;
        if (wy0 >= 0) t.p[t.at(wy0, k)] = X;
        if (has1) {
            t.p[t.at(ry1, k)] = Y;
            if (wy1 >= 0) t.p[t.at(wy1, k)] = Y;
        }
    }
    if (ca.stop_acc) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) stop_part += __shfl_xor(stop_part, off, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = stop_part;
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int w = 0; w < (int)(blockDim.x >> 6); w++) s += wsum[w];
            atomicAdd(ca.stop_acc, s);
        }
    }
}

static Plan make_plan(int n, const float2 *tw) {
    Plan pl;
    pl.n = n;
    pl.nf = 0;
    int m = n;
    while (m % 8 == 0) { pl.radix[pl.nf++] = 8; m /= 8; }
    while (m % 5 == 0) { pl.radix[pl.nf++] = 5; m /= 5; }
    while (m % 4 == 0) { pl.radix[pl.nf++] = 4; m /= 4; }
    while (m % 3 == 0) { pl.radix[pl.nf++] = 3; m /= 3; }
    while (m % 2 == 0) { pl.radix[pl.nf++] = 2; m /= 2; }
    pl.tw = tw;
    // the RL kernels run fft::run<S, false> (no radix-10 butterfly): a 10
    // here -- e.g. a future switch to sgpu_dft.cpp's factorize() -- would be
    // transformed as radix 8 (fft_lds.h, plan_has_radix10)
    if (fft::plan_has_radix10(pl)) {
        std::fprintf(stderr, "sirilgpu: RL FFT plan with a radix-10 pass (not compiled into the RL kernels)\n");
        std::abort();
    }
    return pl;
}

int fft_smooth_len(int need) {
    for (int m = need + (need & 1); m <= fft::kMaxLen; m += 2) {
        int t = m;
        for (int p : {2, 3, 5})
            while (t % p == 0) t /= p;
        if (t == 1) return m;
    }
    return 0;
}

int fft_conv_setup(FftConv &fc, hipStream_t) {
    const int lds = 2 * std::max(fc.n1, fc.n2) * (int)sizeof(float2);   // upper bound
    for (const void *f : {(const void *)k_rlf_rows_fwd, (const void *)k_rlf_cols, (const void *)k_rlf_rows_inv,
                          (const void *)k_rlf_rows_inv_fwd})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    return 0;
}

// the half-spectrum plane's layout: row-major through the transpose kernel
// (default), or column-major, written and read by the row kernels directly
// (SGPU_RL_TRANSPOSE=0, A/B).  Measured the other way round from the DFT
// (profiles/r05x2_ab_rl63_*): 62.4 ms with the transposes, 70.1 ms without --
// one slice's plane (~100 MB) stays in the 256 MB MALL, where the transposes
// run at ~9 TB/s, while the row kernels' 16-byte column stores and loads cost
// a cache line each
static bool rl_transpose_kernel() {
    static const bool t = !std::getenv("SGPU_RL_TRANSPOSE") || std::atoi(std::getenv("SGPU_RL_TRANSPOSE")) != 0;
    return t;
}
static HPlane plane(const FftConv &fc, float2 *p, bool tr) { return HPlane{p, fc.nh1, fc.n2, tr ? 1 : 0}; }

// forward half spectrum of the source, column-major [nh1][n2] in dst and
// transformed along columns (mode 1: stored scaled into `dst`; mode 2: x
// khat and inverse, left in dst)
static void forward_and_cols(const FftConv &fc, const SrcDesc &d, const float2 *khat, float2 *dst, int mode,
                             float scale, hipStream_t s) {
    const Plan p1 = make_plan(fc.n1, fc.tw1), p2 = make_plan(fc.n2, fc.tw2);
    if (rl_transpose_kernel()) {
        hipLaunchKernelGGL(k_rlf_rows_fwd, dim3((fc.n2 + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                           p1, d, plane(fc, fc.t1, false));
        hipLaunchKernelGGL(dft::k_transpose_rect, dim3((fc.nh1 + 31) / 32, (fc.n2 + 31) / 32, 1), dim3(256), 0, s,
                           fc.t1, dst, fc.n2, fc.nh1);
    } else {
        hipLaunchKernelGGL(k_rlf_rows_fwd, dim3((fc.n2 + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                           p1, d, plane(fc, dst, true));
    }
    hipLaunchKernelGGL(k_rlf_cols, dim3(fc.nh1), dim3(fft::kThreads), fft::plan_lds_bytes(p2), s, p2, dst, khat,
                       mode, scale);
}

int fft_conv_taps(const FftConv &fc, const float *taps, int ks, float2 *khat, hipStream_t s) {
    SrcDesc d{taps, fc.W, fc.H, ks / 2, ks, 1, fc.n1, fc.n2};
    forward_and_cols(fc, d, nullptr, khat, 1, (float)(1.0 / ((double)fc.n1 * fc.n2)), s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int fft_conv(const FftConv &fc, const ConvArgs &a, const float2 *khat, int epi, hipStream_t s) {
    if (a.W != fc.W || a.H != fc.H || a.ks / 2 != fc.h) return -1;
    SrcDesc d{a.in, fc.W, fc.H, fc.h, a.ks, 0, fc.n1, fc.n2};
    forward_and_cols(fc, d, khat, fc.t2, 2, 1.f, s);
    const bool tk = rl_transpose_kernel();
    if (tk)
        hipLaunchKernelGGL(dft::k_transpose_rect, dim3((fc.n2 + 31) / 32, (fc.nh1 + 31) / 32, 1), dim3(256), 0, s,
                           fc.t2, fc.t1, fc.nh1, fc.n2);
    const Plan p1 = make_plan(fc.n1, fc.tw1);
    hipLaunchKernelGGL(k_rlf_rows_inv, dim3((fc.H + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                       p1, tk ? plane(fc, fc.t1, false) : plane(fc, fc.t2, true), fc.h, a, epi);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int fft_conv_chain(const FftConv &fc, const ConvArgs &a, const float2 *khat, int epi, bool have, bool next,
                   hipStream_t s) {
    if (a.W != fc.W || a.H != fc.H || a.ks / 2 != fc.h) return -1;
    const Plan p1 = make_plan(fc.n1, fc.tw1), p2 = make_plan(fc.n2, fc.tw2);
    // the in-place kernels keep their outputs in registers per thread: plans
    // with a generic radix (never chosen: 2-3-5-smooth lengths) are refused
    if (next && !fft::plan_inplace(p1)) return -1;
    // the chain keeps the next input's spectra where the row kernels left
    // them: t1 (row-major, transpose kernels) or t2 (column-major, default)
    const bool tk = rl_transpose_kernel();
    const HPlane rows = tk ? plane(fc, fc.t1, false) : plane(fc, fc.t2, true);
    if (!have) {
        SrcDesc d{a.in, fc.W, fc.H, fc.h, a.ks, 0, fc.n1, fc.n2};
        hipLaunchKernelGGL(k_rlf_rows_fwd, dim3((fc.n2 + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                           p1, d, rows);
    }
    if (tk)
        hipLaunchKernelGGL(dft::k_transpose_rect, dim3((fc.nh1 + 31) / 32, (fc.n2 + 31) / 32, 1), dim3(256), 0, s,
                           fc.t1, fc.t2, fc.n2, fc.nh1);
    hipLaunchKernelGGL(k_rlf_cols, dim3(fc.nh1), dim3(fft::kThreads), fft::plan_lds_bytes(p2), s, p2, fc.t2, khat,
                       2, 1.f);
    if (tk)
        hipLaunchKernelGGL(dft::k_transpose_rect, dim3((fc.n2 + 31) / 32, (fc.nh1 + 31) / 32, 1), dim3(256), 0, s,
                           fc.t2, fc.t1, fc.nh1, fc.n2);
    if (next) {
        hipLaunchKernelGGL(k_rlf_rows_inv_fwd, dim3((fc.H + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                           p1, rows, fc.h, a, epi);
        const int l2 = fc.H + 2 * fc.h;      // rows of the extension; the rest must read as zero
        if (l2 < fc.n2) {
            if (tk) {
                if (hipMemsetAsync(fc.t1 + (size_t)l2 * fc.nh1, 0, (size_t)(fc.n2 - l2) * fc.nh1 * sizeof(float2), s) !=
                    hipSuccess)
                    return -1;
            } else if (hipMemset2DAsync(fc.t2 + l2, (size_t)fc.n2 * sizeof(float2), 0,
                                        (size_t)(fc.n2 - l2) * sizeof(float2), (size_t)fc.nh1, s) != hipSuccess) {
                return -1;
            }
        }
    } else {
        hipLaunchKernelGGL(k_rlf_rows_inv, dim3((fc.H + 1) / 2), dim3(fft::kThreads), fft::plan_lds_bytes(p1), s,
                           p1, rows, fc.h, a, epi);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rl
}  // namespace sgpu
