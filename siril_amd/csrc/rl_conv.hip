// rl_conv.hip -- 2-D convolution with a k x k PSF on the matrix cores, for
// Richardson-Lucy deconvolution (filters/deconvolution/deconvolve.hpp) and
// its edge taper (edgetaper.hpp), plus the slice plumbing kernels.
//
// The reference blurs through FFTW: IFFT(FFT(x) . FFT(padcirc(K))), i.e. a
// CIRCULAR convolution over the slice (image.hpp:1233-1293); the naive path
// (k < fft_cutoff) is a correlation with zero borders (image.hpp:498-600),
// which the host turns into a convolution with the flipped kernel.  Both are
// computed here directly as a GEMM on v_mfma_f32_16x16x4_f32:
//   c[oy][ox] = sum_{tr, kc} K[oy + 2h - tr][kc] * T[tr][ox + 2h - kc]
// T = input tile plus halo (LDS), K = taps (LDS).  For a 16-row output block
// the tile rows tr that touch it span 16 + k - 1, so the A operand is a
// banded Toeplitz slice of K (zero outside the band) and B a Hankel slice of
// the tile.  Workgroup = 4 waves = 64 x 64 outputs; a wave owns 32 x 32 =
// 2 x 2 accumulators of 16 x 16, A shared across its column blocks, B across
// its row blocks.  The RL point-wise steps are fused into the epilogue.
#include "rl_conv.h"

#include <stdint.h>

#include <type_traits>

namespace sgpu {
namespace rl {

constexpr int TILE = 64;
constexpr int GUARD = 16;    // floats ahead of the tile: with the taps columns padded to a
                             // multiple of 16 the B column index may reach -15 (A is 0 there)

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int wrapi(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

__host__ __device__ inline int taps_stride(int ks) {
    const int kp = (ks + 15) & ~15;               // K-dim padded to whole chunks (KCHUNK = 16)
    return kp + ((4 - kp) & 63);                  // stride = 4 (mod 64): 16 rows x 4 cols hit 64 banks
}

// kc advances in chunks of CH MFMA steps (4 columns each): the CH operand
// sets of a chunk are loaded together, so the LDS latency of one load
// overlaps the MFMAs of the chunk's earlier steps.
constexpr int CH = 4;
constexpr int KCHUNK = 4 * CH;               // taps columns padded to a multiple of this

template <bool R0, bool R1>
__device__ __forceinline__ void conv_rows(floatx4 (&acc)[2][2], const float *taps, int S, int ks, int nch,
                                          const float *tile, int TW, int t_begin, int t_end, int RB, int CB,
                                          int i, int k, int hk) {
    for (int t = t_begin; t < t_end; ++t) {
        // Two-level accumulation: the taps of one tile row (<= k products per
        // output) go into a fresh row accumulator that is then added to the
        // running sum, so an output's rounding error grows with ~2k additions
        // instead of k^2 chained ones (50 RL iterations at k = 63 drifted to
        // 1.04e-4 of the complex128 restatement with one chain, 10x the f32
        // FFT the reference uses).
        floatx4 racc[2][2];
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int q = 0; q < 2; q++) racc[p][q] = floatx4{0.f, 0.f, 0.f, 0.f};
        // A rows: krow = 16*rb + i + 2h - t (band: 0 <= krow < ks); rows outside
        // the band read a clamped row and are zeroed by a 0/1 mask (no branch)
        const int kr0 = i + 2 * hk - t, kr1 = kr0 + 16;
        // B: tile[RB + t][CB + 16*cb + j + 2h - kc]
        const float *bp = tile + (RB + t) * TW + CB + i + 2 * hk - k;
        // rows t in [15, 2h] (A0) / [31, 2h + 16] (A1) keep every lane's A
        // row inside the band: no clamp and no 0/1 mask multiply there (a
        // wave-uniform branch; the masked form runs only on the band's
        // entry and exit rows)
        auto chunks = [&](auto masked) {
            constexpr bool MS = decltype(masked)::value;
            float m0 = 1.f, m1 = 1.f;
            const float *a0p = taps + kr0 * S + k, *a1p = taps + kr1 * S + k;
            if constexpr (MS) {
                m0 = (kr0 >= 0 && kr0 < ks) ? 1.f : 0.f;
                m1 = (kr1 >= 0 && kr1 < ks) ? 1.f : 0.f;
                a0p = taps + min(max(kr0, 0), ks - 1) * S + k;
                a1p = taps + min(max(kr1, 0), ks - 1) * S + k;
            }
            for (int c = 0; c < nch; ++c) {
                float a0[CH], a1[CH], b0[CH], b1[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int kc = KCHUNK * c + 4 * u;
                    b0[u] = bp[-kc];
                    b1[u] = bp[16 - kc];
                    a0[u] = R0 ? (MS ? a0p[kc] * m0 : a0p[kc]) : 0.f;
                    a1[u] = R1 ? (MS ? a1p[kc] * m1 : a1p[kc]) : 0.f;
                }
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    if (R0) {
                        racc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], b0[u], racc[0][0], 0, 0, 0);
                        racc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], b1[u], racc[0][1], 0, 0, 0);
                    }
                    if (R1) {
                        racc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u], b0[u], racc[1][0], 0, 0, 0);
                        racc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u], b1[u], racc[1][1], 0, 0, 0);
                    }
                }
            }
        };
        const bool edge = (R0 && (t < 15 || t > 2 * hk)) || (R1 && (t < 31 || t > 2 * hk + 16));
        if (edge) chunks(std::true_type{});
        else chunks(std::false_type{});
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (R0) acc[0][q] += racc[0][q];
            if (R1) acc[1][q] += racc[1][q];
        }
    }
}

__global__ __launch_bounds__(256) void k_conv2d_mfma(ConvArgs a, int epi) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int ks = a.ks, hk = ks / 2;
    const int TH = TILE + ks - 1, TW = TILE + ks - 1;
    const int S = taps_stride(ks);
    const int KP = (ks + 15) & ~15;
    float *tile = lds + GUARD;
    float *taps = tile + TH * TW;
    const int X0 = blockIdx.x * TILE, Y0 = blockIdx.y * TILE;
    const int W = a.W, H = a.H;

    for (int idx = threadIdx.x; idx < ks * S; idx += blockDim.x) {
        const int r = idx / S, c = idx - r * S;
        taps[idx] = (c < ks) ? a.taps[r * ks + c] : 0.f;
    }
    if (threadIdx.x < GUARD) lds[threadIdx.x] = 0.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // tile + halo: one wave per row, lanes along the row
    for (int r = wave; r < TH; r += 4) {
        int y = Y0 - hk + r;
        bool yin = true;
        if (a.wrap) y = wrapi(wrapi(y, H), H);
        else yin = (y >= 0 && y < H);
        const float *row = a.in + (long long)(yin ? y : 0) * W;
        for (int c = lane; c < TW; c += 64) {
            int x = X0 - hk + c;
            float v;
            if (a.wrap) {
                v = row[wrapi(wrapi(x, W), W)];
            } else {
                v = (yin && x >= 0 && x < W) ? row[x] : 0.f;
            }
            tile[r * TW + c] = v;
        }
    }
    __syncthreads();

    const int RB = 32 * (wave >> 1), CB = 32 * (wave & 1);
    const int i = lane & 15, k = lane >> 4;
    floatx4 acc[2][2];
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
        for (int q = 0; q < 2; q++) acc[p][q] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nch = KP / KCHUNK;
    // rows t (relative to RB): block 0 uses [0, 16 + 2h), block 1 uses [16, 32 + 2h)
    conv_rows<true, false>(acc, taps, S, ks, nch, tile, TW, 0, 16, RB, CB, i, k, hk);
    conv_rows<true, true>(acc, taps, S, ks, nch, tile, TW, 16, 16 + 2 * hk, RB, CB, i, k, hk);
    conv_rows<false, true>(acc, taps, S, ks, nch, tile, TW, 16 + 2 * hk, 32 + 2 * hk, RB, CB, i, k, hk);

    double stop_part = 0.0;
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int cb = 0; cb < 2; cb++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                // C/D layout of 16x16 MFMA: col = lane & 15, row = 4*(lane >> 4) + reg
                const int oy = Y0 + RB + 16 * rb + 4 * k + r, ox = X0 + CB + 16 * cb + i;
                if (oy >= H || ox >= W) continue;
                const long long p = (long long)oy * W + ox;
                const float c = acc[rb][cb][r];
                rl_epilogue(a, epi, p, ox, oy, c, stop_part);
            }
    if (a.stop_acc) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) stop_part += __shfl_xor(stop_part, off, 64);
        if (lane == 0) atomicAdd(a.stop_acc, stop_part);
    }
}

size_t conv_lds_bytes(int ks) {
    const int TH = TILE + ks - 1, TW = TILE + ks - 1;
    return ((size_t)GUARD + (size_t)TH * TW + (size_t)ks * taps_stride(ks)) * sizeof(float);
}

int max_conv_ks() {
    int ks = 1;
    while (conv_lds_bytes(ks + 2) <= 160 * 1024) ks += 2;
    return ks;
}

int launch_conv(const ConvArgs &a, int epi, hipStream_t s) {
    if (a.ks < 1 || !(a.ks & 1)) return -1;
    const size_t lds = conv_lds_bytes(a.ks);
    if (lds > 160 * 1024) return -1;
    static size_t configured = 0;
    if (lds > 64 * 1024 && lds > configured) {
        if (hipFuncSetAttribute((const void *)k_conv2d_mfma, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds) != hipSuccess)
            return -1;
        configured = lds;
    }
    dim3 grid((a.W + TILE - 1) / TILE, (a.H + TILE - 1) / TILE);
    hipLaunchKernelGGL(k_conv2d_mfma, grid, dim3(256), lds, s, a, epi);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------ regularisers
// One thread per pixel; the few neighbours each output needs are re-read from
// global memory (L2-resident stencil, HBM-bound: one read + one write).

// FFT path (lazy expressions of image_expr.hpp:780-1020 on real(est)):
// grad_x / (|grad| + FLT_EPSILON) at flat index q
__device__ __forceinline__ void tv_unit(const float *e, int W, int H, int q, float &gx, float &gy) {
    const int x = q % W, y = q / W;
    const float dx = (x == W - 1) ? 0.f : e[q + 1] - e[q];
    const float dy = (y == H - 1) ? 0.f : e[q + W] - e[q];
    const float mag = hypotf(dx, dy) + 1.1920929e-7f;
    gx = dx / mag;
    gy = dy / mag;
}
__device__ __forceinline__ float tvx(const float *e, int W, int H, int q) {
    float gx, gy;
    tv_unit(e, W, H, q, gx, gy);
    return gx;
}
__device__ __forceinline__ float tvy(const float *e, int W, int H, int q) {
    float gx, gy;
    tv_unit(e, W, H, q, gx, gy);
    return gy;
}

// naive path (img_t::gradientx / y, sanitized, divided by their hypot)
__device__ __forceinline__ float sanit(float v) { return (v != v || v == 0.f) ? 1.e-9f : v; }
__device__ __forceinline__ void tvn_unit(const float *e, int W, int H, int x, int y, float &gx, float &gy) {
    const int q = y * W + x;
    const float dx = sanit((x < W - 1) ? e[q + 1] - e[q] : 0.f);
    const float dy = sanit((y < H - 1) ? e[q + W] - e[q] : 0.f);
    const float m = hypotf(dx, dy);
    gx = dx / m;
    gy = dy / m;
}
__device__ __forceinline__ float tnx(const float *e, int W, int H, int x, int y) {
    float gx, gy;
    tvn_unit(e, W, H, x, y, gx, gy);
    return gx;
}
__device__ __forceinline__ float tny(const float *e, int W, int H, int x, int y) {
    float gx, gy;
    tvn_unit(e, W, H, x, y, gx, gy);
    return gy;
}

__global__ __launch_bounds__(256) void k_rl_reg(const float *e, float *w, float *gxy_out, int W, int H, int mode) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const int i = y * W + x;
    float r;
    if (mode == REG_W_FFT_TV) {
        // divergence_img_expr_t::operator[] (image_expr.hpp:870-900), with its
        // flat corner indices
        if (x == 0 && y == 0) r = tvx(e, W, H, 0) + tvy(e, W, H, 0);
        else if (x == W - 1 && y == 0) r = -tvx(e, W, H, W - 2) + tvy(e, W, H, W - 1);
        else if (x == 0 && y == H - 1) r = tvx(e, W, H, H - 1) - tvy(e, W, H, H - 2);
        else if (x == W - 1 && y == H - 1)
            r = -tvx(e, W, H, W - 2 + W * (H - 1)) - tvy(e, W, H, W - 1 + W * (H - 2));
        else if (x == 0) r = (tvx(e, W, H, i) + tvy(e, W, H, i)) - tvy(e, W, H, i - W);
        else if (y == 0) r = (tvx(e, W, H, i) - tvx(e, W, H, i - 1)) + tvy(e, W, H, i);
        else if (x == W - 1) r = (-tvx(e, W, H, W - 2 + W * y) + tvy(e, W, H, i)) - tvy(e, W, H, i - W);
        else if (y == H - 1) r = (tvx(e, W, H, i) - tvx(e, W, H, i - 1)) - tvy(e, W, H, x + W * (H - 2));
        else {
            float gx, gy, gxl, gyu, t;
            tv_unit(e, W, H, i, gx, gy);
            tv_unit(e, W, H, i - 1, gxl, t);
            tv_unit(e, W, H, i - W, t, gyu);
            r = ((gx - gxl) + gy) - gyu;
        }
    } else if (mode == REG_W_NAIVE_TV) {
        // img_t::divergence(gx, gy) (image.hpp:992-1060)
        if (x == 0 && y == 0) r = tnx(e, W, H, 0, 0) + tny(e, W, H, 0, 0);
        else if (x == W - 1 && y == 0) r = -tnx(e, W, H, W - 2, 0) + tny(e, W, H, W - 1, 0);
        else if (x == 0 && y == H - 1) r = tnx(e, W, H, 0, H - 1) - tny(e, W, H, 0, H - 2);
        else if (x == W - 1 && y == H - 1) r = -tnx(e, W, H, W - 2, H - 1) - tny(e, W, H, W - 1, H - 2);
        else if (x == 0) r = (tnx(e, W, H, 0, y) + tny(e, W, H, 0, y)) - tny(e, W, H, 0, y - 1);
        else if (y == 0) r = (tnx(e, W, H, x, 0) - tnx(e, W, H, x - 1, 0)) + tny(e, W, H, x, 0);
        else if (x == W - 1) r = (-tnx(e, W, H, W - 2, y) + tny(e, W, H, W - 1, y)) - tny(e, W, H, W - 1, y - 1);
        else if (y == H - 1) r = (tnx(e, W, H, x, H - 1) - tnx(e, W, H, x - 1, H - 1)) - tny(e, W, H, x, H - 2);
        else {
            float gx, gy, gxl, gyu, t;
            tvn_unit(e, W, H, x, y, gx, gy);
            tvn_unit(e, W, H, x - 1, y, gxl, t);
            tvn_unit(e, W, H, x, y - 1, t, gyu);
            r = ((gx - gxl) + gy) - gyu;
        }
    } else {
        const float c = e[i];
        const bool xe = (x == 0 || x == W - 1), ye = (y == 0 || y == H - 1);
        const bool xy_in = (x < W - 1 && y < H - 1);
        if (mode == REG_W_FFT_FH) {
            // gradientxx / yy / xy expressions: (r - 2c) + l, ((br - tr) - bl) + tl
            const float gxx = xe ? 0.f : (e[i + 1] - 2.f * c) + e[i - 1];
            const float gyy = ye ? 0.f : (e[i + W] - 2.f * c) + e[i - W];
            const float gxy = xy_in ? ((e[i + W + 1] - e[i + 1]) - e[i + W]) + c : 0.f;
            const float sumsq = gxx * gxx + gyy * gyy;
            r = sanit(sqrtf(fmaf(2.f, gxy * gxy, sumsq)));
        } else {
            // img_t::gradientxx / yy: (r + l) - 2c; gradientxy as above
            const float gxx = xe ? 0.f : (e[i + 1] + e[i - 1]) - 2.f * c;
            const float gyy = ye ? 0.f : (e[i + W] + e[i - W]) - 2.f * c;
            const float gxy = xy_in ? ((e[i + W + 1] - e[i + 1]) - e[i + W]) + c : 0.f;
            const float xx = fmaxf(1.e-9f, gxx), xy = fmaxf(1.e-9f, gxy), yy = fmaxf(1.e-9f, gyy);
            r = sqrtf(xx * xx + (2.f * (xy * xy) + yy * yy));
            if (gxy_out) gxy_out[i] = gxy;
        }
    }
    w[i] = r;
}

int launch_reg(const float *e, float *w, float *gxy, int W, int H, int mode, hipStream_t s) {
    dim3 grid((W + 63) / 64, (H + 3) / 4);
    hipLaunchKernelGGL(k_rl_reg, grid, dim3(256), 0, s, e, w, gxy, W, H, mode);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- plumbing

__device__ __forceinline__ unsigned f2ord(float v) {
    const unsigned b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

float decode_max(unsigned o) {
    const unsigned b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    float v;
    __builtin_memcpy(&v, &b, 4);
    return v;
}

__global__ __launch_bounds__(256) void k_chan_max(const float *f, long long n, unsigned *bits) {
    unsigned m = 0;
    for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (long long)gridDim.x * blockDim.x) {
        const float v = f[p];
        if (v == v) m = max(m, f2ord(v));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off, 64));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(bits, m);
}

int launch_chan_max(const float *f, long long n, unsigned *bits, hipStream_t s) {
    long long blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_chan_max, dim3((unsigned)blocks), dim3(256), 0, s, f, n, bits);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// add_padding's mirror (utils.hpp:71-112): padded index -> unpadded index
__device__ __forceinline__ int unpad(int p, int n, int pad) {
    const int np = n + 2 * pad;
    int src = p;
    if (p < pad) src = 2 * pad - p;
    else if (p >= np - pad) src = 2 * (np - 1) - 2 * pad - p;
    return src - pad;
}

// whole-sample reflection of process_in_slices (image.hpp:440-450)
__device__ __forceinline__ int reflect(int p, int n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - p - 2;
    return p;
}

__global__ __launch_bounds__(256) void k_extract(const float *f, int rx, int ry, int pad, int Wp, int Hp,
                                                 SliceGeom g, float mx, int div, float *out) {
    const int sx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int sy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (sx >= g.sw || sy >= g.sh) return;
    const int py = reflect(g.y0 - g.pt + sy, Hp), px = reflect(g.x0 - g.pl + sx, Wp);
    const int y = unpad(py, ry, pad), x = unpad(px, rx, pad);
    const float v = f[(long long)y * rx + x];
    out[(long long)sy * g.sw + sx] = div ? v / mx : v;
}

int launch_extract(const float *f, int rx, int ry, int pad, int Wp, int Hp, SliceGeom g, float mx, int div,
                   float *out, hipStream_t s) {
    dim3 grid((g.sw + 63) / 64, (g.sh + 3) / 4);
    hipLaunchKernelGGL(k_extract, grid, dim3(256), 0, s, f, rx, ry, pad, Wp, Hp, g, mx, div, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ __launch_bounds__(256) void k_store(const float *x, int rx, int ry, int pad, SliceGeom g, float mx,
                                               int mul, float *u) {
    const int ax = blockIdx.x * 64 + (threadIdx.x & 63);
    const int ay = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (ax >= g.aw || ay >= g.ah) return;
    const int X = g.x0 + ax - pad, Y = g.y0 + ay - pad;
    if (X < 0 || X >= rx || Y < 0 || Y >= ry) return;
    const float v = x[(long long)(g.pt + ay) * g.sw + g.pl + ax];
    u[(long long)Y * rx + X] = mul ? v * mx : v;
}

int launch_store(const float *x, int rx, int ry, int pad, SliceGeom g, float mx, int mul, float *u,
                 hipStream_t s) {
    dim3 grid((g.aw + 63) / 64, (g.ah + 3) / 4);
    hipLaunchKernelGGL(k_store, grid, dim3(256), 0, s, x, rx, ry, pad, g, mx, mul, u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rl
}  // namespace sgpu
