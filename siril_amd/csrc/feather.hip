// feather.hip -- feathering masks of `stack ... -feather=<dist>` (SURVEY 8f
// rank 2): the producer compute_masks (stacking/blending.c:131-224) and the
// per-block consumer of stack_read_block_data (stacking/median_and_mean.c:
// 483-525), both on HBM-resident frames.
//
//   * k_mask_sample: the 0/255 reference layer (blending.c:138-153) closed by
//     a 7x7 dilate + erode and resized INTER_LINEAR to (int)(0.1 rx) x
//     (int)(0.1 ry) (cvDownscaleBlendMask, opencv/opencv.cpp:587-604).  A
//     linear resize by ~10 reads two rows and two columns of the closed mask
//     per output sample, so a workgroup closes only the 14 source rows around
//     one output row, over the column span of 64 outputs, in LDS (u8), and
//     applies OpenCV's 8-bit fixed-point resize (11-bit coefficients; the
//     baseline SSE2 vertical pass for all but the row tail, the scalar
//     rounding for the tail, as resize.cpp's VResizeLinearVec_32s8u does);
//   * k_mask_dt: distanceTransform(DIST_L2, 3) (opencv.cpp:606) on the
//     zero-bordered (w+2) x (h+2) image: the 3x3 chamfer (0.955, 1.3693) in
//     16-bit fixed point.  The reference's two raster passes are sequential
//     only along each row, t[c] = min(u[c], t[c-1] + a): a min-plus prefix
//     scan, min_k<=c (u[k] - a k) + a c, exact in integers.  One wave per
//     frame walks the rows; each lane owns C adjacent columns in registers,
//     the carry crosses lanes with a 6-step shuffle scan;
//   * k_mask_block: per block and frame, the mask rows of the block's area
//     (read_mask_fits_area convention, image_format_fits.c:4113-4123),
//     cvUpscaleBlendMask (opencv.cpp:611-616: INTER_LINEAR in float, then
//     the vertical flip) and the feather ramp (1 above the distance, else the
//     smootherstep table of init_ramp, blending.c:34-50).
//
// OpenCV is not in this image; the resize and distance-transform arithmetic
// restates OpenCV's generic (non-IPP) code paths, see oracle/feather_ref.py.
// No FMA contraction anywhere in this file: the reference's x86-64 baseline
// build multiplies and adds separately.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "sgpu_internal.h"

#pragma clang fp contract(off)

using sgpu_host::fail;

namespace {

constexpr int kCoefBits = 11;
constexpr int kCoefScale = 1 << kCoefBits;
constexpr int kTileX = 64;          // output columns per k_mask_sample workgroup
constexpr int kRampPace = 1000;     // RAMP_PACE (blending.c:30)
constexpr int kDistMax = 0x7fffffff >> 2;
constexpr int kDistInit = 1 << 30;  // outside the zero-bordered image (never reaches a kept value)

// cv::saturate_cast<short>(float): cvRound (nearest, ties to even), saturated
inline int sat_short(float v) {
    long r = std::lrint(v);
    return (int)std::min(32767L, std::max(-32768L, r));
}

// source index and fraction of OpenCV's INTER_LINEAR resize for each
// destination index (resize.cpp, hal::resize: fx = (float)((d + 0.5) *
// scale - 0.5), cvFloor, fx -= sx).  clamp: the horizontal table (sx < 0 ->
// (0, 0); sx >= src - 1 -> (src - 1, 0)); the vertical one keeps the raw
// fraction and lets the row fetch clamp (clip(sy, 0, h)).
void lin_table(int src, int dst, bool clamp, std::vector<int> &ofs, std::vector<float> &frac) {
    const double inv = (double)dst / (double)src;
    const double scale = 1. / inv;
    ofs.resize(dst);
    frac.resize(dst);
    for (int d = 0; d < dst; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)f;
        s -= (s > f);               // cvFloor
        f -= (float)s;
        if (clamp) {
            if (s < 0) f = 0.f, s = 0;
            if (s + 1 >= src && s >= src - 1) f = 0.f, s = src - 1;
        }
        ofs[d] = s;
        frac[d] = f;
    }
}

// the downscaled mask size (compute_downscaled_mask_size, blending.c:52-59)
inline void mask_size(long rx, long ry, int &rxo, int &ryo) {
    rxo = (int)((double)rx * 0.1);
    ryo = (int)((double)ry * 0.1);
}

}  // namespace

namespace sgpu {

// ---------------------------------------------------------------------------
// k_mask_sample: one output row dy, 64 output columns, one frame
// ---------------------------------------------------------------------------
struct SampleTabs {
    const int *xofs;      // [rxo] clamped source column
    const int *xa;        // [2 rxo] 11-bit coefficients (1 - fx, fx)
    const int *yofs;      // [ryo] raw source row
    const int *yb;        // [2 ryo]
    const int *span;      // [tiles] first source column of the tile's closed span
};

template <typename T>
__device__ __forceinline__ unsigned char nonzero_u8(T v);
template <>
__device__ __forceinline__ unsigned char nonzero_u8<float>(float v) { return v != 0.f ? 255 : 0; }
template <>
__device__ __forceinline__ unsigned char nonzero_u8<unsigned short>(unsigned short v) { return v > 0 ? 255 : 0; }

template <typename T>
__global__ __launch_bounds__(256) void k_mask_sample(const T *frames, long long fstride, int W, int H, SampleTabs t,
                                                     int rxo, int ryo, int xv, int L, unsigned char *dtin) {
    extern __shared__ unsigned char lds[];
    const int f = blockIdx.z, dy = blockIdx.y, tile = blockIdx.x;
    const int d0 = tile * kTileX, d1 = min(d0 + kTileX, rxo);
    const int cs = t.span[tile];                    // closed columns [cs, cs + L)
    const int sy = t.yofs[dy];
    const int r0 = min(max(sy, 0), H - 1);          // clip(sy, 0, h), clip(sy + 1, 0, h)
    const int r1 = min(max(sy + 1, 0), H - 1);
    const int LB = L + 12, LD = L + 6;
    unsigned char *B = lds;                  // 14 rows r0-6 .. r0+7, columns cs-6 ..
    unsigned char *HD = B + 14 * LB;         // 14 rows, columns cs-3 ..
    unsigned char *D = HD + 14 * LD;         // dilated rows r0-3 .. r0+4, columns cs-3 ..
    unsigned char *HE = D + 8 * LD;          // 8 rows, columns cs ..
    const T *fr = frames + (long long)f * fstride;
    for (int i = threadIdx.x; i < 14 * LB; i += blockDim.x) {
        const int rr = i / LB, cc = i - rr * LB;
        const int r = r0 - 6 + rr, c = cs - 6 + cc;
        unsigned char v = 0;                 // dilate: the constant border never wins the max
        if (r >= 0 && r < H && c >= 0 && c < W) v = nonzero_u8<T>(fr[(long long)r * W + c]);
        B[i] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 14 * LD; i += blockDim.x) {
        const int rr = i / LD, cc = i - rr * LD;
        const unsigned char *b = B + rr * LB + cc;
        unsigned char m = b[0];
#pragma unroll
        for (int k = 1; k < 7; k++) m = max(m, b[k]);
        HD[i] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * LD; i += blockDim.x) {
        const int rr = i / LD, cc = i - rr * LD;
        const unsigned char *h = HD + rr * LD + cc;
        unsigned char m = h[0];
#pragma unroll
        for (int k = 1; k < 7; k++) m = max(m, h[k * LD]);
        D[i] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * L; i += blockDim.x) {
        const int rr = i / L, cc = i - rr * L;
        const int c = cs + cc;
        unsigned char m = 255;               // erode: out-of-image columns never win the min
        for (int k = -3; k <= 3; k++)
            if (c + k >= 0 && c + k < W) m = min(m, D[rr * LD + cc + 3 + k]);
        HE[i] = m;
    }
    __syncthreads();
    const int dx = d0 + (int)threadIdx.x;
    if (dx >= d1) return;
    auto closed = [&](int r, int c) -> int {  // erode over rows r-3..r+3 inside the image
        unsigned char m = 255;
        for (int k = -3; k <= 3; k++)
            if (r + k >= 0 && r + k < H) m = min(m, HE[(r + k - (r0 - 3)) * L + (c - cs)]);
        return m;
    };
    const int sx = t.xofs[dx], sx1 = min(sx + 1, W - 1);
    const int a0 = t.xa[2 * dx], a1 = t.xa[2 * dx + 1];
    const int h0 = closed(r0, sx) * a0 + closed(r0, sx1) * a1;    // HResizeLinear (int)
    const int h1 = closed(r1, sx) * a0 + closed(r1, sx1) * a1;
    const int b0 = t.yb[2 * dy], b1 = t.yb[2 * dy + 1];
    int v;
    if (dx < xv) {
        // VResizeLinearVec_32s8u: ((S >> 4) * b) >> 16 per row (mulhi of
        // int16), saturating int16 add, (x + 2) >> 2, pack to u8 unsigned
        int s = ((short)(h0 >> 4) * b0 >> 16) + ((short)(h1 >> 4) * b1 >> 16);
        s = min(max(s, -32768), 32767);
        v = (s + 2) >> 2;
    } else {
        v = (h0 * b0 + h1 * b1 + (1 << (2 * kCoefBits - 1))) >> (2 * kCoefBits);
    }
    v = min(max(v, 0), 255);
    dtin[(long long)f * (ryo + 2) * (rxo + 2) + (long long)(dy + 1) * (rxo + 2) + dx + 1] = (unsigned char)v;
}

// ---------------------------------------------------------------------------
// k_mask_dt: one wave per frame, C columns per lane
// ---------------------------------------------------------------------------
__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, 64); }

template <int C>
__global__ __launch_bounds__(64) void k_mask_dt(const unsigned char *dtin, int Wp, int Hp, int *tmp, float *out,
                                                int hv, int dg) {
    const int f = blockIdx.x, lane = threadIdx.x;
    const unsigned char *src = dtin + (long long)f * Wp * Hp;
    int *tm = tmp + (long long)f * Wp * Hp;
    const int rxo = Wp - 2, ryo = Hp - 2;
    float *o = out + (long long)f * rxo * ryo;
    const int c0 = lane * C;
    int P[C], t[C];
#pragma unroll
    for (int k = 0; k < C; k++) P[k] = kDistInit;
    // forward pass (distanceTransform_3x3 first loop): rows top to bottom,
    // columns left to right
    for (int r = 0; r < Hp; r++) {
        // every lane shuffles (a lane reading an inactive one gets 0)
        const int pl0 = shfl_i(P[C - 1], lane > 0 ? lane - 1 : 0);
        const int pr0 = shfl_i(P[0], lane < 63 ? lane + 1 : 63);
        const int pl = lane > 0 ? pl0 : kDistInit, pr = lane < 63 ? pr0 : kDistInit;
        int m = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < C; k++) {
            const int c = c0 + k;
            const int left = k > 0 ? P[k - 1] : pl, right = k < C - 1 ? P[k + 1] : pr;
            int u = kDistInit;
            if (c < Wp) {
                const bool on = src[(long long)r * Wp + c] != 0;
                u = on ? min(min(left + dg, P[k] + hv), right + dg) : 0;
            }
            m = min(m, u - hv * c);            // running prefix min of u[k] - a k
            t[k] = m;
        }
        // exclusive carry across lanes: inclusive scan of the lane minima
        int agg = m;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(agg, off, 64);
            if (lane >= off) agg = min(agg, v);
        }
        int carry = __shfl_up(agg, 1, 64);
        if (lane == 0) carry = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < C; k++) {
            const int c = c0 + k;
            const int v = min(t[k], carry) + hv * c;
            P[k] = c < Wp ? v : kDistInit;
            if (c < Wp) tm[(long long)r * Wp + c] = v;
        }
    }
    // backward pass: rows bottom to top, columns right to left; the
    // reference's `t0 > HV_DIST` test only skips mins that cannot win
#pragma unroll
    for (int k = 0; k < C; k++) P[k] = kDistInit;
    for (int r = Hp - 1; r >= 0; r--) {
        const int ql0 = shfl_i(P[C - 1], lane > 0 ? lane - 1 : 0);
        const int qr0 = shfl_i(P[0], lane < 63 ? lane + 1 : 63);
        const int ql = lane > 0 ? ql0 : kDistInit, qr = lane < 63 ? qr0 : kDistInit;
        int m = 0x7fffffff;
#pragma unroll
        for (int k = C - 1; k >= 0; k--) {
            const int c = c0 + k;
            const int left = k > 0 ? P[k - 1] : ql, right = k < C - 1 ? P[k + 1] : qr;
            int v = kDistInit;
            if (c < Wp) v = min(min(tm[(long long)r * Wp + c], P[k] + hv), min(left + dg, right + dg));
            m = min(m, v + hv * c);            // running suffix min of v[k] + a k
            t[k] = m;
        }
        int agg = m;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_down(agg, off, 64);
            if (lane + off < 64) agg = min(agg, v);
        }
        int carry = __shfl_down(agg, 1, 64);
        if (lane == 63) carry = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < C; k++) {
            const int c = c0 + k;
            const int v = min(t[k], carry) - hv * c;
            P[k] = c < Wp ? v : kDistInit;
            if (c >= 1 && c <= rxo && r >= 1 && r <= ryo)
                o[(long long)(r - 1) * rxo + (c - 1)] = __int2float_rn(min(v, kDistMax)) * (1.f / 65536.f);
        }
    }
}

// ---------------------------------------------------------------------------
// k_mask_block: the block's ramped mask planes
// ---------------------------------------------------------------------------
struct BlockFrame {
    int y0;      // first plane row holding the area's mask rows
    int ah;      // area.h (0: the frame contributes zeros)
    int base;    // first downscaled row read (ry_o - y_s - h_s)
    int hs;      // downscaled rows read
    int placex;  // canvas column of the frame's column 0
    int flip;    // 1: plane row y0 + i holds upscaled row ah - 1 - i (block reader order)
};

__global__ __launch_bounds__(256) void k_mask_block(const float *masks, int rxo, int ryo, const BlockFrame *bf,
                                                    const int *xofs, const float *xfr, int rx, int cw,
                                                    float *planes, long long pstride, const float *ramp,
                                                    float distf, float invdistf) {
    const int f = blockIdx.z, j = blockIdx.y;
    const int X = blockIdx.x * 256 + threadIdx.x;
    if (X >= cw) return;
    const BlockFrame b = bf[f];
    float v = 0.f;
    const int x = X - b.placex;
    const int i = j - b.y0;
    if (b.ah > 0 && i >= 0 && i < b.ah && x >= 0 && x < rx) {
        const int u = b.flip ? b.ah - 1 - i : i;
        // vertical table of cvUpscaleBlendMask's resize (hs -> ah rows)
        const double scale_y = 1. / ((double)b.ah / (double)b.hs);
        float fy = (float)((u + 0.5) * scale_y - 0.5);
        int sy = (int)fy;
        sy -= (sy > fy);
        fy -= (float)sy;
        const int ra = min(max(sy, 0), b.hs - 1), rb = min(max(sy + 1, 0), b.hs - 1);
        const float *m0 = masks + ((long long)f * ryo + b.base + ra) * rxo;
        const float *m1 = masks + ((long long)f * ryo + b.base + rb) * rxo;
        const int sx = xofs[x], sx1 = min(sx + 1, rxo - 1);
        const float a1 = xfr[x], a0 = 1.f - a1;
        const float s0 = m0[sx] * a0 + m0[sx1] * a1;
        const float s1 = m1[sx] * a0 + m1[sx1] * a1;
        v = s0 * (1.f - fy) + s1 * fy;
        if (v != 0.f) v = v > distf ? 1.f : ramp[(int)((v * invdistf) * (float)kRampPace)];
    }
    planes[(long long)f * pstride + (long long)j * cw + X] = v;
}

}  // namespace sgpu

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" void sgpu_feather_mask_size(long width, long height, long *mask_width, long *mask_height) {
    int rxo = 0, ryo = 0;
    mask_size(width, height, rxo, ryo);
    if (mask_width) *mask_width = rxo;
    if (mask_height) *mask_height = ryo;
}

extern "C" int sgpu_feather_masks_device(sgpu_context *c, const void *d_frames, int elem_size, int nframes,
                                         long width, long height, long frame_stride, float *d_masks) {
    if (!c || !d_frames || !d_masks || nframes < 1 || width < 1 || height < 1 || frame_stride < width * height)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (elem_size != 4 && elem_size != 2) return fail(SGPU_BAD_ARGUMENT, "elem_size: 4 (float) or 2 (uint16)");
    int rxo, ryo;
    mask_size(width, height, rxo, ryo);
    if (rxo < 1 || ryo < 1) return fail(SGPU_BAD_ARGUMENT, "frames smaller than 10 pixels have an empty mask");
    const int Wp = rxo + 2, Hp = ryo + 2;
    int C = 4;
    while (C * 64 < Wp && C < 64) C *= 2;
    if (C * 64 < Wp) return fail(SGPU_BAD_ARGUMENT, "mask wider than 4094 samples (frames wider than 40949)");
    // resize tables: 8-bit coefficients (saturate_cast<short>(w * 2048))
    std::vector<int> xofs, yofs;
    std::vector<float> xf, yf;
    lin_table((int)width, rxo, true, xofs, xf);
    lin_table((int)height, ryo, false, yofs, yf);
    const int tiles = (rxo + kTileX - 1) / kTileX;
    std::vector<int> tab;
    tab.reserve((size_t)3 * rxo + 3 * ryo + tiles);
    tab.insert(tab.end(), xofs.begin(), xofs.end());
    for (int d = 0; d < rxo; d++) {
        tab.push_back(sat_short((1.f - xf[d]) * (float)kCoefScale));
        tab.push_back(sat_short(xf[d] * (float)kCoefScale));
    }
    tab.insert(tab.end(), yofs.begin(), yofs.end());
    for (int d = 0; d < ryo; d++) {
        tab.push_back(sat_short((1.f - yf[d]) * (float)kCoefScale));
        tab.push_back(sat_short(yf[d] * (float)kCoefScale));
    }
    int L = 1;
    for (int q = 0; q < tiles; q++) {
        const int a = xofs[q * kTileX], e = std::min(xofs[std::min((q + 1) * kTileX, rxo) - 1] + 1, (int)width - 1);
        tab.push_back(a);
        L = std::max(L, e - a + 1);
    }
    const size_t lds = (size_t)14 * (L + 12) + (size_t)22 * (L + 6) + (size_t)8 * L;
    if (lds > 64 * 1024) return fail(SGPU_BAD_ARGUMENT, "mask resize span too wide");
    // the vector end of the vertical pass: 16-sample steps, then 8-sample
    // steps while x < width - 8 (VResizeLinearVec_32s8u)
    int xv = 0;
    while (xv <= rxo - 16) xv += 16;
    while (xv < rxo - 8) xv += 8;
    HIP_TRY(hipSetDevice(c->device));
    if (int r = c->fe_tab.ensure(tab.size() * sizeof(int))) return r;
    const size_t dtn = (size_t)nframes * Wp * Hp, dta = ((dtn + 255) / 256) * 256;
    if (int r = c->fe_dt.ensure(dta + dtn * sizeof(int))) return r;
    int *dtab = (int *)c->fe_tab.p;
    HIP_TRY(hipMemcpyAsync(dtab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    unsigned char *dtin = (unsigned char *)c->fe_dt.p;
    int *dtmp = (int *)(dtin + dta);
    HIP_TRY(hipMemsetAsync(dtin, 0, dtn, c->stream));       // the one-pixel black frame
    sgpu::SampleTabs t;
    t.xofs = dtab;
    t.xa = dtab + rxo;
    t.yofs = dtab + 3 * rxo;
    t.yb = dtab + 3 * rxo + ryo;
    t.span = dtab + 3 * rxo + 3 * ryo;
    const dim3 g(tiles, ryo, nframes);
    if (elem_size == 4)
        hipLaunchKernelGGL(sgpu::k_mask_sample<float>, g, dim3(256), lds, c->stream, (const float *)d_frames,
                           (long long)frame_stride, (int)width, (int)height, t, rxo, ryo, xv, L, dtin);
    else
        hipLaunchKernelGGL(sgpu::k_mask_sample<unsigned short>, g, dim3(256), lds, c->stream,
                           (const unsigned short *)d_frames, (long long)frame_stride, (int)width, (int)height, t,
                           rxo, ryo, xv, L, dtin);
    HIP_TRY(hipGetLastError());
    const int hv = (int)std::lrint(0.955f * (float)(1 << 16));      // CV_FLT_TO_FIX(0.955f, DIST_SHIFT)
    const int dg = (int)std::lrint(1.3693f * (float)(1 << 16));
#define SGPU_DT(CC)                                                                                            \
    hipLaunchKernelGGL(sgpu::k_mask_dt<CC>, dim3(nframes), dim3(64), 0, c->stream, dtin, Wp, Hp, dtmp, d_masks, \
                       hv, dg)
    switch (C) {
        case 4: SGPU_DT(4); break;
        case 8: SGPU_DT(8); break;
        case 16: SGPU_DT(16); break;
        case 32: SGPU_DT(32); break;
        default: SGPU_DT(64); break;
    }
#undef SGPU_DT
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));   // the host tables die with this call
    return SGPU_OK;
}

// the mask rows of one block for one frame (stack_read_block_data, median_and_mean.c:406-446, 483-499)
extern "C" int sgpu_feather_block_area(long width, long height, long start_row, long block_height, int shifty,
                                       int registered, int *plane_row, int *area_h, int *mask_row, int *mask_h) {
    if (width < 1 || height < 1 || block_height < 1 || start_row < 0 || !plane_row || !area_h || !mask_row || !mask_h)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    long ay = start_row, ah = block_height, off = 0;
    bool read = true;
    const long ry = height;
    if (registered) {
        if (ay + ah + shifty <= 0 || ay + shifty >= ry) {
            read = false;
        } else if (ay + shifty < 0) {
            ah += ay + shifty;
            ah = std::min(ah, ry);
            off = -(ay + shifty);
            ay = 0;
        } else if (ay + ah + shifty >= ry) {
            ay += shifty;
            ah += ry - (ay + ah);
        } else {
            ay += shifty;
        }
        if (ah <= 0) read = false;
    }
    int rxo, ryo;
    mask_size(width, height, rxo, ryo);
    const double fy = (double)ryo / (double)height;
    const int ys = (int)(fy * (double)ay), hs = (int)(fy * (double)ah);
    *plane_row = (int)off;
    *area_h = 0;
    *mask_row = 0;
    *mask_h = 0;
    // nothing read, or an empty downscaled area (the reference `continue`s
    // and leaves the buffer as it was: zeros here)
    if (!read || ah == 0 || hs == 0 || rxo == 0) return SGPU_OK;
    if (ryo - ys - hs < 0) return fail(SGPU_SEQUENCE_ERROR, "mask area outside the mask");
    *area_h = (int)ah;
    *mask_row = ryo - ys - hs;
    *mask_h = hs;
    return SGPU_OK;
}

extern "C" int sgpu_feather_block_device(sgpu_context *c, const float *d_masks, int nframes, long width,
                                         long height, long start_row, long block_height, const int *shifty,
                                         const int *placex, long canvas_width, float feather, int fits_order,
                                         float *d_planes, long plane_stride) {
    if (!c || !d_masks || !d_planes || nframes < 1 || width < 1 || height < 1 || block_height < 1 ||
        canvas_width < 1 || plane_stride < block_height * canvas_width || !(feather > 0.f))
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    int rxo, ryo;
    mask_size(width, height, rxo, ryo);
    if (rxo < 1 || ryo < 1) return fail(SGPU_BAD_ARGUMENT, "frames smaller than 10 pixels have an empty mask");
    std::vector<sgpu::BlockFrame> bf(nframes);
    for (int f = 0; f < nframes; f++) {
        int off, ah, mrow, mh;
        if (int r = sgpu_feather_block_area(width, height, start_row, block_height, shifty ? shifty[f] : 0,
                                            shifty != nullptr, &off, &ah, &mrow, &mh))
            return r;
        sgpu::BlockFrame &b = bf[f];
        b.ah = ah;
        b.base = mrow;
        b.hs = mh;
        b.placex = placex ? placex[f] : 0;
        // block reader order: rows [off, off + ah) hold the flipped upscale;
        // FITS order reverses the block: rows [h - off - ah, h - off) ascending
        b.flip = fits_order ? 0 : 1;
        b.y0 = fits_order ? (int)(block_height - off - ah) : off;
    }
    std::vector<int> xofs;
    std::vector<float> xf;
    lin_table(rxo, (int)width, true, xofs, xf);
    // init_ramp (blending.c:34-45): r^3 (6 r^2 - 15 r + 10) in float
    std::vector<float> ramp(kRampPace + 1);
    const float norm = 1.f / (float)kRampPace;
    for (int i = 0; i <= kRampPace; i++) {
        const float r = (float)i * norm;
        ramp[i] = r * r * r * (6.f * r * r - 15.f * r + 10.f);
    }
    const size_t nb = bf.size() * sizeof(sgpu::BlockFrame);
    const size_t bytes = nb + xofs.size() * 8 + ramp.size() * 4 + 64;
    HIP_TRY(hipSetDevice(c->device));
    if (int r = c->fe_tab.ensure(bytes)) return r;
    char *p = (char *)c->fe_tab.p;
    sgpu::BlockFrame *dbf = (sgpu::BlockFrame *)p;
    int *dx = (int *)(p + ((nb + 15) / 16) * 16);
    float *dxf = (float *)(dx + xofs.size());
    float *dramp = dxf + xf.size();
    HIP_TRY(hipMemcpyAsync(dbf, bf.data(), nb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dx, xofs.data(), xofs.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dxf, xf.data(), xf.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dramp, ramp.data(), ramp.size() * 4, hipMemcpyHostToDevice, c->stream));
    const float distf = feather, inv = 1.f / distf;
    hipLaunchKernelGGL(sgpu::k_mask_block, dim3((unsigned)((canvas_width + 255) / 256), (unsigned)block_height, nframes),
                       dim3(256), 0, c->stream, d_masks, rxo, ryo, dbf, dx, dxf, (int)width, (int)canvas_width,
                       d_planes, (long long)plane_stride, dramp, distf, inv);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SGPU_OK;
}
