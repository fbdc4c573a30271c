// quality.hip -- frame quality of the DFT registration.
//
// Reference: QualityEstimate_float (algos/quality_float.c:41-147), called on
// the S x S selection of every frame by register_shift_dft
// (registration/shift_methods.c:176,234), then normalizeQualityData
// (:36-54) and the best-frame pick (:241-246).
//
// Per subsample level s = 3, 4, 5 (levels whose sample grid does not change
// are skipped, :131-134), on the (S-1)/s x (S-1)/s grid:
//   k_q_subsample_all  s x s block means of all levels from one read of the
//                  selection (LDS tiles), summed row by row in float as
//                  SubSample does (:153-164), then / (float)(s*s)
//   k_q_smooth     the 3x3 box of _smooth_image_float (:222-250): the
//                  reference smooths in place from line buffers, i.e. every
//                  output reads the unsmoothed neighbours; same summation
//                  order, edges copied
//   k_q_gradient   Gradient (:166-219): pixels >= THRESHOLD_FLOAT inside the
//                  10% margin flag their 3x3 neighbourhood; the flagged
//                  pixels of the margin region sum d1^2 + d2^2 in f64 (d1, d2
//                  float differences).  Per-block f64 partials in a fixed
//                  order; the reference sums in row-major order, so the
//                  result agrees to rounding (relative 1e-12 in the tests).
// Host: dval += q * 9 / s^2 per level, quality = sqrt(dval).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "sgpu_internal.h"

namespace sgpu {
namespace qe {

constexpr float THRESHOLD_FLOAT = 0.156863f;   // algos/quality.h:31
constexpr double QMARGIN = 0.1;                // quality.h:25
constexpr int QSUBSAMPLE_MIN = 3, QSUBSAMPLE_MAX = 5, QSUBSAMPLE_INC = 1;
constexpr int QT = 256;

__global__ __launch_bounds__(QT) void k_q_subsample(const float *frames, long long row_stride, long long frame_stride,
                                                    int s, int xs, int ys, float *buf) {
    const int f = blockIdx.z;
    const long long i = (long long)blockIdx.x * QT + threadIdx.x;
    if (i >= (long long)xs * ys) return;
    const int x = (int)(i % xs), y = (int)(i / xs);
    const float *p = frames + (long long)f * frame_stride + (long long)(y * s) * row_stride + (long long)x * s;
    float v = 0.f;
    for (int r = 0; r < s; ++r) {
        for (int c = 0; c < s; ++c) v += p[c];
        p += row_stride;
    }
    buf[(long long)f * xs * ys + i] = v / (float)(s * s);
}

__global__ __launch_bounds__(QT) void k_q_smooth(const float *in, int xs, int ys, float *out) {
    const int f = blockIdx.z;
    const long long i = (long long)blockIdx.x * QT + threadIdx.x;
    if (i >= (long long)xs * ys) return;
    int x, y;
    if (i < 0x7fffffffLL) {       // 32-bit division when the index fits
        x = (int)((unsigned)i % (unsigned)xs);
        y = (int)((unsigned)i / (unsigned)xs);
    } else {
        x = (int)(i % xs);
        y = (int)(i / xs);
    }
    const float *b = in + (long long)f * xs * ys;
    float r = b[i];
    if (y >= 1 && y < ys - 1 && x >= 1 && x < xs - 1) {
        const float *p = b + (long long)(y - 1) * xs, *c = p + xs, *n = c + xs;
        const float v = (p[x - 1] + p[x]) + (p[x + 1] + c[x - 1]) + (c[x] + c[x + 1]) + (n[x - 1] + n[x]) + n[x + 1];
        r = v * (1.f / 9.f);
    }
    out[(long long)f * xs * ys + i] = r;
}


// Single-read subsample (default; SGPU_QE_FUSED=0 selects k_q_subsample per
// level): every active level's s x s blocks from one LDS tile of TR x TC
// pixels (multiples of 3, 4 and 5, so no block straddles tiles); the sums
// run over LDS in SubSample's order.  60 x 120 tiles (29 KB) keep 5 blocks
// per CU; 60 x 240 tiles were slower (2 blocks per CU).
constexpr int TR = 60, TC = 120;
struct Levels {
    int n;
    int s[3], xs[3], ys[3];
    float *buf[3];
};

template <bool VEC>
__global__ __launch_bounds__(QT) void k_q_subsample_all(const float *frames, long long row_stride,
                                                        long long frame_stride, int width, int height, Levels L) {
    __shared__ float t[TR][TC + 1];
    const int f = blockIdx.z;
    const int r0 = blockIdx.y * TR, c0 = blockIdx.x * TC;
    const float *img = frames + (long long)f * frame_stride;
    if (VEC) {
        // 16-byte loads, all of a thread's loads issued before the LDS stores
        // (host guarantees 16-byte aligned rows and width % 4 == 0, so a
        // float4 is either wholly inside the frame or wholly outside)
        constexpr int Q = TC / 4, NV = TR * Q, PER = (NV + QT - 1) / QT;
        float4 v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int k = threadIdx.x + j * QT, r = k / Q, q = k - r * Q;
            const int y = r0 + r, x = c0 + 4 * q;
            v[j] = (k < NV && y < height && x < width)
                       ? *reinterpret_cast<const float4 *>(img + (long long)y * row_stride + x)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int k = threadIdx.x + j * QT, r = k / Q, q = k - r * Q;
            if (k < NV) {
                t[r][4 * q] = v[j].x;
                t[r][4 * q + 1] = v[j].y;
                t[r][4 * q + 2] = v[j].z;
                t[r][4 * q + 3] = v[j].w;
            }
        }
    } else {
        const int c = threadIdx.x & 127, rr = threadIdx.x >> 7;     // 2 rows of 128 lanes per step
        if (c < TC) {
            const int x = c0 + c;
            for (int r = rr; r < TR; r += 2) {
                const int y = r0 + r;
                t[r][c] = (y < height && x < width) ? img[(long long)y * row_stride + x] : 0.f;
            }
        }
    }
    __syncthreads();
    for (int l = 0; l < L.n; ++l) {
        const int sub = L.s[l], tx = TC / sub, ty = TR / sub;
        for (int k = threadIdx.x; k < tx * ty; k += QT) {
            const int bx = k % tx, by = k / tx;
            const int X = c0 / sub + bx, Y = r0 / sub + by;
            if (X >= L.xs[l] || Y >= L.ys[l]) continue;
            float v = 0.f;
            for (int r = 0; r < sub; ++r)
                for (int cc = 0; cc < sub; ++cc) v += t[by * sub + r][bx * sub + cc];
            L.buf[l][(long long)f * L.xs[l] * L.ys[l] + (long long)Y * L.xs[l] + X] = v / (float)(sub * sub);
        }
    }
}

struct QPart {
    double sum;
    unsigned long long flagged, above;
};

__global__ __launch_bounds__(QT) void k_q_gradient(const float *sm, int xs, int ys, int xb, int yb, QPart *part) {
    const int f = blockIdx.z;
    const float *b = sm + (long long)f * xs * ys;
    const int rw = xs - 2 * xb, rh = ys - 2 * yb;
    const long long nreg = (rw > 0 && rh > 0) ? (long long)rw * rh : 0;
    double sum = 0.0;
    unsigned long long flagged = 0, above = 0;
    // the grid-stride walk in row-major region order, with (x, y) advanced by
    // the stride's quotient / remainder instead of a 64-bit division per pixel
    const long long step = (long long)gridDim.x * QT;
    long long i = (long long)blockIdx.x * QT + threadIdx.x;
    int cx = rw > 0 ? (int)(i % rw) : 0, cy = rw > 0 ? (int)(i / rw) : 0;
    const int sx = rw > 0 ? (int)(step % rw) : 0, sy = rw > 0 ? (int)(step / rw) : 0;
    for (; i < nreg; i += step, cx += sx, cy += sy) {
        if (cx >= rw) {
            cx -= rw;
            ++cy;
        }
        const int x = xb + cx, y = yb + cy;
        const long long o = (long long)y * xs + x;
        if (b[o] >= THRESHOLD_FLOAT) ++above;
        bool map = false;
        for (int dy = -1; dy <= 1 && !map; ++dy) {
            const int yy = y + dy;
            if (yy < yb || yy >= ys - yb) continue;
            for (int dx = -1; dx <= 1; ++dx) {
                const int xx = x + dx;
                if (xx >= xb && xx < xs - xb && b[(long long)yy * xs + xx] >= THRESHOLD_FLOAT) { map = true; break; }
            }
        }
        if (map) {
            const double d1 = (double)(b[o] - b[o + 1]);
            const double d2 = (double)(b[o] - b[o + xs]);
            sum += (d1 * d1 + d2 * d2);
            ++flagged;
        }
    }
    __shared__ double ss[QT];
    __shared__ unsigned long long sf[QT], sa[QT];
    ss[threadIdx.x] = sum;
    sf[threadIdx.x] = flagged;
    sa[threadIdx.x] = above;
    __syncthreads();
    for (int d = QT / 2; d > 0; d >>= 1) {
        if (threadIdx.x < (unsigned)d) {
            ss[threadIdx.x] += ss[threadIdx.x + d];
            sf[threadIdx.x] += sf[threadIdx.x + d];
            sa[threadIdx.x] += sa[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(size_t)f * gridDim.x + blockIdx.x] = QPart{ss[0], sf[0], sa[0]};
}

// Smooth + gradient in one pass (default; SGPU_QE_SPLIT=1 selects the two
// kernels above): a 64 x 16 tile of the margin region per block, the raw
// subsampled values with a 2-pixel halo in LDS, the 3x3 box of k_q_smooth
// (same expression, same edge rule) for the tile with a 1-pixel halo, then
// k_q_gradient's flags and sums.  One partial per tile.
constexpr int GX = 64, GY = 16;
__global__ __launch_bounds__(QT) void k_q_smooth_gradient(const float *in, int xs, int ys, int xb, int yb,
                                                          QPart *part) {
    __shared__ float raw[GY + 4][GX + 4 + 1];
    __shared__ float smt[GY + 2][GX + 2 + 1];
    // smoothed value >= THRESHOLD_FLOAT inside the margin region: the gradient
    // pass's map test is the OR of the 3 x 3 flags around a pixel (the
    // per-pixel loop over the neighbours with its bounds tests and early exit
    // was the kernel's cost)
    __shared__ unsigned char flg[GY + 2][GX + 2 + 2];
    const int f = blockIdx.z;
    const float *b = in + (long long)f * xs * ys;
    const int rw = xs - 2 * xb, rh = ys - 2 * yb;
    const int X0 = xb + blockIdx.x * GX, Y0 = yb + blockIdx.y * GY;
    for (int k = threadIdx.x; k < (GY + 4) * (GX + 4); k += QT) {
        const int r = k / (GX + 4), cc = k - r * (GX + 4);
        const int x = X0 - 2 + cc, y = Y0 - 2 + r;
        raw[r][cc] = (x >= 0 && x < xs && y >= 0 && y < ys) ? b[(long long)y * xs + x] : 0.f;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < (GY + 2) * (GX + 2); k += QT) {
        const int r = k / (GX + 2), cc = k - r * (GX + 2);
        const int x = X0 - 1 + cc, y = Y0 - 1 + r;
        float v = raw[r + 1][cc + 1];
        if (y >= 1 && y < ys - 1 && x >= 1 && x < xs - 1) {
            const float *p = raw[r], *c = raw[r + 1], *n = raw[r + 2];
            const float t = (p[cc] + p[cc + 1]) + (p[cc + 2] + c[cc]) + (c[cc + 1] + c[cc + 2]) + (n[cc] + n[cc + 1]) +
                            n[cc + 2];
            v = t * (1.f / 9.f);
        }
        smt[r][cc] = v;
        flg[r][cc] = (v >= THRESHOLD_FLOAT && y >= yb && y < ys - yb && x >= xb && x < xs - xb) ? 1 : 0;
    }
    __syncthreads();
    double sum = 0.0;
    unsigned long long flagged = 0, above = 0;
    for (int k = threadIdx.x; k < GX * GY; k += QT) {
        const int r = k / GX, cc = k - r * GX;
        if ((int)blockIdx.x * GX + cc >= rw || (int)blockIdx.y * GY + r >= rh) continue;
        const float s0 = smt[r + 1][cc + 1];
        if (s0 >= THRESHOLD_FLOAT) ++above;
        const bool map = ((flg[r][cc] | flg[r][cc + 1]) | (flg[r][cc + 2] | flg[r + 1][cc])) |
                         ((flg[r + 1][cc + 1] | flg[r + 1][cc + 2]) | (flg[r + 2][cc] | flg[r + 2][cc + 1])) |
                         flg[r + 2][cc + 2];
        if (map) {
            const double d1 = (double)(s0 - smt[r + 1][cc + 2]);
            const double d2 = (double)(s0 - smt[r + 2][cc + 1]);
            sum += (d1 * d1 + d2 * d2);
            ++flagged;
        }
    }
    __shared__ double ss[QT];
    __shared__ unsigned long long sf[QT], sa[QT];
    ss[threadIdx.x] = sum;
    sf[threadIdx.x] = flagged;
    sa[threadIdx.x] = above;
    __syncthreads();
    for (int d = QT / 2; d > 0; d >>= 1) {
        if (threadIdx.x < (unsigned)d) {
            ss[threadIdx.x] += ss[threadIdx.x + d];
            sf[threadIdx.x] += sf[threadIdx.x + d];
            sa[threadIdx.x] += sa[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        part[((size_t)f * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = QPart{ss[0], sf[0], sa[0]};
}

// ------------------------------------------------------------------ 16-bit
// QualityEstimate_ushort (algos/quality.c:49-175): WORD subsample rounded
// with round_to_WORD, a histogram stretch by 60000 / max where max is the
// mean of the last three entries of the reference's running top-6 list over
// the interior rows, integer 3x3 smoothing, THRESHOLD_USHRT, and an exact
// integer gradient sum.
constexpr int THRESHOLD_USHRT = 10240;   // algos/quality.h:30

__global__ __launch_bounds__(QT) void k_q16_subsample(const uint16_t *frames, long long row_stride,
                                                      long long frame_stride, int s, int xs, int ys, uint16_t *buf) {
    const int f = blockIdx.z;
    const long long i = (long long)blockIdx.x * QT + threadIdx.x;
    if (i >= (long long)xs * ys) return;
    const int x = (int)(i % xs), y = (int)(i / xs);
    const uint16_t *p = frames + (long long)f * frame_stride + (long long)(y * s) * row_stride + (long long)x * s;
    int v = 0;
    for (int r = 0; r < s; ++r) {
        for (int c = 0; c < s; ++c) v += p[c];
        p += row_stride;
    }
    double t = (double)v / (double)(s * s) + 0.5;        // round_to_WORD (core/proto.h:232-237)
    t = (t > 65535.0) ? 65535.0 : t;
    t = (t < 0.0) ? 0.0 : t;
    buf[(long long)f * xs * ys + i] = (uint16_t)t;
}

// The running top list is order dependent (a value enters only above the
// current third entry), so it is replayed in scan order by one wave per
// frame: each 64-sample chunk is filtered with a ballot against the current
// third entry (almost always empty past the first rows) and the survivors
// are inserted one by one in lane order.  Output: the stretch divisor.
__global__ __launch_bounds__(64) void k_q16_maxp(const uint16_t *buf, int xs, int ys, int *maxv) {
    const int f = blockIdx.x;
    const uint16_t *b = buf + (long long)f * xs * ys;
    int m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;   // wave-uniform
    const long long beg = (long long)xs, end = (long long)xs * (ys - 1);   // rows 1 .. ys-2
    for (long long base = beg; base < end; base += 64) {
        const long long i = base + threadIdx.x;
        const int v = (i < end) ? (int)b[i] : 0;
        unsigned long long cand = __ballot(v > m2 && v < 65530);
        while (cand) {
            const int lane = __ffsll((long long)cand) - 1;
            cand &= cand - 1;
            const int w = __shfl(v, lane, 64);
            if (w > m2) {                                  // the list may have moved within the chunk
                if (w > m0) { m5 = m4; m4 = m3; m3 = m2; m2 = m1; m1 = m0; m0 = w; }
                else if (w > m1) { m5 = m4; m4 = m3; m3 = m2; m2 = m1; m1 = w; }
                else { m5 = m4; m4 = m3; m3 = m2; m2 = w; }
            }
        }
    }
    if (threadIdx.x == 0) maxv[f] = (m3 + m4 + m5) / 3;
}

__device__ __forceinline__ int q16_stretch(int v, int mx) {
    if (mx <= 0) return v;
    const double mult = 60000.0 / (double)mx;
    unsigned int u = (unsigned int)((double)v * mult);
    return (int)(u > 65535u ? 65535u : u);
}

// _smooth_image_16 (:250-276) on the stretched values: every output reads the
// unsmoothed neighbours (line buffers); edges keep the stretched value
__global__ __launch_bounds__(QT) void k_q16_smooth(const uint16_t *in, int xs, int ys, const int *maxv,
                                                   uint16_t *out) {
    const int f = blockIdx.z;
    const long long i = (long long)blockIdx.x * QT + threadIdx.x;
    if (i >= (long long)xs * ys) return;
    const int x = (int)(i % xs), y = (int)(i / xs);
    const uint16_t *b = in + (long long)f * xs * ys;
    const int mx = maxv[f];
    int r = q16_stretch(b[i], mx);
    if (y >= 1 && y < ys - 1 && x >= 1 && x < xs - 1) {
        unsigned int v = 0;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) v += (unsigned int)q16_stretch(b[(long long)(y + dy) * xs + x + dx], mx);
        r = (int)(v / 9u);
    }
    out[(long long)f * xs * ys + i] = (uint16_t)r;
}

struct QPart16 {
    unsigned long long sum, flagged, above;
};

__global__ __launch_bounds__(QT) void k_q16_gradient(const uint16_t *sm, int xs, int ys, int xb, int yb,
                                                     QPart16 *part) {
    const int f = blockIdx.z;
    const uint16_t *b = sm + (long long)f * xs * ys;
    const int rw = xs - 2 * xb, rh = ys - 2 * yb;
    const long long nreg = (rw > 0 && rh > 0) ? (long long)rw * rh : 0;
    unsigned long long sum = 0, flagged = 0, above = 0;
    // the grid-stride walk in row-major region order, with (x, y) advanced by
    // the stride's quotient / remainder instead of a 64-bit division per pixel
    const long long step = (long long)gridDim.x * QT;
    long long i = (long long)blockIdx.x * QT + threadIdx.x;
    int cx = rw > 0 ? (int)(i % rw) : 0, cy = rw > 0 ? (int)(i / rw) : 0;
    const int sx = rw > 0 ? (int)(step % rw) : 0, sy = rw > 0 ? (int)(step / rw) : 0;
    for (; i < nreg; i += step, cx += sx, cy += sy) {
        if (cx >= rw) {
            cx -= rw;
            ++cy;
        }
        const int x = xb + cx, y = yb + cy;
        const long long o = (long long)y * xs + x;
        if (b[o] >= THRESHOLD_USHRT) ++above;
        bool map = false;
        for (int dy = -1; dy <= 1 && !map; ++dy) {
            const int yy = y + dy;
            if (yy < yb || yy >= ys - yb) continue;
            for (int dx = -1; dx <= 1; ++dx) {
                const int xx = x + dx;
                if (xx >= xb && xx < xs - xb && b[(long long)yy * xs + xx] >= THRESHOLD_USHRT) { map = true; break; }
            }
        }
        if (map) {
            const long long d1 = (long long)b[o] - (long long)b[o + 1];
            const long long d2 = (long long)b[o] - (long long)b[o + xs];
            sum += (unsigned long long)(d1 * d1 + d2 * d2);
            ++flagged;
        }
    }
    __shared__ unsigned long long ss[QT], sf[QT], sa[QT];
    ss[threadIdx.x] = sum;
    sf[threadIdx.x] = flagged;
    sa[threadIdx.x] = above;
    __syncthreads();
    for (int d = QT / 2; d > 0; d >>= 1) {
        if (threadIdx.x < (unsigned)d) {
            ss[threadIdx.x] += ss[threadIdx.x + d];
            sf[threadIdx.x] += sf[threadIdx.x + d];
            sa[threadIdx.x] += sa[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(size_t)f * gridDim.x + blockIdx.x] = QPart16{ss[0], sf[0], sa[0]};
}

}  // namespace qe
}  // namespace sgpu

using namespace sgpu::qe;

extern "C" int sgpu_quality_estimate_device(sgpu_context *c, const float *d_frames, int nframes, int width,
                                            int height, long row_stride, long frame_stride, double *quality) {
    if (!c || !d_frames || nframes <= 0 || width <= 0 || height <= 0 || row_stride < width || !quality ||
        (nframes > 1 && frame_stride < row_stride * (long)height))
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_quality_estimate_device: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const int region_w = width - 1, region_h = height - 1;   // quality_float.c:54-55
    // the levels QualityEstimate_float visits (:66-75, :131-134)
    Levels L = {};
    for (int subsample = QSUBSAMPLE_MIN; subsample <= QSUBSAMPLE_MAX;) {
        const int xs = region_w / subsample, ys = region_h / subsample;
        if (xs < 2 || ys < 2) break;
        L.s[L.n] = subsample;
        L.xs[L.n] = xs;
        L.ys[L.n] = ys;
        L.n++;
        do {
            subsample += QSUBSAMPLE_INC;
        } while (width / subsample == xs && height / subsample == ys);
    }
    std::vector<double> dval((size_t)nframes, 0.0);
    const int nblk_g = 64;
    const char *qs = std::getenv("SGPU_QE_SPLIT");     // "1": separate smooth + gradient kernels (A/B knob)
    const bool split = qs && qs[0] == '1';
    if (L.n > 0) {
        size_t off[3], tot = 0, poff[4] = {0, 0, 0, 0};
        unsigned gx[3], gy[3];
        for (int l = 0; l < L.n; ++l) {
            off[l] = tot;
            tot += (size_t)L.xs[l] * L.ys[l] * nframes;
            const int yb = (int)((double)L.ys[l] * QMARGIN) + 1, xb = (int)((double)L.xs[l] * QMARGIN) + 1;
            const int rw = L.xs[l] - 2 * xb, rh = L.ys[l] - 2 * yb;
            gx[l] = split ? nblk_g : (unsigned)std::max(1, (rw + GX - 1) / GX);
            gy[l] = split ? 1 : (unsigned)std::max(1, (rh + GY - 1) / GY);
            poff[l + 1] = poff[l] + (size_t)gx[l] * gy[l] * nframes;
        }
        const size_t big = (size_t)L.xs[0] * L.ys[0] * nframes;
        int rc;
        if ((rc = c->qe_buf.ensure((tot + big) * sizeof(float))) ||
            (rc = c->qe_part.ensure(sizeof(QPart) * poff[L.n])))
            return rc;
        float *base = (float *)c->qe_buf.p, *sm = base + tot;
        for (int l = 0; l < L.n; ++l) L.buf[l] = base + off[l];
        const char *fz = std::getenv("SGPU_QE_FUSED");   // "0": one pass per level (A/B knob)
        if (!(fz && fz[0] == '0')) {
            const dim3 tg((unsigned)((width + TC - 1) / TC), (unsigned)((height + TR - 1) / TR), (unsigned)nframes);
            const char *qv = std::getenv("SGPU_QE_VEC");     // "0": scalar loads (A/B knob)
            const bool vec = !(qv && qv[0] == '0') && ((uintptr_t)d_frames % 16 == 0) && row_stride % 4 == 0 &&
                             (nframes == 1 || frame_stride % 4 == 0) && width % 4 == 0;
            if (vec)
                hipLaunchKernelGGL(k_q_subsample_all<true>, tg, dim3(QT), 0, c->stream, d_frames,
                                   (long long)row_stride, (long long)frame_stride, width, height, L);
            else
                hipLaunchKernelGGL(k_q_subsample_all<false>, tg, dim3(QT), 0, c->stream, d_frames,
                                   (long long)row_stride, (long long)frame_stride, width, height, L);
        } else {
            for (int l = 0; l < L.n; ++l) {
                const long long n = (long long)L.xs[l] * L.ys[l];
                const dim3 g((unsigned)((n + QT - 1) / QT), 1, (unsigned)nframes);
                hipLaunchKernelGGL(k_q_subsample, g, dim3(QT), 0, c->stream, d_frames, (long long)row_stride,
                                   (long long)frame_stride, L.s[l], L.xs[l], L.ys[l], L.buf[l]);
            }
        }
        for (int l = 0; l < L.n; ++l) {
            const int xs = L.xs[l], ys = L.ys[l];
            const int yb = (int)((double)ys * QMARGIN) + 1, xb = (int)((double)xs * QMARGIN) + 1;
            QPart *pl = (QPart *)c->qe_part.p + poff[l];
            if (split) {
                const long long n = (long long)xs * ys;
                const dim3 g((unsigned)((n + QT - 1) / QT), 1, (unsigned)nframes);
                hipLaunchKernelGGL(k_q_smooth, g, dim3(QT), 0, c->stream, L.buf[l], xs, ys, sm);
                hipLaunchKernelGGL(k_q_gradient, dim3(nblk_g, 1, nframes), dim3(QT), 0, c->stream, sm, xs, ys, xb,
                                   yb, pl);
            } else {
                hipLaunchKernelGGL(k_q_smooth_gradient, dim3(gx[l], gy[l], nframes), dim3(QT), 0, c->stream,
                                   L.buf[l], xs, ys, xb, yb, pl);
            }
        }
        HIP_TRY(hipGetLastError());
        std::vector<QPart> hp(poff[L.n]);
        HIP_TRY(hipMemcpyAsync(hp.data(), c->qe_part.p, hp.size() * sizeof(QPart), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (int l = 0; l < L.n; ++l) {
            for (int f = 0; f < nframes; ++f) {
                double sum = 0.0;
                unsigned long long fl = 0, ab = 0;
                const size_t nb = (size_t)gx[l] * gy[l];
                for (size_t b = 0; b < nb; ++b) {
                    const QPart &p = hp[poff[l] + (size_t)f * nb + b];
                    sum += p.sum;
                    fl += p.flagged;
                    ab += p.above;
                }
                // Gradient: -1 without significant pixels (:187-190, :205-209)
                const double q = (ab == 0 || fl == 0) ? -1.0 : sum / (double)fl / 10.0;
                dval[(size_t)f] += (q * ((double)(QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (L.s[l] * L.s[l])));
            }
        }
    }
    for (int f = 0; f < nframes; ++f) quality[f] = std::sqrt(dval[(size_t)f]);
    return SGPU_OK;
}

extern "C" int sgpu_quality_estimate(sgpu_context *c, const float *frames, int nframes, int width, int height,
                                     double *quality) {
    if (!c || !frames || nframes <= 0 || width <= 0 || height <= 0 || !quality)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_quality_estimate: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t fbytes = sizeof(float) * (size_t)width * height;
    int rc;
    if ((rc = c->qe_io.ensure(fbytes * nframes))) return rc;
    HIP_TRY(hipMemcpyAsync(c->qe_io.p, frames, fbytes * nframes, hipMemcpyHostToDevice, c->stream));
    return sgpu_quality_estimate_device(c, (const float *)c->qe_io.p, nframes, width, height, width,
                                        (long)width * height, quality);
}

// normalizeQualityData (registration/shift_methods.c:36-54): quality in place
// over the sequence, q_min / q_max as register_shift_dft tracked them.
extern "C" void sgpu_normalize_quality(double *quality, int n, double q_min, double q_max) {
    double diff = q_max - q_min;
    if (diff == 0) {
        q_min = 0;
        diff = (q_max == 0.) ? 1. : q_max;
    }
    for (int i = 0; i < n; ++i) {
        quality[i] -= q_min;
        quality[i] /= diff;
        if (quality[i] < 0 || std::isnan(quality[i])) quality[i] = -1.0;
    }
}

// QualityEstimate_ushort for DATA_USHORT frames (QualityEstimate dispatches on
// the fit type, algos/quality.c:39-45).  The gradient sums are exact integers
// (the reference's double sum equals them whenever it is itself exact).
extern "C" int sgpu_quality_estimate_u16_device(sgpu_context *c, const uint16_t *d_frames, int nframes, int width,
                                                int height, long row_stride, long frame_stride, double *quality) {
    if (!c || !d_frames || nframes <= 0 || width <= 0 || height <= 0 || row_stride < width || !quality ||
        (nframes > 1 && frame_stride < row_stride * (long)height))
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_quality_estimate_u16_device: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const int region_w = width - 1, region_h = height - 1;   // quality.c:61-64
    std::vector<double> dval((size_t)nframes, 0.0);
    const int nblk_g = 64;
    for (int subsample = QSUBSAMPLE_MIN; subsample <= QSUBSAMPLE_MAX;) {
        const int xs = region_w / subsample, ys = region_h / subsample;
        if (xs < 2 || ys < 2) break;
        const long long n = (long long)xs * ys;
        int rc;
        const size_t bytes = 2 * (size_t)n * nframes * sizeof(uint16_t);
        if ((rc = c->qe_buf.ensure(bytes + (size_t)nframes * sizeof(int))) ||
            (rc = c->qe_part.ensure(sizeof(QPart16) * nblk_g * nframes)))
            return rc;
        uint16_t *buf = (uint16_t *)c->qe_buf.p, *sm = buf + n * nframes;
        int *maxv = (int *)((char *)c->qe_buf.p + bytes);
        const dim3 g((unsigned)((n + QT - 1) / QT), 1, (unsigned)nframes);
        hipLaunchKernelGGL(k_q16_subsample, g, dim3(QT), 0, c->stream, d_frames, (long long)row_stride,
                           (long long)frame_stride, subsample, xs, ys, buf);
        hipLaunchKernelGGL(k_q16_maxp, dim3((unsigned)nframes), dim3(64), 0, c->stream, buf, xs, ys, maxv);
        hipLaunchKernelGGL(k_q16_smooth, g, dim3(QT), 0, c->stream, buf, xs, ys, maxv, sm);
        const int yb = (int)((double)ys * QMARGIN) + 1, xb = (int)((double)xs * QMARGIN) + 1;
        hipLaunchKernelGGL(k_q16_gradient, dim3(nblk_g, 1, nframes), dim3(QT), 0, c->stream, sm, xs, ys, xb, yb,
                           (QPart16 *)c->qe_part.p);
        HIP_TRY(hipGetLastError());
        std::vector<QPart16> hp((size_t)nblk_g * nframes);
        HIP_TRY(hipMemcpyAsync(hp.data(), c->qe_part.p, hp.size() * sizeof(QPart16), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (int f = 0; f < nframes; ++f) {
            unsigned long long sum = 0, fl = 0, ab = 0;
            for (int b = 0; b < nblk_g; ++b) {
                const QPart16 &p = hp[(size_t)f * nblk_g + b];
                sum += p.sum;
                fl += p.flagged;
                ab += p.above;
            }
            // Gradient: -1 without significant pixels (:216-219, :232-236)
            const double q = (ab == 0 || fl == 0) ? -1.0 : (double)sum / (double)fl / 10.0;
            dval[(size_t)f] += (q * ((double)(QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (subsample * subsample)));
        }
        do {
            subsample += QSUBSAMPLE_INC;
        } while (width / subsample == xs && height / subsample == ys);
    }
    for (int f = 0; f < nframes; ++f) quality[f] = std::sqrt(dval[(size_t)f]);
    return SGPU_OK;
}

extern "C" int sgpu_quality_estimate_u16(sgpu_context *c, const uint16_t *frames, int nframes, int width, int height,
                                         double *quality) {
    if (!c || !frames || nframes <= 0 || width <= 0 || height <= 0 || !quality)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_quality_estimate_u16: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t fbytes = sizeof(uint16_t) * (size_t)width * height;
    int rc;
    if ((rc = c->qe_io.ensure(fbytes * nframes))) return rc;
    HIP_TRY(hipMemcpyAsync(c->qe_io.p, frames, fbytes * nframes, hipMemcpyHostToDevice, c->stream));
    return sgpu_quality_estimate_u16_device(c, (const uint16_t *)c->qe_io.p, nframes, width, height, width,
                                            (long)width * height, quality);
}
