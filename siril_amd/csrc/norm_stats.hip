// norm_stats.hip -- per-frame normalization estimators for stacking
// (SURVEY.md §8f rank 1), DATA_FLOAT planes resident in HBM.
//
// Reference: compute_normalization -> _compute_estimators_for_image
// (stacking/normalization.c:107-146, 249-294) -> statistics_internal_float
// with STATS_NORM / STATS_LITENORM (algos/statistics_float.c:281-480):
//   data     = samples != 0 and not NaN            (:231-252)
//   median   = histogram_median_float(data)        (sorting.c:644-649 ->
//              rt/rt_algo.cc:38-172, 65536-bin histogram, float interpolation)
//   mad      = same percentile of |x - (float)median|     (:79-101)
//   IKSSlite = filter to [median -/+ 6 mad] (double, stored float), its
//              median, its MAD, sqrt(bwmv)*0.991              (:199-229, :103-127)
// and compute_factors_from_estimators (normalization.c:150-185).
//
// Every frame of a batch is processed by the same launches (grid.y = frame).
// A stage is one streaming pass over the frame (HBM-bound):
//   k_minmax<M>  count, min, max of the stage's values (one atomic per block)
//   k_hist<M>    65536-bin histogram, LDS-private as packed u16 pairs
//                (128 KB; a block covers < 65536 samples so no u16 overflows),
//                non-empty bin pairs flushed with 64-bit global atomics
//   k_select     one block per frame: prefix scan of the histogram, the
//                reference's float interpolation, next stage's parameters,
//                histogram and min/max reset for the next stage
//   k_bwmv       per-block f64 partials in a fixed order, k_bwmv_final sums
//                them in a fixed order (deterministic run to run)
// Stage values: M=0 x; M=1 |x - median|; M=2 x in [lo,hi]; M=3 |x - loc| in [lo,hi].
// DATA_USHORT (statistics_internal_ushort, algos/statistics.c:231-449):
// stages 0/1 are exact integer histograms (k_hist16 / k_select16:
// histogram_median and siril_stats_ushort_mad are order statistics), the
// IKSS stages run on (float)x * (float)(1/65535.0) converted on load.
// No host round trip between stages: each kernel reads the previous stage's
// results from the per-frame state in device memory.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "sgpu_internal.h"

namespace sgpu {
namespace ns {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int HB = 65536;          // histoSize cap, rt_algo.cc:82
constexpr int HIST_THREADS = 1024;
// samples per histogram block.  A packed u16 counter overflows only if more
// than 65535 samples of one block land in one bin: every add checks the old
// counter, and a block that saw a wrap redoes its chunk with direct global
// atomics (exact; only degenerate, near-constant frames take that path).
constexpr int HIST_PER_BLOCK = 4 * 63 * HIST_THREADS;
constexpr int RED_THREADS = 256;

struct FrameState {
    unsigned long long cnt;        // stage sample count
    unsigned int mn, mx;           // ordered-int encoded min / max of the stage's values
    unsigned long long ngood;      // non-zero, non-NaN samples
    unsigned long long kept;       // IKSS samples
    float median, mad, loc, mad2;  // stage results
    float lo, hi;                  // IKSS bounds
    double scale;
    double dmedian;                // DATA_USHORT: histogram_median (integer order statistics)
    float mad16;                   // DATA_USHORT: siril_stats_ushort_mad
    int medi;                      // round_to_int(dmedian)
    int status;                    // 0 ok, 1 = reference returns NULL stats
    int pad;
};

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
// statistics.c:421-426: newdata[i] = (float)data[i] * (float)(1.0 / USHRT_MAX_DOUBLE)
constexpr float INV_U16 = (float)(1.0 / 65535.0);

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(unsigned short u) { return (float)u * INV_U16; }

// 16-byte (float) / 8-byte (u16) vector of 4 samples
template <typename T> struct Vec4;
template <> struct Vec4<float> { typedef f4v type; };
template <> struct Vec4<unsigned short> { typedef u16x4 type; };

__device__ __forceinline__ unsigned f2o(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(unsigned o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

template <int M>
__device__ __forceinline__ bool stage_value(float x, const FrameState &s, float &v) {
    bool ok = (x != 0.f) && !isnan(x);
    if (M >= 2) ok = ok && (x >= s.lo) && (x <= s.hi);
    if (M == 1) v = fabsf(x - s.median);
    else if (M == 3) v = fabsf(x - s.loc);
    else v = x;
    return ok;
}

__global__ __launch_bounds__(64) void k_init(FrameState *st, int nframes) {
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= nframes) return;
    FrameState s = {};
    s.mn = 0xffffffffu;
    s.mx = 0u;
    st[f] = s;
}

template <int M, typename T>
__global__ __launch_bounds__(RED_THREADS) void k_minmax(const T *frames, long long stride, long long npix,
                                                        FrameState *st, int vec) {
    const int f = blockIdx.y;
    FrameState s = st[f];
    if (s.status) return;
    const T *x = frames + (long long)f * stride;
    unsigned long long cnt = 0;
    unsigned mn = 0xffffffffu, mx = 0u;
    auto take = [&](T xr) {
        float v;
        if (stage_value<M>(to_f(xr), s, v)) {
            ++cnt;
            const unsigned o = f2o(v);
            mn = min(mn, o);
            mx = max(mx, o);
        }
    };
    const long long tid = (long long)blockIdx.x * RED_THREADS + threadIdx.x;
    const long long nth = (long long)gridDim.x * RED_THREADS;
    if (vec) {   // 4-sample loads: frames aligned, npix and stride multiples of 4
        typedef typename Vec4<T>::type V;
        const V *x4 = reinterpret_cast<const V *>(x);
        for (long long i = tid; i < npix / 4; i += nth) {
            const V q = __builtin_nontemporal_load(x4 + i);
            take(q.x); take(q.y); take(q.z); take(q.w);
        }
    } else {
        for (long long i = tid; i < npix; i += nth) take(__builtin_nontemporal_load(x + i));
    }
    for (int d = 32; d > 0; d >>= 1) {
        cnt += __shfl_xor(cnt, d);
        mn = min(mn, (unsigned)__shfl_xor((int)mn, d));
        mx = max(mx, (unsigned)__shfl_xor((int)mx, d));
    }
    __shared__ unsigned long long sc[RED_THREADS / 64];
    __shared__ unsigned smn[RED_THREADS / 64], smx[RED_THREADS / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sc[w] = cnt; smn[w] = mn; smx[w] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < RED_THREADS / 64; ++k) { cnt += sc[k]; mn = min(mn, smn[k]); mx = max(mx, smx[k]); }
        if (cnt) {
            atomicAdd(&st[f].cnt, cnt);
            atomicMin(&st[f].mn, mn);
            atomicMax(&st[f].mx, mx);
        }
    }
}

template <int M, typename T>
__global__ __launch_bounds__(HIST_THREADS) void k_hist(const T *frames, long long stride, long long npix,
                                                       const FrameState *st, unsigned *hist, int vec) {
    const int f = blockIdx.y;
    const FrameState s = st[f];
    if (s.status || s.cnt == 0) return;
    const float lo = o2f(s.mn), hi = o2f(s.mx);
    if (fabsf(hi - lo) == 0.f) return;   // rt_algo.cc:74-77 fast exit, no histogram
    const long long i0 = (long long)blockIdx.x * HIST_PER_BLOCK;
    if (i0 >= npix) return;
    const unsigned hs = s.cnt < (unsigned long long)HB ? (unsigned)s.cnt : (unsigned)HB;
    const float scale = (float)(hs - 1) / (hi - lo);   // rt_algo.cc:84
    __shared__ unsigned h2[HB / 2];
    for (int k = threadIdx.x; k < HB / 2; k += HIST_THREADS) h2[k] = 0u;
    __syncthreads();
    const T *x = frames + (long long)f * stride;
    const long long i1 = min(npix, i0 + HIST_PER_BLOCK);
    bool ovf = false;
    // static_cast<uint16_t>(float) as the x86-64 build does it:
    // 32-bit truncation, low 16 bits (rt_algo.cc:94)
    auto bin = [&](float v) { return (unsigned)(int)(scale * (v - lo)) & 0xffffu; };
    auto put = [&](T xr) {
        float v;
        if (stage_value<M>(to_f(xr), s, v)) {
            const unsigned b = bin(v), sh = (b & 1u) * 16;
            const unsigned old = atomicAdd(&h2[b >> 1], 1u << sh);
            ovf |= ((old >> sh) & 0xffffu) == 0xffffu;
        }
    };
    if (vec) {   // HIST_PER_BLOCK is a multiple of 4
        typedef typename Vec4<T>::type V;
        const V *x4 = reinterpret_cast<const V *>(x);
        for (long long i = i0 / 4 + threadIdx.x; i < i1 / 4; i += HIST_THREADS) {
            const V q = __builtin_nontemporal_load(x4 + i);
            put(q.x); put(q.y); put(q.z); put(q.w);
        }
    } else {
        for (long long i = i0 + threadIdx.x; i < i1; i += HIST_THREADS) put(__builtin_nontemporal_load(x + i));
    }
    if (__syncthreads_or(ovf)) {   // a packed counter wrapped: exact slow path for this chunk
        unsigned *g = hist + (size_t)f * HB;
        for (long long i = i0 + threadIdx.x; i < i1; i += HIST_THREADS) {
            float v;
            if (stage_value<M>(to_f(x[i]), s, v)) atomicAdd(&g[bin(v)], 1u);
        }
        return;
    }
    // one 64-bit atomic per bin pair: bins 2k, 2k+1 are the low and high
    // words of g2[k] (a bin total stays far below 2^32, so no carry crosses)
    unsigned long long *g2 = reinterpret_cast<unsigned long long *>(hist + (size_t)f * HB);
    for (int k = threadIdx.x; k < HB / 2; k += HIST_THREADS) {
        const unsigned v = h2[k];
        if (v) atomicAdd(&g2[k], ((unsigned long long)(v >> 16) << 32) | (v & 0xffffu));
    }
}

// One block per frame.  `stage` selects where the percentile goes and what
// the next stage needs.  Clears the histogram and the min/max/count.
__global__ __launch_bounds__(1024) void k_select(FrameState *st, unsigned *hist, int stage) {
    const int f = blockIdx.x;
    FrameState s = st[f];
    unsigned *h = hist + (size_t)f * HB;
    constexpr int PER = HB / 1024;
    __shared__ unsigned long long part[1024];
    __shared__ float res;
    if (s.status) return;
    const unsigned long long n = s.cnt;
    const float lo = o2f(s.mn), hi = o2f(s.mx);
    const bool flat = (n == 0) || (fabsf(hi - lo) == 0.f);
    unsigned long long mine = 0;
    if (!flat)
        for (int j = 0; j < PER; ++j) mine += h[threadIdx.x * PER + j];
    part[threadIdx.x] = mine;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {          // inclusive Hillis-Steele scan
        const unsigned long long a = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
        __syncthreads();
        part[threadIdx.x] += a;
        __syncthreads();
    }
    if (threadIdx.x == 0) res = lo;
    __syncthreads();
    if (!flat) {
        const unsigned hs = n < (unsigned long long)HB ? (unsigned)n : (unsigned)HB;
        const float scale = (float)(hs - 1) / (hi - lo);
        const float thr = 0.5f * (float)n;             // rt_algo.cc:137
        unsigned long long count = part[threadIdx.x] - mine;   // prefix before my bins
        // k is one past the first bin whose inclusive prefix, as float, reaches thr
        if ((float)count < thr && (float)part[threadIdx.x] >= thr) {
            for (int j = 0; j < PER; ++j) {
                if ((float)count < thr) {
                    const unsigned hj = h[threadIdx.x * PER + j];
                    count += hj;
                    if ((float)count >= thr) {
                        const unsigned long long k = (unsigned long long)threadIdx.x * PER + j + 1;
                        const unsigned long long count_ = count - hj;
                        const float c0 = (float)count - thr;
                        const float c1 = thr - (float)count_;
                        float out = ((c1 * (float)k) + (c0 * (float)(k - 1))) / (c0 + c1);
                        out /= scale;
                        out += lo;
                        const float m = (hi < out) ? hi : out;   // rtengine::LIM
                        res = (m < lo) ? lo : m;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (!flat)
        for (int j = 0; j < PER; ++j) h[threadIdx.x * PER + j] = 0u;
    if (threadIdx.x == 0) {
        const float r = res;
        FrameState &o = st[f];
        o.cnt = 0;
        o.mn = 0xffffffffu;
        o.mx = 0u;
        if (n == 0) { o.status = 1; return; }   // no good pixel / IKSS kept == 0
        if (stage == 0) { o.median = r; o.ngood = n; }
        else if (stage == 1) {
            o.mad = r;
            // IKSSlite: xlow = median - 6.0 * mad evaluated in double (statistics_float.c:203-204)
            o.lo = (float)((double)s.median - 6.0 * (double)r);
            o.hi = (float)((double)s.median + 6.0 * (double)r);
        } else if (stage == 2) { o.loc = r; o.kept = n; }
        else {
            o.mad2 = r;
            if (r == 0.0f) o.status = 1;       // "MAD is null" (statistics_float.c:217-220)
        }
    }
}


// DATA_USHORT stages 0/1 (statistics.c:356-388): exact 65536-value histogram
// of the samples > 0 (M=0) or of |x - round_to_int(median)| (M=1); counts
// the samples too.  Same LDS layout / flush as k_hist.
template <int M>
__global__ __launch_bounds__(HIST_THREADS) void k_hist16(const unsigned short *frames, long long stride,
                                                         long long npix, FrameState *st, unsigned *hist, int vec) {
    const int f = blockIdx.y;
    const FrameState s = st[f];
    if (s.status) return;
    const long long i0 = (long long)blockIdx.x * HIST_PER_BLOCK;
    if (i0 >= npix) return;
    __shared__ unsigned h2[HB / 2];
    __shared__ unsigned long long wc[HIST_THREADS / 64];
    for (int k = threadIdx.x; k < HB / 2; k += HIST_THREADS) h2[k] = 0u;
    __syncthreads();
    const unsigned short *x = frames + (long long)f * stride;
    const long long i1 = min(npix, i0 + HIST_PER_BLOCK);
    unsigned cnt = 0;
    bool ovf = false;
    auto bin = [&](unsigned short u) {
        return (M == 0) ? (unsigned)u : (unsigned)(unsigned short)abs((int)u - s.medi);
    };
    auto put = [&](unsigned short u) {
        if (u > 0) {
            const unsigned b = bin(u), sh = (b & 1u) * 16;
            ++cnt;
            const unsigned old = atomicAdd(&h2[b >> 1], 1u << sh);
            ovf |= ((old >> sh) & 0xffffu) == 0xffffu;
        }
    };
    if (vec) {
        const u16x4 *x4 = reinterpret_cast<const u16x4 *>(x);
        for (long long i = i0 / 4 + threadIdx.x; i < i1 / 4; i += HIST_THREADS) {
            const u16x4 q = __builtin_nontemporal_load(x4 + i);
            put(q.x); put(q.y); put(q.z); put(q.w);
        }
    } else {
        for (long long i = i0 + threadIdx.x; i < i1; i += HIST_THREADS) put(__builtin_nontemporal_load(x + i));
    }
    unsigned long long c = cnt;
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < HIST_THREADS / 64; ++k) t += wc[k];
        if (t) atomicAdd(&st[f].cnt, t);
    }
    if (__syncthreads_or(ovf)) {   // a packed counter wrapped: exact slow path for this chunk
        unsigned *g = hist + (size_t)f * HB;
        for (long long i = i0 + threadIdx.x; i < i1; i += HIST_THREADS) {
            const unsigned short u = x[i];
            if (u > 0) atomicAdd(&g[bin(u)], 1u);
        }
        return;
    }
    unsigned long long *g2 = reinterpret_cast<unsigned long long *>(hist + (size_t)f * HB);
    for (int k = threadIdx.x; k < HB / 2; k += HIST_THREADS) {
        const unsigned v = h2[k];
        if (v) atomicAdd(&g2[k], ((unsigned long long)(v >> 16) << 32) | (v & 0xffffu));
    }
}

// histogram_median (sorting.c:575-641): exact order statistics a[k-1], a[k]
// (k = n/2) of the counted values; (a[k-1] + a[k]) / 2.0 for even n.
__global__ __launch_bounds__(1024) void k_select16(FrameState *st, unsigned *hist, int stage) {
    const int f = blockIdx.x;
    const FrameState s = st[f];
    unsigned *h = hist + (size_t)f * HB;
    constexpr int PER = HB / 1024;
    __shared__ unsigned long long part[1024];
    __shared__ int v1, v2;
    if (s.status) return;
    const unsigned long long n = s.cnt;
    unsigned long long mine = 0;
    for (int j = 0; j < PER; ++j) mine += h[threadIdx.x * PER + j];
    part[threadIdx.x] = mine;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const unsigned long long a = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
        __syncthreads();
        part[threadIdx.x] += a;
        __syncthreads();
    }
    if (threadIdx.x == 0) { v1 = 0; v2 = 0; }
    __syncthreads();
    const unsigned long long k = n / 2;
    // smallest v with prefix(v) > t, for t = k-1 (even n) and t = k
    const unsigned long long before = part[threadIdx.x] - mine;
    for (int w = 0; w < 2; ++w) {
        if (w == 0 && (n % 2 != 0 || k == 0)) continue;
        const unsigned long long t = (w == 0) ? k - 1 : k;
        if (before <= t && part[threadIdx.x] > t) {
            unsigned long long c = before;
            for (int j = 0; j < PER; ++j) {
                c += h[threadIdx.x * PER + j];
                if (c > t) { if (w == 0) v1 = threadIdx.x * PER + j; else v2 = threadIdx.x * PER + j; break; }
            }
        }
    }
    __syncthreads();
    for (int j = 0; j < PER; ++j) h[threadIdx.x * PER + j] = 0u;
    if (threadIdx.x == 0) {
        FrameState &o = st[f];
        o.cnt = 0;
        if (n == 0) { o.status = 1; return; }
        const double r = (n % 2 == 0) ? (double)(v1 + v2) / 2.0 : (double)v2;
        if (stage == 0) {
            o.dmedian = r;
            o.ngood = n;
            o.medi = (int)(r + 0.5);                       // round_to_int, r >= 0
        } else {
            o.mad16 = (float)r;
            // IKSS inputs scaled to [0,1] (statistics.c:425-429), then IKSSlite's bounds
            const float med = (float)o.dmedian * INV_U16;
            const float mad = o.mad16 * INV_U16;
            o.lo = (float)((double)med - 6.0 * (double)mad);
            o.hi = (float)((double)med + 6.0 * (double)mad);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(RED_THREADS) void k_bwmv(const T *frames, long long stride, long long npix,
                                                      const FrameState *st, double2 *partial, int vec) {
    const int f = blockIdx.y;
    const FrameState s = st[f];
    if (s.status) return;
    const T *x = frames + (long long)f * stride;
    const float median = s.loc, factor = 1.f / (9.f * s.mad2);
    double up = 0.0, down = 0.0;
    auto acc = [&](T xr) {
        const float v = to_f(xr);
        if (v != 0.f && !isnan(v) && v >= s.lo && v <= s.hi) {
            const float i_med = v - median;
            const float yi = i_med * factor;
            const float yi2 = fabsf(yi) < 1.f ? yi * yi : 1.f;
            const float t = (1 - yi2) * (1 - yi2);
            const float u = i_med * t;
            up += (double)(u * u);
            down += (double)((1 - yi2) * (1 - 5 * yi2));
        }
    };
    const long long tid = (long long)blockIdx.x * RED_THREADS + threadIdx.x;
    const long long nth = (long long)gridDim.x * RED_THREADS;
    if (vec) {
        typedef typename Vec4<T>::type V;
        const V *x4 = reinterpret_cast<const V *>(x);
        for (long long i = tid; i < npix / 4; i += nth) {
            const V q = __builtin_nontemporal_load(x4 + i);
            acc(q.x); acc(q.y); acc(q.z); acc(q.w);
        }
    } else {
        for (long long i = tid; i < npix; i += nth) acc(__builtin_nontemporal_load(x + i));
    }
    __shared__ double su[RED_THREADS], sd[RED_THREADS];
    su[threadIdx.x] = up;
    sd[threadIdx.x] = down;
    __syncthreads();
    for (int d = RED_THREADS / 2; d > 0; d >>= 1) {
        if (threadIdx.x < (unsigned)d) {
            su[threadIdx.x] += su[threadIdx.x + d];
            sd[threadIdx.x] += sd[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[(size_t)f * gridDim.x + blockIdx.x] = make_double2(su[0], sd[0]);
}

__global__ __launch_bounds__(RED_THREADS) void k_bwmv_final(FrameState *st, const double2 *partial, int nblk) {
    const int f = blockIdx.x;
    if (st[f].status) return;
    __shared__ double su[RED_THREADS], sd[RED_THREADS];
    double up = 0.0, down = 0.0;
    for (int b = threadIdx.x; b < nblk; b += RED_THREADS) {
        up += partial[(size_t)f * nblk + b].x;
        down += partial[(size_t)f * nblk + b].y;
    }
    su[threadIdx.x] = up;
    sd[threadIdx.x] = down;
    __syncthreads();
    for (int d = RED_THREADS / 2; d > 0; d >>= 1) {
        if (threadIdx.x < (unsigned)d) {
            su[threadIdx.x] += su[threadIdx.x + d];
            sd[threadIdx.x] += sd[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double n = (double)st[f].kept;
        const double dn = sd[0];
        const double bwmv = dn ? n * (su[0] / (dn * dn)) : 0.0;   // statistics_float.c:124
        st[f].scale = sqrt(bwmv) * .991;                          // :225
    }
}

}  // namespace ns
}  // namespace sgpu

using namespace sgpu::ns;

namespace {

template <typename T>
int launch_stats(sgpu_context *c, const T *d_frames, int nframes, long long npix, long long stride, int lite,
                 FrameState *st, unsigned *hist, double2 *partial, int nblk) {
    hipStream_t s = c->stream;
    const int vec = (npix % 4 == 0) && (stride % 4 == 0) && (((uintptr_t)d_frames & (4 * sizeof(T) - 1)) == 0);
    const dim3 rg((unsigned)nblk, (unsigned)nframes);
    const dim3 hg((unsigned)((npix + HIST_PER_BLOCK - 1) / HIST_PER_BLOCK), (unsigned)nframes);
    hipLaunchKernelGGL(k_init, dim3((nframes + 63) / 64), dim3(64), 0, s, st, nframes);
    if constexpr (sizeof(T) == 4) {
        hipLaunchKernelGGL((k_minmax<0, T>), rg, dim3(RED_THREADS), 0, s, d_frames, stride, npix, st, vec);
        hipLaunchKernelGGL((k_hist<0, T>), hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select, dim3(nframes), dim3(1024), 0, s, st, hist, 0);
        hipLaunchKernelGGL((k_minmax<1, T>), rg, dim3(RED_THREADS), 0, s, d_frames, stride, npix, st, vec);
        hipLaunchKernelGGL((k_hist<1, T>), hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select, dim3(nframes), dim3(1024), 0, s, st, hist, 1);
    } else {
        hipLaunchKernelGGL(k_hist16<0>, hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select16, dim3(nframes), dim3(1024), 0, s, st, hist, 0);
        hipLaunchKernelGGL(k_hist16<1>, hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select16, dim3(nframes), dim3(1024), 0, s, st, hist, 1);
    }
    if (!lite) {
        hipLaunchKernelGGL((k_minmax<2, T>), rg, dim3(RED_THREADS), 0, s, d_frames, stride, npix, st, vec);
        hipLaunchKernelGGL((k_hist<2, T>), hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select, dim3(nframes), dim3(1024), 0, s, st, hist, 2);
        hipLaunchKernelGGL((k_minmax<3, T>), rg, dim3(RED_THREADS), 0, s, d_frames, stride, npix, st, vec);
        hipLaunchKernelGGL((k_hist<3, T>), hg, dim3(HIST_THREADS), 0, s, d_frames, stride, npix, st, hist, vec);
        hipLaunchKernelGGL(k_select, dim3(nframes), dim3(1024), 0, s, st, hist, 3);
        hipLaunchKernelGGL(k_bwmv<T>, rg, dim3(RED_THREADS), 0, s, d_frames, stride, npix, st, partial, vec);
        hipLaunchKernelGGL(k_bwmv_final, dim3(nframes), dim3(RED_THREADS), 0, s, st, partial, nblk);
    }
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}

template <typename T>
int norm_stats_device(sgpu_context *c, const T *d_frames, int nframes, long npix, long frame_stride, int lite,
                      double *stats, long *ngood, int *status) {
    HIP_TRY(hipSetDevice(c->device));
    const int nblk = (int)std::min<long long>(512, std::max<long long>(1, npix / (RED_THREADS * 64)));
    const size_t st_bytes = sizeof(FrameState) * (size_t)nframes;
    const size_t hist_bytes = sizeof(unsigned) * (size_t)HB * nframes;
    const size_t part_bytes = sizeof(double2) * (size_t)nblk * nframes;
    int rc;
    if ((rc = c->ns_state.ensure(st_bytes)) || (rc = c->ns_hist.ensure(hist_bytes)) ||
        (rc = c->ns_part.ensure(part_bytes)))
        return rc;
    HIP_TRY(hipMemsetAsync(c->ns_hist.p, 0, hist_bytes, c->stream));
    if ((rc = launch_stats<T>(c, d_frames, nframes, npix, frame_stride, lite, (FrameState *)c->ns_state.p,
                              (unsigned *)c->ns_hist.p, (double2 *)c->ns_part.p, nblk)))
        return rc;
    std::vector<FrameState> h((size_t)nframes);
    HIP_TRY(hipMemcpyAsync(h.data(), c->ns_state.p, st_bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const bool u16 = sizeof(T) == 2;
    const double normValue = u16 ? 65535.0 : 1.0;     // USHRT_MAX_DOUBLE / float images
    for (int f = 0; f < nframes; ++f) {
        const FrameState &s = h[(size_t)f];
        stats[4 * f + 0] = u16 ? s.dmedian : (double)s.median;   // stat->median
        stats[4 * f + 1] = u16 ? (double)s.mad16 : (double)s.mad;  // stat->mad
        stats[4 * f + 2] = lite ? 0.0 : (double)s.loc * normValue;  // stat->location
        stats[4 * f + 3] = lite ? 0.0 : s.scale * normValue;        // stat->scale
        if (ngood) ngood[f] = (long)s.ngood;
        if (status) status[f] = s.status;
    }
    return SGPU_OK;
}

template <typename T>
int norm_stats_host(sgpu_context *c, const T *frames, int nframes, long npix, long frame_stride, int lite,
                    double *stats, long *ngood, int *status) {
    HIP_TRY(hipSetDevice(c->device));
    // stage frames through HBM in batches of at most 1 GiB
    const size_t fbytes = sizeof(T) * (size_t)npix;
    const int batch = (int)std::max<size_t>(1, std::min<size_t>((size_t)nframes, ((size_t)1 << 30) / fbytes));
    int rc;
    if ((rc = c->ns_io.ensure(fbytes * batch))) return rc;
    for (int f0 = 0; f0 < nframes; f0 += batch) {
        const int nb = std::min(batch, nframes - f0);
        HIP_TRY(hipMemcpy2DAsync(c->ns_io.p, fbytes, frames + (size_t)f0 * frame_stride,
                                 sizeof(T) * (size_t)frame_stride, fbytes, nb, hipMemcpyHostToDevice, c->stream));
        if ((rc = norm_stats_device<T>(c, (const T *)c->ns_io.p, nb, npix, npix, lite, stats + 4 * f0,
                                       ngood ? ngood + f0 : nullptr, status ? status + f0 : nullptr)))
            return rc;
    }
    return SGPU_OK;
}

}  // namespace

#define NS_ARGS_OK(frames) (c && (frames) && nframes > 0 && npix > 0 && frame_stride >= npix && stats)

extern "C" int sgpu_norm_stats_device(sgpu_context *c, const float *d_frames, int nframes, long npix,
                                      long frame_stride, int lite, double *stats, long *ngood, int *status) {
    if (!NS_ARGS_OK(d_frames)) return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_stats_device: bad arguments");
    return norm_stats_device<float>(c, d_frames, nframes, npix, frame_stride, lite, stats, ngood, status);
}

extern "C" int sgpu_norm_stats(sgpu_context *c, const float *frames, int nframes, long npix, long frame_stride,
                               int lite, double *stats, long *ngood, int *status) {
    if (!NS_ARGS_OK(frames)) return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_stats: bad arguments");
    return norm_stats_host<float>(c, frames, nframes, npix, frame_stride, lite, stats, ngood, status);
}

extern "C" int sgpu_norm_stats_u16_device(sgpu_context *c, const uint16_t *d_frames, int nframes, long npix,
                                          long frame_stride, int lite, double *stats, long *ngood, int *status) {
    if (!NS_ARGS_OK(d_frames))
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_stats_u16_device: bad arguments");
    return norm_stats_device<unsigned short>(c, d_frames, nframes, npix, frame_stride, lite, stats, ngood, status);
}

extern "C" int sgpu_norm_stats_u16(sgpu_context *c, const uint16_t *frames, int nframes, long npix,
                                   long frame_stride, int lite, double *stats, long *ngood, int *status) {
    if (!NS_ARGS_OK(frames)) return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_stats_u16: bad arguments");
    return norm_stats_host<unsigned short>(c, frames, nframes, npix, frame_stride, lite, stats, ngood, status);
}

// compute_factors_from_estimators (stacking/normalization.c:150-185) for one
// layer, after _compute_estimators_for_image (:107-146) picked the estimators.
extern "C" int sgpu_norm_factors(int normalize, int lite, int nframes, int ref_index, const double *stats,
                                 const double *ref_stats, double *offset, double *mul, double *scale) {
    if (nframes <= 0 || ref_index < 0 || ref_index >= nframes || !stats || !offset || !mul || !scale)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_factors: bad arguments");
    if (!ref_stats) ref_stats = stats;
    auto loc_of = [&](const double *s, int i) { return lite ? s[4 * i + 0] : s[4 * i + 2]; };
    auto scl_of = [&](const double *s, int i) { return lite ? 1.5 * s[4 * i + 1] : s[4 * i + 3]; };
    for (int i = 0; i < nframes; ++i) {
        offset[i] = 0.0;
        mul[i] = 1.0;
        scale[i] = 1.0;
    }
    if (normalize == SGPU_NO_NORM) return SGPU_OK;
    const bool additive = normalize == SGPU_ADDITIVE || normalize == SGPU_ADDITIVE_SCALING;
    const bool scaling = normalize == SGPU_ADDITIVE_SCALING || normalize == SGPU_MULTIPLICATIVE_SCALING;
    if (!additive && normalize != SGPU_MULTIPLICATIVE && !scaling)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_norm_factors: unknown normalization");
    // estimators (the reference stores them in the coefficient arrays first)
    std::vector<double> e_loc((size_t)nframes), e_scl((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        e_loc[(size_t)i] = loc_of(stats, i);
        e_scl[(size_t)i] = scaling ? scl_of(stats, i) : 1.0;
    }
    const double loc0 = loc_of(ref_stats, ref_index);
    const double scl0 = scaling ? scl_of(ref_stats, ref_index) : 1.0;
    for (int i = 0; i < nframes; ++i) {
        double sc = 1.0;
        if (scaling) sc = (e_scl[(size_t)i] == 0) ? 1 : scl0 / e_scl[(size_t)i];
        scale[i] = sc;
        if (additive) offset[i] = sc * e_loc[(size_t)i] - loc0;
        else mul[i] = (e_loc[(size_t)i] == 0) ? 1 : loc0 / e_loc[(size_t)i];
    }
    return SGPU_OK;
}
