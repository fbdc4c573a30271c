// bgnoise.hip -- background noise of a frame (imstats bgnoise), the
// estimator -weight=noise divides by (median_and_mean.c:1111-1135).
//
// The reference takes it from siril_fits_img_stats_float / _ushort
// (algos/quantize.c:139-205, 71-137) -> FnNoise1_float / FnNoise1_ushort
// (:1343-1488, :1202-1341), a CFITSIO estimator: per image row, the first-
// order differences of consecutive valid pixels (non-zero, and not NaN for
// float), their mean and RMS (FnDiffMeanSigma_*, :327-422), up to NITER = 3
// rounds of SIGMA_CLIP = 5 clipping around the mean; the row's RMS; the
// median of the rows' values times 0.70710678.  Float data are in [0, 1]
// units (normValue 1, statistics_float.c:389-400), 16-bit data in ADU.
//
// One thread per row, in the reference's sequential order: the float sums
// (double accumulation of float differences and their squares) are not exact
// in general, so the order is kept rather than reassociated.  The clipped
// survivors are never compacted: each round re-streams the row and applies
// the earlier rounds' tests in sequence, which selects the same subsequence
// in the same order as the reference's in-place compaction.  The median over
// rows runs on the host (<= a few thousand values per frame).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "sgpu_internal.h"

namespace sgpu {
namespace bn {

constexpr int kNiter = 3;          // NITER (quantize.c:39)
constexpr double kClip = 5.;       // SIGMA_CLIP (quantize.c:38)

__device__ __forceinline__ bool valid(float v) { return v != 0.f && !isnan(v); }
__device__ __forceinline__ bool valid(unsigned short v) { return v != 0; }

// one streaming pass over the row's differences: the survivors of tests
// [0, nt) (float: |d - (float)mean| < 5 sd, d - mean in float; int: in
// double), their count (array length), non-NaN count and double sums
template <class T>
__device__ void diff_pass(const T *row, int W, int nt, const double *tm, const double *ts, long &narr, long &ngood,
                          double &sum, double &sum2) {
    narr = ngood = 0;
    sum = sum2 = 0.0;
    int ii = 0;
    while (ii < W && !valid(row[ii])) ii++;
    if (ii == W) return;
    T v1 = row[ii];
    for (ii++; ii < W; ii++) {
        const T x = row[ii];
        if (!valid(x)) continue;
        bool keep = true;
        if constexpr (sizeof(T) == 4) {
            const float d = (float)v1 - (float)x;
            for (int j = 0; j < nt; j++) keep = keep && ((double)fabsf(d - (float)tm[j]) < kClip * ts[j]);
            if (keep) {
                narr++;
                if (!isnan(d)) {
                    ngood++;
                    const double t = (double)d;
                    sum += t;
                    sum2 += t * t;
                }
            }
        } else {
            const int d = (int)v1 - (int)x;
            for (int j = 0; j < nt; j++) keep = keep && (fabs((double)d - tm[j]) < kClip * ts[j]);
            if (keep) {
                narr++;
                ngood++;
                const double t = (double)d;
                sum += t;
                sum2 += t * t;
            }
        }
        v1 = x;
    }
}

// FnDiffMeanSigma_float / _int on the pass's sums
__device__ void mean_sigma(long n, double sum, double sum2, double &mean, double &sd) {
    if (n > 1) {
        mean = sum / n;
        sd = sqrt((sum2 / n) - (mean * mean));
    } else if (n == 1) {
        mean = sum;
        sd = 0.0;
    } else {
        mean = 0.0;
        sd = 0.0;
    }
}

// per row: the clipped RMS of the differences, or -1 when the row has fewer
// than two differences (the reference skips it)
template <class T>
__global__ __launch_bounds__(256) void k_row_noise(const T *frames, long long fstride, int W, int H, int nframes,
                                                   double *out) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)nframes * H) return;
    const int f = (int)(gid / H), r = (int)(gid % H);
    const T *row = frames + f * fstride + (long long)r * W;
    double tm[kNiter], ts[kNiter];
    long narr, ngood;
    double sum, sum2, mean, sd;
    diff_pass(row, W, 0, tm, ts, narr, ngood, sum, sum2);
    if (narr < 2) {
        out[gid] = -1.0;
        return;
    }
    mean_sigma(ngood, sum, sum2, mean, sd);
    if (sd > 0.) {
        long nvals = narr;
        for (int it = 0; it < kNiter; it++) {
            tm[it] = mean;
            ts[it] = sd;
            diff_pass(row, W, it + 1, tm, ts, narr, ngood, sum, sum2);
            if (narr == nvals) break;
            nvals = narr;
            mean_sigma(ngood, sum, sum2, mean, sd);
        }
    }
    out[gid] = sd;
}

}  // namespace bn
}  // namespace sgpu

namespace {

// median of the rows' values (qsort + middle pair for float,
// quickmedian_double for 16-bit: the same value) times 0.70710678
double frame_noise(std::vector<double> &v) {
    if (v.empty()) return 0.0;
    double x;
    if (v.size() == 1) {
        x = v[0];
    } else {
        std::sort(v.begin(), v.end());
        const size_t n = v.size();
        x = (v[(n - 1) / 2] + v[n / 2]) / 2.;
    }
    return .70710678 * x;
}

template <class T>
int bgnoise_device(sgpu_context *c, const T *d_frames, int nframes, int width, int height, long frame_stride,
                   double *noise) {
    if (!c || !d_frames || nframes <= 0 || width <= 0 || height <= 0 || frame_stride < (long)width * height || !noise)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_bgnoise: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    if (width < 3) {                       // rows must have at least 3 pixels (quantize.c:1362-1366)
        for (int f = 0; f < nframes; f++) noise[f] = 0.0;
        return SGPU_OK;
    }
    const size_t nrow = (size_t)nframes * height;
    if (int rc = c->bn_rows.ensure(nrow * sizeof(double))) return rc;
    double *d_rows = (double *)c->bn_rows.p;
    hipLaunchKernelGGL((sgpu::bn::k_row_noise<T>), dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, c->stream,
                       d_frames, (long long)frame_stride, width, height, nframes, d_rows);
    HIP_TRY(hipGetLastError());
    std::vector<double> rows(nrow);
    HIP_TRY(hipMemcpyAsync(rows.data(), d_rows, nrow * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int f = 0; f < nframes; f++) {
        std::vector<double> v;
        v.reserve(height);
        for (int r = 0; r < height; r++) {
            const double x = rows[(size_t)f * height + r];
            if (!(x < 0.0)) v.push_back(x);
        }
        noise[f] = frame_noise(v);
    }
    return SGPU_OK;
}

template <class T>
int bgnoise_host(sgpu_context *c, const T *frames, int nframes, int width, int height, long frame_stride,
                 double *noise) {
    if (!c || !frames || nframes <= 0 || width <= 0 || height <= 0 || frame_stride < (long)width * height || !noise)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_bgnoise: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t fbytes = sizeof(T) * (size_t)width * height;
    const int batch = (int)std::max<size_t>(1, std::min<size_t>((size_t)nframes, ((size_t)1 << 30) / fbytes));
    if (int rc = c->ns_io.ensure(fbytes * batch)) return rc;
    for (int f0 = 0; f0 < nframes; f0 += batch) {
        const int nb = std::min(batch, nframes - f0);
        HIP_TRY(hipMemcpy2DAsync(c->ns_io.p, fbytes, frames + (size_t)f0 * frame_stride,
                                 sizeof(T) * (size_t)frame_stride, fbytes, nb, hipMemcpyHostToDevice, c->stream));
        if (int rc = bgnoise_device<T>(c, (const T *)c->ns_io.p, nb, width, height, (long)width * height, noise + f0))
            return rc;
    }
    return SGPU_OK;
}

}  // namespace

extern "C" int sgpu_bgnoise_device(sgpu_context *c, const float *d_frames, int nframes, int width, int height,
                                   long frame_stride, double *noise) {
    return bgnoise_device<float>(c, d_frames, nframes, width, height, frame_stride, noise);
}
extern "C" int sgpu_bgnoise_u16_device(sgpu_context *c, const uint16_t *d_frames, int nframes, int width, int height,
                                       long frame_stride, double *noise) {
    return bgnoise_device<unsigned short>(c, (const unsigned short *)d_frames, nframes, width, height, frame_stride,
                                          noise);
}
extern "C" int sgpu_bgnoise(sgpu_context *c, const float *frames, int nframes, int width, int height,
                            long frame_stride, double *noise) {
    return bgnoise_host<float>(c, frames, nframes, width, height, frame_stride, noise);
}
extern "C" int sgpu_bgnoise_u16(sgpu_context *c, const uint16_t *frames, int nframes, int width, int height,
                                long frame_stride, double *noise) {
    return bgnoise_host<unsigned short>(c, (const unsigned short *)frames, nframes, width, height, frame_stride,
                                        noise);
}
