// stack_partial.hip -- partial sums of a frame shard for the no-rejection
// mean stack (mean_and_reject with NO_REJEC: median_and_mean.c:1083-1097,
// rejection_float.c:116-142), the data path of the frame-sharded multi-GPU
// stack: every rank holds a contiguous range of frames, accumulates per
// pixel the f64 sum and the count of its non-zero (present) samples in frame
// order, the partials are all-reduced over RCCL, and k_mean_finish turns
// them into the mean.  The reference's mean is sum/kept over the non-zero
// samples of the whole column; splitting the f64 sum by frame ranges gives
// the same double whenever the double sums are exact (f32 samples within a
// 2^29 dynamic range, e.g. Siril's [0, 1] data above 2^-20), which is the
// same condition under which the reference's own omp-simd reduction order
// does not matter.  The guard: the partial pass also keeps the smallest and
// largest |x| of the present samples (all-reduced with MIN / MAX), and
// k_mean_finish flags every pixel whose sums are not provably exact in every
// order -- all |x| on the grid of ulp(min |x|) and every partial sum within
// 2^53 of it: ceil(log2 count) + e(max) - e(min) + 24 <= 53 -- so the caller
// recomputes those few pixels from their gathered columns in frame order
// (siril_amd/distributed.py), as the exact kernel does for the sorted path.
#include <hip/hip_runtime.h>

#include "sgpu_internal.h"
#include "sgpu_kparams.h"
#include "stack_sorted_impl.h"

namespace sgpu {

template <bool VEC>
__global__ __launch_bounds__(256) void k_mean_partial(KParams p, double *sum, int *count, float *amin,
                                                      float *amax) {
    constexpr int PX = VEC ? 4 : 1;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long pix0 = t * PX;
    if (pix0 >= p.npix) return;
    double s[PX];
    int k[PX];
    float lo[PX], hi[PX];
#pragma unroll
    for (int q = 0; q < PX; q++) {
        s[q] = 0.0;
        k[q] = 0;
        lo[q] = f_inf();
        hi[q] = 0.f;
    }
    const int N = p.nframes;
    if (VEC) {
        const float *src = p.frames + pix0;
        for (int f = 0; f < N; f++) {
            const float4 v4 = *reinterpret_cast<const float4 *>(src + (long long)f * p.frame_stride);
            const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int q = 0; q < PX; q++) {
                float x = v[q];
                if (p.norm == ADDITIVE || p.norm == ADDITIVE_SCALING) {
                    x = (x != 0.f) ? (float)(x * p.scale[f] - p.offset[f]) : 0.f;
                } else if (p.norm == MULTIPLICATIVE || p.norm == MULTIPLICATIVE_SCALING) {
                    x = (float)((x * p.scale[f]) * p.mul[f]);
                }
                if (x != 0.f) {
                    s[q] += (double)x;
                    k[q]++;
                    lo[q] = fminf(lo[q], fabsf(x));
                    hi[q] = fmaxf(hi[q], fabsf(x));
                }
            }
        }
    } else {
        const int x = (int)(pix0 % p.W);
        for (int f = 0; f < N; f++) {
            const float v = gather_sample(p, f, pix0, x);
            if (v != 0.f) {
                s[0] += (double)v;
                k[0]++;
                lo[0] = fminf(lo[0], fabsf(v));
                hi[0] = fmaxf(hi[0], fabsf(v));
            }
        }
    }
#pragma unroll
    for (int q = 0; q < PX; q++) {
        const long long pix = pix0 + q;
        if (pix >= p.npix) break;
        sum[pix] += s[q];
        count[pix] += k[q];
        if (amin) {
            amin[pix] = fminf(amin[pix], lo[q]);
            amax[pix] = fmaxf(amax[pix], hi[q]);
        }
    }
}

// exponent of a float's leading bit (subnormals: the grid 2^-149 = 2^(-126-23))
__device__ __forceinline__ int fexp(float a) {
    const int e = (int)((__float_as_uint(a) >> 23) & 0xffu);
    return e == 0 ? -126 : e - 127;
}

// every order of the count additions gives the same double (see the header)
__device__ __forceinline__ bool sums_exact(int count, float amin, float amax) {
    if (count <= 1) return true;
    const int cl = 32 - __clz(count - 1);            // ceil(log2 count)
    return cl + fexp(amax) - fexp(amin) + 24 <= 53;
}

// mean of the present samples, clamped to [0, 1] unless output_norm
// (set_float_in_interval, core/proto.h:384-388); a column without a present
// sample is all zeros, whose quickmedian (median_and_mean.c:1040-1041) is 0.
__global__ __launch_bounds__(256) void k_mean_finish(const double *sum, const int *count, const float *amin,
                                                     const float *amax, long long npix, float *out,
                                                     int output_norm, unsigned char *flag) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    if (flag) flag[i] = sums_exact(count[i], amin[i], amax[i]) ? 0 : 1;
    float fr = count[i] > 0 ? (float)(sum[i] / (double)count[i]) : 0.f;
    if (!output_norm) {
        fr = (fr < 0.f) ? 0.f : fr;
        fr = (fr > 1.f) ? 1.f : fr;
    }
    out[i] = fr;
}

// the (shifted, normalized) samples of the listed pixels, frame-major:
// out[f * k + j] = sample f of pixel idx[j] (gather_sample)
__global__ __launch_bounds__(256) void k_gather_columns(KParams p, const long long *idx, long long k,
                                                        float *out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= k * p.nframes) return;
    const int f = (int)(t / k);
    const long long j = t % k;
    const long long pix = idx[j];
    out[t] = gather_sample(p, f, pix, (int)(pix % p.W));
}

}  // namespace sgpu

extern "C" int sgpu_mean_partial_device(sgpu_context *c, const float *d_frames, int N, long W, long rows,
                                        long frame_stride, const sgpu_stack_params *P, double *d_sum,
                                        int *d_count);

namespace sgpu_host {
int prepare_params(sgpu_context *c, int N, long W, const sgpu_stack_params *P, sgpu::KParams &k, bool &xf);
}

extern "C" int sgpu_mean_partial_guard_device(sgpu_context *c, const float *d_frames, int N, long W, long rows,
                                              long frame_stride, const sgpu_stack_params *P, double *d_sum,
                                              int *d_count, float *d_amin, float *d_amax);

extern "C" int sgpu_mean_partial_device(sgpu_context *c, const float *d_frames, int N, long W, long rows,
                                        long frame_stride, const sgpu_stack_params *P, double *d_sum,
                                        int *d_count) {
    return sgpu_mean_partial_guard_device(c, d_frames, N, W, rows, frame_stride, P, d_sum, d_count, nullptr,
                                          nullptr);
}

extern "C" int sgpu_mean_partial_guard_device(sgpu_context *c, const float *d_frames, int N, long W, long rows,
                                              long frame_stride, const sgpu_stack_params *P, double *d_sum,
                                              int *d_count, float *d_amin, float *d_amax) {
    using sgpu_host::fail;
    if ((d_amin == nullptr) != (d_amax == nullptr)) return fail(SGPU_BAD_ARGUMENT, "amin and amax go together");
    if (!c || !P || !d_frames || !d_sum || !d_count) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    if (P->method != SGPU_METHOD_MEAN || P->type_of_rejection != SGPU_NO_REJEC || P->weights)
        return fail(SGPU_BAD_ARGUMENT, "partial sums are the unweighted no-rejection mean only");
    if (W * rows >= (1L << 31)) return fail(SGPU_BAD_ARGUMENT, "block too large");
    HIP_TRY(hipSetDevice(c->device));
    sgpu::KParams k;
    bool xf;
    c->ev_used = 0;
    if (int r = sgpu_host::prepare_params(c, N, W, P, k, xf)) return r;
    k.frames = d_frames;
    k.frame_stride = frame_stride;
    k.npix = (long long)W * rows;
    const bool vec = !P->shiftx && W % 4 == 0 && frame_stride % 4 == 0 && ((uintptr_t)d_frames % 16) == 0;
    const long long threads = vec ? (k.npix + 3) / 4 : k.npix;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    sgpu_host::mark(c);
    if (vec)
        hipLaunchKernelGGL(sgpu::k_mean_partial<true>, dim3(grid), dim3(256), 0, c->stream, k, d_sum, d_count, d_amin,
                           d_amax);
    else
        hipLaunchKernelGGL(sgpu::k_mean_partial<false>, dim3(grid), dim3(256), 0, c->stream, k, d_sum, d_count,
                           d_amin, d_amax);
    HIP_TRY(hipGetLastError());
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    return SGPU_OK;
}

extern "C" int sgpu_mean_finish_guard_device(sgpu_context *c, const double *d_sum, const int *d_count,
                                             const float *d_amin, const float *d_amax, long npix, float *d_out,
                                             int output_norm, unsigned char *d_flag) {
    using sgpu_host::fail;
    if (!c || !d_sum || !d_count || !d_out || npix < 0) return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (d_flag && (!d_amin || !d_amax)) return fail(SGPU_BAD_ARGUMENT, "the guard needs amin and amax");
    if (npix == 0) return SGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(sgpu::k_mean_finish, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, c->stream,
                       d_sum, d_count, d_amin, d_amax, (long long)npix, d_out, output_norm, d_flag);
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}

extern "C" int sgpu_mean_finish_device(sgpu_context *c, const double *d_sum, const int *d_count, long npix,
                                       float *d_out, int output_norm) {
    return sgpu_mean_finish_guard_device(c, d_sum, d_count, nullptr, nullptr, npix, d_out, output_norm, nullptr);
}

extern "C" int sgpu_gather_columns_device(sgpu_context *c, const float *d_frames, int N, long W, long rows,
                                          long frame_stride, const sgpu_stack_params *P, const long long *d_idx,
                                          long long k, float *d_out) {
    using sgpu_host::fail;
    if (!c || !P || !d_frames || (k > 0 && (!d_idx || !d_out))) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1 || k < 0) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (k == 0) return SGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    sgpu::KParams kp;
    bool xf;
    c->ev_used = 0;
    if (int r = sgpu_host::prepare_params(c, N, W, P, kp, xf)) return r;
    kp.frames = d_frames;
    kp.frame_stride = frame_stride;
    kp.npix = (long long)W * rows;
    const long long t = k * N;
    hipLaunchKernelGGL(sgpu::k_gather_columns, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, c->stream, kp,
                       d_idx, k, d_out);
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}
