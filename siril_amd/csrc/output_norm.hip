// output_norm.hip -- norm_to_0_1_range (stacking/median_and_mean.c:557-582),
// the whole-image post-pass of a 32-bit stack with args->output_norm
// (:1774-1775).
//
// Reference: min / max over the non-zero samples of indices 1..n-1 (the loop
// starts at i = 1; `tmp < mini` / `tmp > maxi`, so NaN never wins), then
// x = (x == 0) ? 0 : (x - mini) / (maxi - mini) in float.  Min and max are
// order-independent, so one streaming pass with ordered-integer atomics (one
// pair per block) gives exactly the reference's values; the second pass is
// elementwise.  Two HBM passes over the image (8 B per pixel read, 4 written).
#include <hip/hip_runtime.h>

#include "sgpu_internal.h"

namespace sgpu {

// float -> unsigned key with the same order (finite values and infinities)
__device__ __forceinline__ unsigned fkey(float f) {
    const unsigned u = __builtin_bit_cast(unsigned, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
    const unsigned u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __builtin_bit_cast(float, u);
}

__global__ void k_onorm_init(unsigned *mm) {
    mm[0] = fkey(3.40282347e+38f);    // FLT_MAX
    mm[1] = fkey(-3.40282347e+38f);   // -1.f * FLT_MAX
}

__global__ __launch_bounds__(256) void k_onorm_minmax(const float *img, long long n, unsigned *mm) {
    unsigned lo = 0xffffffffu, hi = 0u;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = 1 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float t = img[i];
        if (t != 0.f && t == t) {
            const unsigned k = fkey(t);
            lo = k < lo ? k : lo;
            hi = k > hi ? k : hi;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const unsigned a = __shfl_xor(lo, m, 64), b = __shfl_xor(hi, m, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    __shared__ unsigned slo[4], shi[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        slo[w] = lo;
        shi[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 1; j < (int)(blockDim.x >> 6); j++) {
            lo = slo[j] < lo ? slo[j] : lo;
            hi = shi[j] > hi ? shi[j] : hi;
        }
        if (lo != 0xffffffffu) atomicMin(mm, lo);
        if (hi != 0u) atomicMax(mm + 1, hi);
    }
}

__global__ __launch_bounds__(256) void k_onorm_apply(float *img, long long n, const unsigned *mm) {
    const float mini = fkey_inv(mm[0]), maxi = fkey_inv(mm[1]);
    const float range = maxi - mini;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float x = img[i];
        img[i] = (x == 0.f) ? 0.f : (x - mini) / range;
    }
}

}  // namespace sgpu

extern "C" int sgpu_norm_to_0_1_range_device(sgpu_context *c, float *d_img, long n) {
    if (!c || !d_img || n < 0) return sgpu_host::fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (n == 0) return SGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (int r = c->onorm.ensure(2 * sizeof(unsigned))) return r;
    unsigned *mm = (unsigned *)c->onorm.p;
    const unsigned grid = (unsigned)std::min<long>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(sgpu::k_onorm_init, dim3(1), dim3(1), 0, c->stream, mm);
    hipLaunchKernelGGL(sgpu::k_onorm_minmax, dim3(grid), dim3(256), 0, c->stream, d_img, (long long)n, mm);
    hipLaunchKernelGGL(sgpu::k_onorm_apply, dim3(grid), dim3(256), 0, c->stream, d_img, (long long)n, mm);
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}
