// stack_mean.hip -- NO_REJEC mean stack (mean_and_reject with NO_REJEC,
// median_and_mean.c:1083-1097 / rejection_float.c:128-142,350-351).
//
// Streaming kernel, HBM-bound: each thread owns 4 adjacent output pixels and
// walks the N frames with 16-byte loads (frame-major input, so a wave reads
// 1 KiB contiguous per frame).  Zero samples are missing; the mean of the
// non-zero samples is accumulated in double in frame order -- the exact
// summation order of the reference.  All-zero columns (kept == 0: the
// reference returns quickmedian of the stack) go to the exact kernel.
#include <hip/hip_runtime.h>
#include "sgpu_kparams.h"
#include "stack_sorted_impl.h"

namespace sgpu {

template <bool VEC>
__global__ __launch_bounds__(256) void k_stack_mean(KParams p) {
    constexpr int PX = VEC ? 4 : 1;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long pix0 = t * PX;
    int rl = 0, rh = 0;
    if (pix0 < p.npix) {
        double sum[PX];
        int kept[PX];
#pragma unroll
        for (int q = 0; q < PX; q++) { sum[q] = 0.0; kept[q] = 0; }
        const int N = p.nframes;
        if (VEC) {
            // no shift, W % 4 == 0, npix % 4 == 0 (host-checked)
            const float *src = p.frames + pix0;
            for (int f = 0; f < N; f++) {
                const float4 v4 = *reinterpret_cast<const float4 *>(src + (long long)f * p.frame_stride);
                float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                for (int q = 0; q < PX; q++) {
                    float x = v[q];
                    if (p.norm == ADDITIVE || p.norm == ADDITIVE_SCALING) {
                        x = (x != 0.f) ? (float)(x * p.scale[f] - p.offset[f]) : 0.f;
                    } else if (p.norm == MULTIPLICATIVE || p.norm == MULTIPLICATIVE_SCALING) {
                        x = (float)((x * p.scale[f]) * p.mul[f]);
                    }
                    if (x != 0.f) { sum[q] += (double)x; kept[q]++; }
                }
            }
        } else {
            const int x = (int)(pix0 % p.W);
            for (int f = 0; f < N; f++) {
                const float v = gather_sample(p, f, pix0, x);
                if (v != 0.f) { sum[0] += (double)v; kept[0]++; }
            }
        }
#pragma unroll
        for (int q = 0; q < PX; q++) {
            const long long pix = pix0 + q;
            if (pix >= p.npix) break;
            if (kept[q] == 0) {
                const int slot = atomicAdd(p.fb_count, 1);
                p.fb_list[slot] = (int)pix;
                continue;
            }
            double res = sum[q] / (double)kept[q];
            if (p.weights) {
                // all kept samples are within [pmin, pmax]; recompute min/max
                const int x = (int)(pix % p.W);
                float pmin = __builtin_huge_valf(), pmax = -__builtin_huge_valf();
                for (int f = 0; f < N; f++) {
                    const float v = gather_sample(p, f, pix, x);
                    if (v != 0.f) {
                        pmin = (pmin > v) ? v : pmin;
                        pmax = (pmax < v) ? v : pmax;
                    }
                }
                res = weighted_mean(p, pix, x, pmin, pmax, kept[q]);
            }
            write_result(p, pix, res, 0, 0);
        }
    }
    (void)rl; (void)rh;
}

int launch_stack_mean(const KParams &p, hipStream_t s) {
    const bool vec = (p.shiftx == nullptr) && (p.W % 4 == 0) && (p.npix % 4 == 0) &&
                     (p.frame_stride % 4 == 0) && ((uintptr_t)p.frames % 16 == 0);
    const long long threads = vec ? (p.npix + 3) / 4 : p.npix;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    if (vec) hipLaunchKernelGGL(k_stack_mean<true>, dim3(grid), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_stack_mean<false>, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sgpu
