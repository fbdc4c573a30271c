// stack_mean.hip -- NO_REJEC mean stack (mean_and_reject with NO_REJEC,
// median_and_mean.c:1083-1097 / rejection_float.c:128-142,350-351; the
// DATA_USHORT twin :1020-1034 with apply_rejection_ushort :717-736).
//
// Streaming kernels, HBM-bound (9.7 GB per 100 x 6000 x 4000 f32 stack).
// Each thread owns 4 adjacent output pixels (16-bit: 8) and walks the N
// frames with 16-byte non-temporal loads (frame-major input: a wave reads
// 1 KiB contiguous per frame); the frame loop is unrolled by kUnroll with all
// of a group's loads issued before the first is used, so every wave keeps
// kUnroll KiB in flight (one load per wave in flight left the round-4 kernel
// latency-bound).  Zero samples are missing (the reference's compaction).
//
// Float sums are accumulated in double in frame order -- the reference's
// sequential order.  For kept >= STACK_SIMD_N_THRESHOLD (16) the reference
// sums with `#pragma omp simd reduction` (:1085-1090), whose order is the
// build's vectorisation; the kernel proves per pixel that the float result
// does not depend on the order (SumGuard of stack_sorted_impl.h: the f64 sum
// is exact in every order, or (float)(q - e) == (float)(q + e) for the
// order-error bound e) and records the pixels it cannot prove in fb2_list
// (sgpu_last_order_sensitive): their value is the sequential order's.
// Weighted means are sequential sums in the reference (:1056-1069): no guard.
// 16-bit sums are integers (gint64 in the reference): exact in any order.
//
// All-zero columns (kept == 0: the reference returns quickmedian of the stack)
// go to the exact kernel through fb_list.
#include <hip/hip_runtime.h>
#include "sgpu_kparams.h"
#include "stack_sorted_impl.h"

namespace sgpu {

constexpr int kUnroll = 8;     // frames whose loads are in flight together per thread
typedef float vf4 __attribute__((ext_vector_type(4)));      // nontemporal builtins take clang vectors
typedef uint32_t vu4 __attribute__((ext_vector_type(4)));

// normalization of one float sample, as gather_sample (stack_sorted_impl.h)
template <int NK>
__device__ __forceinline__ float norm_f(float v, double sc, double of, double mu) {
    if constexpr (NK == 1) return (v != 0.f) ? (float)(v * sc - of) : 0.f;   // ADDITIVE(_SCALING)
    else if constexpr (NK == 2) return (float)((v * sc) * mu);               // MULTIPLICATIVE(_SCALING)
    else return v;
}

// one f32 sample into a pixel's accumulators
struct MeanAcc {
    double sum;
    int kept;
    float amin, amax;          // min / max |x| over the kept samples
    unsigned sgn;              // OR of the samples' bits: sign bit set if any x < 0 (or -0)
    __device__ __forceinline__ void init() { sum = 0.0; kept = 0; amin = __builtin_huge_valf(); amax = 0.f; sgn = 0u; }
    __device__ __forceinline__ void add(float x) {
        const bool nz = x != 0.f;
        sum += (double)x;                         // + (double)0 leaves the sum unchanged
        kept += nz ? 1 : 0;
        const float ax = fabsf(x);
        amin = fminf(amin, nz ? ax : __builtin_huge_valf());
        amax = fmaxf(amax, ax);
        sgn |= __builtin_bit_cast(uint32_t, x);
    }
    // true when the float conversion of sum / kept is the same in every
    // summation order of the kept samples (stack_sorted_impl.h SumGuard)
    __device__ __forceinline__ bool order_free(double q) const {
        if (kept < 16) return true;               // the reference's own sequential branch (:1091-1094)
        if (ebits(amax) - ebits(amin) + 24 + ceil_log2(kept) <= 53) return true;   // exact in f64
        // any summation tree of depth d is within gamma_d sum|x| of the exact
        // sum: the kernel's chain (kept) and the reference's (<= kept), plus
        // slack for the division and q +- e
        const double c = (double)(2 * kept + 16) * 0x1p-53;
        const double sabs = (sgn & 0x80000000u) ? (double)kept * (double)amax : sum;
        return f32_stable(q, (c * sabs + fabs(sum) * 0x1p-50) / (double)kept);
    }
};

template <int NK>
__global__ __launch_bounds__(256) void k_stack_mean_vec(KParams p) {
    constexpr int PX = 4;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long pix0 = t * PX;
    const bool live = pix0 < p.npix;          // npix % 4 == 0 (host-checked): all 4 or none
    MeanAcc a[PX];
#pragma unroll
    for (int q = 0; q < PX; q++) a[q].init();
    const int N = p.nframes;
    if (live) {
        const vf4 *src = reinterpret_cast<const vf4 *>(p.frames + pix0);
        const long long fs4 = p.frame_stride / 4;
        int f = 0;
        for (; f + kUnroll <= N; f += kUnroll) {
            vf4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(src + (long long)(f + u) * fs4);
#pragma unroll
            for (int u = 0; u < kUnroll; u++) {
                double sc = 1.0, of = 0.0, mu = 1.0;
                if constexpr (NK == 1) { sc = p.scale[f + u]; of = p.offset[f + u]; }
                if constexpr (NK == 2) { sc = p.scale[f + u]; mu = p.mul[f + u]; }
                a[0].add(norm_f<NK>(v[u].x, sc, of, mu));
                a[1].add(norm_f<NK>(v[u].y, sc, of, mu));
                a[2].add(norm_f<NK>(v[u].z, sc, of, mu));
                a[3].add(norm_f<NK>(v[u].w, sc, of, mu));
            }
        }
        for (; f < N; f++) {
            const vf4 v = __builtin_nontemporal_load(src + (long long)f * fs4);
            double sc = 1.0, of = 0.0, mu = 1.0;
            if constexpr (NK == 1) { sc = p.scale[f]; of = p.offset[f]; }
            if constexpr (NK == 2) { sc = p.scale[f]; mu = p.mul[f]; }
            a[0].add(norm_f<NK>(v.x, sc, of, mu));
            a[1].add(norm_f<NK>(v.y, sc, of, mu));
            a[2].add(norm_f<NK>(v.z, sc, of, mu));
            a[3].add(norm_f<NK>(v.w, sc, of, mu));
        }
    }
    float r[PX];
#pragma unroll
    for (int q = 0; q < PX; q++) {
        const long long pix = pix0 + q;
        double res = a[q].sum / (double)(a[q].kept > 0 ? a[q].kept : 1);
        // wave-uniform calls: every lane takes part in the ballots
        const int fslot = wave_append(p.fb_count, live && a[q].kept == 0);
        if (fslot >= 0) p.fb_list[fslot] = (int)pix;
        const int oslot = wave_append(p.fb2_count, live && a[q].kept > 0 && !p.weights && !a[q].order_free(res));
        if (oslot >= 0) p.fb2_list[oslot] = (int)pix;
        if (live && a[q].kept > 0 && p.weights) {
            const int x = (int)(pix % p.W);
            float pmin = __builtin_huge_valf(), pmax = -__builtin_huge_valf();
            for (int f = 0; f < N; f++) {
                const float v = gather_sample(p, f, pix, x);
                if (v != 0.f) {
                    pmin = (pmin > v) ? v : pmin;
                    pmax = (pmax < v) ? v : pmax;
                }
            }
            res = weighted_mean(p, pix, x, pmin, pmax, a[q].kept);
        }
        float fr = (float)res;
        if (!p.output_norm) {                     // set_float_in_interval, proto.h:384-388
            fr = (fr < 0.f) ? 0.f : fr;
            fr = (fr > 1.f) ? 1.f : fr;
        }
        r[q] = fr;
    }
    if (!live) return;
    // kept == 0 pixels are rewritten by the exact kernel (same stream, later)
    const vf4 rv = {r[0], r[1], r[2], r[3]};
    __builtin_nontemporal_store(rv, reinterpret_cast<vf4 *>(p.out + pix0));
    if (p.rej_lo) {
#pragma unroll
        for (int q = 0; q < PX; q++) p.rej_lo[pix0 + q] = 0;
    }
    if (p.rej_hi) {
#pragma unroll
        for (int q = 0; q < PX; q++) p.rej_hi[pix0 + q] = 0;
    }
}

// shifted frames (per-frame x shift: no 16-byte alignment) -- one pixel per
// thread through gather_sample, same accumulators and guard
__global__ __launch_bounds__(256) void k_stack_mean_px(KParams p) {
    const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = pix < p.npix;
    MeanAcc a;
    a.init();
    const int x = live ? (int)(pix % p.W) : 0;
    if (live)
        for (int f = 0; f < p.nframes; f++) a.add(gather_sample(p, f, pix, x));
    double res = a.sum / (double)(a.kept > 0 ? a.kept : 1);
    const int fslot = wave_append(p.fb_count, live && a.kept == 0);
    if (fslot >= 0) p.fb_list[fslot] = (int)pix;
    const int oslot = wave_append(p.fb2_count, live && a.kept > 0 && !p.weights && !a.order_free(res));
    if (oslot >= 0) p.fb2_list[oslot] = (int)pix;
    if (!live || a.kept == 0) return;
    if (p.weights) {
        float pmin = __builtin_huge_valf(), pmax = -__builtin_huge_valf();
        for (int f = 0; f < p.nframes; f++) {
            const float v = gather_sample(p, f, pix, x);
            if (v != 0.f) {
                pmin = (pmin > v) ? v : pmin;
                pmax = (pmax < v) ? v : pmax;
            }
        }
        res = weighted_mean(p, pix, x, pmin, pmax, a.kept);
    }
    write_result(p, pix, res, 0, 0);
}

// ---- DATA_USHORT: integer sums (gint64 in the reference, exact in any order)

// the WORD the reference stores for a sample (gather_sample16 without the
// shift): round_to_WORD of the normalization affine, null samples null
template <int NK>
__device__ __forceinline__ uint32_t norm_w(uint32_t w, double sc, double of, double mu) {
    if constexpr (NK == 0) return w;
    else {
        if (w == 0u) return 0u;
        double t = (NK == 1) ? (double)w * sc - of : ((double)w * sc) * mu;
        t = t + 0.5;                                   // round_to_WORD, proto.h:232-237
        t = (t > 65535.0) ? 65535.0 : t;
        t = (t < 0.0) ? 0.0 : t;
        return (uint32_t)t;
    }
}

template <int NK>
__global__ __launch_bounds__(256) void k_stack_mean16_vec(KParams p) {
    constexpr int PX = 8;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long pix0 = t * PX;
    const bool live = pix0 < p.npix;          // npix % 8 == 0 (host-checked)
    uint32_t sum[PX];
    int kept[PX];
#pragma unroll
    for (int q = 0; q < PX; q++) { sum[q] = 0u; kept[q] = 0; }
    const int N = p.nframes;
    auto acc = [&](const vu4 v, int f) {
        double sc = 1.0, of = 0.0, mu = 1.0;
        if constexpr (NK == 1) { sc = p.scale[f]; of = p.offset[f]; }
        if constexpr (NK == 2) { sc = p.scale[f]; mu = p.mul[f]; }
        const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const uint32_t lo = norm_w<NK>(wds[h] & 0xffffu, sc, of, mu);
            const uint32_t hi = norm_w<NK>(wds[h] >> 16, sc, of, mu);
            sum[2 * h] += lo;
            kept[2 * h] += lo != 0u;
            sum[2 * h + 1] += hi;
            kept[2 * h + 1] += hi != 0u;
        }
    };
    if (live) {
        const vu4 *src = reinterpret_cast<const vu4 *>(p.frames16 + pix0);
        const long long fs8 = p.frame_stride / 8;
        int f = 0;
        for (; f + kUnroll <= N; f += kUnroll) {
            vu4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(src + (long long)(f + u) * fs8);
#pragma unroll
            for (int u = 0; u < kUnroll; u++) acc(v[u], f + u);
        }
        for (; f < N; f++) acc(__builtin_nontemporal_load(src + (long long)f * fs8), f);
    }
#pragma unroll
    for (int q = 0; q < PX; q++) {
        const long long pix = pix0 + q;
        const int fslot = wave_append(p.fb_count, live && kept[q] == 0);
        if (fslot >= 0) p.fb_list[fslot] = (int)pix;
        if (!live || kept[q] == 0) continue;
        double res = (double)sum[q] / (double)kept[q];
        if (p.weights) {
            const int x = (int)(pix % p.W);
            float pmin = __builtin_huge_valf(), pmax = -__builtin_huge_valf();
            for (int f = 0; f < N; f++) {
                const float v = gather_sample16(p, f, pix, x);
                if (v != 0.f) {
                    pmin = (pmin > v) ? v : pmin;
                    pmax = (pmax < v) ? v : pmax;
                }
            }
            res = weighted_mean<1>(p, pix, x, pmin, pmax, kept[q]);
        }
        write_result16(p, pix, res, 0, 0);
    }
}

__global__ __launch_bounds__(256) void k_stack_mean16_px(KParams p) {
    const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = pix < p.npix;
    uint32_t sum = 0u;
    int kept = 0;
    const int x = live ? (int)(pix % p.W) : 0;
    if (live)
        for (int f = 0; f < p.nframes; f++) {
            const uint32_t w = (uint32_t)gather_sample16(p, f, pix, x);
            sum += w;
            kept += w != 0u;
        }
    const int fslot = wave_append(p.fb_count, live && kept == 0);
    if (fslot >= 0) p.fb_list[fslot] = (int)pix;
    if (!live || kept == 0) return;
    double res = (double)sum / (double)kept;
    if (p.weights) {
        float pmin = __builtin_huge_valf(), pmax = -__builtin_huge_valf();
        for (int f = 0; f < p.nframes; f++) {
            const float v = gather_sample16(p, f, pix, x);
            if (v != 0.f) {
                pmin = (pmin > v) ? v : pmin;
                pmax = (pmax < v) ? v : pmax;
            }
        }
        res = weighted_mean<1>(p, pix, x, pmin, pmax, kept);
    }
    write_result16(p, pix, res, 0, 0);
}

static int norm_kind(int norm) {
    if (norm == ADDITIVE || norm == ADDITIVE_SCALING) return 1;
    if (norm == MULTIPLICATIVE || norm == MULTIPLICATIVE_SCALING) return 2;
    return 0;
}

// p.fb2_list / fb2_count must be set (order-sensitive pixels; float only)
int launch_stack_mean(const KParams &p, hipStream_t s) {
    const int nk = norm_kind(p.norm);
    if (p.frames16) {
        // N * 65535 must fit the u32 sums
        if (p.nframes > 65536) return -1;
        const bool vec = (p.shiftx == nullptr) && (p.npix % 8 == 0) && (p.frame_stride % 8 == 0) &&
                         ((uintptr_t)p.frames16 % 16 == 0);
        const long long threads = vec ? p.npix / 8 : p.npix;
        const unsigned grid = (unsigned)((threads + 255) / 256);
        if (!vec) hipLaunchKernelGGL(k_stack_mean16_px, dim3(grid), dim3(256), 0, s, p);
        else if (nk == 1) hipLaunchKernelGGL(k_stack_mean16_vec<1>, dim3(grid), dim3(256), 0, s, p);
        else if (nk == 2) hipLaunchKernelGGL(k_stack_mean16_vec<2>, dim3(grid), dim3(256), 0, s, p);
        else hipLaunchKernelGGL(k_stack_mean16_vec<0>, dim3(grid), dim3(256), 0, s, p);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (!p.fb2_list || !p.fb2_count) return -1;
    const bool vec = (p.shiftx == nullptr) && (p.npix % 4 == 0) && (p.frame_stride % 4 == 0) &&
                     ((uintptr_t)p.frames % 16 == 0) && ((uintptr_t)p.out % 16 == 0);
    const long long threads = vec ? p.npix / 4 : p.npix;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    if (!vec) hipLaunchKernelGGL(k_stack_mean_px, dim3(grid), dim3(256), 0, s, p);
    else if (nk == 1) hipLaunchKernelGGL(k_stack_mean_vec<1>, dim3(grid), dim3(256), 0, s, p);
    else if (nk == 2) hipLaunchKernelGGL(k_stack_mean_vec<2>, dim3(grid), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_stack_mean_vec<0>, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sgpu
