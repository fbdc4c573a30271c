// stack_exact.hip -- exact sequential per-pixel stack ("exact path").
//
// Runs on the GPU for the pixels the sorted path defers (fb_list): columns
// with NaN/Inf, the kept==0 / median==0 corner cases, rejection rounds whose
// outcome depends on the element order left by quickselect (the `N - r <= 4`
// cutoff, rejection_float.c:188,239,279), MAD (not yet on the sorted path),
// and any N above the largest sorted-path instantiation.  One thread runs the
// reference's sequential algorithm on one column held in a per-thread slice
// of a global scratch buffer, reproducing the in-place permutations of
// quickmedian_float (sorting.c:240-273), sortnet_median_float (:468-513) and
// quicksort_f (:110-135), so the visiting order -- and therefore the result --
// is the reference's.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include "sgpu_kparams.h"
#include "stack_sorted_impl.h"

namespace sgpu {
namespace ex {

__device__ __forceinline__ void swapf(float &a, float &b) { float t = a; a = b; b = t; }

// sortnet_median_float comparator lists, sorting.c:468-513 (pairs i,j; swap if a[i] > a[j])
__constant__ unsigned char kNet[] = {
    /*2*/ 0,1,
    /*3*/ 0,1, 1,2, 0,1,
    /*4*/ 0,1, 2,3, 0,2, 1,3, 1,2,
    /*5*/ 0,1, 2,3, 1,3, 2,4, 0,2, 1,4, 1,2, 3,4, 2,3,
    /*6*/ 0,1, 2,3, 4,5, 0,2, 3,5, 1,4, 0,1, 2,3, 4,5, 1,2, 3,4, 2,3,
    /*7*/ 1,2, 3,4, 5,6, 0,2, 4,6, 3,5, 2,6, 1,5, 0,4, 2,5, 0,3, 2,4, 1,3, 0,1, 2,3, 4,5,
    /*8*/ 0,1, 2,3, 4,5, 6,7, 0,2, 1,3, 4,6, 5,7, 1,2, 5,6, 0,4, 1,5, 2,6, 3,7, 2,4, 3,5,
          1,2, 3,4, 5,6};
__constant__ short kNetOff[9] = {0, 0, 0, 1, 4, 9, 18, 30, 46};
__constant__ short kNetLen[9] = {0, 0, 1, 3, 5, 9, 12, 16, 19};

__device__ double sortnet_median(float *a, int n) {
    const int k = n / 2;
    if (n == 1) return a[0];
    if (n < 2 || n > 8) return 0.0;
    const unsigned char *p = kNet + 2 * kNetOff[n];
    for (int c = 0; c < kNetLen[n]; c++) {
        const int i = p[2 * c], j = p[2 * c + 1];
        if (a[i] > a[j]) swapf(a[i], a[j]);
    }
    return (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
}

__device__ double quickmedian(float *a, int n) {
    if (n < 9) return sortnet_median(a, n);
    const int k = n / 2;
    int left = 0, right = n - 1;
    while (left < right) {
        int p = (left + right) / 2;
        const float pivot = a[p];
        a[p] = a[right];
        a[right] = pivot;
        p = left;
        // Lomuto's loop with its memory latency off the chain: iteration i
        // writes only a[p] and a[i] (p <= i), so a[i + 1] can be read one
        // iteration ahead, and a[p] -- the element a swap moves to i -- is
        // re-read right after p advances, a whole iteration before its use.
        // Same swaps in the same order as sorting.c:257-263.
        float cur = a[left], ap = cur;
        for (int i = left; i < right; i++) {
            const float nxt = a[i + 1];          // i + 1 <= right: in range (a[right] is the pivot)
            if (cur < pivot) {
                a[i] = ap;                       // swapf(a[p], a[i])
                a[p] = cur;
                p++;
                ap = (p == i + 1) ? nxt : a[p];
            }
            cur = nxt;
        }
        a[right] = a[p];
        a[p] = pivot;
        if (p < k) left = p + 1;
        else right = p;
    }
    return (n % 2 == 0) ? ((double)a[k - 1] + a[k]) / 2.0 : (double)a[k];
}

__device__ void insertion_sort(float *a, int n) {
    for (int i = 1; i < n; i++) {
        const float v = a[i];
        int j = i - 1;
        while (j >= 0 && a[j] > v) { a[j + 1] = a[j]; --j; }
        a[j + 1] = v;
    }
}

// quicksort_f with an explicit stack; sub-arrays are disjoint, so the order
// they are processed in does not change the result (smaller side first keeps
// the stack at log2(n)).
__device__ void quicksort(float *a0, int n0) {
    int sb[64], sn[64], top = 0;
    sb[0] = 0; sn[0] = n0; top = 1;
    while (top > 0) {
        --top;
        float *a = a0 + sb[top];
        const int n = sn[top];
        if (n <= 32) { insertion_sort(a, n); continue; }
        const float pivot = a[n / 2];
        int l = 0, r = n - 1;
        while (l <= r) {
            if (a[l] < pivot) { l++; continue; }
            if (a[r] > pivot) { r--; continue; }
            swapf(a[l], a[r]);
            l++; r--;
        }
        const int nl = r + 1, bl = sb[top] + 0;      // [0, r]
        const int nr = n - l, br = sb[top] + l;      // [l, n)
        if (nl > nr) {
            sb[top] = bl; sn[top] = nl; top++;
            sb[top] = br; sn[top] = nr; top++;
        } else {
            sb[top] = br; sn[top] = nr; top++;
            sb[top] = bl; sn[top] = nl; top++;
        }
    }
}

__device__ float sd(const float *x, int n, float *mean_out) {     // statistics.h:80-106
    double s = 0.0, q = 0.0;
    // sequential f64 chains (the restated order); unrolled so the reads of
    // a group are issued together ahead of the dependent adds
#pragma unroll 8
    for (int i = 0; i < n; i++) s += (double)x[i];
    const float mean = (float)(s / n);
#pragma unroll 8
    for (int i = 0; i < n; i++) { const float d = x[i] - mean; q += (double)(d * d); }
    if (mean_out) *mean_out = mean;
    return sqrtf((float)(q / (n - 1)));
}

// findMinMaxPercentile (rt/rt_algo.cc:38-172) at 0.5, single thread.
// `h` is n uint32 of scratch.
__device__ float hist_percentile(const float *x, int n, uint32_t *h) {
    float lo = x[0], hi = x[0];
    for (int i = 1; i < n; ++i) {
        lo = (x[i] < lo) ? x[i] : lo;
        hi = (hi < x[i]) ? x[i] : hi;
    }
    if (fabsf(hi - lo) == 0.f) return lo;
    const unsigned hs = (unsigned)(n < 65536 ? n : 65536);
    const float scale = (hs - 1) / (hi - lo);
    for (unsigned i = 0; i < hs; i++) h[i] = 0;
    for (int i = 0; i < n; ++i) {
        int b = (int)(scale * (x[i] - lo));
        b = b < 0 ? 0 : (b > (int)hs - 1 ? (int)hs - 1 : b);   // device-side bound (data NaN-free here)
        h[(uint16_t)b]++;
    }
    size_t k = 0, count = 0;
    float out = 0.f;
    for (int pass = 0; pass < 2; pass++) {
        const float thr = 0.5f * n;
        while (count < thr) count += h[k++];
        if (k > 0) {
            const size_t before = count - h[k - 1];
            const float c0 = count - thr, c1 = thr - before;
            out = (c1 * k + c0 * (k - 1)) / (c0 + c1);
        } else {
            out = k;
        }
        out /= scale;
        out += lo;
        const float m = (hi < out) ? hi : out;
        out = (lo < m) ? m : lo;
    }
    return out;
}

__device__ double mad(const float *x, int n, double m, float *tmp, uint32_t *h) {
    const float med = (float)m;
    for (int i = 0; i < n; i++) tmp[i] = fabsf(x[i] - med);
    return hist_percentile(tmp, n, h);
}

__device__ int compact(float *s, const int *rej, int n) {
    int o = 0;
    for (int p = 0; p < n; p++)
        if (!rej[p]) s[o++] = s[p];
    return o;
}

__device__ __forceinline__ int sclip(float x, float s, float slo, float shi, float m, int rej[2]) {
    if (m - x > s * slo) { rej[0]++; return -1; }
    if (x - m > s * shi) { rej[1]++; return 1; }
    return 0;
}

struct Work {           // per-thread slices of the scratch buffer
    float *stack, *o_stack, *w_stack, *tmp;
    int *rejected;
    uint32_t *hist;
};

// apply_rejection_float (rejection_float.c:100-354), no drizzle
__device__ int apply_rejection(const KParams &p, Work &wk, int nb, int crej[2], long long pix, int x) {
    int N = nb, r = 0, firstloop = 1, kept = 0, changed, n;
    double median = 0.0;
    float *stack = wk.stack, *w = wk.w_stack;
    int *rejected = wk.rejected;
    const float slo = p.sig0, shi = p.sig1;
    for (int f = 0; f < N; f++) wk.o_stack[f] = stack[f];
    for (int f = 0; f < N; f++)
        if (stack[f] != 0.f && (!p.drizz || plane_at(p, p.drizz, f, pix, x) != 0.f)) {   // :117-135
            if (f != kept) stack[kept] = stack[f];
            kept++;
        }
    if (kept <= 1) return kept;
    const int removed = N - kept;
    N = kept;
    switch (p.rtype) {
        case PERCENTILE: case SIGMA: case MAD:
            median = quickmedian(stack, N);
            if (median == 0.0) return 0;
            break;
        default: break;
    }
    switch (p.rtype) {
        case PERCENTILE: {
            const float mf = (float)median;
            for (int f = 0; f < N; f++) {
                const float x = stack[f];
                if (mf - x > mf * slo) { crej[0]++; rejected[f] = -1; }
                else if (x - mf > mf * shi) { crej[1]++; rejected[f] = 1; }
                else rejected[f] = 0;
            }
            N = compact(stack, rejected, N);
            break;
        }
        case SIGMA: case MAD:
            do {
                float var;
                if (p.rtype == SIGMA) var = sd(stack, N, nullptr);
                else var = (float)mad(stack, N, median, wk.tmp, wk.hist);
                if (!firstloop) median = quickmedian(stack, N);
                else firstloop = 0;
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        rejected[f] = sclip(stack[f], var, slo, shi, (float)median, crej);
                        if (rejected[f]) r++;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case SIGMEDIAN: {
            int it = 0;
            do {
                const float sigma = sd(stack, N, nullptr);
                const float mf = (float)quickmedian(stack, N);
                n = 0;
                for (int f = 0; f < N; f++)
                    if (sclip(stack[f], sigma, slo, shi, mf, crej)) { stack[f] = mf; n++; }
            } while (n > 0 && ++it < 100000);
            break;
        }
        case WINSORIZED:
            do {
                float sigma0, sigma = sd(stack, N, nullptr);
                const float mf = (float)quickmedian(stack, N);
                for (int j = 0; j < N; j++) w[j] = stack[j];
                int it = 0;
                do {
                    const float m0 = mf - 1.5f * sigma, m1 = mf + 1.5f * sigma;
                    for (int j = 0; j < N; j++) {
                        const float a = (m0 > w[j]) ? m0 : w[j];
                        w[j] = (m1 < a) ? m1 : a;
                    }
                    sigma0 = sigma;
                    sigma = 1.134f * sd(w, N, nullptr);
                } while (fabsf(sigma - sigma0) > sigma0 * 0.0005f && ++it < 100000);
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        rejected[f] = sclip(stack[f], sigma, slo, shi, mf, crej);
                        if (rejected[f] != 0) r++;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case LINEARFIT:
            do {
                quicksort(stack, N);
                // siril_fit_linear (siril_fit_linear.c:24-50), x[i] = 1/(i+1)
                float m_y = stack[0];
                for (int i = 1; i < N; i++) m_y += (stack[i] - m_y) * (1.f / (i + 1));
                float m_dxdy = 0.f, dx = -p.m_x;
                for (int i = 0; i < N; i++, dx += 1.f) {
                    const float dy = stack[i] - m_y;
                    m_dxdy += (dx * dy - m_dxdy) * (1.f / (i + 1));
                }
                const float a = m_dxdy * p.m_dx2;      // slope
                const float b = m_y - p.m_x * a;       // intercept
                float sigma = 0.f;
                for (int f = 0; f < N; f++) sigma += fabsf(stack[f] - (a * f + b));
                sigma /= (float)N;
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        const float x = stack[f];
                        if (a * f + b - x > sigma * slo) { crej[0]++; rejected[f] = -1; r++; }
                        else if (x - a * f - b > sigma * shi) { crej[1]++; rejected[f] = 1; r++; }
                        else rejected[f] = 0;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case GESDT: {
            quicksort(stack, N);
            const int lhs = (N - 1) / 2, rhs = N / 2;      // gsl median from sorted data
            median = (lhs == rhs) ? (double)stack[lhs] : (stack[lhs] + stack[rhs]) / 2.0;
            int max_out = (int)((float)nb * p.sig0);
            if (removed >= max_out) return kept;
            max_out -= removed;
            if (max_out > N - 2) max_out = N - 2;   // device bound: the reference is undefined past it
            // ESD records reuse tmp (x) and hist (i | out<<31)
            float *ox = wk.tmp;
            uint32_t *oi = wk.hist;
            for (int j = 0; j < N; j++) { w[j] = stack[j]; rejected[j] = 0; }
            int cold = 0;
            for (int it = 0, size = N; it < max_out; it++, size--) {
                float avg;
                const float s = sd(w, size, &avg);
                float dev = avg - w[0];
                const float d2 = w[size - 1] - avg;
                int im;
                if (d2 > dev) { dev = d2; im = size - 1; } else im = 0;
                const float g = dev / s;
                const int out = g > p.crit[it + removed];
                ox[it] = w[im];
                const int idx = (im == 0) ? cold++ : im;
                oi[it] = (uint32_t)idx | ((uint32_t)out << 31);
                for (int q = im; q < size - 1; q++) w[q] = w[q + 1];
            }
            int i = max_out - 1;                          // confirm_outliers
            while (i > 1 && !(oi[i] >> 31)) i--;
            for (int j = i; j >= 0; j--) {
                const int idx = (int)(oi[j] & 0x7fffffffu);
                if (ox[j] >= median) { rejected[idx] = 1; crej[1]++; }
                else { rejected[idx] = -1; crej[0]++; }
            }
            N = compact(stack, rejected, N);
            break;
        }
        default:
            break;
    }
    return N;
}

// mean_and_reject, float branch (median_and_mean.c:1038-1099)
__device__ double mean_and_reject(const KParams &p, Work &wk, int n, int rej[2], long long pix, int x) {
    const int kept = apply_rejection(p, wk, n, rej, pix, x);
    if (kept == 0) return quickmedian(wk.stack, n);
    if (is_weighted(p)) {
        float pmin = FLT_MAX, pmax = -FLT_MAX;
        for (int f = 0; f < kept; ++f) {
            if (pmin > wk.stack[f]) pmin = wk.stack[f];
            if (pmax < wk.stack[f]) pmax = wk.stack[f];
        }
        double sum = 0.0, norm = 0.0;
        for (int f = 0; f < n; ++f) {
            const float v = wk.o_stack[f];
            if (v >= pmin && v <= pmax && v != 0.f) {
                const double w = sample_weight(p, f, pix, x);
                sum += (double)v * w;
                norm += w;
            }
        }
        if (norm == 0. || sum == 0.) {
            sum = 0.;
            for (int f = 0; f < n; ++f) {
                const float v = wk.o_stack[f];
                if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
            }
            return sum / (double)kept;
        }
        return sum / norm;
    }
    double sum = 0.0;
    for (int f = 0; f < kept; ++f) sum += (double)wk.stack[f];
    return sum / (double)kept;
}

}  // namespace ex

// Per-thread body: `base` is the thread's 6 * N words of scratch (global
// memory or LDS), pixels tid, tid + nthreads, ... of the launch's list.
__device__ __forceinline__ void exact_body(const KParams &p, int all_pixels, float *base, long long tid,
                                           long long nthreads) {
    const int N = p.nframes;
    ex::Work wk;
    wk.stack = base;
    wk.o_stack = base + N;
    wk.w_stack = base + 2LL * N;
    wk.tmp = base + 3LL * N;
    wk.rejected = (int *)(base + 4LL * N);
    wk.hist = (uint32_t *)(base + 5LL * N);
    const long long count = all_pixels ? p.npix : (long long)*p.fb_count;
    unsigned long long c0 = 0, c1 = 0;
    for (long long i = tid; i < count; i += nthreads) {
        const long long pix = all_pixels ? i : (long long)p.fb_list[i];
        const int x = (int)(pix % p.W);
        // the column's N frame reads in groups of 16 in flight (one at a time
        // they were N dependent HBM round trips: most of a deferred N = 400
        // pixel's time)
        for (int f0 = 0; f0 < N; f0 += 16) {
            float g[16];
#pragma unroll
            for (int u = 0; u < 16; u++) g[u] = (f0 + u < N) ? gather_sample(p, f0 + u, pix, x) : 0.f;
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (f0 + u < N) wk.stack[f0 + u] = g[u];
        }
        int rej[2] = {0, 0};
        double res;
        if (p.rtype == KMEDIAN) res = ex::quickmedian(wk.stack, N);
        else res = ex::mean_and_reject(p, wk, N, rej, pix, x);
        write_result(p, pix, res, rej[0], rej[1]);
        c0 += rej[0];
        c1 += rej[1];
    }
    add_counts64(p, c0, c1);
}

// scratch per thread: 6 * N words of the global scratch buffer
__global__ __launch_bounds__(64) void k_stack_exact(KParams p, int all_pixels) {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * blockDim.x;
    if (tid >= p.scratch_threads) return;
    exact_body(p, all_pixels, p.scratch + tid * 6LL * p.nframes, tid, nthreads);
}

// Same with the scratch in LDS (blockDim.x threads x 6 * N words of dynamic
// LDS): every access of the sequential loops (quickselect swaps, sd passes,
// compaction) is an LDS round trip instead of an L2 / HBM one, which is what
// bounds a thread's latency -- a few deferred pixels of a 100-deep column
// took ~2.4 ms with global scratch.
__global__ __launch_bounds__(64) void k_stack_exact_lds(KParams p, int all_pixels) {
    extern __shared__ float lds_scratch[];
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * blockDim.x;
    exact_body(p, all_pixels, lds_scratch + threadIdx.x * 6 * p.nframes, tid, nthreads);
}

// ---------------------------------------------------------------------------
// Small columns (N <= NW = 16 / 32), SIGMA and WINSORIZED: the same
// sequential algorithm with only the array that is indexed by data -- the
// stack quickselect permutes and the rounds compact -- in LDS (N words per
// thread, [slot][thread] so a wave's lanes hit consecutive banks); the
// Winsorized copy w_stack lives in registers (its loops run in index order,
// unrolled to NW with the tail masked), the clip decisions are fused into the
// compaction pass (a decision reads stack[f] before any write reaches f) and
// o_stack is re-gathered for the weighted mean.  At N = 12 the old kernel's
// 6 N words per thread held the CU to 2 waves per SIMD; this one runs at the
// register-bound occupancy (stack dark|bias rej 3 3 masters, where a low
// sigma leaves the cutoff order-dependent for a third of the pixels).
namespace exs {

// strided LDS view of one thread's stack
struct SV {
    float *b;
    int t;
    __device__ __forceinline__ float &operator[](int i) const { return b[i * t]; }
};

__device__ __forceinline__ double quickmedian(SV a, int n) {     // sorting.c:240-273, 468-513
    if (n < 9) {
        const int k = n / 2;
        if (n == 1) return a[0];
        if (n < 2) return 0.0;
        const unsigned char *pn = ex::kNet + 2 * ex::kNetOff[n];
        for (int c = 0; c < ex::kNetLen[n]; c++) {
            const int i = pn[2 * c], j = pn[2 * c + 1];
            const float ai = a[i], aj = a[j];
            if (ai > aj) { a[i] = aj; a[j] = ai; }
        }
        return (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
    }
    const int k = n / 2;
    int left = 0, right = n - 1;
    while (left < right) {
        int q = (left + right) / 2;
        const float pivot = a[q];
        a[q] = a[right];
        a[right] = pivot;
        q = left;
        for (int i = left; i < right; i++) {
            const float ai = a[i];
            if (ai < pivot) {
                a[i] = a[q];
                a[q] = ai;
                q++;
            }
        }
        a[right] = a[q];
        a[q] = pivot;
        if (q < k) left = q + 1;
        else right = q;
    }
    return (n % 2 == 0) ? ((double)a[k - 1] + a[k]) / 2.0 : (double)a[k];
}

__device__ __forceinline__ float sd_lds(SV x, int n) {            // statistics.h:80-106
    double s = 0.0, q = 0.0;
    for (int i = 0; i < n; i++) s += (double)x[i];
    const float mean = (float)(s / n);
    for (int i = 0; i < n; i++) {
        const float d = x[i] - mean;
        q += (double)(d * d);
    }
    return sqrtf((float)(q / (n - 1)));
}

template <int NW>
__device__ __forceinline__ float sd_reg(const float (&w)[NW], int n) {
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int i = 0; i < NW; i++)
        if (i < n) s += (double)w[i];
    const float mean = (float)(s / n);
#pragma unroll
    for (int i = 0; i < NW; i++)
        if (i < n) {
            const float d = w[i] - mean;
            q += (double)(d * d);
        }
    return sqrtf((float)(q / (n - 1)));
}

// one rejection round's clip decisions fused with the compaction
__device__ __forceinline__ int clip_compact(SV a, int n, int &r, float s, float slo, float shi, float m,
                                            int crej[2]) {
    int o = 0;
    for (int f = 0; f < n; f++) {
        const float x = a[f];
        int rej = 0;
        if (!(n - r <= 4)) {
            rej = ex::sclip(x, s, slo, shi, m, crej);
            if (rej) r++;
        }
        if (!rej) a[o++] = x;
    }
    return o;
}

template <int NW>
__device__ int apply_rejection(const KParams &p, SV stack, int nb, int crej[2], long long pix, int x) {
    int N = nb, r = 0, kept = 0;
    const float slo = p.sig0, shi = p.sig1;
    for (int f = 0; f < N; f++) {                       // :116-136
        const float v = stack[f];
        if (v != 0.f && (!p.drizz || plane_at(p, p.drizz, f, pix, x) != 0.f)) {
            if (f != kept) stack[kept] = v;
            kept++;
        }
    }
    if (kept <= 1) return kept;
    N = kept;
    bool changed;
    if (p.rtype == PERCENTILE) {                        // :147-173
        const double median = quickmedian(stack, N);
        if (median == 0.0) return 0;
        const float mf = (float)median;
        int o = 0;
        for (int f = 0; f < N; f++) {
            const float x = stack[f];
            int rej = 0;
            if (mf - x > mf * slo) { crej[0]++; rej = 1; }
            else if (x - mf > mf * shi) { crej[1]++; rej = 1; }
            if (!rej) stack[o++] = x;
        }
        return o;
    }
    if (p.rtype == SIGMEDIAN) {                         // :210-222 (no compaction)
        int it = 0, nrep;
        do {
            const float sigma = sd_lds(stack, N);
            const float mf = (float)quickmedian(stack, N);
            nrep = 0;
            for (int f = 0; f < N; f++)
                if (ex::sclip(stack[f], sigma, slo, shi, mf, crej)) {
                    stack[f] = mf;
                    nrep++;
                }
        } while (nrep > 0 && ++it < 100000);
        return N;
    }
    if (p.rtype == SIGMA) {                             // :147-157, 174-209
        double median = quickmedian(stack, N);
        if (median == 0.0) return 0;
        bool firstloop = true;
        do {
            const float var = sd_lds(stack, N);
            if (!firstloop) median = quickmedian(stack, N);
            firstloop = false;
            const int out = clip_compact(stack, N, r, var, slo, shi, (float)median, crej);
            changed = N != out;
            N = out;
        } while (changed && N > 3);
    } else {                                            // WINSORIZED, :223-259
        float w[NW];
        do {
            float sigma0, sigma = sd_lds(stack, N);
            const float mf = (float)quickmedian(stack, N);
#pragma unroll
            for (int j = 0; j < NW; j++) w[j] = j < N ? stack[j] : 0.f;
            int it = 0;
            do {
                const float m0 = mf - 1.5f * sigma, m1 = mf + 1.5f * sigma;
#pragma unroll
                for (int j = 0; j < NW; j++) {
                    const float a = (m0 > w[j]) ? m0 : w[j];
                    w[j] = (m1 < a) ? m1 : a;
                }
                sigma0 = sigma;
                sigma = 1.134f * sd_reg<NW>(w, N);
            } while (fabsf(sigma - sigma0) > sigma0 * 0.0005f && ++it < 100000);
            const int out = clip_compact(stack, N, r, sigma, slo, shi, mf, crej);
            changed = N != out;
            N = out;
        } while (changed && N > 3);
    }
    return N;
}

template <int NW>
__device__ double mean_and_reject(const KParams &p, SV stack, int n, int rej[2], long long pix, int x) {
    const int kept = apply_rejection<NW>(p, stack, n, rej, pix, x);
    if (kept == 0) return quickmedian(stack, n);        // median_and_mean.c:1040
    if (is_weighted(p)) {                               // :1043-1082, o_stack re-gathered
        float pmin = FLT_MAX, pmax = -FLT_MAX;
        for (int f = 0; f < kept; ++f) {
            const float v = stack[f];
            if (pmin > v) pmin = v;
            if (pmax < v) pmax = v;
        }
        double sum = 0.0, norm = 0.0;
        for (int f = 0; f < n; ++f) {
            const float v = gather_sample(p, f, pix, x);
            if (v >= pmin && v <= pmax && v != 0.f) {
                const double w = sample_weight(p, f, pix, x);
                sum += (double)v * w;
                norm += w;
            }
        }
        if (norm == 0. || sum == 0.) {
            sum = 0.;
            for (int f = 0; f < n; ++f) {
                const float v = gather_sample(p, f, pix, x);
                if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
            }
            return sum / (double)kept;
        }
        return sum / norm;
    }
    double sum = 0.0;
    for (int f = 0; f < kept; ++f) sum += (double)stack[f];
    return sum / (double)kept;
}

}  // namespace exs

template <int NW>
__global__ __launch_bounds__(64) void k_stack_exact_small(KParams p, int all_pixels) {
    extern __shared__ float lds_stack[];
    const int T = blockDim.x;
    const long long tid = (long long)blockIdx.x * T + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * T;
    const exs::SV stack{lds_stack + threadIdx.x, T};
    const int N = p.nframes;
    const long long count = all_pixels ? p.npix : (long long)*p.fb_count;
    unsigned long long c0 = 0, c1 = 0;
    for (long long i = tid; i < count; i += nthreads) {
        const long long pix = all_pixels ? i : (long long)p.fb_list[i];
        const int x = (int)(pix % p.W);
        for (int f = 0; f < N; f++) stack[f] = gather_sample(p, f, pix, x);
        int rej[2] = {0, 0};
        const double res = exs::mean_and_reject<NW>(p, stack, N, rej, pix, x);
        write_result(p, pix, res, rej[0], rej[1]);
        c0 += rej[0];
        c1 += rej[1];
    }
    add_counts64(p, c0, c1);
}
template __global__ void k_stack_exact_small<16>(KParams, int);
template __global__ void k_stack_exact_small<32>(KParams, int);

}  // namespace sgpu

// ====================================================================== 16-bit
// DATA_USHORT: apply_rejection_ushort (median_and_mean.c:703-954) and the
// ushort branch of mean_and_reject (:961-1036), sequential per pixel.
namespace sgpu {
namespace ex16 {

typedef uint16_t WORD;

__device__ __forceinline__ void swapw(WORD &a, WORD &b) { WORD t = a; a = b; b = t; }

__constant__ unsigned char kNet9[] = {1,8, 2,7, 3,6, 4,5, 1,4, 5,8, 0,2, 6,7, 2,6, 7,8, 0,3, 4,5,
                                      0,1, 3,5, 6,7, 2,4, 1,3, 5,7, 4,6, 1,2, 3,4, 5,6, 7,8, 2,3, 4,5};

__device__ double sortnet_median(WORD *a, int n) {      // sorting.c:366-410
    const int k = n / 2;
    if (n == 1) return a[0];
    if (n < 2 || n > 9) return 0.0;
    const unsigned char *p = (n == 9) ? kNet9 : ex::kNet + 2 * ex::kNetOff[n];
    const int len = (n == 9) ? 25 : ex::kNetLen[n];
    for (int c = 0; c < len; c++) {
        const int i = p[2 * c], j = p[2 * c + 1];
        if (a[i] > a[j]) swapw(a[i], a[j]);
    }
    return (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
}

__device__ double quickmedian(WORD *a, int n) {         // sorting.c:195-230
    if (n < 9) return sortnet_median(a, n);
    const int k = n / 2;
    int left = 0, right = n - 1;
    while (left < right) {
        int p = (left + right) / 2;
        const WORD pivot = a[p];
        a[p] = a[right];
        a[right] = pivot;
        p = left;
        for (int i = left; i < right; i++)
            if (a[i] < pivot) { swapw(a[p], a[i]); p++; }
        a[right] = a[p];
        a[p] = pivot;
        if (p < k) left = p + 1;
        else right = p;
    }
    return (n % 2 == 0) ? ((double)a[k - 1] + (double)a[k]) / 2.0 : (double)a[k];
}

__device__ void sort(WORD *a, int n) {                   // quicksort_s: result is the sorted array
    for (int i = 1; i < n; i++) {                        // (insertion sort; equal keys are identical)
        const WORD v = a[i];
        int j = i - 1;
        while (j >= 0 && a[j] > v) { a[j + 1] = a[j]; --j; }
        a[j + 1] = v;
    }
}

// histogram_median (sorting.c:577-642) on a scratch copy: exact order
// statistics of the values; sortnet below 10 elements (permutes `a`).
__device__ double histogram_median(WORD *a, int n, WORD *tmp) {
    if (n < 10) return sortnet_median(a, n);
    for (int i = 0; i < n; i++) tmp[i] = a[i];
    sort(tmp, n);
    const int k = n / 2;
    return (n % 2 == 0) ? (double)((int)tmp[k - 1] + (int)tmp[k]) / 2.0 : (double)tmp[k];
}

__device__ float sd32(const WORD *d, int n) {            // siril_stats_ushort_sd_32, statistics.c:115-127
    uint32_t isum = 0;
    for (int i = 0; i < n; ++i) isum += d[i];
    const float mean = (float)(((double)isum) / ((double)n));
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
        const float px = (float)d[i];
        acc += (px - mean) * (px - mean);
    }
    return sqrtf((float)(acc / (n - 1)));
}

__device__ float sd_m(const WORD *d, int n, float *m) {  // median_and_mean.c:647-660
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += d[i];
    const float mean = (float)(acc / n);
    acc = 0.0;
    for (int i = 0; i < n; ++i) acc += (d[i] - mean) * (d[i] - mean);
    if (m) *m = mean;
    return sqrtf((float)(acc / (n - 1)));
}

__device__ int round_to_int(double x) {                  // proto.h:208-213
    x = (x > 2147483647.0 - 0.5) ? 2147483647.0 - 0.5 : x;
    x = (x < -2147483648.0 + 0.5) ? -2147483648.0 + 0.5 : x;
    return (int)(x + ((x >= 0.0) ? 0.5 : -0.5));
}
__device__ WORD roundf_to_word(float f) {                // proto.h:341-346
    f = f + 0.5f;
    f = (f > 65535.f) ? 65535.f : f;
    f = (f < 0.0f) ? 0.0f : f;
    return (WORD)f;
}
__device__ WORD round_to_word(double x) {                // proto.h:232-237
    x = x + 0.5;
    x = (x > 65535.0) ? 65535.0 : x;
    x = (x < 0.0) ? 0.0 : x;
    return (WORD)x;
}

__device__ float mad(const WORD *d, int n, double m, WORD *tmp, WORD *tmp2) {   // statistics.c:133-154
    const int med = round_to_int(m);
    for (int i = 0; i < n; i++) tmp[i] = (WORD)abs((int)d[i] - med);
    return (float)histogram_median(tmp, n, tmp2);
}

__device__ __forceinline__ int sclip(WORD x, float slo, float shi, float s, float m, int rej[2]) {
    if (m - x > slo * s) { rej[0]++; return -1; }
    if (x - m > shi * s) { rej[1]++; return 1; }
    return 0;
}

__device__ int compact(WORD *s, const int *rej, int n) {
    int o = 0;
    for (int p = 0; p < n; p++)
        if (!rej[p]) s[o++] = s[p];
    return o;
}

struct Work {
    WORD *stack, *o_stack, *w_stack, *tmp, *tmp2;
    float *yf;
    int *rejected;
};

__device__ int apply_rejection(const KParams &p, Work &wk, int nb, int crej[2], long long pix, int x) {
    int N = nb, r = 0, firstloop = 1, kept = 0, changed, n;
    float median = 0.f;
    WORD *stack = wk.stack, *w = wk.w_stack;
    int *rejected = wk.rejected;
    const float slo = p.sig0, shi = p.sig1;
    for (int f = 0; f < N; f++) wk.o_stack[f] = stack[f];
    for (int f = 0; f < N; f++)
        if (stack[f] != 0 && (!p.drizz || plane_at(p, p.drizz, f, pix, x) != 0.f)) {   // median_and_mean.c:716-731
            if (f != kept) stack[kept] = stack[f];
            kept++;
        }
    if (kept <= 1) return kept;
    const int removed = N - kept;
    N = kept;
    switch (p.rtype) {
        case PERCENTILE: case SIGMA: case MAD: case SIGMEDIAN: case WINSORIZED:
            median = (float)quickmedian(stack, N);
            if (median == 0.f) return 0;
            break;
        default: break;
    }
    switch (p.rtype) {
        case PERCENTILE:
            for (int f = 0; f < N; f++) {
                const WORD x = stack[f];
                if ((median - (float)x) / median > slo) { crej[0]++; rejected[f] = -1; }
                else if (((float)x - median) / median > shi) { crej[1]++; rejected[f] = 1; }
                else rejected[f] = 0;
            }
            N = compact(stack, rejected, N);
            break;
        case SIGMA: case MAD:
            do {
                float var;
                if (p.rtype == SIGMA) var = sd32(stack, N);
                else var = mad(stack, N, median, wk.tmp, wk.tmp2);
                if (!firstloop) median = (float)quickmedian(stack, N);
                else firstloop = 0;
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        rejected[f] = sclip(stack[f], slo, shi, var, median, crej);
                        if (rejected[f]) r++;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case SIGMEDIAN: {
            int it = 0;
            do {
                const float sigma = sd32(stack, N);
                if (!firstloop) median = (float)quickmedian(stack, N);
                else firstloop = 0;
                n = 0;
                for (int f = 0; f < N; f++)
                    if (sclip(stack[f], slo, shi, sigma, median, crej)) { stack[f] = (WORD)median; n++; }
            } while (n > 0 && ++it < 100000);
            break;
        }
        case WINSORIZED:
            do {
                float sigma0, sigma = sd32(stack, N);
                if (!firstloop) median = (float)quickmedian(stack, N);
                else firstloop = 0;
                for (int j = 0; j < N; j++) w[j] = stack[j];
                int it = 0;
                do {
                    const WORD m0 = roundf_to_word(median - 1.5f * sigma);
                    const WORD m1 = roundf_to_word(median + 1.5f * sigma);
                    for (int j = 0; j < N; ++j) {
                        w[j] = w[j] < m0 ? m0 : w[j];
                        w[j] = w[j] > m1 ? m1 : w[j];
                    }
                    sigma0 = sigma;
                    sigma = 1.134f * sd32(w, N);
                } while (fabs(sigma - sigma0) > sigma0 * 0.0005f && ++it < 100000);
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        rejected[f] = sclip(stack[f], slo, shi, sigma, median, crej);
                        if (rejected[f] != 0) r++;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case LINEARFIT:
            do {
                sort(stack, N);
                for (int f = 0; f < N; f++) wk.yf[f] = (float)stack[f];
                float m_y = wk.yf[0];
                for (int i = 1; i < N; i++) m_y += (wk.yf[i] - m_y) * (1.f / (i + 1));
                float m_dxdy = 0.f, dx = -p.m_x;
                for (int i = 0; i < N; i++, dx += 1.f) {
                    const float dy = wk.yf[i] - m_y;
                    m_dxdy += (dx * dy - m_dxdy) * (1.f / (i + 1));
                }
                const float a = m_dxdy * p.m_dx2;
                const float b = m_y - p.m_x * a;
                float sigma = 0.f;
                for (int f = 0; f < N; f++) sigma += fabsf(stack[f] - (a * f + b));
                sigma /= (float)N;
                for (int f = 0; f < N; f++) {
                    if (N - r <= 4) rejected[f] = 0;
                    else {
                        const WORD x = stack[f];
                        if (a * f + b - x > sigma * slo) { crej[0]++; rejected[f] = -1; r++; }
                        else if (x - a * f - b > sigma * shi) { crej[1]++; rejected[f] = 1; r++; }
                        else rejected[f] = 0;
                    }
                }
                const int out = compact(stack, rejected, N);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        case GESDT: {
            sort(stack, N);
            {
                const int lhs = (N - 1) / 2, rhs = N / 2;
                median = (lhs == rhs) ? (float)stack[lhs] : (float)((stack[lhs] + stack[rhs]) / 2.0);
            }
            int max_out = (int)((float)nb * p.sig0);
            if (removed >= max_out) return kept;
            max_out -= removed;
            if (max_out > N - 2) max_out = N - 2;
            float *ox = (float *)wk.yf;
            int *oi = (int *)wk.tmp;      // tmp + tmp2 give N ints of room
            for (int j = 0; j < N; j++) { w[j] = stack[j]; rejected[j] = 0; }
            int cold = 0;
            for (int it = 0, size = N; it < max_out; it++, size--) {
                float avg;
                const float s = sd_m(w, size, &avg);
                float dev = avg - w[0];
                const float d2 = w[size - 1] - avg;
                int im;
                if (d2 > dev) { dev = d2; im = size - 1; } else im = 0;
                const float g = dev / s;
                const int out = g > p.crit[it + removed];
                ox[it] = w[im];
                const int idx = (im == 0) ? cold++ : im;
                oi[it] = idx | (out << 30);
                for (int q = im; q < size - 1; q++) w[q] = w[q + 1];
            }
            int i = max_out - 1;
            while (i > 1 && !((oi[i] >> 30) & 1)) i--;
            const double md = median;
            for (int j = i; j >= 0; j--) {
                const int idx = oi[j] & 0x3fffffff;
                if (ox[j] >= md) { rejected[idx] = 1; crej[1]++; }
                else { rejected[idx] = -1; crej[0]++; }
            }
            N = compact(stack, rejected, N);
            break;
        }
        default:
            break;
    }
    return N;
}

__device__ double mean_and_reject(const KParams &p, Work &wk, int n, int rej[2], long long pix, int x) {
    const int kept = apply_rejection(p, wk, n, rej, pix, x);
    if (kept == 0) return quickmedian(wk.stack, n);
    if (is_weighted(p)) {
        WORD pmin = 65535, pmax = 0;
        for (int f = 0; f < kept; ++f) {
            const WORD px = wk.stack[f];
            if (pmin > px) pmin = px;
            if (pmax < px) pmax = px;
        }
        double sum = 0.0, norm = 0.0;
        for (int f = 0; f < n; ++f) {
            const WORD v = wk.o_stack[f];
            if (v >= pmin && v <= pmax && v > 0) {
                const double w = sample_weight(p, f, pix, x);
                sum += (double)v * w;
                norm += w;
            }
        }
        if (norm == 0. || sum == 0.) {
            sum = 0.;
            for (int f = 0; f < n; ++f) {
                const WORD v = wk.o_stack[f];
                if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
            }
            return sum / (double)kept;
        }
        return sum / norm;
    }
    long long sum = 0;
    for (int f = 0; f < kept; ++f) sum += wk.stack[f];
    return sum / (double)kept;
}

// one normalized 16-bit sample, median_and_mean.c:1615-1686 (round_to_WORD)
__device__ WORD gather16(const KParams &p, int f, long long pix, int x) {
    long long idx = pix;
    if (p.shiftx) {
        const int s = p.shiftx[f];
        if (s && (x - s >= p.W || x - s < 0)) return 0;
        idx -= s;
    }
    const WORD v = p.frames16[(long long)f * p.frame_stride + idx];
    switch (p.norm) {
        default:
        case NO_NORM: return v;
        case ADDITIVE: case ADDITIVE_SCALING:
            if (v > 0) return round_to_word((double)v * p.scale[f] - p.offset[f]);
            return 0;
        case MULTIPLICATIVE: case MULTIPLICATIVE_SCALING:
            return round_to_word((double)v * p.scale[f] * p.mul[f]);
    }
}

}  // namespace ex16

// 16-bit sequences through the sequential path: every pixel (all_pixels) or
// the pixels the 16-bit sorted path deferred (fb_list); scratch per thread =
// 6 * N words (WORD stack/o_stack/w_stack/tmp/tmp2 + float yf + int rejected)
__device__ __forceinline__ void exact16_body(const KParams &p, int all_pixels, float *base, long long tid,
                                             long long nthreads) {
    const int N = p.nframes;
    ex16::Work wk;
    ex16::WORD *wb = (ex16::WORD *)base;           // 5 WORD arrays in 2.5 N words
    wk.stack = wb;
    wk.o_stack = wb + N;
    wk.w_stack = wb + 2LL * N;
    wk.tmp = wb + 3LL * N;
    wk.tmp2 = wb + 4LL * N;
    wk.yf = base + 3LL * N;
    wk.rejected = (int *)(base + 4LL * N);
    unsigned long long c0 = 0, c1 = 0;
    const long long count = all_pixels ? p.npix : (long long)*p.fb_count;
    for (long long i = tid; i < count; i += nthreads) {
        const long long pix = all_pixels ? i : (long long)p.fb_list[i];
        const int x = (int)(pix % p.W);
        for (int f0 = 0; f0 < N; f0 += 16) {       // 16 frame reads in flight (as exact_body)
            ex16::WORD g[16];
#pragma unroll
            for (int u = 0; u < 16; u++) g[u] = (f0 + u < N) ? ex16::gather16(p, f0 + u, pix, x) : (ex16::WORD)0;
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (f0 + u < N) wk.stack[f0 + u] = g[u];
        }
        int rej[2] = {0, 0};
        double res;
        if (p.rtype == KMEDIAN) res = ex16::quickmedian(wk.stack, N);
        else res = ex16::mean_and_reject(p, wk, N, rej, pix, x);
        if (p.out_f32) {
            float fr = (float)res * .000015259022f;          // double_ushort_to_float_range
            if (!p.output_norm) {
                fr = (fr < 0.f) ? 0.f : fr;
                fr = (fr > 1.f) ? 1.f : fr;
            }
            p.out[pix] = fr;
        }
        if (p.out16) p.out16[pix] = ex16::round_to_word(res * p.out16_mul);   // normalize_to16bit
        if (p.rej_lo) p.rej_lo[pix] = (uint16_t)(rej[0] > 65535 ? 65535 : rej[0]);
        if (p.rej_hi) p.rej_hi[pix] = (uint16_t)(rej[1] > 65535 ? 65535 : rej[1]);
        c0 += rej[0];
        c1 += rej[1];
    }
    add_counts64(p, c0, c1);
}

__global__ __launch_bounds__(64) void k_stack_exact16(KParams p, int all_pixels) {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * blockDim.x;
    if (tid >= p.scratch_threads) return;
    exact16_body(p, all_pixels, p.scratch + tid * 6LL * p.nframes, tid, nthreads);
}

__global__ __launch_bounds__(64) void k_stack_exact16_lds(KParams p, int all_pixels) {
    extern __shared__ float lds_scratch[];
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * blockDim.x;
    exact16_body(p, all_pixels, lds_scratch + threadIdx.x * 6 * p.nframes, tid, nthreads);
}

}  // namespace sgpu

// ---------------------------------------------------------------------------
// Small 16-bit columns (N <= NW), SIGMA and WINSORIZED: k_stack_exact_small's
// layout for apply_rejection_ushort (median_and_mean.c:703-954): the WORD
// stack in LDS (one word per slot: the dword array holds the sample widened),
// w_stack in registers, clip decisions fused into the compaction, o_stack
// re-gathered for the weighted mean; the ushort rules (initial median == 0
// for both types, sd32, roundf_to_WORD Winsorize bounds, integer mean).
namespace sgpu {
namespace exs16 {

typedef uint16_t WORD;

struct SVW {
    unsigned *b;
    int t;
    struct Ref {
        unsigned *q;
        __device__ __forceinline__ operator WORD() const { return (WORD)*q; }
        __device__ __forceinline__ Ref &operator=(WORD v) { *q = v; return *this; }
        __device__ __forceinline__ Ref &operator=(const Ref &o) { *q = *o.q; return *this; }
    };
    __device__ __forceinline__ Ref operator[](int i) const { return Ref{b + i * t}; }
};

__device__ __forceinline__ double quickmedian(SVW a, int n) {     // sorting.c:195-230, 366-410
    if (n < 9) {
        const int k = n / 2;
        if (n == 1) return (WORD)a[0];
        if (n < 2) return 0.0;
        const unsigned char *pn = ex::kNet + 2 * ex::kNetOff[n];
        for (int c = 0; c < ex::kNetLen[n]; c++) {
            const int i = pn[2 * c], j = pn[2 * c + 1];
            const WORD ai = a[i], aj = a[j];
            if (ai > aj) { a[i] = aj; a[j] = ai; }
        }
        return (n % 2 == 0) ? ((WORD)a[k - 1] + (WORD)a[k]) / 2.0 : (double)(WORD)a[k];
    }
    const int k = n / 2;
    int left = 0, right = n - 1;
    while (left < right) {
        int q = (left + right) / 2;
        const WORD pivot = a[q];
        a[q] = (WORD)a[right];
        a[right] = pivot;
        q = left;
        for (int i = left; i < right; i++) {
            const WORD ai = a[i];
            if (ai < pivot) {
                a[i] = (WORD)a[q];
                a[q] = ai;
                q++;
            }
        }
        a[right] = (WORD)a[q];
        a[q] = pivot;
        if (q < k) left = q + 1;
        else right = q;
    }
    return (n % 2 == 0) ? ((double)(WORD)a[k - 1] + (double)(WORD)a[k]) / 2.0 : (double)(WORD)a[k];
}

__device__ __forceinline__ float sd32_lds(SVW d, int n) {           // statistics.c:115-127
    uint32_t isum = 0;
    for (int i = 0; i < n; ++i) isum += (WORD)d[i];
    const float mean = (float)(((double)isum) / ((double)n));
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
        const float px = (float)(WORD)d[i];
        acc += (px - mean) * (px - mean);
    }
    return sqrtf((float)(acc / (n - 1)));
}

template <int NW>
__device__ __forceinline__ float sd32_reg(const unsigned (&w)[NW], int n) {
    uint32_t isum = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i)
        if (i < n) isum += w[i];
    const float mean = (float)(((double)isum) / ((double)n));
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i)
        if (i < n) {
            const float px = (float)w[i];
            acc += (px - mean) * (px - mean);
        }
    return sqrtf((float)(acc / (n - 1)));
}

__device__ __forceinline__ int clip_compact(SVW a, int n, int &r, float s, float slo, float shi, float m,
                                            int crej[2]) {
    int o = 0;
    for (int f = 0; f < n; f++) {
        const WORD x = a[f];
        int rej = 0;
        if (!(n - r <= 4)) {
            rej = ex16::sclip(x, slo, shi, s, m, crej);
            if (rej) r++;
        }
        if (!rej) a[o++] = x;
    }
    return o;
}

template <int NW>
__device__ int apply_rejection(const KParams &p, SVW stack, int nb, int crej[2], long long pix, int x) {
    int N = nb, r = 0, kept = 0;
    const float slo = p.sig0, shi = p.sig1;
    for (int f = 0; f < N; f++) {                       // :716-731
        const WORD v = stack[f];
        if (v != 0 && (!p.drizz || plane_at(p, p.drizz, f, pix, x) != 0.f)) {
            if (f != kept) stack[kept] = v;
            kept++;
        }
    }
    if (kept <= 1) return kept;
    N = kept;
    float median = (float)quickmedian(stack, N);        // :747-756
    if (median == 0.f) return 0;
    bool firstloop = true, changed;
    if (p.rtype == PERCENTILE) {                        // :758-771 (the WORD division form)
        int o = 0;
        for (int f = 0; f < N; f++) {
            const WORD x = stack[f];
            int rej = 0;
            if ((median - (float)x) / median > slo) { crej[0]++; rej = 1; }
            else if (((float)x - median) / median > shi) { crej[1]++; rej = 1; }
            if (!rej) stack[o++] = x;
        }
        return o;
    }
    if (p.rtype == SIGMEDIAN) {                         // :800-829: the median written back as a WORD
        int it = 0, nrep;
        do {
            const float sigma = sd32_lds(stack, N);
            if (!firstloop) median = (float)quickmedian(stack, N);
            firstloop = false;
            nrep = 0;
            for (int f = 0; f < N; f++)
                if (ex16::sclip((WORD)stack[f], slo, shi, sigma, median, crej)) {
                    stack[f] = (WORD)median;
                    nrep++;
                }
        } while (nrep > 0 && ++it < 100000);
        return N;
    }
    if (p.rtype == SIGMA) {                             // :758-786
        do {
            const float var = sd32_lds(stack, N);
            if (!firstloop) median = (float)quickmedian(stack, N);
            firstloop = false;
            const int out = clip_compact(stack, N, r, var, slo, shi, median, crej);
            changed = N != out;
            N = out;
        } while (changed && N > 3);
    } else {                                            // WINSORIZED, :830-873
        unsigned w[NW];
        do {
            float sigma0, sigma = sd32_lds(stack, N);
            if (!firstloop) median = (float)quickmedian(stack, N);
            firstloop = false;
#pragma unroll
            for (int j = 0; j < NW; j++) w[j] = j < N ? (unsigned)(WORD)stack[j] : 0u;
            int it = 0;
            do {
                const unsigned m0 = ex16::roundf_to_word(median - 1.5f * sigma);
                const unsigned m1 = ex16::roundf_to_word(median + 1.5f * sigma);
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    w[j] = w[j] < m0 ? m0 : w[j];
                    w[j] = w[j] > m1 ? m1 : w[j];
                }
                sigma0 = sigma;
                sigma = 1.134f * sd32_reg<NW>(w, N);
            } while (fabs(sigma - sigma0) > sigma0 * 0.0005f && ++it < 100000);
            const int out = clip_compact(stack, N, r, sigma, slo, shi, median, crej);
            changed = N != out;
            N = out;
        } while (changed && N > 3);
    }
    return N;
}

template <int NW>
__device__ double mean_and_reject(const KParams &p, SVW stack, int n, int rej[2], long long pix, int x) {
    const int kept = apply_rejection<NW>(p, stack, n, rej, pix, x);
    if (kept == 0) return quickmedian(stack, n);
    if (is_weighted(p)) {
        WORD pmin = 65535, pmax = 0;
        for (int f = 0; f < kept; ++f) {
            const WORD px = stack[f];
            if (pmin > px) pmin = px;
            if (pmax < px) pmax = px;
        }
        double sum = 0.0, norm = 0.0;
        for (int f = 0; f < n; ++f) {
            const WORD v = ex16::gather16(p, f, pix, x);
            if (v >= pmin && v <= pmax && v > 0) {
                const double w = sample_weight(p, f, pix, x);
                sum += (double)v * w;
                norm += w;
            }
        }
        if (norm == 0. || sum == 0.) {
            sum = 0.;
            for (int f = 0; f < n; ++f) {
                const WORD v = ex16::gather16(p, f, pix, x);
                if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
            }
            return sum / (double)kept;
        }
        return sum / norm;
    }
    long long sum = 0;
    for (int f = 0; f < kept; ++f) sum += (WORD)stack[f];
    return sum / (double)kept;
}

}  // namespace exs16

template <int NW>
__global__ __launch_bounds__(64) void k_stack_exact16_small(KParams p, int all_pixels) {
    extern __shared__ unsigned lds_w[];
    const int T = blockDim.x;
    const long long tid = (long long)blockIdx.x * T + threadIdx.x;
    const long long nthreads = (long long)gridDim.x * T;
    const exs16::SVW stack{lds_w + threadIdx.x, T};
    const int N = p.nframes;
    const long long count = all_pixels ? p.npix : (long long)*p.fb_count;
    unsigned long long c0 = 0, c1 = 0;
    for (long long i = tid; i < count; i += nthreads) {
        const long long pix = all_pixels ? i : (long long)p.fb_list[i];
        const int x = (int)(pix % p.W);
        for (int f = 0; f < N; f++) stack[f] = ex16::gather16(p, f, pix, x);
        int rej[2] = {0, 0};
        const double res = exs16::mean_and_reject<NW>(p, stack, N, rej, pix, x);
        if (p.out_f32) {
            float fr = (float)res * .000015259022f;          // double_ushort_to_float_range
            if (!p.output_norm) {
                fr = (fr < 0.f) ? 0.f : fr;
                fr = (fr > 1.f) ? 1.f : fr;
            }
            p.out[pix] = fr;
        }
        if (p.out16) p.out16[pix] = ex16::round_to_word(res * p.out16_mul);   // normalize_to16bit
        if (p.rej_lo) p.rej_lo[pix] = (uint16_t)(rej[0] > 65535 ? 65535 : rej[0]);
        if (p.rej_hi) p.rej_hi[pix] = (uint16_t)(rej[1] > 65535 ? 65535 : rej[1]);
        c0 += rej[0];
        c1 += rej[1];
    }
    add_counts64(p, c0, c1);
}
template __global__ void k_stack_exact16_small<16>(KParams, int);
template __global__ void k_stack_exact16_small<32>(KParams, int);

}  // namespace sgpu

// fold the striped per-wave rejection totals of one launch into `counts`
// (sgpu_kparams.h kCountStripes; sgpu_capi.cpp run_launch)
namespace sgpu {
__global__ __launch_bounds__(256) void k_fold_counts(const unsigned long long *stripes, unsigned long long *counts) {
    unsigned long long a = 0, b = 0;
    for (int i = threadIdx.x; i < kCountStripes; i += blockDim.x) {
        a += stripes[(size_t)i * 8];
        b += stripes[(size_t)i * 8 + 1];
    }
    __shared__ unsigned long long sa[256], sbb[256];
    sa[threadIdx.x] = a;
    sbb[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            sa[threadIdx.x] += sa[threadIdx.x + o];
            sbb[threadIdx.x] += sbb[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counts[0] += sa[0];
        counts[1] += sbb[0];
    }
}
}  // namespace sgpu
