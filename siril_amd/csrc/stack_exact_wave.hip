// stack_exact_wave.hip -- the exact sequential path with a whole WAVE per
// deferred pixel (SIGMA, WINSORIZED, PERCENTILE and the median stack, N of
// 33..1024).
//
// The one-thread kernel (stack_exact.hip) runs the reference's loops on one
// lane: every step of quickmedian_float's Lomuto partition, of the clip loop
// and of the compaction is a dependent LDS round trip, ~1.1 ms for one
// deferred 400-frame SIGMA pixel (config 4's whole exact tail, since all of
// its few pixels run side by side).  Here the 64 lanes of a wave share one
// column in LDS and reproduce the same permutations with data-parallel steps:
//   * compaction (zeros, rejected samples): stable, by ballot prefix counts;
//   * the clip loop's `N - r <= 4` cutoff (rejection_float.c:188): sample f
//     is rejected iff it is a candidate and r0 + (candidates before f) <
//     N - 4, a prefix count again;
//   * Lomuto's partition (sorting.c:257-263) as a closed form: the samples
//     below the pivot keep their order at the front; the block of the others
//     is a queue that every later small sample rotates by one, so its final
//     content is read off a tape T (T[q] = the large sample of step j0 + q,
//     or T[h] for a small step that found h small steps before it since the
//     first large one j0) whose references are resolved by pointer jumping
//     (log2 rounds);
//   * the f64 sums (statistics.h:80-106 sd, the means) stay sequential on
//     lane 0 in the reference's order -- they are the ones order matters for.
// Same results as the one-thread kernel bit for bit (the permutation of every
// pass, hence every later sum order and cutoff, is the reference's).
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include "sgpu_kparams.h"
#include "stack_sorted_impl.h"

namespace sgpu {
namespace exw {

constexpr int kMaxC = 16;        // samples per lane: N <= 1024

// diagnostic build (-DSGPU_EXW_PROF=1): per-phase cycles of the first pixel
// of block 0, printed by its lane 0 -- [0] gather [1] null compaction
// [2] quickmedian [3] sd [4] clip + compaction [5] mean; [6] partition passes
// [7] pointer-jumping rounds
#ifndef SGPU_EXW_PROF
#define SGPU_EXW_PROF 0
#endif
#if SGPU_EXW_PROF
__device__ unsigned long long g_exw_prof[8];
#define EXW_T0() const unsigned long long exw_t0_ = __builtin_readcyclecounter()
#define EXW_ON() (blockIdx.x == 0 && (threadIdx.x & 63) == 0)
#define EXW_ACC(k) do { if (EXW_ON()) sgpu::exw::g_exw_prof[k] += __builtin_readcyclecounter() - exw_t0_; } while (0)
#define EXW_CNT(k) do { if (EXW_ON()) sgpu::exw::g_exw_prof[k] += 1; } while (0)
#else
#define EXW_T0() ((void)0)
#define EXW_ACC(k) ((void)0)
#define EXW_CNT(k) ((void)0)
#endif

// sortnet_median_float comparator lists (sorting.c:468-513), pairs i, j
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

// LDS writes of some lanes visible to every lane of the wave
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
// set bits of the lanes below this one
__device__ __forceinline__ int below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ int popc(unsigned long long m) { return (int)__popcll(m); }

struct Col {
    float *st;       // the stack (compacted / permuted in place, as the reference's)
    float *os;       // o_stack: the gathered column in frame order
    float *w;        // w_stack (Winsorized copy)
    float *val;      // partition tape values
    int *par;        // partition tape references
    double *wt;      // sample weights (weighted mean; aliases val / par)
};

// sortnet_median_float on lane 0 (n <= 8), result on every lane
__device__ __forceinline__ double sortnet_median(float *a, int n) {
    double r = 0.0;
    if (lane_id() == 0) {
        const int k = n / 2;
        if (n == 1) {
            r = a[0];
        } else if (n >= 2 && n <= 8) {
            const unsigned char *pn = kNet + 2 * kNetOff[n];
            for (int c = 0; c < kNetLen[n]; c++) {
                const int i = pn[2 * c], j = pn[2 * c + 1];
                const float ai = a[i], aj = a[j];
                if (ai > aj) { a[i] = aj; a[j] = ai; }
            }
            r = (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
        }
    }
    wsync();
    return __shfl(r, 0, 64);
}

// One Lomuto pass of quickmedian_float (sorting.c:249-266) over [left, right]
// with the middle pivot; returns the pivot's final index p.
__device__ __forceinline__ int partition(float *a, int left, int right, float *val, int *par) {
    const int lane = lane_id();
    const int mid = (left + right) / 2;
    const float pivot = a[mid];
    const float ar = a[right];
    wsync();
    if (lane == 0) {
        a[mid] = ar;
        a[right] = pivot;
    }
    wsync();
    const int m = right - left;                 // the scanned range [left, right)
    const int nc = (m + 63) >> 6;
    // Every LDS phase below issues its reads four chunks at a time with
    // clamped indices and no branch between them, so a phase costs one LDS
    // round trip per four chunks (a branch per chunk serialised them: ~11 K
    // cycles per pass at m = 400).
    float x[kMaxC];                             // the scanned samples (a[] is unchanged until the writes)
    unsigned long long sm[kMaxC];               // small-sample ballots (wave-uniform)
    int S = 0, j0 = -1;
#pragma unroll
    for (int q0 = 0; q0 < kMaxC; q0 += 4) {
        if (q0 < nc) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                x[q0 + u] = a[left + (j < m ? j : m - 1)];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                const bool valid = j < m;
                const bool small = valid && x[q0 + u] < pivot;
                sm[q0 + u] = __ballot(small);
                const unsigned long long lm = __ballot(valid && !small);
                if (j0 < 0 && lm) j0 = (q0 + u) * 64 + (int)__builtin_ctzll(lm);
                S += popc(sm[q0 + u]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                x[q0 + u] = 0.f;
                sm[q0 + u] = 0ull;
            }
        }
    }
    if (j0 >= 0) {
        // tape T over the steps j0..m-1: a large step appends its sample, a
        // small one re-appends the queue head T[h] (h: small steps in [j0, j))
        const int M = m - j0;
        int pre = 0;                                     // smalls in the chunks before
#pragma unroll
        for (int q = 0; q < kMaxC; q++) {
            if (q < nc) {
                const int j = q * 64 + lane;
                const bool small = (sm[q] >> lane) & 1ull;
                if (j < m && j >= j0) {
                    const int t = j - j0;
                    if (small) {
                        par[t] = pre + below(sm[q]) - j0;   // every sample before j0 is small
                    } else {
                        par[t] = t;
                        val[t] = x[q];
                    }
                }
                pre += popc(sm[q]);
            }
        }
        wsync();
        // pointer jumping to the large step each reference ends at: every
        // reference points to a strictly earlier tape index and a chain is a
        // few references long, so a few rounds.  A read may already see this
        // round's writes (still an ancestor); a round without a change means
        // every entry points to a root.
        const int ncm = (M + 63) >> 6;
        for (int round = 0; round < 64; round++) {
            bool ch = false;
#pragma unroll
            for (int q0 = 0; q0 < kMaxC; q0 += 4) {
                if (q0 < ncm) {
                    int p1[4], p2[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int t = (q0 + u) * 64 + lane;
                        p1[u] = par[t < M ? t : M - 1];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) p2[u] = par[p1[u]];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int t = (q0 + u) * 64 + lane;
                        if (t < M && p2[u] != p1[u]) {
                            par[t] = p2[u];
                            ch = true;
                        }
                    }
                }
            }
            wsync();
            EXW_CNT(7);
            if (!__ballot(ch)) break;
        }
        // final content: smalls in order at [left, left + S), the queue
        // T[H .. H + K) after them (H: small steps from j0 on)
        const int H = S - j0, K = m - S;
        float lq[kMaxC];
#pragma unroll
        for (int q0 = 0; q0 < kMaxC; q0 += 4) {
            if (q0 < nc) {
                int r1[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int t = (q0 + u) * 64 + lane;
                    r1[u] = par[H + (t < K ? t : 0)];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) lq[q0 + u] = val[r1[u]];
            } else {
#pragma unroll
                for (int u = 0; u < 4; u++) lq[q0 + u] = 0.f;
            }
        }
        wsync();
        pre = 0;
#pragma unroll
        for (int q = 0; q < kMaxC; q++) {
            if (q < nc) {
                const int j = q * 64 + lane;
                const bool small = (sm[q] >> lane) & 1ull;
                if (j < m && small) a[left + pre + below(sm[q])] = x[q];
                pre += popc(sm[q]);
                if (j < K) a[left + S + j] = lq[q];
            }
        }
        wsync();
    }
    const int p = left + S;                              // all small: p == right
    // a[right] = a[p]; a[p] = pivot (sorting.c:264-265)
    const float ap = a[p];
    wsync();
    if (lane == 0) {
        a[right] = ap;
        a[p] = pivot;
    }
    wsync();
    return p;
}

// quickmedian_float (sorting.c:240-273) in place
__device__ __noinline__ double quickmedian_(float *a, int n, float *val, int *par);
__device__ __forceinline__ double quickmedian(float *a, int n, float *val, int *par) {
    EXW_T0();
    const double r = quickmedian_(a, n, val, par);
    EXW_ACC(2);
    return r;
}
__device__ __noinline__ double quickmedian_(float *a, int n, float *val, int *par) {
    if (n < 9) return sortnet_median(a, n);
    const int k = n / 2;
    int left = 0, right = n - 1;
    while (left < right) {
        EXW_CNT(6);
        const int p = partition(a, left, right, val, par);
        if (p < k) left = p + 1;
        else right = p;
    }
    return (n % 2 == 0) ? ((double)a[k - 1] + a[k]) / 2.0 : (double)a[k];
}

// siril_stats_float_sd (statistics.h:80-106), sequential f64 sums on lane 0
__device__ __forceinline__ float sd(const float *x, int n) {
    EXW_T0();
    float r = 0.f;
    if (lane_id() == 0) {
        double s = 0.0, q = 0.0;
#pragma unroll 8
        for (int i = 0; i < n; i++) s += (double)x[i];
        const float mean = (float)(s / n);
#pragma unroll 8
        for (int i = 0; i < n; i++) {
            const float d = x[i] - mean;
            q += (double)(d * d);
        }
        r = sqrtf((float)(q / (n - 1)));
    }
    r = __shfl(r, 0, 64);
    EXW_ACC(3);
    return r;
}

// Stable compaction of a[0, n) to the samples `keep` accepts; returns their count
template <class F>
__device__ __forceinline__ int compact(float *a, int n, F keep) {
    const int lane = lane_id();
    const int nc = (n + 63) >> 6;
    float x[kMaxC];
    bool k[kMaxC];
#pragma unroll
    for (int q0 = 0; q0 < kMaxC; q0 += 4) {
        if (q0 < nc) {                        // reads of four chunks in flight together
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                x[q0 + u] = a[j < n ? j : n - 1];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                k[q0 + u] = j < n && keep(j, x[q0 + u]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                x[q0 + u] = 0.f;
                k[q0 + u] = false;
            }
        }
    }
    wsync();
    int base = 0;
#pragma unroll
    for (int q = 0; q < kMaxC; q++) {
        if (q < nc) {
            const unsigned long long m = __ballot(k[q]);
            if (k[q]) a[base + below(m)] = x[q];
            base += popc(m);
        }
    }
    wsync();
    return base;
}

// The clip pass and compaction of one round (SIGMA / WINSORIZED,
// rejection_float.c:182-199 / :238-248): candidates by sigma_clipping_float
// (:49-60), the `N - r <= 4` cutoff in index order, the stable compaction.
// PCT: percentile_clipping (:62-74), no cutoff.  Returns the new N.
template <bool PCT>
__device__ __forceinline__ int clip_round(float *a, int N, int &r, float s, float slo, float shi, float m, int crej[2]) {
    const int lane = lane_id();
    const int nc = (N + 63) >> 6;
    float x[kMaxC];
    int cand[kMaxC];
#pragma unroll
    for (int q0 = 0; q0 < kMaxC; q0 += 4) {
        if (q0 < nc) {                        // reads of four chunks in flight together
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                x[q0 + u] = a[j < N ? j : N - 1];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = q0 + u;
            const int j = q * 64 + lane;
            cand[q] = 0;
            if (q < nc && j < N) {
                if (m - x[q] > s * slo) cand[q] = -1;
                else if (x[q] - m > s * shi) cand[q] = 1;
            } else {
                x[q] = 0.f;
            }
        }
    }
    wsync();
    int pre = 0, base = 0, lo = 0, hi = 0;
    const int lim = N - 4 - r;                     // rejections allowed before the cutoff
#pragma unroll
    for (int q = 0; q < kMaxC; q++) {
        if (q < nc) {
            const unsigned long long cm = __ballot(cand[q] != 0);
            const bool rej = cand[q] != 0 && (PCT || pre + below(cm) < lim);
            lo += popc(__ballot(rej && cand[q] < 0));
            hi += popc(__ballot(rej && cand[q] > 0));
            const unsigned long long km = __ballot(q * 64 + lane < N && !rej);
            if (q * 64 + lane < N && !rej) a[base + below(km)] = x[q];
            base += popc(km);
            pre += popc(cm);
        }
    }
    wsync();
    r += lo + hi;
    crej[0] += lo;
    crej[1] += hi;
    return base;
}

// w[j] = st[j] and the Winsorized clamp of w (rejection_float.c:228-234),
// reads of four chunks in flight together
__device__ __forceinline__ void copy_col(float *w, const float *st, int n) {
    const int lane = lane_id(), nc = (n + 63) >> 6;
#pragma unroll
    for (int q0 = 0; q0 < kMaxC; q0 += 4) {
        if (q0 < nc) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                v[u] = st[j < n ? j : n - 1];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                if (j < n) w[j] = v[u];
            }
        }
    }
    wsync();
}
__device__ __forceinline__ void clamp_col(float *w, int n, float m0, float m1) {
    const int lane = lane_id(), nc = (n + 63) >> 6;
#pragma unroll
    for (int q0 = 0; q0 < kMaxC; q0 += 4) {
        if (q0 < nc) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                v[u] = w[j < n ? j : n - 1];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = (q0 + u) * 64 + lane;
                const float a = (m0 > v[u]) ? m0 : v[u];
                if (j < n) w[j] = (m1 < a) ? m1 : a;
            }
        }
    }
    wsync();
}

// apply_rejection_float (rejection_float.c:100-354) for SIGMA, WINSORIZED and
// PERCENTILE, no drizzle weights other than the null test
__device__ __forceinline__ int apply_rejection(const KParams &p, Col &c, int nb, int crej[2], long long pix, int x) {
    const float slo = p.sig0, shi = p.sig1;
    // compaction of the null samples (:117-135)
    EXW_T0();
    const int kept = compact(c.st, nb, [&](int f, float v) {
        return v != 0.f && (!p.drizz || plane_at(p, p.drizz, f, pix, x) != 0.f);
    });
    EXW_ACC(1);
    if (kept <= 1) return kept;
    int N = kept, r = 0;
    bool changed;
    switch (p.rtype) {
        case PERCENTILE: {
            const double median = quickmedian(c.st, N, c.val, c.par);
            if (median == 0.0) return 0;
            const float mf = (float)median;
            EXW_T0();
            N = clip_round<true>(c.st, N, r, mf, slo, shi, mf, crej);
            EXW_ACC(4);
            break;
        }
        case SIGMA: {
            double median = quickmedian(c.st, N, c.val, c.par);
            if (median == 0.0) return 0;
            bool first = true;
            do {
                const float var = sd(c.st, N);
                if (!first) median = quickmedian(c.st, N, c.val, c.par);
                first = false;
                EXW_T0();
                const int out = clip_round<false>(c.st, N, r, var, slo, shi, (float)median, crej);
                EXW_ACC(4);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        }
        case WINSORIZED:
            do {
                float sigma0, sigma = sd(c.st, N);
                const float mf = (float)quickmedian(c.st, N, c.val, c.par);
                copy_col(c.w, c.st, N);
                int it = 0;
                do {
                    const float m0 = mf - 1.5f * sigma, m1 = mf + 1.5f * sigma;
                    clamp_col(c.w, N, m0, m1);
                    sigma0 = sigma;
                    sigma = 1.134f * sd(c.w, N);
                } while (fabsf(sigma - sigma0) > sigma0 * 0.0005f && ++it < 100000);
                EXW_T0();
                const int out = clip_round<false>(c.st, N, r, sigma, slo, shi, mf, crej);
                EXW_ACC(4);
                changed = N != out;
                N = out;
            } while (changed && N > 3);
            break;
        default:
            break;
    }
    return N;
}

// mean_and_reject, float branch (median_and_mean.c:1038-1099)
__device__ __forceinline__ double mean_and_reject(const KParams &p, Col &c, int n, int crej[2], long long pix, int x) {
    const int lane = lane_id();
    const int kept = apply_rejection(p, c, n, crej, pix, x);
    if (kept == 0) return quickmedian(c.st, n, c.val, c.par);
    double res = 0.0;
    if (is_weighted(p)) {
        float pmin = FLT_MAX, pmax = -FLT_MAX;
        for (int f = lane; f < kept; f += 64) {
            const float v = c.st[f];
            if (pmin > v) pmin = v;
            if (pmax < v) pmax = v;
        }
#pragma unroll
        for (int lm = 32; lm >= 1; lm >>= 1) {
            const float a = __shfl_xor(pmin, lm, 64), b = __shfl_xor(pmax, lm, 64);
            if (pmin > a) pmin = a;
            if (pmax < b) pmax = b;
        }
        // the sample weights, gathered by every lane (sequential reads would
        // be n dependent HBM round trips); the sums stay sequential
        for (int f = lane; f < n; f += 64) c.wt[f] = sample_weight(p, f, pix, x);
        wsync();
        if (lane == 0) {
            double sum = 0.0, norm = 0.0;
            for (int f = 0; f < n; ++f) {
                const float v = c.os[f];
                if (v >= pmin && v <= pmax && v != 0.f) {
                    const double w = c.wt[f];
                    sum += (double)v * w;
                    norm += w;
                }
            }
            if (norm == 0. || sum == 0.) {
                sum = 0.;
                for (int f = 0; f < n; ++f) {
                    const float v = c.os[f];
                    if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
                }
                res = sum / (double)kept;
            } else {
                res = sum / norm;
            }
        }
    } else if (lane == 0) {
        double sum = 0.0;
#pragma unroll 8
        for (int f = 0; f < kept; ++f) sum += (double)c.st[f];
        res = sum / (double)kept;
    }
    return __shfl(res, 0, 64);
}

}  // namespace exw

// One wave per pixel (block = 64 lanes), grid-stride over the deferred list
// (or every pixel: all_pixels).  Dynamic LDS: 5 words per frame (even N).
__global__ __launch_bounds__(64) void k_stack_exact_wave(KParams p, int all_pixels) {
    extern __shared__ float lds_col[];
    const int N = p.nframes;
    const int n2 = (N + 1) & ~1;                 // even row: the weights below are 8-byte aligned
    exw::Col c;
    c.st = lds_col;
    c.os = lds_col + n2;
    c.w = lds_col + 2 * n2;
    c.val = lds_col + 3 * n2;
    c.par = (int *)(lds_col + 4 * n2);
    c.wt = (double *)(lds_col + 3 * n2);       // aliases val + par (2 n2 words), used after them
    const int lane = exw::lane_id();
    const long long count = all_pixels ? p.npix : (long long)*p.fb_count;
    unsigned long long c0 = 0, c1 = 0;
    for (long long i = blockIdx.x; i < count; i += gridDim.x) {
        const long long pix = all_pixels ? i : (long long)p.fb_list[i];
        const int x = (int)(pix % p.W);
        // the column's reads all in flight (up to 16 per lane), then stored
        EXW_T0();
        {
            float g[exw::kMaxC];
#pragma unroll
            for (int q = 0; q < exw::kMaxC; q++) {
                const int f = q * 64 + lane;
                g[q] = f < N ? gather_sample(p, f, pix, x) : 0.f;
            }
#pragma unroll
            for (int q = 0; q < exw::kMaxC; q++) {
                const int f = q * 64 + lane;
                if (f < N) {
                    c.st[f] = g[q];
                    c.os[f] = g[q];
                }
            }
        }
        exw::wsync();
        EXW_ACC(0);
        int rej[2] = {0, 0};
        double res;
        if (p.rtype == KMEDIAN) res = exw::quickmedian(c.st, N, c.val, c.par);
        else res = exw::mean_and_reject(p, c, N, rej, pix, x);
#if SGPU_EXW_PROF
        if (i == 0 && lane == 0 && blockIdx.x == 0) {
            unsigned long long *g = exw::g_exw_prof;
            printf("EXW_PROF N=%d gather %llu null %llu qmedian %llu sd %llu clip %llu mean %llu passes %llu jumps %llu\n",
                   N, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]);
        }
#endif
        if (lane == 0) {
            write_result(p, pix, res, rej[0], rej[1]);
            c0 += rej[0];
            c1 += rej[1];
        }
        exw::wsync();                            // the next pixel's gather overwrites the column
    }
    add_counts64(p, c0, c1);
}

}  // namespace sgpu
