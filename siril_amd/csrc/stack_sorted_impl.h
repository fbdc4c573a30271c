// stack_sorted_impl.h -- per-pixel rejection stack on a register-resident,
// sorted column ("sorted path").
//
// Layout: a group of G consecutive lanes owns one output pixel; lane g holds
// E = NP/G samples of the pixel's N-deep column in VGPRs.  After the gather
// the column is sorted with a fully unrolled bitonic network (in-lane
// compare-exchanges, plus __shfl_xor exchanges across the G lanes), so every
// order statistic the reference asks quickselect for is an indexed read of
// the sorted column, and every rejection round of SIGMA / WINSORIZED /
// PERCENTILE removes a prefix and a suffix: the kept set is an index window
// [lo, hi).
//
// Exactness vs. the reference (stacking/rejection_float.c:100-354):
//   * order statistics, the n<9 float-add median (sorting.c:512) and the
//     n>=9 double median (sorting.c:272) are reproduced exactly;
//   * the Winsorized clamp is iterated in place in the reference
//     (w = min(m1, max(m0, w)), rejection_float.c:232-234); a chain of clamps
//     is itself one clamp, so we carry the composed bounds [L, U] and apply
//     them to the sorted column -- bit-identical w values, no second array;
//   * f32 arithmetic is unfused (-ffp-contract=off), double accumulation as
//     in statistics.h:80-106; only the summation order differs (ascending
//     order here; the reference's is the quickselect permutation, and an
//     OpenMP SIMD reduction from 24 samples on, itself build-dependent).
//     Every f64 sum is only ever used through a float conversion ((float)
//     (sum / N) in siril_stats_float_sd and the output, (float)(vsum / (N-1))
//     before sqrtf), so the result is order-independent whenever that
//     conversion is: the sum-order guard (SumGuard below) proves it per pixel
//     and per pass -- the sum is exact in any order (samples within a 2^29
//     dynamic range), or the float is the same for every value within the
//     error bound of ANY summation order -- and defers the pixel otherwise;
//   * the `N - r <= 4` cutoff (rejection_float.c:188,239) depends on the
//     order quickselect leaves the column in.  When a round's candidates
//     would cross the cutoff, or a column holds NaN/Inf, or the reference
//     would take its kept==0 path (quickmedian of the mutated stack,
//     median_and_mean.c:1040), the pixel is deferred to the exact sequential
//     kernel (stack_exact.hip) through fb_list.  Such a pixel's result is
//     therefore exactly the reference's.
//
// Both a device kernel and a host build (G == 1, tests only) are produced
// from this header: SG_HD functions have no device-only dependency for G==1.
#pragma once
#include <utility>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "sgpu_kparams.h"

#define SG_HD __host__ __device__ __forceinline__

// tuning knobs (build-time): independent f64 accumulator chains per lane
#ifndef SGPU_NACC
#define SGPU_NACC 2
#endif
#ifndef SGPU_OPAQUE_FINAL
#define SGPU_OPAQUE_FINAL 1
#endif
#ifndef SGPU_RANGE_FIRST
#define SGPU_RANGE_FIRST 1
#endif
#ifndef SGPU_RECLAMP
#define SGPU_RECLAMP 1
#endif
// timing ablations (diagnostic builds only; results are wrong with any set):
// SGPU_ABL_NOSORT skips the column sort, SGPU_ABL_ITERS=k runs exactly k
// Winsorized inner iterations per round, SGPU_ABL_NOREJ skips the rejection
#ifndef SGPU_MEDIAN_SELECT
#define SGPU_MEDIAN_SELECT 1      // median stack: pruned selection network (0: the full sort; A/B)
#endif
#ifndef SGPU_ABL_NOSORT
#define SGPU_ABL_NOSORT 0
#endif
#ifndef SGPU_ABL_ITERS
#define SGPU_ABL_ITERS 0
#endif
#ifndef SGPU_ABL_NOREJ
#define SGPU_ABL_NOREJ 0
#endif
// widest lane group that transposes the sorted column to the interleaved
// layout (padding-free passes); wider groups keep the block layout
#ifndef SGPU_IL_SIGMA_MAXG
#define SGPU_IL_SIGMA_MAXG 2      // interleaved SIGMA / PERCENTILE columns up to this G (A/B)
#endif
#ifndef SGPU_IL_MAXG
#define SGPU_IL_MAXG 16
#endif
// slot granularity of the wave-uniform pass ends (4; 2 measured 7x slower:
// the column loops no longer fully unroll)
#ifndef SGPU_LATE_PIX
#define SGPU_LATE_PIX 1
#endif
#ifndef SGPU_GATHER_STOP
#define SGPU_GATHER_STOP 1
#endif
#ifndef SGPU_STOP_GRAN
#define SGPU_STOP_GRAN 4
#endif
// A/B: the compare form of count_sigma on the device
#ifndef SGPU_COUNT_CMP
#define SGPU_COUNT_CMP 0
#endif

namespace sgpu {

SG_HD float f_inf() { return __builtin_huge_valf(); }

// Diagnostic section timer (-DSGPU_PROF=1 builds only): every lane adds the
// shader clock elapsed since its previous mark to the section it closes; the
// kernel sums the lanes into KParams::prof.  Sections: 0 gather, 1 sort,
// 2 round median + fill, 3 first sd (+ moments), 4 interval loop, 5 clip
// counts, 6 exact inner loop + count, 7 round tail, 8 final mean + write,
// 9 other types' rejection.
#ifndef SGPU_PROF
#define SGPU_PROF 0
#endif
struct ProfAcc {
    unsigned long long t, acc[12];
};
#if SGPU_PROF && defined(__HIP_DEVICE_COMPILE__)
#define SG_PMARK(pa, k)                                                      \
    do {                                                                     \
        if (pa) {                                                            \
            const unsigned long long now_ = __builtin_readcyclecounter();    \
            (pa)->acc[k] += now_ - (pa)->t;                                  \
            (pa)->t = now_;                                                  \
        }                                                                    \
    } while (0)
#else
#define SG_PMARK(pa, k) do { } while (0)
#endif

// Make a value opaque to the optimizer: stops LICM from hoisting one window
// predicate per column element out of the Winsorized loops (that hoist alone
// costs ~E registers).
SG_HD void opaque(int &x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#else
    asm volatile("" : "+r"(x));
#endif
}

SG_HD void opaquef(float &x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#else
    asm volatile("" : "+r"(x));
#endif
}

// Make the column registers opaque (no code emitted): stops GVN/PRE from
// keeping E f32->f64 conversions of one pass alive (2E registers) to reuse
// them in a later pass over the same values.
template <int E> SG_HD void opaque_col(float (&v)[E]) {
#pragma unroll
    for (int e = 0; e < E; e++) {
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(v[e]));
#else
        asm volatile("" : "+r"(v[e]));
#endif
    }
}

// ------------------------------------------------------------ group primitives
// xor-exchange inside a lane group: DPP quad permutes for masks 1 and 2,
// ds_swizzle (xor mode, no LDS traffic) for 4, 8 and 16.
template <int MASK> __device__ __forceinline__ int xchg_i(int v) {
    if constexpr (MASK == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    else if constexpr (MASK == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
    else return __builtin_amdgcn_ds_swizzle(v, (MASK << 10) | 0x1F);                        // and 0x1F, xor MASK
}
template <int G, int MASK> SG_HD float gxchg(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G > 1) return __builtin_bit_cast(float, xchg_i<MASK>(__builtin_bit_cast(int, v)));
#endif
    return v;
}
template <int G, int MASK> SG_HD double gxchg(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G > 1) {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
        const int lo = xchg_i<MASK>((int)(u & 0xffffffffu)), hi = xchg_i<MASK>((int)(u >> 32));
        return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
    }
#endif
    return v;
}
template <int G, int MASK> SG_HD int gxchg(int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G > 1) return xchg_i<MASK>(v);
#endif
    return v;
}
template <int G, int MASK> SG_HD uint32_t gxchg(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G > 1) return (uint32_t)xchg_i<MASK>((int)v);
#endif
    return v;
}
// run-time mask (a constant after unrolling: the switch folds away)
template <int G> SG_HD float gxchg_rt(float v, int mask) {
    switch (mask) {
        case 1: return gxchg<G, 1>(v);
        case 2: return gxchg<G, 2>(v);
        case 4: return gxchg<G, 4>(v);
        case 8: return gxchg<G, 8>(v);
        default: return gxchg<G, 16>(v);
    }
}
// butterfly sum over the G lanes; a+b == b+a, so every lane ends with the same bits
template <int G, typename T> SG_HD T gsum_t(T v) {
    if constexpr (G >= 2) v += gxchg<G, 1>(v);
    if constexpr (G >= 4) v += gxchg<G, 2>(v);
    if constexpr (G >= 8) v += gxchg<G, 4>(v);
    if constexpr (G >= 16) v += gxchg<G, 8>(v);
    if constexpr (G >= 32) v += gxchg<G, 16>(v);
    return v;
}
template <int G> SG_HD float gbcast(float v, int src) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (G > 1) return __shfl(v, src, G);
#endif
    return v;
}
template <int G> SG_HD int gbcast(int v, int src) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (G > 1) return __shfl(v, src, G);
#endif
    return v;
}

// ---------------------------------------------------------------- sorting
// xor-exchange with any lane mask < 32 (the merge's flip stage pairs lane g
// with g ^ (2R - 1)): DPP quad permutes for 1, 2, 3, ds_swizzle otherwise.
template <int MASK> __device__ __forceinline__ int xchg_any(int v) {
    if constexpr (MASK == 1 || MASK == 2) return xchg_i<MASK>(v);
    else if constexpr (MASK == 3) return __builtin_amdgcn_mov_dpp(v, 0x1B, 0xF, 0xF, false); // quad_perm [3,2,1,0]
    else return __builtin_amdgcn_ds_swizzle(v, (MASK << 10) | 0x1F);
}
template <int G, int MASK> SG_HD float gxchg_any(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G > 1) return __builtin_bit_cast(float, xchg_any<MASK>(__builtin_bit_cast(int, v)));
#endif
    return v;
}
// min(a, o) when c = -Inf, max(a, o) when c = +Inf: one v_med3_f32 replaces
// min + max + a lane-dependent select in the cross-lane merge stages
SG_HD float lane_minmax(float a, float o, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(a, o, c);
#else
    return c < 0.f ? fminf(a, o) : fmaxf(a, o);
#endif
}
SG_HD void cmpx(float &a, float &b) {
    const float mn = fminf(a, b), mx = fmaxf(a, b);
    a = mn;
    b = mx;
}
// Batcher's odd-even merge sort of the E in-lane slots, ascending (543
// compare-exchanges at E = 64 against the bitonic network's 672, and no
// direction selects: every comparator puts the minimum at the lower slot).
// RS: slots e >= RS hold +Inf on entry (padding known at compile time): every
// comparator whose upper slot is >= RS is then a no-op (min(x, +Inf) = x
// stays low, +Inf stays high) and is left out -- the upper slots are never
// written, so the invariant holds through the whole network (E = 128 with
// 100 real slots: 1104 of 1471 comparators; E = 64 with 52: 423 of 543).
template <int E, int RS = E> SG_HD void oem_sort(float (&v)[E]) {
    static_assert(RS >= 1 && RS <= E, "real slots");
#pragma unroll
    for (int lp = 0; (1 << lp) < E; lp++) {
        const int p = 1 << lp;
#pragma unroll
        for (int lk = lp; lk >= 0; lk--) {
            const int k = 1 << lk;
#pragma unroll
            for (int j = k % p; j + k < E; j += 2 * k) {
#pragma unroll
                for (int i = 0; i < k; i++) {
                    if (i + j + k < RS && (i + j) / (2 * p) == (i + j + k) / (2 * p)) cmpx(v[i + j], v[i + j + k]);
                }
            }
        }
    }
}
// The same network pruned to the outputs [LO, HI) (round 6: the median
// stack reads two ranks of the sorted column).  OemNet lists oem_sort's
// comparators in order at compile time; OemUse walks them backwards from the
// wanted outputs: a comparator none of whose outputs is needed later is left
// out, one whose min (max) output alone is needed becomes a single fminf
// (fmaxf).  The comparators are expanded by a fold over their indices, so
// every slot index is a constant (no dynamic register indexing).  At E = 128,
// RS = 104 and ranks [47, 53): 1 806 of 2 314 min / max operations.
template <int E, int RS> struct OemNet {
    static constexpr int count() {
        int n = 0;
        for (int lp = 0; (1 << lp) < E; lp++)
            for (int lk = lp; lk >= 0; lk--) {
                const int p = 1 << lp, k = 1 << lk;
                for (int j = k % p; j + k < E; j += 2 * k)
                    for (int i = 0; i < k; i++)
                        if (i + j + k < RS && (i + j) / (2 * p) == (i + j + k) / (2 * p)) n++;
            }
        return n;
    }
    static constexpr int N = count();
    short a[N], b[N];
    constexpr OemNet() : a(), b() {
        int n = 0;
        for (int lp = 0; (1 << lp) < E; lp++)
            for (int lk = lp; lk >= 0; lk--) {
                const int p = 1 << lp, k = 1 << lk;
                for (int j = k % p; j + k < E; j += 2 * k)
                    for (int i = 0; i < k; i++)
                        if (i + j + k < RS && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                            a[n] = (short)(i + j);
                            b[n] = (short)(i + j + k);
                            n++;
                        }
            }
    }
};
// one evaluation per specialisation (variable templates), not per comparator
template <int E, int RS> inline constexpr OemNet<E, RS> kOemNet{};
template <int E, int RS, int LO, int HI> struct OemUse {
    unsigned char use[OemNet<E, RS>::N];      // bit 0: min output needed, bit 1: max output needed
    constexpr OemUse() : use() {
        bool need[E] = {};
        for (int r = LO; r < HI; r++) need[r] = true;
        for (int c = OemNet<E, RS>::N - 1; c >= 0; c--) {
            const int a = kOemNet<E, RS>.a[c], b = kOemNet<E, RS>.b[c];
            use[c] = (unsigned char)((need[a] ? 1 : 0) | (need[b] ? 2 : 0));
            if (use[c]) need[a] = need[b] = true;
        }
    }
};
template <int E, int RS, int LO, int HI> inline constexpr OemUse<E, RS, LO, HI> kOemUse{};
template <int E, int RS, int LO, int HI, int C> SG_HD void oem_sel_step(float (&v)[E]) {
    constexpr int a = kOemNet<E, RS>.a[C], b = kOemNet<E, RS>.b[C];
    constexpr unsigned us = kOemUse<E, RS, LO, HI>.use[C];
    if constexpr (us == 3) {
        cmpx(v[a], v[b]);
    } else if constexpr (us == 1) {
        v[a] = fminf(v[a], v[b]);
    } else if constexpr (us == 2) {
        v[b] = fmaxf(v[a], v[b]);
    }
}
template <int E, int RS, int LO, int HI, int... Cs>
SG_HD void oem_sel_all(float (&v)[E], std::integer_sequence<int, Cs...>) {
    (oem_sel_step<E, RS, LO, HI, Cs>(v), ...);
}
template <int E, int RS, int LO, int HI> SG_HD void oem_select(float (&v)[E]) {
    oem_sel_all<E, RS, LO, HI>(v, std::make_integer_sequence<int, OemNet<E, RS>::N>{});
}

template <int NP, int G, int R> SG_HD void sort_merge_lanes(float (&v)[NP / G], int g);
// Sort of the NP-element column spread as E = NP/G per lane (element index
// i = g*E + e), ascending: every lane sorts its slots, then runs of R lanes
// are merged into 2R lanes -- a flip stage (element I of the 2R-lane block
// against 2RE-1-I: lane g ^ (2R-1), slot E-1-e; every lane sends the same
// register, so the exchange is one DPP/swizzle per slot) followed by the
// half-cleaners (lane masks R/2..1, then in-lane distances E/2..1).  All
// runs stay ascending, so no stage needs a direction select.
template <int NP, int G, int RS = NP / G> SG_HD void sort_column(float (&v)[NP / G], int g) {
    constexpr int E = NP / G;
    oem_sort<E, RS>(v);
    if constexpr (G > 1) {
        sort_merge_lanes<NP, G, 1>(v, g);
    }
}

// Bitonic sort of the NP-element column spread as E = NP/G per lane; element
// index i = g*E + e.  Ascending.  (Kept as the reference network for the
// sort_column A/B: SGPU_SORT_BITONIC=1.)
template <int NP, int G> SG_HD void bitonic_sort(float (&v)[NP / G], int g) {
    constexpr int E = NP / G;
    constexpr int LOGNP = __builtin_ctz(NP);
    // affine loop counters (log2 k, log2 j) so the loops fully unroll and
    // every slot index is a compile-time constant (no scratch)
#pragma unroll
    for (int lk = 1; lk <= LOGNP; lk++) {
        const int k = 1 << lk;
#pragma unroll
        for (int lj = lk - 1; lj >= 0; lj--) {
            const int j = 1 << lj;
            if (j >= E) {
                // partner lives in lane g ^ (j/E), same slot e.  k > j >= E, so
                // the direction bit (i & k) is a lane bit: uniform per lane.
                const bool up = ((g * E) & k) == 0;
                const bool lower = (g & (j / E)) == 0;
                const bool take_min = (lower == up);
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const float o = gxchg_rt<G>(v[e], j / E);
                    const float mn = fminf(v[e], o), mx = fmaxf(v[e], o);
                    v[e] = take_min ? mn : mx;
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int l = e ^ j;
                    if (l > e) {
                        const float a = v[e], b = v[l];
                        const float mn = fminf(a, b), mx = fmaxf(a, b);
                        bool up;
                        if (k < E) up = (e & k) == 0;            // compile-time
                        else up = ((g * E) & k) == 0;            // lane bit (k >= E)
                        v[e] = up ? mn : mx;
                        v[l] = up ? mx : mn;
                    }
                }
            }
        }
    }
}

template <int NP, int G, int R> SG_HD void sort_merge_lanes(float (&v)[NP / G], int g) {
    constexpr int E = NP / G;
    if constexpr (R < G) {
        {
            const float c = (g & R) == 0 ? -f_inf() : f_inf();   // lower half keeps the minimum
            // slots e and E-1-e in place (a temporary copy of the column
            // would double the live registers)
#pragma unroll
            for (int e = 0; e < E / 2; e++) {
                const float a = v[e], b = v[E - 1 - e];
                const float ra = gxchg_any<G, 2 * R - 1>(a), rb = gxchg_any<G, 2 * R - 1>(b);
                v[e] = lane_minmax(a, rb, c);
                v[E - 1 - e] = lane_minmax(b, ra, c);
            }
        }
#pragma unroll
        for (int m = R / 2; m >= 1; m >>= 1) {
            const float c = (g & m) == 0 ? -f_inf() : f_inf();
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = lane_minmax(v[e], gxchg_rt<G>(v[e], m), c);
        }
#pragma unroll
        for (int j = E / 2; j >= 1; j >>= 1) {
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int l = e ^ j;
                if (l > e) cmpx(v[e], v[l]);
            }
        }
        sort_merge_lanes<NP, G, 2 * R>(v, g);
    }
}

#ifndef SGPU_SORT_BITONIC
#define SGPU_SORT_BITONIC 0
#endif
// RS: a bound on the slots per lane that can hold samples (slots e >= RS are
// +Inf padding in every lane: frames e*G + g >= N); the host guarantees
// ceil(N / G) <= RS (rs_pick)
template <int NP, int G, int RS = NP / G> SG_HD void sort_col(float (&v)[NP / G], int g) {
    if constexpr (SGPU_SORT_BITONIC) bitonic_sort<NP, G>(v, g);
    else sort_column<NP, G, RS>(v, g);
}
// real-slot bound of a launch: the smallest compiled bound >= ceil(N / G)
// (steps of 4 at E = 64, of 8 at E = 128: the variants of
// stack_sorted_rs*.hip), or E (full network)
inline int rs_pick(int E, int G, int N) {
    if (E != 64 && E != 128) return E;
    const int step = E == 64 ? 4 : 8;
    const int need = (N + G - 1) / G;
    const int rs = (need + step - 1) / step * step;
    return rs < E ? rs : E;
}

// ------------------------------------------------------ indexed (dynamic) read
// Select v[idx] for a per-lane dynamic idx without scratch: a binary tree of
// bitfield selects (v_bfi_b32, E-1 of them).  Written on the bit patterns so
// the compiler cannot turn the tree back into an indexed (scratch/LDS) load.
SG_HD float bsel(uint32_t m, float a_if0, float b_if1) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(b_if1), "v"(a_if0));
    return r;
#else
    const uint32_t a = __builtin_bit_cast(uint32_t, a_if0), b = __builtin_bit_cast(uint32_t, b_if1);
    return __builtin_bit_cast(float, (b & m) | (a & ~m));
#endif
}
// depth-first over halves: only O(log E) partial results are live at once
template <int LO, int LEN, int E>
SG_HD float sel_range(const float (&v)[E], const uint32_t (&m)[16]) {
    if constexpr (LEN == 1) {
        return v[LO];
    } else {
        constexpr int L = __builtin_ctz(LEN) - 1;   // idx bit choosing the half
        const float a = sel_range<LO, LEN / 2, E>(v, m);
        const float b = sel_range<LO + LEN / 2, LEN / 2, E>(v, m);
        return bsel(m[L], a, b);
    }
}
template <int E> SG_HD float sel(const float (&v)[E], int idx) {
    uint32_t m[16];
#pragma unroll
    for (int b = 0; b < 16; b++) m[b] = 0u - (uint32_t)((idx >> b) & 1);
    return sel_range<0, E, E>(v, m);
}
// Wave-uniform index: a tree of scalar branches picks the one register to
// read (no VALU select work at all).
template <int LO, int LEN, int E> SG_HD float selu_range(const float (&v)[E], int idx) {
    if constexpr (LEN == 1) {
        return v[LO];
    } else {
        if (idx & (LEN / 2)) return selu_range<LO + LEN / 2, LEN / 2, E>(v, idx);
        return selu_range<LO, LEN / 2, E>(v, idx);
    }
}
template <int E> SG_HD float selu(const float (&v)[E], int idx) {
#if defined(__HIP_DEVICE_COMPILE__)
    idx = __builtin_amdgcn_readfirstlane(idx);
#endif
    return selu_range<0, E, E>(v, idx);
}

// Slot layout of the sorted column inside a lane group.  Block (IL = false):
// lane g holds sorted indices [g*E, (g+1)*E) -- what bitonic_sort produces.
// Interleaved (IL = true): lane g holds indices g, g+G, g+2G, ... so the
// padding slots (index >= N) are the same trailing slots e >= ceil(N/G) in
// every lane and the per-iteration passes can stop there (wave-uniform).
// G == 1: both layouts coincide.
template <int E, int G, bool IL> SG_HD int slot_index(int g, int e) {
    return IL ? e * G + g : g * E + e;
}
// Pass loops stop at slot `elim` (a multiple of SGPU_STOP_GRAN, wave-uniform)
// in chunks of SGPU_STOP_GRAN.
#define SG_STOP4(e, elim) if (((e) & (SGPU_STOP_GRAN - 1)) == 0 && (e) >= (elim)) break

// element `idx` of the group's sorted column (idx uniform across the group)
template <int E, int G, bool IL = false> SG_HD float ostat(const float (&v)[E], int idx) {
    if constexpr (IL) {
        const float s = sel<E>(v, idx / G);
        return gbcast<G>(s, idx & (G - 1));
    } else {
        const float s = sel<E>(v, idx & (E - 1));
        return gbcast<G>(s, idx / E);
    }
}

// Block -> interleaved layout for G == 2: lane 0 keeps its even-offset
// samples and takes lane 1's even ones; lane 1 the odd ones (one DPP
// exchange per slot pair).
template <int E> SG_HD void to_interleaved2(float (&v)[E], int g) {
    float nv[E];
#pragma unroll
    for (int k = 0; k < E / 2; k++) {
        const float send = (g == 0) ? v[2 * k + 1] : v[2 * k];
        const float recv = gxchg<2, 1>(send);
        nv[k] = (g == 0) ? v[2 * k] : recv;
        nv[E / 2 + k] = (g == 0) ? recv : v[2 * k + 1];
    }
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = nv[e];
}

// Block -> interleaved layout for any G (2, 4, 8, ...): a G x G transpose of
// every group of G consecutive slots across the G lanes (log2 G stages of
// xor-exchanges, recursive 2x2 block transposes), then a compile-time slot
// renaming: block index i = g*E + G*q + j lands in lane j, slot g*E/G + q.
template <int E, int G> SG_HD void to_interleaved(float (&v)[E], int g) {
    static_assert(E % G == 0, "slots per lane must be a multiple of G");
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
#pragma unroll
        for (int q = 0; q < E / G; q++) {
#pragma unroll
            for (int j = 0; j < G; j++) {
                if (j & m) continue;
                float &a = v[q * G + j], &b = v[q * G + (j | m)];
                const bool hi = (g & m) != 0;
                const float send = hi ? a : b;
                const float recv = gxchg_rt<G>(send, m);
                a = hi ? recv : a;
                b = hi ? b : recv;
            }
        }
    }
    // lane j now holds, at slot q*G + g', the element of lane g' (block index
    // g'*E + G*q + j): rename it to slot g'*E/G + q
    float nv[E];
#pragma unroll
    for (int q = 0; q < E / G; q++)
#pragma unroll
        for (int gg = 0; gg < G; gg++) nv[gg * (E / G) + q] = v[q * G + gg];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = nv[e];
}

// quickmedian_float (sorting.c:240-273) / sortnet_median_float (:468-513)
// on the sorted window [lo, lo+n): exact order statistics with the
// reference's rounding: float add below 9 elements, double add from 9.
template <int E, int G, bool IL = false> SG_HD double median_win(const float (&v)[E], int lo, int n) {
    if (n <= 0) return 0.0;                   // sortnet default branch
    const int k = n / 2;
    const bool even = (n & 1) == 0;
    const float b = ostat<E, G, IL>(v, lo + k);
    // make the second select depend on the first: the two trees are then
    // evaluated one after the other instead of side by side (register peak)
    int z = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(z) : "v"(b));
#endif
    const float a = ostat<E, G, IL>(v, lo + k - (even ? 1 : 0) + z);
    if (!even) return (double)b;
    if (n < 9) return (a + b) / 2.0;          // float add (sorting.c:512)
    return ((double)a + b) / 2.0;             // double add (sorting.c:272)
}

// ------------------------------------------------------------ sum-order guard
// The reference sums in its own order (statistics.h:80-106: the quickselect
// permutation, an OpenMP SIMD reduction from 24 samples on; mean_and_reject's
// mean, median_and_mean.c:1083-1097, likewise), this kernel in sorted order
// over lanes and chains.  Any two orders of m additions differ by at most
// 2 gamma_m sum|terms| (gamma_m = m u / (1 - m u), u = 2^-53); the sums are
// only consumed through a float conversion, so the float result is the
// reference's whenever either
//   * the sum is exact in every order: all terms are multiples of the
//     smallest sample's ulp and the total stays below 2^53 of them (positive
//     samples whose binade span + 24 + ceil(log2 m) <= 53: every subset,
//     clamp or median fill of the window stays in [vmin, vmax]), or
//   * (float)(q - e) == (float)(q + e) for the computed quotient q and e its
//     bound (rounding is monotone: every value in between converts to the
//     same float).
// Otherwise the pass reports -2 and the pixel is deferred to the exact
// sequential kernel (the reference's own sequential order).  c = (2m + 16) u
// also covers the division, the fill-slot correction and the rounding of
// q +- e themselves.
struct SumGuard {
    int exact;       // sums of window samples (and of their clamps) are exact in f64
    int pos;         // every sample > 0: sum|x| = sum x, the bound is relative
    double xabs_c;   // c * m * max|x| over the column: bound for mixed-sign columns
    double c;        // (2m + 16) * 2^-53: relative bound for sums of non-negative terms
};
SG_HD int ebits(float x) {
    const int e = (int)((__builtin_bit_cast(uint32_t, x) >> 23) & 0xffu);
    return e ? e : 1;                                   // subnormals: granularity 2^-149
}
SG_HD int ceil_log2(int m) { return m <= 1 ? 0 : 32 - __builtin_clz((unsigned)(m - 1)); }
// vmin / vmax: smallest and largest sample any sum of the pixel can see;
// m: terms per sum (visited slots + corrections); depth: additions on the
// longest path of this kernel's summation tree (a chain of E / NACC slots,
// the chain and lane combines, the fill correction); n: the reference's
// (sequential or SIMD-lane) chain length bound.  Any summation tree of depth
// d is within gamma_d sum|x| of the exact sum, so two orders differ by at
// most (d_gpu + d_ref) u sum|x| (+ slack for the division and q +- e).
SG_HD SumGuard make_guard(float vmin, float vmax, int m, int depth, int n) {
    SumGuard sg;
    const float amax = fabsf(vmin) > fabsf(vmax) ? fabsf(vmin) : fabsf(vmax);
    sg.pos = vmin > 0.f;
    sg.exact = sg.pos && (ebits(vmax) - ebits(vmin) + 24 + ceil_log2(m) <= 53);
    sg.c = (double)(depth + n + 16) * 0x1p-53;
    sg.xabs_c = sg.c * (double)m * (double)amax;
    return sg;
}
// order-error bound of a sum of samples whose computed value is `sum` and
// whose terms (window samples, clamps, fills) lie within [xlo, xhi]: relative
// for positive columns, else m * max(|xlo|, |xhi|) (the window's own ends)
SG_HD double sum_bound(const SumGuard &sg, double sum, float xlo, float xhi, int m) {
    if (sg.pos) return sum * sg.c;
    const float a = fabsf(xlo) > fabsf(xhi) ? fabsf(xlo) : fabsf(xhi);
    return sg.c * (double)m * (double)a;
}
// (float)x is the same float for every value within e of q (a non-finite
// quotient -- 0 / 0, x / 0 -- is one in every order)
SG_HD bool f32_stable(double q, double e) { return !(q - q == 0.0) || (float)(q - e) == (float)(q + e); }

// siril_stats_float_sd (statistics.h:80-106) over the window [lo, hi), with
// the samples optionally clamped to [L, U] (Winsorized w_stack).
template <int E, int G, bool CLAMP>
SG_HD float sd_win(const float (&v)[E], int g, int lo, int hi, float L, float U, const SumGuard &sg) {
    opaque(lo);
    opaque(hi);
    // four independent f64 chains per lane (a single chain is latency-bound);
    // the reference's summation order is already not reproduced (see header)
    double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = g * E + e;
        float x = v[e];
        if (CLAMP) x = fminf(U, fmaxf(L, x));
        const float xm = (i >= lo && i < hi) ? x : 0.f;
        s[e % SGPU_NACC] += (double)xm;
    }
    const double st = gsum_t<G>((s[0] + s[1]) + (s[2] + s[3]));
    const int n = hi - lo;
    const double qm = st / n;
    if (!sg.exact && !f32_stable(qm, ((sg.pos ? st * sg.c : sg.xabs_c) + fabs(st) * 0x1p-50) / n)) return -2.f;
    const float mean = (float)qm;
    double q[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = g * E + e;
        float x = v[e];
        if (CLAMP) x = fminf(U, fmaxf(L, x));
        const float d = x - mean;
        const float dd = (i >= lo && i < hi) ? d * d : 0.f;
        q[e % SGPU_NACC] += (double)dd;
    }
    const double qt = gsum_t<G>((q[0] + q[1]) + (q[2] + q[3]));
    const double qv = qt / (n - 1);
    if (!f32_stable(qv, qv * sg.c)) return -2.f;
    return sqrtf((float)qv);
}

// roundf_to_WORD (core/proto.h:341-346) kept in float: the 16-bit Winsorize
// bounds (median_and_mean.c:840-841) are whole numbers in [0, 65535]
SG_HD float roundf_to_word_f(float f) {
    f = f + 0.5f;
    f = (f > 65535.f) ? 65535.f : f;
    f = (f < 0.0f) ? 0.0f : f;
    return truncf(f);
}

// clamp(x, L, U) for L <= U and non-NaN x: min(U, max(L, x)) in one v_med3_f32
// (no operand canonicalisation, unlike fminf/fmaxf)
SG_HD float med3(float x, float L, float U) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(x, L, U);
#else
    return fminf(U, fmaxf(L, x));
#endif
}

// Every slot outside the window [lo, hi) takes the value `fill` (the window
// median): once per rejection round, so that the per-iteration sd passes
// below need no window predicate at all.
template <int E, int G, bool IL>
SG_HD void fill_outside(float (&v)[E], int g, int lo, int hi, float fill, int elim) {
    // in-window iff 0 <= slot - lo < hi - lo (one unsigned compare).  The
    // add/compare/select triple is one asm block so the compiler cannot hoist
    // E window compares (an SGPR pair each) above the pass and spill them.
    const unsigned n = (unsigned)(hi - lo);
    const int base = (IL ? g : g * E) - lo;
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
#if defined(__HIP_DEVICE_COMPILE__)
        int t;
        asm("v_add_u32 %0, %2, %3\n\t"
            "v_cmp_gt_u32 vcc, %4, %0\n\t"
            "v_cndmask_b32 %1, %5, %1, vcc"
            : "=&v"(t), "+v"(v[e])
            : "i"(IL ? e * G : e), "v"(base), "v"(n), "v"(fill)
            : "vcc");
#else
        const unsigned t = (unsigned)(base + (IL ? e * G : e));
        v[e] = (t < n) ? v[e] : fill;
#endif
    }
}

typedef float sg_f2 __attribute__((ext_vector_type(2)));


// a / b correctly rounded from y = RN(1/b): q0 = RN(a*y), e = a - q0*b (exact
// with an fma), q = RN(q0 + e*y) (Markstein's theorem; checked bit for bit
// against a / b on 22 M random pairs, b = 1..1100).  Three f64 ops instead of
// the ten of the general division sequence, per sd pass.
SG_HD double div_rn(double a, double b, double y) {
    const double q0 = a * y;
    const double e = fma(-q0, b, a);
    return fma(e, y, q0);
}

// siril_stats_float_sd (statistics.h:80-106) over the n-sample window of a
// column whose k = G*elim - n other visited slots all hold `fill` (slots
// from elim on are never visited), samples optionally
// clamped to [L, U] (Winsorized w_stack).  L <= fill <= U (fill is the median
// the clamp bounds are built around), so a fill slot adds exactly
// (double)fill to the first sum and (double)fl(fl(fill - mean)^2) to the
// second: both are taken back out in f64 (k * f32 value is exact in f64).
// Sums are exact whenever the reference's own double sums are exact; fill ~
// mean keeps the second correction small.  Returns a negative value when
// sigma is not finite (caller defers the pixel).
template <int NP, int G, bool CLAMP>
SG_HD float sd_filled(const float (&v)[NP / G], int n, float fill, float L, float U, int elim, double rn,
                      double rn1, const SumGuard &sg, float xlo = 0.f, float xhi = 0.f) {
    constexpr int E = NP / G;
    const double k = (double)(G * elim - n);
    double st, stot;
    // a fill slot after the clamp (equal to fill for the float path, where
    // L <= fill <= U; the 16-bit path's rounded bounds may not bracket it)
    const float fe = CLAMP ? med3(fill, L, U) : fill;
    {
        double s[SGPU_NACC];
#pragma unroll
        for (int c = 0; c < SGPU_NACC; c++) s[c] = 0.0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            SG_STOP4(e, elim);
            const float x = CLAMP ? med3(v[e], L, U) : v[e];
            s[e % SGPU_NACC] += (double)x;
        }
        st = s[0];
#pragma unroll
        for (int c = 1; c < SGPU_NACC; c++) st += s[c];
        st = gsum_t<G>(st);
        stot = st;                                             // positive columns: sum |x|
        st -= k * (double)fe;
    }
    const double qm = div_rn(st, (double)n, rn);
    if (!sg.exact && !f32_stable(qm, (sum_bound(sg, stot, xlo, xhi, G * elim) + fabs(st) * 0x1p-50) * rn))
        return -2.f;
    const float mean = (float)qm;                              // (float)(sum / N)
#if SGPU_RECLAMP
    // recompute the clamp in the second pass instead of keeping E clamped
    // values alive across the reduction (register pressure)
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(L), "+v"(U));
#endif
#endif
    double q[SGPU_NACC];
#pragma unroll
    for (int c = 0; c < SGPU_NACC; c++) q[c] = 0.0;
    static_assert(E % 2 == 0, "pairs");
#pragma unroll
    for (int e = 0; e < E; e += 2) {
        SG_STOP4(e, elim);
        sg_f2 x;
        x.x = CLAMP ? med3(v[e], L, U) : v[e];
        x.y = CLAMP ? med3(v[e + 1], L, U) : v[e + 1];
        const sg_f2 d = x - (sg_f2)(mean);
        const sg_f2 dd = d * d;                 // v_pk_add_f32 / v_pk_mul_f32
        q[e % SGPU_NACC] += (double)dd.x;
        q[(e + 1) % SGPU_NACC] += (double)dd.y;
    }
    double qt = q[0];
#pragma unroll
    for (int c = 1; c < SGPU_NACC; c++) qt += q[c];
    const float df = fe - mean;
    const double fq = k * (double)(df * df);
    qt = gsum_t<G>(qt);
    const double qabs = qt;                                    // every term >= 0
    qt -= fq;
    const double qv = div_rn(qt, (double)(n - 1), rn1);
    const double eq = qabs * (sg.c * rn1);                     // sg.c * rn1: loop-invariant
    if ((float)(qv - eq) != (float)(qv + eq)) return -2.f;     // f32_stable (qv finite: n >= 2, no NaN)
    const float sd = sqrtf((float)qv);
    return (sd - sd == 0.f) ? sd : -1.f;
}

template <int E, int G> SG_HD double sum_all(const float (&v)[E], int elim) {
    double s[SGPU_NACC];
#pragma unroll
    for (int c = 0; c < SGPU_NACC; c++) s[c] = 0.0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
        s[e % SGPU_NACC] += (double)v[e];
    }
    double st = s[0];
#pragma unroll
    for (int c = 1; c < SGPU_NACC; c++) st += s[c];
    return gsum_t<G>(st);
}

template <int E, int G, bool IL = false>
SG_HD double sum_win(const float (&v)[E], int g, int lo, int hi, int elim = E) {
    opaque(lo);
    opaque(hi);
    double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
        const int i = slot_index<E, G, IL>(g, e);
        const float xm = (i >= lo && i < hi) ? v[e] : 0.f;
        s[e % SGPU_NACC] += (double)xm;
    }
    return gsum_t<G>((s[0] + s[1]) + (s[2] + s[3]));
}

// Count sigma_clipping_float (rejection_float.c:49-60) low/high candidates
// over the visited slots.  Low candidates are a prefix and high ones a suffix
// of the sorted window (fl(m - x) and fl(x - m) are monotone in x).  No window
// predicate: slots outside the window hold the fill m (never a candidate:
// fl(m - m) = 0 is not > a threshold >= 0) or +Inf (always a high candidate;
// the caller subtracts those).  With both thresholds >= 0 a low candidate
// (x < m) is never a high one, so the reference's `else` needs no test.
// SIGNBIT: the sign-bit form below (device); false keeps the compare form
// (the MAD kernels' register allocation spills with the sign-bit form:
// mad100 37.6 -> 80 ms, measured).
template <int E, int G, bool SIGNBIT = true>
SG_HD void count_sigma(const float (&v)[E], float mf, float tl, float th, int &cl, int &ch,
                       int elim) {
#if defined(__HIP_DEVICE_COMPILE__) && !SGPU_COUNT_CMP
  if constexpr (SIGNBIT) {
    // Sign-bit form (no compares, no VCC round trips):
    // fl(mf - x) = -fl(x - mf) (round-to-nearest is symmetric), so with
    // d = fl(x - mf):  low  <=> d < -tl <=> fl(d + tl) < 0,
    //                  high <=> d > th  <=> fl(th - d) < 0,
    // and a float sum is < 0 exactly when its sign bit is set once -0 is
    // impossible: tl + 0 and th + 0 turn a -0 threshold into +0, and
    // x + (+0) / (+0) - x never round to -0 for x != -0.  +Inf slots give
    // fl(d + tl) = +Inf (not low) and fl(th - d) = -Inf (high), as the
    // compare form does.
    // Two slots per asm block: the scheduler cannot hoist the E differences
    // ahead of the pass (which spilled the N = 400 SIGMA column), and an
    // ext_vector (packed) form of this loop was miscompiled (the sign bit of
    // element .y taken from element .x).
    const float tlp = tl + 0.f, thp = th + 0.f;
    static_assert(E % 2 == 0, "pairs");
    unsigned a = 0, b = 0;
#pragma unroll
    for (int e = 0; e < E; e += 2) {
        SG_STOP4(e, elim);
        float d0, d1, t0, t1;
        asm("v_sub_f32 %2, %6, %8\n\t"          // d = x - mf
            "v_sub_f32 %3, %7, %8\n\t"
            "v_add_f32 %4, %2, %9\n\t"          // d + tl
            "v_add_f32 %5, %3, %9\n\t"
            "v_sub_f32 %2, %10, %2\n\t"         // th - d
            "v_sub_f32 %3, %10, %3\n\t"
            "v_lshrrev_b32 %4, 31, %4\n\t"
            "v_lshrrev_b32 %5, 31, %5\n\t"
            "v_lshrrev_b32 %2, 31, %2\n\t"
            "v_lshrrev_b32 %3, 31, %3\n\t"
            "v_add3_u32 %0, %0, %4, %5\n\t"
            "v_add3_u32 %1, %1, %2, %3"
            : "+v"(a), "+v"(b), "=&v"(d0), "=&v"(d1), "=&v"(t0), "=&v"(t1)
            : "v"(v[e]), "v"(v[e + 1]), "v"(mf), "v"(tlp), "v"(thp));
    }
    cl = gsum_t<G>((int)a);
    ch = gsum_t<G>((int)b);
    return;
  }
#endif
  {
    int a = 0, b = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
        const float x = v[e];
        a += (mf - x > tl) ? 1 : 0;
        b += (x - mf > th) ? 1 : 0;
    }
    cl = gsum_t<G>(a);
    ch = gsum_t<G>(b);
  }
}

// siril_stats_float_mad (statistics_float.c:79-101) -> histogram_median_float
// (sorting.c:644-649) -> findMinMaxPercentile at 0.5 (rt/rt_algo.cc:38-172)
// on the n window samples of a sorted column whose other visited slots hold
// +Inf: t = |x - mp| (float), lo / hi = min / max of t, scale = (n - 1) /
// (hi - lo), bin = (uint16)(scale * (t - lo)), and the 50th percentile
// interpolated inside the first bin k-1 whose cumulative count reaches
// thr = 0.5f * n.  The histogram walk becomes a bisection over the bin index
// b of count(b) = #{t : scale * (t - lo) < b + 1} (trunc(w) <= b <=> w < b+1
// for w >= 0; +Inf slots never count).  hi is at an end of the sorted window
// (t is convex in x), passed in as |x_first - mp| and |x_last - mp|.
template <int E, int G>
SG_HD float mad_sorted(const float (&v)[E], int n, float mp, float tfirst, float tlast, int elim) {
    float lo = f_inf();
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
        const float t = fabsf(v[e] - mp);
        lo = (t < lo) ? t : lo;
    }
    if constexpr (G >= 2) { const float o = gxchg<G, 1>(lo); lo = (o < lo) ? o : lo; }
    if constexpr (G >= 4) { const float o = gxchg<G, 2>(lo); lo = (o < lo) ? o : lo; }
    if constexpr (G >= 8) { const float o = gxchg<G, 4>(lo); lo = (o < lo) ? o : lo; }
    if constexpr (G >= 16) { const float o = gxchg<G, 8>(lo); lo = (o < lo) ? o : lo; }
    if constexpr (G >= 32) { const float o = gxchg<G, 16>(lo); lo = (o < lo) ? o : lo; }
    const float hi = (tfirst < tlast) ? tlast : tfirst;
    if (fabsf(hi - lo) == 0.f) return lo;
    const unsigned hs = (unsigned)n;                       // n < 65536
    const float scale = (float)(hs - 1) / (hi - lo);
    const float thr = 0.5f * (float)n;
    // count(b) for one bin bound (one pass)
    auto count_le = [&](int b) {
        const float lim = (float)(b + 1);
        int c = 0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            SG_STOP4(e, elim);
            const float w = scale * (fabsf(v[e] - mp) - lo);
            c += (w < lim) ? 1 : 0;
        }
        return gsum_t<G>(c);
    };
    int blo = 0, bhi = (int)hs - 1;                        // count(hs - 1) = n >= thr
    while (blo < bhi) {
        const int mid = (blo + bhi) >> 1;
        if ((float)count_le(mid) >= thr) bhi = mid;
        else blo = mid + 1;
    }
    const int k = blo + 1;
    const int count = count_le(blo);
    const int before = blo > 0 ? count_le(blo - 1) : 0;
    const float c0 = (float)count - thr, c1 = thr - (float)before;
    float out = (c1 * (float)k + c0 * (float)(k - 1)) / (c0 + c1);
    out /= scale;
    out += lo;
    const float m = (hi < out) ? hi : out;                 // rtengine::LIM
    return (lo < m) ? m : lo;
}

// siril_stats_ushort_mad (statistics.c:133-154) on the n window samples of a
// sorted 16-bit column (exact floats; other visited slots +Inf): t = |x - c|
// with c = round_to_int(median), whose median histogram_median / sortnet
// return as the k-th smallest t (n odd) or the mean of the (k-1)-th and k-th
// (n even), k = n/2, in double.  The k-th smallest is found by bisection over
// the integer values 0..tmax of count(t <= b); the (k-1)-th is the same value
// unless fewer than k samples lie below it, then the largest t below it.
template <int E, int G>
SG_HD float mad_u16_sorted(const float (&v)[E], int n, float c, float tmax, int elim) {
    auto count_le = [&](float b) {
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            SG_STOP4(e, elim);
            cnt += (fabsf(v[e] - c) <= b) ? 1 : 0;
        }
        return gsum_t<G>(cnt);
    };
    const int k = n / 2;
    int blo = 0, bhi = (int)tmax;                        // count(tmax) = n > k
    while (blo < bhi) {
        const int mid = (blo + bhi) >> 1;
        if (count_le((float)mid) >= k + 1) bhi = mid;
        else blo = mid + 1;
    }
    const float tk = (float)blo;
    if (n & 1) return tk;
    float tk1 = tk;
    if (count_le(tk - 1.f) < k) {
        // fewer than k samples strictly below tk: the (k-1)-th is tk itself
    } else {
        float m = -1.f;
#pragma unroll
        for (int e = 0; e < E; e++) {
            SG_STOP4(e, elim);
            const float t = fabsf(v[e] - c);
            m = (t < tk && t > m) ? t : m;
        }
        if constexpr (G >= 2) { const float o = gxchg<G, 1>(m); m = (o > m) ? o : m; }
        if constexpr (G >= 4) { const float o = gxchg<G, 2>(m); m = (o > m) ? o : m; }
        if constexpr (G >= 8) { const float o = gxchg<G, 4>(m); m = (o > m) ? o : m; }
        if constexpr (G >= 16) { const float o = gxchg<G, 8>(m); m = (o > m) ? o : m; }
        if constexpr (G >= 32) { const float o = gxchg<G, 16>(m); m = (o > m) ? o : m; }
        tk1 = m;
    }
    return (float)(((double)tk1 + (double)tk) / 2.0);
}

// ------------------------------------------------------------- per pixel
struct PixCfg {
    int nframes;
    float sig0, sig1;
    const float *crit;
    float m_x, m_dx2;
    int elim;        // slots per lane the interleaved passes visit (multiple of 4)
    ProfAcc *pa;     // diagnostic section timer (SGPU_PROF builds), or null
};
struct PixOut {
    int fallback;    // 1: defer to the exact sequential kernel
    double res;      // mean_and_reject() / quickmedian_float() result
    int rl, rh;      // rejected low / high
    int nkept;       // kept samples (apply_rejection_float return value)
    float pmin, pmax;// range of the kept samples (weighted mean)
};

// Iteration safety caps: the reference loops have none (WINSORIZED inner loop,
// SIGMEDIAN); a pixel hitting a cap is deferred to the exact kernel, which
// applies a much larger cap.
constexpr int kWinsorCap = 1000;
constexpr int kSigmedCap = 1000;

// The `N - r <= 4` rule of one rejection round: returns 1 when the outcome
// depends on the element order (pixel must be deferred), else applies it.
SG_HD int cutoff_round(int n, int &r, int cl, int ch, int &lo, int &hi, int &rl, int &rh,
                       bool &changed) {
    const int c = cl + ch;
    if (n - r <= 4) {            // no more rejections this round (:188-190)
        changed = false;
        return 0;
    }
    if (r + c > n - 4) return 1;  // candidates straddle the cutoff: order-dependent
    r += c;
    rl += cl;
    rh += ch;
    lo += cl;
    hi -= ch;
    changed = (c > 0);
    return 0;
}

// U16: DATA_USHORT column (apply_rejection_ushort, median_and_mean.c:703-954)
// held as exact floats.  Differences from the float path on the types the
// 16-bit sorted path runs (SIGMA, WINSORIZED, median): the initial median==0
// test also covers WINSORIZED (:747-756) and the Winsorize bounds are
// roundf_to_WORD(median -/+ 1.5 sigma) (:840-841); integer sums are exact in
// f64, and sd32 (statistics.c:115-127) is the float-path formula.
template <int NP, int G, int RT, int U16 = 0>
SG_HD PixOut pixel_sorted(float (&v)[NP / G], int g, int kept, const PixCfg &c) {
    constexpr int E = NP / G;
    // interleaved layout (padding-free passes) unless the type re-sorts
    // (SIGMEDIAN, LINEARFIT) or walks the block layout (GESDT, G == 1 anyway)
    // (measured at N = 400: the transpose pays for the Winsorized iteration
    // passes, 90.9 -> 83.0 ms at G = 8, not for SIGMA's few passes, 51.8 ->
    // 53.8 ms at G = 4)
    constexpr bool IL = (G == 1) || (RT != SIGMEDIAN && (G == 2 || (RT == WINSORIZED && G <= SGPU_IL_MAXG) ||
                                                         ((RT == SIGMA || RT == PERCENTILE) && G <= SGPU_IL_SIGMA_MAXG)));
    const int elim = IL ? c.elim : E;
    if constexpr (IL && G == 2) to_interleaved2<E>(v, g);
    else if constexpr (IL && G > 2) to_interleaved<E, G>(v, g);
    PixOut o;
    o.fallback = 0;
    o.res = 0.0;
    o.rl = o.rh = 0;
    o.nkept = 0;
    o.pmin = o.pmax = 0.f;
    const float slo = c.sig0, shi = c.sig1;

    if constexpr (RT == KMEDIAN) {
        // stack_median: quickmedian_float over all N samples, zeros included.
        // N is wave-uniform, so are the order-statistic indices.
        const int n = c.nframes, k = n / 2;
        o.res = median_win<E, G, IL>(v, 0, n);
        (void)k;
        return o;
    }
    // apply_rejection_float: kept <= 1 returns kept (:140-142); kept == 0 makes
    // mean_and_reject take a quickmedian of the stack -> exact kernel.
    if (kept == 0) { o.fallback = 1; return o; }
    if (kept == 1) {
        o.res = (double)ostat<E, G, IL>(v, 0);
        o.pmin = o.pmax = (float)o.res;
        o.nkept = 1;
        return o;
    }
    int lo = 0, hi = kept;
    // sum-order guard of the pixel: every sum below sees samples of
    // [vmin, vmax] (window subsets, their Winsorize clamps, median fills)
    const SumGuard sg = make_guard(ostat<E, G, IL>(v, 0), ostat<E, G, IL>(v, kept - 1), G * E + 2,
                                   (E + SGPU_NACC - 1) / SGPU_NACC + SGPU_NACC + ceil_log2(G) + 4, kept);

    if constexpr (RT == NO_REJEC || SGPU_ABL_NOREJ) {
        // handled here only for completeness (the streaming kernel is used)
    } else if constexpr (RT == PERCENTILE) {               // :148-173
        const double med = median_win<E, G, IL>(v, 0, kept);
        if (med == 0.0) { o.fallback = 1; return o; }
        const float mf = (float)med;
        int cl, ch;
        if constexpr (U16) {
            // WORD percentile_clipping (median_and_mean.c:589-603) divides by
            // the median: (m - x) / m > plow, (x - m) / m > phigh
            if (!(mf > 0.f)) { o.fallback = 1; return o; }
            int a = 0, b = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                SG_STOP4(e, elim);
                const float x = v[e];
                const bool l = (mf - x) / mf > slo;
                a += l ? 1 : 0;
                b += (!l && (x - mf) / mf > shi) ? 1 : 0;
            }
            cl = gsum_t<G>(a);
            ch = gsum_t<G>(b);
        } else {
            const float tl = mf * slo, th = mf * shi;   // s = median (:159-170)
            if (!(tl >= 0.f && th >= 0.f)) { o.fallback = 1; return o; }
            count_sigma<E, G>(v, mf, tl, th, cl, ch, elim);
        }
        ch -= G * elim - kept;                          // +Inf slots past the kept samples
        o.rl = cl;
        o.rh = ch;
        lo = cl;
        hi = kept - ch;
        if (hi - lo <= 0) { o.fallback = 1; return o; }
    } else if constexpr (RT == SIGMA) {                    // :149-209
        double med = median_win<E, G, IL>(v, 0, kept);
        if (med == 0.0) { o.fallback = 1; return o; }
        int r = 0;
        bool first = true, changed;
        do {
            // sd and median are independent reads of the window: take the
            // median first, it is the fill of the out-of-window slots
            if (!first) med = median_win<E, G, IL>(v, lo, hi - lo);
            first = false;
            const float mf = (float)med;
            float xlo = 0.f, xhi = 0.f;                  // window ends (mixed-sign columns' bound)
            if (!sg.pos) { xlo = ostat<E, G, IL>(v, lo); xhi = ostat<E, G, IL>(v, hi - 1); }
            fill_outside<E, G, IL>(v, g, lo, hi, mf, elim);
            const float var = sd_filled<NP, G, false>(v, hi - lo, mf, 0.f, 0.f, elim, 1.0 / (hi - lo),
                                                      1.0 / (hi - lo - 1), sg, xlo, xhi);
            if (var < 0.f) { o.fallback = 1; return o; }
            int cl, ch;
            const float tl = var * slo, th = var * shi;
            if (!(tl >= 0.f && th >= 0.f)) { o.fallback = 1; return o; }
            count_sigma<E, G>(v, mf, tl, th, cl, ch, elim);
            if (cutoff_round(hi - lo, r, cl, ch, lo, hi, o.rl, o.rh, changed)) {
                o.fallback = 1;
                return o;
            }
        } while (changed && hi - lo > 3);
    } else if constexpr (RT == WINSORIZED) {               // :223-259
        int r = 0;
        bool changed, first = true;
        do {
            const float mf = (float)median_win<E, G, IL>(v, lo, hi - lo);
            if (U16 && first && mf == 0.f) { o.fallback = 1; return o; }
            first = false;
            float xlo = 0.f, xhi = 0.f;                  // window ends (mixed-sign columns' bound)
            if (!sg.pos) { xlo = ostat<E, G, IL>(v, lo); xhi = ostat<E, G, IL>(v, hi - 1); }
            fill_outside<E, G, IL>(v, g, lo, hi, mf, elim);
            const int n = hi - lo;
            const double rn = 1.0 / n, rn1 = 1.0 / (n - 1);     // once per round
            SG_PMARK(c.pa, 2);
            float sigma = sd_filled<NP, G, false>(v, n, mf, 0.f, 0.f, elim, rn, rn1, sg, xlo, xhi);
            SG_PMARK(c.pa, 3);
            if (sigma < 0.f) { o.fallback = 1; return o; }
            int cl, ch;
            float L = -f_inf(), U = f_inf(), sigma0;
            int it = 0;
            do {
                float m0 = mf - 1.5f * sigma, m1 = mf + 1.5f * sigma;
                if (U16) {
                    m0 = roundf_to_word_f(m0);
                    m1 = roundf_to_word_f(m1);
                }
                L = fminf(m1, fmaxf(m0, L));   // composed clamp bounds
                U = fminf(m1, fmaxf(m0, U));
                sigma0 = sigma;
                const float sw = sd_filled<NP, G, true>(v, n, mf, L, U, elim, rn, rn1, sg, xlo, xhi);
                if (sw < 0.f || ++it > kWinsorCap) { o.fallback = 1; return o; }
                sigma = 1.134f * sw;
#if SGPU_ABL_ITERS
            } while (it < SGPU_ABL_ITERS);
#else
            } while (fabsf(sigma - sigma0) > sigma0 * 0.0005f);
#endif
            const float tl = sigma * slo, th = sigma * shi;
            if (!(tl >= 0.f && th >= 0.f)) { o.fallback = 1; return o; }
            count_sigma<E, G>(v, mf, tl, th, cl, ch, elim);
            SG_PMARK(c.pa, 6);
            if (cutoff_round(hi - lo, r, cl, ch, lo, hi, o.rl, o.rh, changed)) {
                o.fallback = 1;
                return o;
            }
            SG_PMARK(c.pa, 7);
        } while (changed && hi - lo > 3);
    } else if constexpr (RT == SIGMEDIAN) {                // :210-222
        // outliers are replaced by the median; re-sort keeps the column ordered
        int n, it = 0;
        bool first = true;
        do {
            const float sigma = sd_win<E, G, false>(v, g, 0, kept, 0.f, 0.f, sg);
            if (sigma < 0.f) { o.fallback = 1; return o; }     // order-dependent rounding
            const float mf = (float)median_win<E, G>(v, 0, kept);
            // 16-bit: median == 0 returns 0 kept (:747-756); the replacement
            // `stack[frame] = median` stores a float into a WORD (truncation)
            if (U16 && first && mf == 0.f) { o.fallback = 1; return o; }
            first = false;
            const float rep = U16 ? truncf(mf) : mf;
            int cl = 0, ch = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int i = g * E + e;
                const float x = v[e];
                const bool in = i < kept;
                const bool l = in && (mf - x > sigma * slo);
                const bool h = in && !l && (x - mf > sigma * shi);
                cl += l ? 1 : 0;
                ch += h ? 1 : 0;
                v[e] = (l || h) ? rep : x;
            }
            cl = gsum_t<G>(cl);
            ch = gsum_t<G>(ch);
            o.rl += cl;
            o.rh += ch;
            n = cl + ch;
            if (n > 0) sort_col<NP, G>(v, g);
            if (++it > kSigmedCap) { o.fallback = 1; return o; }
        } while (n > 0);
    } else if constexpr (RT == LINEARFIT) {                // :260-300, G == 1 only
        static_assert(G == 1, "LINEARFIT sorted path is single-lane");
        int r = 0, n = kept;
        bool changed;
        do {
            // siril_fit_linear on the sorted column (siril_fit_linear.c:24-50).
            // Every loop stops at slot elim (>= N >= n for every lane, wave-
            // uniform): the slots past it only ever hold +Inf.
            float m_y = v[0];
#pragma unroll
            for (int i = 1; i < E; i++) {
                SG_STOP4(i, elim);
                if (i < n) m_y += (v[i] - m_y) * (1.f / (float)(i + 1));
            }
            float m_dxdy = 0.f, dx = -c.m_x;
#pragma unroll
            for (int i = 0; i < E; i++) {
                SG_STOP4(i, elim);
                if (i < n) {
                    const float dy = v[i] - m_y;
                    m_dxdy += (dx * dy - m_dxdy) * (1.f / (float)(i + 1));
                    dx += 1.f;
                }
            }
            const float b = m_dxdy * c.m_dx2;   // slope
            const float a = m_y - c.m_x * b;    // intercept
            float sigma = 0.f;
#pragma unroll
            for (int i = 0; i < E; i++) {
                SG_STOP4(i, elim);
                if (i < n) sigma += fabsf(v[i] - (b * (float)i + a));
            }
            sigma /= (float)n;
            int rej = 0;
#pragma unroll
            for (int i = 0; i < E; i++) {
                SG_STOP4(i, elim);
                if (i < n && n - r > 4) {
                    const float x = v[i];
                    const float fi = (float)i;
                    int s = 0;
                    if (b * fi + a - x > sigma * slo) { o.rl++; s = 1; }
                    else if (x - b * fi - a > sigma * shi) { o.rh++; s = 1; }
                    if (s) { r++; rej++; v[i] = f_inf(); }
                }
            }
            changed = rej > 0;
            if (changed) sort_col<NP, G>(v, g);   // order-preserving compaction
            n -= rej;
        } while (changed && n > 3);
        hi = n;
    } else if constexpr (RT == GESDT) {                    // :301-348, G == 1 only
        static_assert(G == 1, "GESDT sorted path is single-lane");
        // gsl_stats_float_median_from_sorted_data: float add of the middle pair
        const int lhs = (kept - 1) / 2, rhs = kept / 2;
        const float ml = sel<E>(v, lhs), mr = sel<E>(v, rhs);
        const double median = (lhs == rhs) ? (double)ml : (ml + mr) / 2.0;
        int max_out = (int)((float)c.nframes * c.sig0);
        const int removed = c.nframes - kept;
        // the window sum below is kept by subtraction: exact only when every
        // sum of the column is (sum-order guard); otherwise defer
        if (removed < max_out && !sg.exact) { o.fallback = 1; return o; }
        if (removed < max_out) {
            max_out -= removed;
            // pass 1: the Grubbs sequence.  The window [wl, wh) loses its first
            // or last sample each iteration; its f64 sum is kept by
            // subtraction (exact whenever the reference's own double sums
            // are, the condition every sd pass here already relies on), so an
            // iteration is one squared-deviation pass plus the two end
            // samples.  The decisions (which end, above the median?) are kept
            // as bits for the confirmation replay.
            constexpr int MW = (E + 31) / 32;
            uint32_t hbits[MW], gbits[MW];
#pragma unroll
            for (int w = 0; w < MW; w++) hbits[w] = gbits[w] = 0u;
            int last = -1;
            {
                double S = sum_win<E, G, true>(v, g, 0, kept, elim);
                int wl = 0, wh = kept;
                for (int it = 0; it < max_out; it++) {
                    const int n = wh - wl;
                    const float avg = (float)(S / (double)n);   // siril_stats_float_sd's mean
                    double q[4] = {0.0, 0.0, 0.0, 0.0};
                    const unsigned un = (unsigned)n;
#pragma unroll
                    for (int e = 0; e < E; e++) {
                        SG_STOP4(e, elim);
                        const float d = v[e] - avg;
                        const float dd = ((unsigned)(e - wl) < un) ? d * d : 0.f;
                        q[e & 3] += (double)dd;
                    }
                    const double qv = ((q[0] + q[1]) + (q[2] + q[3])) / (double)(n - 1);
                    if (!f32_stable(qv, qv * sg.c)) { o.fallback = 1; return o; }
                    const float sd = sqrtf((float)qv);
                    const float lo_v = sel<E>(v, wl), hi_v = sel<E>(v, wh - 1);
                    float dev = avg - lo_v;
                    const float d2 = hi_v - avg;
                    const bool high = d2 > dev;
                    if (high) dev = d2;
                    const float G_ = dev / sd;
                    if (G_ > c.crit[it + removed]) last = it;
                    const float x = high ? hi_v : lo_v;
#pragma unroll
                    for (int w = 0; w < MW; w++) {
                        const uint32_t bit = ((it >> 5) == w) ? (1u << (it & 31)) : 0u;
                        hbits[w] |= high ? bit : 0u;
                        gbits[w] |= ((double)x >= median) ? bit : 0u;
                    }
                    S -= (double)x;
                    if (high) wh--; else wl++;
                }
            }
            // confirm_outliers (median_and_mean.c:685-701)
            int i_conf = max_out - 1;
            if (i_conf > 1) i_conf = (last > 1) ? last : 1;
            // pass 2: replay the recorded sequence, mark confirmed indices
            uint32_t mask[MW];
#pragma unroll
            for (int w = 0; w < MW; w++) mask[w] = 0u;
            {
                int cold = 0;
                for (int it = 0; it <= i_conf; it++) {
                    uint32_t hw = 0u, gw = 0u;
#pragma unroll
                    for (int w = 0; w < MW; w++) {
                        hw |= ((it >> 5) == w) ? hbits[w] : 0u;
                        gw |= ((it >> 5) == w) ? gbits[w] : 0u;
                    }
                    const bool high = (hw >> (it & 31)) & 1u;
                    const int size = kept - it;
                    const int idx = high ? size - 1 : cold++;   // reference index semantics
                    if ((gw >> (it & 31)) & 1u) o.rh++; else o.rl++;
#pragma unroll
                    for (int w = 0; w < MW; w++)
                        mask[w] |= ((idx >> 5) == w) ? (1u << (idx & 31)) : 0u;
                }
            }
            // compaction + mean over unmarked indices of [0, kept)
            double s = 0.0;
            int n = 0;
            float pmin = f_inf(), pmax = -f_inf();
#pragma unroll
            for (int e = 0; e < E; e++) {
                const bool keep = e < kept && !((mask[e >> 5] >> (e & 31)) & 1u);
                const float xm = keep ? v[e] : 0.f;
                s += (double)xm;
                n += keep ? 1 : 0;
                if (keep) { pmin = fminf(pmin, v[e]); pmax = fmaxf(pmax, v[e]); }
            }
            if (n == 0) { o.fallback = 1; return o; }
            o.res = s / (double)n;                            // exact sums (sg.exact)
            o.nkept = n;
            o.pmin = pmin;
            o.pmax = pmax;
            return o;
        }
    } else if constexpr (RT == MAD) {                      // :149-209 with var = MAD
        // the MAD of each round is taken around the PREVIOUS round's median
        // (var before `median = quickmedian(...)`, rejection_float.c:178-186)
        double med = median_win<E, G, IL>(v, 0, kept);
        if (med == 0.0) { o.fallback = 1; return o; }
        int r = 0;
        bool first = true, changed;
        do {
            const int n = hi - lo;
            const float mp = (float)med;
            fill_outside<E, G, IL>(v, g, lo, hi, f_inf(), elim);   // out-of-window: +Inf
            float var;
            if constexpr (U16) {
                // siril_stats_ushort_mad (statistics.c:133-154): the exact
                // median of |x - round_to_int(m)| over the window
                const float cm = (float)(int)((double)mp + 0.5);       // m > 0
                const float tf = fabsf(ostat<E, G, IL>(v, lo) - cm), tl_ = fabsf(ostat<E, G, IL>(v, hi - 1) - cm);
                var = mad_u16_sorted<E, G>(v, n, cm, tf > tl_ ? tf : tl_, elim);
            } else {
                const float tf = fabsf(ostat<E, G, IL>(v, lo) - mp), tl_ = fabsf(ostat<E, G, IL>(v, hi - 1) - mp);
                var = mad_sorted<E, G>(v, n, mp, tf, tl_, elim);
            }
            if (!first) med = median_win<E, G, IL>(v, lo, n);
            first = false;
            const float mf = (float)med;
            int cl, ch;
            const float tl = var * slo, th = var * shi;
            if (!(tl >= 0.f && th >= 0.f) || !(var - var == 0.f)) { o.fallback = 1; return o; }
            count_sigma<E, G, false>(v, mf, tl, th, cl, ch, elim);
            ch -= G * elim - n;                            // the +Inf slots outside the window
            if (cutoff_round(n, r, cl, ch, lo, hi, o.rl, o.rh, changed)) {
                o.fallback = 1;
                return o;
            }
        } while (changed && hi - lo > 3);
    }
    // mean of the kept window (median_and_mean.c:1083-1097)
    SG_PMARK(c.pa, 9);
#if SGPU_OPAQUE_FINAL
    opaque_col<E>(v);
#endif
    const int n = hi - lo;
    o.nkept = n;
    // (range first: evaluating the two select trees after the sum doubles
    // the register peak and spills)
    double st;
#if SGPU_RANGE_FIRST
    o.pmin = ostat<E, G, IL>(v, lo);
    o.pmax = ostat<E, G, IL>(v, hi - 1);
    fill_outside<E, G, IL>(v, g, lo, hi, 0.f, elim);   // out-of-window slots add 0
    st = sum_all<E, G>(v, elim);
#else
    st = sum_win<E, G, IL>(v, g, lo, hi, elim);
    o.pmin = ostat<E, G, IL>(v, lo);
    o.pmax = ostat<E, G, IL>(v, hi - 1);
#endif
    o.res = st / (double)n;
    // the output is (float)mean (median_and_mean.c:1725-1727): order-independent
    // when the sum is exact or the float is stable under the order error
    if (!U16 && !sg.exact && !f32_stable(o.res, (sum_bound(sg, st, o.pmin, o.pmax, G * elim) + fabs(st) * 0x1p-50) / n))
        o.fallback = 1;
    return o;
}

// ------------------------------------------------------------------ gather
// One sample of the column, median_and_mean.c:1615-1686: registration x-shift
// (zero outside the frame) then normalization in double, zeros kept at zero
// for the additive modes.
__device__ __forceinline__ float gather_sample(const KParams &p, int f, long long pix, int x) {
    long long idx = pix;
    if (p.shiftx) {
        const int s = p.shiftx[f];
        if (s && (x - s >= p.W || x - s < 0)) return 0.f;
        idx -= s;
    }
    const float v = p.frames[(long long)f * p.frame_stride + idx];
    switch (p.norm) {
        default:
        case NO_NORM:
            return v;
        case ADDITIVE:
        case ADDITIVE_SCALING:
            if (v != 0.f) {
                const double t = v * p.scale[f];
                return (float)(t - p.offset[f]);
            }
            return 0.f;
        case MULTIPLICATIVE:
        case MULTIPLICATIVE_SCALING: {
            const double t = v * p.scale[f];
            return (float)(t * p.mul[f]);
        }
    }
}

// 16-bit twin: the WORD the reference stores for the sample (zero outside the
// frame, round_to_WORD of the normalization affine, null samples null).
__device__ __forceinline__ float gather_sample16(const KParams &p, int f, long long pix, int x) {
    long long idx = pix;
    if (p.shiftx) {
        const int s = p.shiftx[f];
        if (s && (x - s >= p.W || x - s < 0)) return 0.f;
        idx -= s;
    }
    const float v = (float)p.frames16[(long long)f * p.frame_stride + idx];
    if (p.norm == NO_NORM || v == 0.f) return v;
    double t;
    switch (p.norm) {
        default:
        case ADDITIVE:
        case ADDITIVE_SCALING:
            t = (double)v * p.scale[f] - p.offset[f];
            break;
        case MULTIPLICATIVE:
        case MULTIPLICATIVE_SCALING:
            t = ((double)v * p.scale[f]) * p.mul[f];
            break;
    }
    t = t + 0.5;                                   // round_to_WORD, proto.h:232-237
    t = (t > 65535.0) ? 65535.0 : t;
    t = (t < 0.0) ? 0.0 : t;
    return (float)(uint32_t)t;
}

// A per-sample weight plane (data->drizz / data->mask) at the sample's
// shifted index (median_and_mean.c:1687-1692).  Out-of-frame samples read 0
// here; the reference keeps the previous pixel's weight there, but those
// samples are zero and never counted.
__device__ __forceinline__ float plane_at(const KParams &p, const float *pl, int f, long long pix, int x) {
    long long idx = pix;
    if (p.shiftx) {
        const int s = p.shiftx[f];
        if (s && (x - s >= p.W || x - s < 0)) return 0.f;
        idx -= s;
    }
    return pl[(long long)f * p.frame_stride + idx];
}
// weight of sample f in the weighted mean: n = 1 (x drizzle) (x mask)
// (x frame weight), in the reference's order (median_and_mean.c:1060-1066)
__device__ __forceinline__ double sample_weight(const KParams &p, int f, long long pix, int x) {
    double n = 1.;
    if (p.drizz) n *= plane_at(p, p.drizz, f, pix, x);
    if (p.mask) n *= plane_at(p, p.mask, f, pix, x);
    if (p.weights) n *= p.weights[f];
    return n;
}
__device__ __forceinline__ bool is_weighted(const KParams &p) { return p.weights || p.drizz || p.mask; }

// weighted branch of mean_and_reject, median_and_mean.c:1043-1082 (float)
// and :967-1016 (DATA_USHORT: the same formula on the stored WORDs), over the
// ORIGINAL frame order (o_stack), re-gathered sequentially by one lane.
template <int U16 = 0>
__device__ __forceinline__ double weighted_mean(const KParams &p, long long pix, int x, float pmin,
                                                float pmax, int kept) {
    double sum = 0.0, norm = 0.0;
    for (int f = 0; f < p.nframes; f++) {
        const float val = U16 ? gather_sample16(p, f, pix, x) : gather_sample(p, f, pix, x);
        if (val >= pmin && val <= pmax && val != 0.f) {
            const double w = sample_weight(p, f, pix, x);
            sum += (double)val * w;
            norm += w;
        }
    }
    if (norm == 0. || sum == 0.) {
        sum = 0.;
        for (int f = 0; f < p.nframes; f++) {
            const float val = U16 ? gather_sample16(p, f, pix, x) : gather_sample(p, f, pix, x);
            if (val >= pmin && val <= pmax && val > 0) sum += (double)val;
        }
        return sum / (double)kept;
    }
    return sum / norm;
}

__device__ __forceinline__ void write_result(const KParams &p, long long pix, double res, int rl,
                                             int rh) {
    float fr = (float)res;
    if (!p.output_norm) {                       // set_float_in_interval, proto.h:384-388
        fr = (fr < 0.f) ? 0.f : fr;
        fr = (fr > 1.f) ? 1.f : fr;
    }
    p.out[pix] = fr;
    if (p.rej_lo) p.rej_lo[pix] = (uint16_t)(rl > 65535 ? 65535 : rl);   // truncate_to_WORD
    if (p.rej_hi) p.rej_hi[pix] = (uint16_t)(rh > 65535 ? 65535 : rh);
}

// 16-bit output (k_stack_exact16 epilogue): float image in [0,1] via
// double_ushort_to_float_range and/or round_to_WORD (proto.h:232-237)
__device__ __forceinline__ void write_result16(const KParams &p, long long pix, double res, int rl,
                                               int rh) {
    if (p.out_f32) {
        float fr = (float)res * .000015259022f;
        if (!p.output_norm) {
            fr = (fr < 0.f) ? 0.f : fr;
            fr = (fr > 1.f) ? 1.f : fr;
        }
        p.out[pix] = fr;
    }
    if (p.out16) {
        const double r = res * p.out16_mul;     // normalize_to16bit (x1 is exact)
        double t = r + 0.5;
        t = (t > 65535.0) ? 65535.0 : t;
        t = (t < 0.0) ? 0.0 : t;
        p.out16[pix] = (uint16_t)t;
    }
    if (p.rej_lo) p.rej_lo[pix] = (uint16_t)(rl > 65535 ? 65535 : rl);
    if (p.rej_hi) p.rej_hi[pix] = (uint16_t)(rh > 65535 ? 65535 : rh);
}

// wave-level reduction of the rejection counters: one atomic per wave
// Append to a device list from the active lanes of a wave: one atomic per
// wave (its ballot's popcount) instead of one per lane -- thousands of
// same-address atomics serialise across the XCDs.  Every active lane must
// call it; lanes with pred == false get -1.
__device__ __forceinline__ int wave_append(int *counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m == 0ull) return -1;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, (int)__popcll(m));
    base = __shfl(base, leader, 64);
    return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// a thread's 64-bit totals at the end of a sequential kernel (lanes may have
// left early, so no wave reduction): one atomic pair per thread, spread over
// the stripes by the global thread index (or on `counts`)
__device__ __forceinline__ void add_counts64(const KParams &p, unsigned long long a, unsigned long long b) {
    if (!(a | b)) return;
    unsigned long long *dst = p.counts;
    if (p.cstripe) {
        const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
        dst = p.cstripe + (size_t)(t % kCountStripes) * 8;
    }
    atomicAdd(dst, a);
    atomicAdd(dst + 1, b);
}

__device__ __forceinline__ void add_counts(const KParams &p, int rl, int rh) {
    unsigned long long a = (unsigned)rl, b = (unsigned)rh;
#pragma unroll
    for (int lm = 5; lm >= 0; lm--) {
        a += __shfl_xor(a, 1 << lm, 64);
        b += __shfl_xor(b, 1 << lm, 64);
    }
    if ((threadIdx.x & 63) == 0 && (a | b)) {
        unsigned long long *dst = p.counts;
        if (p.cstripe) {
            const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
            dst = p.cstripe + (size_t)(w % kCountStripes) * 8;
        }
        atomicAdd(dst, a);
        atomicAdd(dst + 1, b);
    }
}

// Column gather.  XF == 0: plain frames.  XF == 1: registration x-shift and
// normalization, median_and_mean.c:1615-1686, folded into one formula with
// per-frame (scale, mul, offset) prepared by the host:
//     additive:        (float)((v*scale)*1   - offset), v != 0
//     multiplicative:  (float)((v*scale)*mul - 0)
// (x*1 and x-0 are exact, so both reproduce the reference's rounding); null
// samples stay null.  The shift table holds 0 for unshifted frames.
// All E loads of a lane are issued before the first use.
//
// Padding slots (frame >= N) read 0 through the buffer range check: the
// descriptor of slot e covers only the frames that exist from its base frame
// on, so the rejection types (DROP_ZERO: zero = missing) need no per-slot
// liveness predicate at all -- a dead slot is just a missing sample.  The
// median stack keeps zeros, so there dead slots are forced to +Inf.
// U16: 16-bit frames (p.frames16), samples converted exactly to float; with
// XF the registration shift and the normalization to WORD (round_to_WORD of
// the same affine, as the reference stores DATA_USHORT stacks).
// RS: slots e >= RS are padding in every lane (the launch's real-slot bound,
// rs_pick): no load and no conversion for them, they are +Inf outright.
#ifndef SGPU_GATHER_SLOTSTEP
#define SGPU_GATHER_SLOTSTEP 1
#endif
template <int XF, int E, int G, bool DROP_ZERO, int U16 = 0, int RS = E, bool SLOTSTEP = SGPU_GATHER_SLOTSTEP>
__device__ __forceinline__ void gather_column(const KParams &p, float (&v)[E], long long pix, int x,
                                              int g, int &kept, int &bad) {
    const int N = p.nframes;
    const uint32_t off = (uint32_t)pix;   // host guarantees npix < 2^30
    constexpr uint32_t ES = U16 ? 2u : 4u;  // bytes per sample
    // lane g of the group reads frames e*G + g: the descriptor is built on the
    // wave-uniform frame e*G (SGPRs, no waterfall loop) and the lane's frame
    // offset g*frame_stride goes into the 32-bit VGPR byte offset (the
    // launcher checks (G-1)*stride*4 + npix*4 < 2^32)
    const uint32_t fbytes = (uint32_t)(p.frame_stride * ES);
    const uint32_t lane_off = (uint32_t)g * fbytes;
    float raw[E];
    // NaN / Inf detector: fma(x, 0, acc) turns NaN once any sample is NaN or
    // infinite (one instruction a slot; the x - x == 0 test and its count
    // were three).  Measured with the compile-time padding selects below
    // (profiles/r06x3_ab_gather_trim.txt): config 2 11.58 -> 11.46 ms,
    // sigma100 8.16 -> 8.03 ms, median100 unchanged.
    float nacc = 0.f;
    // slots whose base frame is past the last frame are padding in every lane
    // (frames e*G + g): no load at all for them (a wave-uniform stop at
    // ceil(N / G), in chunks of SGPU_STOP_GRAN), they read as missing.
    // Measured (profiles/r03n_ab.txt): winsorized400 70.7 -> 52.8 ms, sigma100
    // 11.9 -> 9.9, winsorized100 17.3 -> 16.3; but the E = 128, G = 4 column
    // (N = 257..512 SIGMA / PERCENTILE) spills more SGPRs with it, 43.2 -> 46.1
    // ms, so that shape keeps the plain loop
    // (Round 6: dropping the stop under a compile-time real-slot bound -- its
    // exits rematerialise the zeros of the slots not yet loaded, ~550 v_mov
    // per lane in the prep kernel -- measured slower: config 2 15.6 vs 12.0
    // ms with the same prep otherwise, profiles/r06g_ab.txt.  The grouped
    // issue of the loads between the exits is worth more than the moves.)
    constexpr bool GSTOP = SGPU_GATHER_STOP && !(E == 128 && G == 4);
    const int elg = GSTOP ? (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1) : E;
    // (no zero-initialisation of raw: the stop's exits then had to
    // rematerialise the zeros of every slot not yet loaded on the path that
    // continues -- ~480 v_mov per lane in the prep kernel at N = 100; the
    // conversion below selects 0 for the slots past the stop instead)
    // Per-slot descriptors in few scalar instructions (round 6): the slot's
    // base address advances by one 64-bit add per slot (not a multiply of
    // the frame index), and its record count is one of the G + 1 values
    // (frames present from the base frame on: 0 .. G) picked by a clamp.  A
    // slot with no frame present keeps its (unused) base and 0 records, so
    // every lane's load is dropped.  (The per-slot multiplies, clamps of the
    // base frame and their hazard nops were ~17 scalar instructions a slot:
    // 1 559 of the median kernel's 4 300 instructions per wave.)  Measured
    // (profiles/r06r_ab_gather_slotstep.txt): sigma100 8.08 -> 7.96 ms,
    // median100 2.07 -> 2.04 ms, but the moment path's prep kernel 0.5 %
    // slower (11.50 -> 11.58 ms), so prep keeps the clamped form (SLOTSTEP
    // false).
    uint32_t nrec_c[G + 1];
    nrec_c[0] = 0u;
#pragma unroll
    for (int c = 1; c <= G; c++) nrec_c[c] = (uint32_t)(c - 1) * fbytes + (uint32_t)p.npix * ES;
    const char *slot_base = U16 ? (const char *)p.frames16 : (const char *)p.frames;
    const long long slot_step = (long long)G * p.frame_stride * ES;
#pragma unroll
    for (int e = 0; e < RS; e++) {
        if constexpr (GSTOP) {
            SG_STOP4(e, elg);
        }
        const int f0 = e * G;                            // uniform base frame
        uint32_t nrec;
        const char *fpb;
        if constexpr (SLOTSTEP) {
            const int rem = N - f0;                      // frames present from f0 on, unclamped
            nrec = nrec_c[0];
#pragma unroll
            for (int c = 1; c <= G; c++) nrec = (c == G ? rem >= c : rem == c) ? nrec_c[c] : nrec;
            fpb = slot_base;
            slot_base += slot_step;
        } else {                                         // base frame clamped to N - 1, multiplied out
            const int fb = f0 < N ? f0 : N - 1;
            const int cnt = f0 < N ? (N - f0 < G ? N - f0 : G) : 0;
            nrec = cnt > 0 ? (uint32_t)(cnt - 1) * fbytes + (uint32_t)p.npix * ES : 0u;
            fpb = (U16 ? (const char *)p.frames16 : (const char *)p.frames) + (long long)fb * p.frame_stride * ES;
        }
        uint32_t o = off;
        if (XF) {
            const int fe = min(f0 + g, N - 1);
            const int sh = p.shiftx[fe];
            const int xs = x - sh;
            o = (xs >= 0 && xs < p.W) ? off - (uint32_t)sh : off;
        }
        if constexpr (U16) {
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(fpb), (short)0, (int)nrec, 0x00020000);
            raw[e] = (float)(uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsrc, (int)(lane_off + o * 2u), 0, 0);
        } else {
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(fpb), (short)0, (int)nrec, 0x00020000);
            raw[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(lane_off + o * 4u), 0, 0));
        }
    }
#pragma unroll
    for (int e = RS; e < E; e++) v[e] = f_inf();
#pragma unroll
    for (int e = 0; e < RS; e++) {
        float val = (!GSTOP || e < elg) ? raw[e] : 0.f;   // past the stop: a missing sample
        if (XF) {
            const int fe = min(e * G + g, N - 1);
            const int sh = p.shiftx[fe];
            const int xs = x - sh;
            const bool outside = !(xs >= 0 && xs < p.W);   // sh == 0 is never outside
            if constexpr (U16) {
                // normalized WORD samples (median_and_mean.c:1665-1684):
                // round_to_WORD((v * pscale) * pmul - poffset) of the non-null
                // samples (the host's one formula; x * 1 and x - 0 are exact)
                if (p.norm != NO_NORM && val != 0.f) {
                    double t = (double)val * p.scale[fe] * p.mul[fe] - p.offset[fe];
                    t = t + 0.5;
                    t = (t > 65535.0) ? 65535.0 : t;
                    t = (t < 0.0) ? 0.0 : t;
                    val = (float)(uint32_t)t;
                }
                val = outside ? 0.f : val;
            } else {
                const double t = (double)val * p.scale[fe] * p.mul[fe] - p.offset[fe];
                val = (outside || val == 0.f) ? 0.f : (float)t;
            }
            // drizzle: a sample with a null weight is removed like a null
            // pixel (rejection_float.c:117-126)
            if (p.drizz && !outside && p.drizz[(long long)fe * p.frame_stride + (pix - sh)] == 0.f) val = 0.f;
        }
        // NaN/Inf detector: x - x is 0 for every finite x, NaN otherwise
        nacc = __builtin_fmaf(val, 0.f, nacc);
        if (DROP_ZERO) {
            const bool z = (val == 0.f);                  // null sample = missing
            kept += z ? 0 : 1;
            v[e] = z ? f_inf() : val;
        } else {
            constexpr int FMIN = RS < E ? G * (RS - (E == 64 ? 4 : 8)) + 1 : 0;   // frames every N of the bucket has
            v[e] = (e * G + G - 1 < FMIN || e * G + g < N) ? val : f_inf();
        }
    }
    bad |= (nacc != nacc) ? 1 : 0;
}

// One pixel of the sorted path (gather, sort, rejection, output); rl / rh
// receive its counts (lane 0 of the group).
template <int NP, int G, int RT, int XF, int U16, bool LATE = false, int RS = NP / G>
__device__ __forceinline__ void stack_pixel(const KParams &p, long long pix, int g, int &rl, int &rh) {
    constexpr int E = NP / G;
    constexpr bool DZ = (RT != KMEDIAN);
    const int x = (int)(pix % p.W);
    const int N = p.nframes;
    float v[E];
    int kept = 0, bad = 0;
    ProfAcc pacc, *pa = nullptr;
#if SGPU_PROF
    if (p.prof) {
        pa = &pacc;
        pacc.t = __builtin_readcyclecounter();
        for (int q = 0; q < 12; q++) pacc.acc[q] = 0;
    }
#endif
    gather_column<XF, E, G, DZ, U16, RS>(p, v, pix, x, g, kept, bad);
    SG_PMARK(pa, 0);
    bad = gsum_t<G>(bad);
    kept = gsum_t<G>(kept);
    PixOut o;
    if (bad) {
        o.fallback = 1;
    } else {
#if !SGPU_ABL_NOSORT
        if constexpr (RT == KMEDIAN && G == 1 && RS < E && SGPU_MEDIAN_SELECT) {
            // the median stack reads ranks N/2 - 1 and N/2 only: the network
            // pruned to what N in this real-slot bucket (rs_pick: N in
            // (RS - step, RS]) can read
            constexpr int step = E == 64 ? 4 : 8;
            oem_select<E, RS, (RS - step + 1) / 2 - 1, RS / 2 + 1>(v);
        } else {
            sort_col<NP, G, RS>(v, g);
        }
#endif
        SG_PMARK(pa, 1);
        // interleaved passes visit ceil(N/G) slots per lane, rounded to 4
        const int el = (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
        PixCfg c{N, p.sig0, p.sig1, p.crit, p.m_x, p.m_dx2, el < E ? el : E, pa};
        o = pixel_sorted<NP, G, RT, U16>(v, g, kept, c);
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (LATE) {
        // the direct launch re-derives its pixel (and the address arithmetic
        // of the write) from the work-item id after the rejection, instead of
        // keeping the 64-bit index and pointers live across it: the large
        // columns' kernels spilled exactly those (NP = 512: 11 dwords a lane)
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        pix = ((long long)blockIdx.x * blockDim.x + tid) / G;
    }
#endif
    if (o.fallback) {
        if (g == 0) {
            const int slot = wave_append(p.fb_count, true);
            p.fb_list[slot] = (int)pix;
        }
    } else if (g == 0) {
        double res = o.res;
        if (RT != KMEDIAN && is_weighted(p))
            res = weighted_mean<U16>(p, pix, (int)(pix % p.W), o.pmin, o.pmax, o.nkept);
        if constexpr (U16) write_result16(p, pix, res, o.rl, o.rh);
        else write_result(p, pix, res, o.rl, o.rh);
        rl += o.rl;
        rh += o.rh;
    }
    SG_PMARK(pa, 8);
#if SGPU_PROF
    if (pa) {
        for (int q = 0; q < 12; q++) {
            unsigned long long a = pacc.acc[q];
            for (int lm = 5; lm >= 0; lm--) a += __shfl_xor(a, 1 << lm, 64);
            if ((threadIdx.x & 63) == 0) atomicAdd(p.prof + q, a);
        }
    }
#endif
}

// LIST = 0: every pixel of the block; LIST = 1: the pixels of p.fb2_list
// (the moment path's fallbacks, stack_wz.h), grid-stride over the list.
// RS: real-slot bound of the direct launch's sort network (sort_col).
template <int NP, int G, int RT, int XF, int W, int U16 = 0, int LIST = 0, int RS = NP / G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_sorted(KParams p) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int g = (int)(gid % G);
    int rl = 0, rh = 0;
    if constexpr (LIST) {
        const long long n = *p.fb2_count, stride = (long long)gridDim.x * blockDim.x / G;
        for (long long i = gid / G; i < n; i += stride) stack_pixel<NP, G, RT, XF, U16>(p, p.fb2_list[i], g, rl, rh);
    } else {
        const long long pix = gid / G;
        if (pix < p.npix)
            stack_pixel<NP, G, RT, XF, U16, (SGPU_LATE_PIX && NP >= 256), RS>(p, pix, g, rl, rh);
    }
    add_counts(p, rl, rh);
}

}  // namespace sgpu
