// stack_wz.h -- WINSORIZED (float) stack on moments: the column lives in
// registers only for the gather, the sort and ONE pass; every rejection round
// after that is scalar work on the window's moments plus reads of a few ranks
// from an LDS copy of the sorted column's ends and middle.
//
// Why: the reference (rejection_float.c:223-259) runs, per round, an sd pass
// pair, a quickselect median, and per clamp iteration two more O(N) passes
// (siril_stats_float_sd of w_stack); the register-resident sorted path
// (stack_sorted_impl.h) still pays a median select, a fill pass, two sd
// passes, a count pass per round and two passes per iteration.  Here:
//   * ranks: the sorted column's low KT, middle KM and high KT ranks go to
//     LDS (RankStore); medians, tail samples, clip candidates and the window
//     ends are single LDS reads;
//   * moments: W1 = sum (x - c0), W2 = sum (x - c0)^2 over the window (one
//     f64 pass, c0 the first median); a round's clipped samples are
//     subtracted, the clamped tails of an iteration are taken out of them
//     (the samples below L / above U are a prefix / suffix of the window);
//   * sigma: every sd the reference computes -- the round's first sd and the
//     1.134 sd of each clamp iteration -- is known from the moments up to the
//     reference's own float rounding, so it is carried as an interval that
//     provably holds the reference's float (var_bounds below); the stop test
//     and the final clip must have one outcome over the intervals;
//   * mean: sum x = W1 + n c0, exact whenever the sum-order guard proves the
//     window's sums exact, else checked for float stability.
// DATA_USHORT columns (apply_rejection_ushort, median_and_mean.c:831-860; U16
// template flag): the same path on the WORD samples held as exact floats.
// The differences are the ones the 16-bit sorted path has: the Winsorize
// bounds are roundf_to_WORD(median -/+ 1.5 sigma) (:840-841; monotone, so
// the sigma interval maps to integer bound intervals), a first median of 0
// leaves no sample (:747-756: the exact kernel takes the pixel), the sd is
// siril_stats_ushort_sd_32 (statistics.c:115-127: the float-path formula on
// integers) and the mean is the exact integer sum over kept (:1020-1034).
// Any undecidable step, or a rank outside the stored ranges, sends the pixel
// to the register-resident kernel (second launch over the list fb2_list),
// whose own deferrals go to the exact sequential kernel as before.  So every
// pixel's result is the one the sorted path -- i.e. the reference -- gives.
#pragma once
#include "stack_sorted_impl.h"

// Ranks stored per end (KT) and around the median (KM) at N <= 128.  Sized
// from the ranks the rounds visit (scripts/wzstat on the benchmark recipe:
// depth from an end p50 / p99 / p99.9 = 7 / 13-14 / 15-16, from the middle
// 1 / 3 / 4; 16 / 8 hold every read of 99.5 % of the moment-path pixels) so
// that the rounds kernel can stage a wave's records in LDS (R = 40 slots,
// 10 KB per wave, 4 waves / SIMD): config 2 13.65 -> 12.78 ms with the LDS
// rounds (24 / 16 with global reads: 13.65; 16 / 8 with global reads: 14.35,
// the extra fallbacks unpaid; profiles/r05r_ab_*.log)
#ifndef SGPU_WZ_KT
#define SGPU_WZ_KT 16
#endif
#ifndef SGPU_WZ_KM
#define SGPU_WZ_KM 8
#endif
// instrumentation hook of the host statistics tool (scripts/wzstat): empty in
// every product build
#ifndef SGPU_WZ_TRACE
#define SGPU_WZ_TRACE(ev) ((void)0)
#endif

namespace sgpu {

SG_HD unsigned umul24(unsigned a, unsigned b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul24(a, b);
#else
    return (a & 0xffffffu) * (b & 0xffffffu);
#endif
}

// sqrtf bounds: RN(sqrt(x)) lies in [sqrt_lo(x), sqrt_hi(x)] (the device's
// v_sqrt_f32 is within 1 ulp; the neighbours of its result bracket the
// correctly rounded root; zero stays exact)
SG_HD float fnext(float r) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, r) + 1u); }
SG_HD float fprev(float r) { return r > 0.f ? __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, r) - 1u) : 0.f; }
SG_HD float fsqrt_raw(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
SG_HD float sqrt_lo(float x) { return x < 0x1p-100f ? 0.f : fprev(fsqrt_raw(x)); }
SG_HD float sqrt_hi(float x) { return x == 0.f ? 0.f : (x < 0x1p-100f ? 0x1p-49f : fnext(fsqrt_raw(x))); }

// sigma_clipping_float's candidates (rejection_float.c:49-60) for a sigma
// known only to lie in an interval: thresholds tl in [tl0, tl1], th in
// [th0, th1].  Low candidates (mf - x > tl) are a prefix of the sorted window
// and high ones (x - mf > th) a suffix, so they are counted by walking the
// stored ranks from each end under the larger thresholds; the first sample
// that is not a candidate there must not be one under the smaller ones
// either.  Returns 0 (cl / ch set), 1 ambiguous, 2 a walk left the stored
// ranks (count with passes instead).
template <class TS>
SG_HD int wz_clip_counts(const TS &ts, int lo, int hi, float mf, float tl0, float th0, float tl1, float th1,
                         int &cl, int &ch) {
    float x;
    int k = 0;
    for (;;) {
        if (lo + k >= hi || !ts.fetch(lo + k, x)) return 2;
        if (!(mf - x > tl1)) break;
        k++;
    }
    if (mf - x > tl0) return 1;
    cl = k;
    k = 0;
    for (;;) {
        if (hi - 1 - k < lo + cl || !ts.fetch(hi - 1 - k, x)) return 2;
        if (!(x - mf > th1)) break;
        k++;
    }
    if (x - mf > th0) return 1;
    ch = k;
    return 0;
}

// Ranks kept per pixel: [0, KT), [mid0, mid0 + KM) around kept/2 and
// [kept - KT, kept).  LDS layout [rank slot][pixel of the wave]: the wave's
// pixels read consecutive words (no bank conflicts).
template <int NP, int G>
struct RankStore {
    static constexpr int E = NP / G;
    static constexpr int PW = 64 / G;                      // pixels per wave
    static constexpr int KT = NP <= 128 ? SGPU_WZ_KT : NP / 4;   // ranks per end
    static constexpr int KM = NP <= 128 ? SGPU_WZ_KM : 16; // ranks around the median
    static constexpr int R = 2 * KT + KM;                  // slots per pixel
    float *base;                                           // rank slot j of this pixel at base[j * stride + p]
    long long stride, p;                                   // LDS: the wave's pixels; global: the launch's
    int kept, mid0, mid1, hi0;                             // stored: [0, KT), [mid0, mid1), [hi0, kept)
    // stores the interleaved sorted column (lane g, slot e = rank e*G + g);
    // the slot loops cover the wave's range of `kept` (kmin..kmax, uniform),
    // the rank tests are per pixel
    SG_HD void store(const float (&v)[E], int g, int kmin, int kmax) {
        mid0 = kept / 2 - KM / 2;
        hi0 = kept - KT;
        hi0 = hi0 < 0 ? 0 : hi0;
        const int eh0 = (kmin - KT) / G - 1, eln = (kmax + G - 1) / G;
        const int em0 = (kmin / 2 - KM / 2) / G - 1, em1 = (kmax / 2 + KM / 2) / G + 1;
        // what the slot loops can reach of this pixel's ranges
        hi0 = hi0 > eh0 * G ? hi0 : (eh0 > 0 ? eh0 * G : 0);
        mid1 = mid0 + KM < (em1 + 1) * G ? mid0 + KM : (em1 + 1) * G;
        mid0 = mid0 > em0 * G ? mid0 : em0 * G;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const int r = e * G + g;
            if (e < (KT + G - 1) / G) {
                if (r < KT && r < kept) base[r * stride + p] = v[e];
            }
            if (e >= eh0 && e < eln) {
                if (r >= hi0 && r < kept) base[(KT + KM + r - (kept - KT)) * stride + p] = v[e];
            }
            if (e >= em0 && e <= em1) {
                if (r >= mid0 && r < mid1 && r < kept) base[(KT + r - (kept / 2 - KM / 2)) * stride + p] = v[e];
            }
        }
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // The same store into the HBM record of the prep kernel, with the rank
    // tests moved into buffer descriptors: one raw-buffer descriptor per
    // region (low [0, KT), middle [KT, KT + KM), high [KT + KM, R)), whose
    // record count is the region's size, and a per-lane 32-bit byte offset
    // (the pixel's column + the rank's slot within the region, wrapping
    // modulo 2^32 when the slot is negative).  A rank outside its region --
    // below it (a huge unsigned offset) or above it -- is past the record
    // count, and the hardware drops the store; so every slot of the
    // wave-uniform loops is stored unconditionally: one 32-bit add per store
    // instead of a 64-bit multiply, a compare and an exec-mask branch.  The
    // regions then hold exactly what store() puts there (plus +Inf in slots of
    // ranks >= kept, which fetch never reads).  Needs NP * stride * 4 <=
    // 2^32 (negative slots >= -NP stay above the record count), which the
    // launcher enforces (stack_sorted_inst.h).
    __device__ void store_buf(const float (&v)[E], int g, int kmin, int kmax) {
        mid0 = kept / 2 - KM / 2;
        hi0 = kept - KT;
        hi0 = hi0 < 0 ? 0 : hi0;
        const int eh0 = (kmin - KT) / G - 1, eln = (kmax + G - 1) / G;
        const int em0 = (kmin / 2 - KM / 2) / G - 1, em1 = (kmax / 2 + KM / 2) / G + 1;
        hi0 = hi0 > eh0 * G ? hi0 : (eh0 > 0 ? eh0 * G : 0);
        mid1 = mid0 + KM < (em1 + 1) * G ? mid0 + KM : (em1 + 1) * G;
        mid0 = mid0 > em0 * G ? mid0 : em0 * G;
        const uint32_t S4 = (uint32_t)stride * 4u;
        const uint32_t pb = (uint32_t)p * 4u;
        const auto rlo = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)((uint32_t)KT * S4), 0x00020000);
        const auto rmid = __builtin_amdgcn_make_buffer_rsrc(base + (long long)KT * stride, (short)0,
                                                            (int)((uint32_t)KM * S4), 0x00020000);
        const auto rhi = __builtin_amdgcn_make_buffer_rsrc(base + (long long)(KT + KM) * stride, (short)0,
                                                           (int)((uint32_t)KT * S4), 0x00020000);
        const uint32_t blo = pb + (uint32_t)g * S4;
        const uint32_t bhi = pb + (uint32_t)(g + KT - kept) * S4;
        const uint32_t bmid = pb + (uint32_t)(g - (kept / 2 - KM / 2)) * S4;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const uint32_t eo = (uint32_t)(e * G) * S4;
            const uint32_t x = __builtin_bit_cast(uint32_t, v[e]);     // the b32 store takes the bits
            if (e < (KT + G - 1) / G) __builtin_amdgcn_raw_buffer_store_b32(x, rlo, (int)(blo + eo), 0, 0);
            if (e >= eh0 && e < eln) __builtin_amdgcn_raw_buffer_store_b32(x, rhi, (int)(bhi + eo), 0, 0);
            if (e >= em0 && e <= em1) __builtin_amdgcn_raw_buffer_store_b32(x, rmid, (int)(bmid + eo), 0, 0);
        }
    }
#endif
    // rank r (0 <= r < kept); false when not stored (the pixel falls back).
    // Branch-free: the slot is selected, one load is issued (slot 0 when the
    // rank is not stored), so the rounds' fetch loops carry no divergent
    // control flow per range test.
    SG_HD bool fetch(int r, float &x) const {
        const bool lo_ok = r < KT && r < kept, hi_ok = r >= hi0 && r < kept, mid_ok = r >= mid0 && r < mid1;
        const int slot = lo_ok ? r : hi_ok ? KT + KM + r - (kept - KT) : KT + r - (kept / 2 - KM / 2);
        const bool ok = lo_ok || hi_ok || mid_ok;
        // slot < R and stride = the chunk's pixels < 2^23 with R * stride <
        // 2^32 (both enforced by the launcher, stack_sorted_inst.h): one
        // full-rate 24-bit multiply whose 32-bit product cannot wrap; the
        // pixel's base address is loop-invariant (a 64-bit multiply per fetch
        // was quarter-rate work)
        x = (base + p)[umul24((unsigned)(ok ? slot : 0), (unsigned)stride)];
        return ok;
    }
};

// Bounds of the reference's (float)(vsum / (n - 1)) (siril_stats_float_sd,
// statistics.h:80-106) for the window's samples clamped to [L, U], L in
// [Llo, Lhi], U in [Ulo, Uhi] (no clamp: a = c = 0, widths 0).  R1 / R2:
// moments about c0 of the samples between the clamps at the inner corner
// (Lhi, Ulo); a / c: samples below Lhi / above Ulo; E1 / E2: bounds of the
// absolute f64 errors of R1 / R2.  The argument:
//   * the reference sums fl(fl(w - mean)^2) in f64, mean = (float)(sum w / n);
//     each term is within (1 + u)^3 of (w - mean)^2 (u = 2^-24), the f64 sum
//     within its order bound (sg.c) of the exact one, and
//     sum (w - mean)^2 = V*(L, U) + n (mean - mean*)^2, mean* the exact mean,
//     |mean - mean*| <= half an ulp + the order error of sum w;
//   * V*(L, U) = sum (w - mean*)^2 decreases as L rises or U falls
//     (dV*/dL = 2 a(L) (L - mean*) <= 0): it is smallest at the inner corner,
//     computed here from the moments, and grows by at most
//     2 a |L - mean*| dL + 2 c |U - mean*| dU towards (Llo, Uhi);
//   * every float step after the f64 sum -- the (float) conversion, sqrtf
//     (bracketed by sqrt_lo / sqrt_hi), 1.134f *, 1.5f *, m -+ t, min / max --
//     is monotone, so interval ends map to interval ends.
SG_HD void var_bounds(double R1, double R2, float E1, float E2, int a, int c, int n, float c0, float Llo, float Lhi,
                      float Ulo, float Uhi, bool clamped, float eps, float sgc, double rn, double rn1,
                      float &varlo, float &varhi) {
    const float af = (float)a, cf = (float)c;
    double VA, DA;
    float lAf = 0.f, uAf = 0.f, dL = 0.f, dU = 0.f, wmax;
    if (clamped) {
        const double lA = (double)Lhi - (double)c0, uA = (double)Ulo - (double)c0;
        DA = (double)a * lA + (double)c * uA + R1;
        const double QA = (double)a * (lA * lA) + (double)c * (uA * uA) + R2;
        VA = QA - DA * DA * rn;
        lAf = fabsf((float)lA) * 1.0000002f;
        uAf = fabsf((float)uA) * 1.0000002f;
        // widths of the clamp intervals: fl(Lhi - Llo) <= (1 + 2^-24)(Lhi - Llo)
        // (Lhi >= Llo), so the f32 difference times 1 + 2^-22.3 bounds them
        // from above like the f64 form did
        dL = (Lhi - Llo) * 1.0000002f;
        dU = (Uhi - Ulo) * 1.0000002f;
        wmax = fmaxf(fabsf(Llo), fabsf(Uhi));
    } else {
        DA = R1;
        VA = R2 - DA * DA * rn;
        // |w| <= max |x| over the window: |c0| + the moments' spread bound
        wmax = fabsf(c0) + sqrtf((float)R2 * 1.0001f + E2) * 1.0001f;
    }
    const float rnf = (float)rn * 1.0000002f;
    const float DAf = fabsf((float)DA) * 1.0000002f;
    const float fe1 = E1 + eps * (af * lAf + cf * uAf);
    const float fe2 = E2 + eps * (af * lAf * lAf + cf * uAf * uAf);
    const float eV = fe2 + eps * DAf * DAf * rnf + (2.f * DAf + fe1) * fe1 * rnf;
    const float dev = (DAf + af * dL + cf * dU + fe1) * rnf;
    const float dB = 2.f * af * (lAf + dL + dev) * dL + 2.f * cf * (uAf + dU + dev) * dU;
    const float dmu = wmax * (0x1p-23f + sgc) + fe1 * rnf + 0x1p-120f;
    const float u3c = 3.0000002f * 0x1p-24f + sgc + 0x1p-49f;
    const float eHi = (eV + dB + (float)n * dmu * dmu) * (1.f + 0x1p-18f);
    const double Vlo = (VA - (double)(eV * (1.f + 0x1p-18f))) * (1.0 - (double)u3c) - (double)n * 0x1p-125;
    const double Vhi = (VA + (double)eHi) * (1.0 + (double)u3c) + (double)n * 0x1p-125;
    varlo = (float)((Vlo > 0.0 ? Vlo : 0.0) * rn1);
    varhi = (Vhi - Vhi == 0.0) ? (float)(Vhi * rn1) : f_inf();
}

// median_win's rounding (sorting.c:240-273, 468-513) on two fetched ranks
SG_HD float median_from(float a, float b, int n) {
    if (n & 1) return b;
    if (n < 9) return (float)((double)(a + b) / 2.0);
    return (float)(((double)a + b) / 2.0);
}

// Rejection state of one pixel between rounds (kept in HBM between the
// launches of the round-wise rounds kernel) and the per-pixel constants the
// rounds read (recomputed from the stored ranks at every launch).
struct WzState {
    double W1, W2;           // window moments about c0
    float E1, E2;            // their absolute error bounds
    int lo, hi, r, rl, rh;   // window, cutoff counter, rejected low / high
    int pad;
};
struct WzConst {
    SumGuard sg;
    float c0, eps, sgc, slo_, shi_;
    int kept;
    bool exact_w1;
};

// The per-pixel constants (the preamble of the reference's loop): 0, or 1
// when the extreme ranks are not stored.  m: samples the moments pass visited.
template <class RS>
SG_HD int wz_consts(const RS &rs, int kept, float c0, int m, float slo_, float shi_, WzConst &k, float &ymax,
                    float &vmin) {
    float vmax;
    if (!rs.fetch(0, vmin) || !rs.fetch(kept - 1, vmax)) return 1;
    k.sg = make_guard(vmin, vmax, m + 2, (m + SGPU_NACC - 1) / SGPU_NACC + SGPU_NACC + 9, kept);
    k.eps = (float)(4 * m + 64) * 0x1p-53f;
    k.sgc = (float)k.sg.c * 1.0001f;
    k.c0 = c0;
    k.slo_ = slo_;
    k.shi_ = shi_;
    k.kept = kept;
    ymax = fmaxf(fabsf(vmin - c0), fabsf(vmax - c0)) * 1.0001f;
    // every y and every partial sum of them on the grid of ulp(vmin) / 2 (c0
    // may be a midpoint) within 2^53 of it
    k.exact_w1 = vmin > 0.f && (ebits(vmax) - ebits(vmin) + 26 + ceil_log2(kept) <= 53);
    return 0;
}

#ifndef SGPU_WZ_BATCH
#define SGPU_WZ_BATCH 0          // 1: four-rank batched walks (measured slower, 16.2-17.2 vs 15.8 ms: A/B only)
#endif

// Four consecutive ranks of one end of the window (r, r + d, r + 2d, r + 3d;
// d = +1 from the low end, -1 from the high end), fetched as one batch of
// independent loads and consumed in order: the walks of a round pay one load
// latency per four samples instead of one per sample.  ok: bit j set when
// rank j of the batch is stored (negative ranks are never fetched).
struct RankRun {
    float x0, x1, x2, x3;
    unsigned ok;
    int left;
};
template <class RS>
SG_HD void run_fill(const RS &rs, RankRun &b, int r, int d) {
    float *x[4] = {&b.x0, &b.x1, &b.x2, &b.x3};
    b.ok = 0u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int rj = r + j * d;
        const bool ok = rs.fetch(rj < 0 ? 0 : rj, *x[j]) && rj >= 0;
        b.ok |= ok ? (1u << j) : 0u;
    }
    b.left = 4;
}
SG_HD void run_pop(RankRun &b) {
    b.x0 = b.x1;
    b.x1 = b.x2;
    b.x2 = b.x3;
    b.ok >>= 1;
    b.left--;
}

// take sample x out of the moments (one clamped or clipped sample)
SG_HD void wz_take(float x, float c0, float eps, double &M1, double &M2, float &F1, float &F2) {
    const double y = (double)x - (double)c0;
    M1 -= y;
    M2 = fma(-y, y, M2);
    F1 += eps * fabsf((float)y);
    F2 += eps * (float)(y * y);
}

// One rejection round of the pixel on moments (rejection_float.c:223-259,
// one pass of its do-while).  Returns 0 (st updated; more: another round
// follows), 1: the sorted kernel takes the pixel, 2: the exact kernel takes
// it (order-dependent cutoff, as the sorted path decides).
template <int U16 = 0, class RS>
SG_HD int wz_round(const RS &rs, const WzConst &k, WzState &st, bool &more) {
    const float c0 = k.c0, eps = k.eps, sgc = k.sgc;
    int lo = st.lo, hi = st.hi;
    const int n = hi - lo;
    const double rn = 1.0 / n, rn1 = 1.0 / (n - 1);
#if SGPU_WZ_BATCH
    // one batch of independent loads: the median pair and four ranks at each
    // end of the window (the window ends, the first samples the clamps and
    // the clip walk reach)
    float ma, mb;
    const bool okm = rs.fetch(lo + n / 2 - ((n & 1) ? 0 : 1), ma) & rs.fetch(lo + n / 2, mb);
    RankRun e0, e1;                        // ranks lo.. and hi-1.. as of the round start
    run_fill(rs, e0, lo, 1);
    run_fill(rs, e1, hi - 1, -1);
    if (!okm || !(e0.ok & e1.ok & 1u)) return 1;
    const float mf = median_from(ma, mb, n);
    SGPU_WZ_TRACE(0);
    const float xw0 = e0.x0, xw1 = e1.x0;
#else
    float ma, mb;
    if (!rs.fetch(lo + n / 2 - ((n & 1) ? 0 : 1), ma) || !rs.fetch(lo + n / 2, mb)) return 1;
    const float mf = median_from(ma, mb, n);
    SGPU_WZ_TRACE(0);
    float xw0, xw1;
    if (!rs.fetch(lo, xw0) || !rs.fetch(hi - 1, xw1)) return 1;
#endif
    // the round's first sd (siril_stats_float_sd of the window, :226)
    float vlo, vhi;
    const bool flat = xw0 == xw1;         // constant window: every sd below is exactly 0
    var_bounds(st.W1, st.W2, st.E1, st.E2, 0, 0, n, c0, 0.f, 0.f, 0.f, 0.f, false, eps, sgc, rn, rn1, vlo, vhi);
    if (flat) vlo = vhi = 0.f;
    float slo = sqrt_lo(vlo), shi = sqrt_hi(vhi);
    // clamp iterations (:229-237)
    float Llo = -f_inf(), Lhi = -f_inf(), Ulo = f_inf(), Uhi = f_inf();
    int a = 0, c = 0;
    double R1 = st.W1, R2 = st.W2;
    float F1 = st.E1, F2 = st.E2;
#if SGPU_WZ_BATCH
    RankRun wl = e0, wh = e1;             // next samples to clamp: wl.x0 = rank lo + a, wh.x0 = rank hi - 1 - c
#else
    float nlo = xw0, nhi = xw1;           // next samples to clamp: ranks lo + a, hi - 1 - c
#endif
    for (int it = 0;;) {
        const float tlo = 1.5f * slo, thi = 1.5f * shi;
        float m0lo = mf - thi, m0hi = mf - tlo, m1lo = mf + tlo, m1hi = mf + thi;
        if (U16) {   // roundf_to_WORD of every end (monotone)
            m0lo = roundf_to_word_f(m0lo);
            m0hi = roundf_to_word_f(m0hi);
            m1lo = roundf_to_word_f(m1lo);
            m1hi = roundf_to_word_f(m1hi);
        }
        Llo = fminf(m1lo, fmaxf(m0lo, Llo));
        Lhi = fminf(m1hi, fmaxf(m0hi, Lhi));
        Ulo = fminf(m1lo, fmaxf(m0lo, Ulo));
        Uhi = fminf(m1hi, fmaxf(m0hi, Uhi));
#if SGPU_WZ_BATCH
        while (wl.x0 < Lhi) {
            wz_take(wl.x0, c0, eps, R1, R2, F1, F2);
            if (++a + c >= n) return 1;
            run_pop(wl);
            if (wl.left == 0) run_fill(rs, wl, lo + a, 1);
            if (!(wl.ok & 1u)) return 1;
        }
        while (wh.x0 > Ulo) {
            wz_take(wh.x0, c0, eps, R1, R2, F1, F2);
            if (a + ++c >= n) return 1;
            run_pop(wh);
            if (wh.left == 0) run_fill(rs, wh, hi - 1 - c, -1);
            if (!(wh.ok & 1u)) return 1;
        }
#else
        while (nlo < Lhi) {
            wz_take(nlo, c0, eps, R1, R2, F1, F2);
            if (++a + c >= n || !rs.fetch(lo + a, nlo)) return 1;
        }
        while (nhi > Ulo) {
            wz_take(nhi, c0, eps, R1, R2, F1, F2);
            if (a + ++c >= n || !rs.fetch(hi - 1 - c, nhi)) return 1;
        }
#endif
        SGPU_WZ_TRACE(1);
        var_bounds(R1, R2, F1, F2, a, c, n, c0, Llo, Lhi, Ulo, Uhi, true, eps, sgc, rn, rn1, vlo, vhi);
        if (flat) vlo = vhi = 0.f;
        if (!(vhi - vhi == 0.f)) return 1;
        const float s0lo = slo, s0hi = shi;
        slo = 1.134f * sqrt_lo(vlo);
        shi = 1.134f * sqrt_hi(vhi);
        const float A = slo - s0hi, B = shi - s0lo;      // fl(sigma - sigma0) in [A, B]
        const float dmin = A > 0.f ? A : (B < 0.f ? -B : 0.f);
        const float dmax = fmaxf(fabsf(A), fabsf(B));
        if (dmin > s0hi * 0.0005f) {
            if (++it > kWinsorCap) return 1;
            continue;
        }
        if (dmax <= s0lo * 0.0005f) break;
        return 1;
    }
    // sigma_clipping_float (:238-246) with sigma in [slo, shi]
    int cl = 0, ch = 0;
#if SGPU_WZ_BATCH
    // the clip candidates are the window's first ranks from each end: walked
    // from the round-start batches (more only past four candidates), and
    // taken out of the moments as they are counted -- the same samples, in
    // the same order (lows ascending, then highs descending), that the
    // round-3 form subtracted after cutoff_round; a pixel that leaves below
    // (ambiguous, order-dependent cutoff) discards st
    if (n - st.r > 4) {
        const float tl0 = slo * k.slo_, th0 = slo * k.shi_, tl1 = shi * k.slo_, th1 = shi * k.shi_;
        if (!(tl0 >= 0.f && th0 >= 0.f)) return 2;
        float x;
        RankRun b = e0;
        for (int j = 0;; j++) {
            if (lo + j >= hi) return 1;
            if (b.left == 0) run_fill(rs, b, lo + j, 1);
            if (!(b.ok & 1u)) return 1;
            x = b.x0;
            if (!(mf - x > tl1)) break;
            wz_take(x, c0, eps, st.W1, st.W2, st.E1, st.E2);
            run_pop(b);
            cl++;
        }
        if (mf - x > tl0) return 1;
        b = e1;
        for (int j = 0;; j++) {
            if (hi - 1 - j < lo + cl) return 1;
            if (b.left == 0) run_fill(rs, b, hi - 1 - j, -1);
            if (!(b.ok & 1u)) return 1;
            x = b.x0;
            if (!(x - mf > th1)) break;
            wz_take(x, c0, eps, st.W1, st.W2, st.E1, st.E2);
            run_pop(b);
            ch++;
        }
        if (x - mf > th0) return 1;
    }
    bool changed;
    if (cutoff_round(n, st.r, cl, ch, lo, hi, st.rl, st.rh, changed)) return 2;
#else
    if (n - st.r > 4) {
        const float tl0 = slo * k.slo_, th0 = slo * k.shi_, tl1 = shi * k.slo_, th1 = shi * k.shi_;
        if (!(tl0 >= 0.f && th0 >= 0.f)) return 2;
        if (wz_clip_counts(rs, lo, hi, mf, tl0, th0, tl1, th1, cl, ch)) return 1;
    }
    // the clipped samples leave the moments (before the window moves)
    const int lo0 = lo, hi0 = hi;
    bool changed;
    if (cutoff_round(n, st.r, cl, ch, lo, hi, st.rl, st.rh, changed)) return 2;
    for (int j = 0; j < lo - lo0 + (hi0 - hi); j++) {
        float x;
        const int rk = j < lo - lo0 ? lo0 + j : hi0 - 1 - (j - (lo - lo0));
        if (!rs.fetch(rk, x)) return 1;
        wz_take(x, c0, eps, st.W1, st.W2, st.E1, st.E2);
    }
#endif
    st.lo = lo;
    st.hi = hi;
    more = changed && hi - lo > 3;
    return 0;
}

// mean of the kept window (median_and_mean.c:1083-1097): sum x = W1 + n c0
template <class RS>
SG_HD int wz_final(const RS &rs, const WzConst &k, const WzState &st, PixOut &o) {
    const int n = st.hi - st.lo;
    o.rl = st.rl;
    o.rh = st.rh;
    if (!rs.fetch(st.lo, o.pmin) || !rs.fetch(st.hi - 1, o.pmax)) return 1;
    const double s = st.W1 + (double)n * (double)k.c0;
    o.res = s / (double)n;
    o.nkept = n;
    if (!k.exact_w1) {
        const double e = (double)st.E1 * 1.0001 + sum_bound(k.sg, s, o.pmin, o.pmax, n) + fabs(s) * 0x1p-50;
        if (!f32_stable(o.res, e / n)) return 1;
    }
    return 0;
}

// Start of a pixel: 3 when o is final already (kept == 1), 1 for the sorted
// kernel, else 0 with k / st ready for the rounds.
template <int U16 = 0, class RS>
SG_HD int wz_start(const RS &rs, int kept, double W1, double W2, float c0, int m, float slo_, float shi_,
                   WzConst &k, WzState &st, PixOut &o) {
    o.rl = o.rh = 0;
    o.res = 0.0;
    o.nkept = 0;
    o.pmin = o.pmax = 0.f;
    o.fallback = 0;
    if (kept == 1) {                        // apply_rejection_float returns kept <= 1 (:140-142)
        float v0;
        if (!rs.fetch(0, v0)) return 1;
        o.res = (double)v0;
        o.pmin = o.pmax = v0;
        o.nkept = 1;
        return 3;
    }
    if (U16 && c0 == 0.f) return 4;         // 16-bit: median 0 -> no sample kept (:747-756): exact kernel
    float ymax, vmin;
    if (wz_consts(rs, kept, c0, m, slo_, shi_, k, ymax, vmin)) return 1;
    st.W1 = W1;
    st.W2 = W2;
    st.E1 = k.eps * (float)kept * ymax;
    st.E2 = k.eps * (float)W2;
    st.lo = 0;
    st.hi = kept;
    st.r = st.rl = st.rh = 0;
    st.pad = 0;
    return 0;
}

// Second half of a pixel: from the stored ranks and the window moments (W1,
// W2 about c0) to the result, every round in one call.  Returns the route
// (0 result in o, 1 sorted kernel, 2 exact kernel).  m: samples the moments
// pass visited.  (A one-phase-per-call state machine with lane refill, so
// that lanes do not wait for the slowest pixel of their wave, was built and
// measured slower: 25.1 vs 17.1 ms for config 2 -- every trip pays every
// phase some lane is in.  The round-wise launches below refill at round
// granularity instead.)
template <int U16 = 0, class RS>
SG_HD int wz_finish(const RS &rs, int kept, double W1, double W2, float c0, int m, float slo_, float shi_,
                    PixOut &o) {
    WzConst k;
    WzState st;
    int rc = wz_start<U16>(rs, kept, W1, W2, c0, m, slo_, shi_, k, st, o);
    if (rc == 3) return 0;
    if (rc == 4) return 2;
    if (rc) return rc;
    bool more = true;
    while (more)
        if ((rc = wz_round<U16>(rs, k, st, more))) return rc;
    return wz_final(rs, k, st, o);
}

// First half: sort the gathered column, store its ranks, and the window
// moments about the first median c0 (one f64 pass; ranks >= kept hold +Inf
// and add 0).  Returns 2 for the exact kernel (kept == 0), else 0.
// GBUF: the record is the prep kernel's HBM one (RankStore::store_buf).
template <int NP, int G, int RSL = NP / G, bool GBUF = false>
SG_HD int wz_prepare(float (&v)[NP / G], int g, int kept, int kmin, int N, RankStore<NP, G> &rs, double &W1,
                     double &W2, float &c0) {
    constexpr int E = NP / G;
    if (kept == 0) return 2;                // quickmedian of the whole stack (median_and_mean.c:1040)
    sort_col<NP, G, RSL>(v, g);
    if constexpr (G == 2) to_interleaved2<E>(v, g);
    else if constexpr (G > 2) to_interleaved<E, G>(v, g);
    rs.kept = kept;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GBUF) rs.store_buf(v, g, kmin, N);
    else rs.store(v, g, kmin, N);
#else
    rs.store(v, g, kmin, N);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GBUF) {
        // c0 from the middle slots only: the two ranks median_win reads,
        // (kept - 1) / 2 .. kept / 2, lie in slots [(kmin / 2 - 1) / G,
        // (N / 2) / G] over the wave (kept in [kmin, N]), a wave-uniform
        // window of a few slots -- a select chain over it instead of two
        // 63-deep select trees over the whole column
        const int ra = kept / 2 - ((kept & 1) ? 0 : 1), rb = kept / 2;
        const int ew0 = (kmin / 2 - 1) / G, ew1 = (N / 2) / G;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int e = 0; e < E; e++) {
            if (e >= ew0 && e <= ew1) {
                sa = (e == ra / G) ? v[e] : sa;
                sb = (e == rb / G) ? v[e] : sb;
            }
        }
        c0 = median_from(gbcast<G>(sa, ra & (G - 1)), gbcast<G>(sb, rb & (G - 1)), kept);
    } else {
        c0 = (float)median_win<E, G, true>(v, 0, kept);
    }
#else
    c0 = (float)median_win<E, G, true>(v, 0, kept);
#endif
    const int el = (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
    const int elim = el < E ? el : E;
    double s1[SGPU_NACC], s2[SGPU_NACC];
#pragma unroll
    for (int q = 0; q < SGPU_NACC; q++) s1[q] = s2[q] = 0.0;
    const double cd = (double)c0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        SG_STOP4(e, elim);
        const float xe = v[e] < f_inf() ? v[e] : c0;
        const double y = (double)xe - cd;
        s1[e % SGPU_NACC] += y;
        s2[e % SGPU_NACC] = fma(y, y, s2[e % SGPU_NACC]);
    }
    W1 = s1[0];
    W2 = s2[0];
#pragma unroll
    for (int q = 1; q < SGPU_NACC; q++) {
        W1 += s1[q];
        W2 += s2[q];
    }
    W1 = gsum_t<G>(W1);
    W2 = gsum_t<G>(W2);
    return 0;
}

// One pixel after the gather (single-kernel form: LDS rank store; hostsim).
template <int NP, int G, int U16 = 0>
SG_HD int wz_pixel(float (&v)[NP / G], int g, int kept, int kmin, int N, float slo_, float shi_,
                   RankStore<NP, G> &rs, PixOut &o) {
    constexpr int E = NP / G;
    double W1, W2;
    float c0;
    o.rl = o.rh = 0;
    if (wz_prepare<NP, G>(v, g, kept, kmin, N, rs, W1, W2, c0)) return 2;
    return wz_finish<U16>(rs, kept, W1, W2, c0, G * E, slo_, shi_, o);
}

// The kernel: one pixel per group of G lanes (interleaved layout after the
// sort), 4 waves per block.
template <int NP, int G, int XF, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_wz(KParams p) {
    constexpr int E = NP / G;
    using RS = RankStore<NP, G>;
    __shared__ float s_rank[4 * RS::PW * RS::R];
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long pix = gid / G;
    const int g = (int)(gid % G);
    int rl = 0, rh = 0;
    if (pix < p.npix) {       // group-uniform
        const int x = (int)(pix % p.W);
        int kept = 0, bad = 0;
        RS rs;
        rs.base = s_rank + (threadIdx.x >> 6) * (RS::PW * RS::R);
        rs.stride = RS::PW;
        rs.p = (int)(threadIdx.x & 63) / G;
        PixOut o;
        int route;
        {
            float v[E];
            gather_column<XF, E, G, true>(p, v, pix, x, g, kept, bad);
            bad = gsum_t<G>(bad);
            kept = gsum_t<G>(kept);
            // the wave's smallest kept (uniform: the rank store's slot
            // loops; any value keeps the store and its reads consistent)
            int kmin = kept;
#pragma unroll
            for (int lm = 32; lm >= 1; lm >>= 1) kmin = min(kmin, __shfl_xor(kmin, lm, 64));
            kmin = __builtin_amdgcn_readfirstlane(kmin);
            route = bad ? 2 : wz_pixel<NP, G>(v, g, kept, kmin, p.nframes, p.sig0, p.sig1, rs, o);
        }
        if (route == 1) {
            if (g == 0) {
                const int slot = wave_append(p.fb2_count, true);
                p.fb2_list[slot] = (int)pix;
            }
        } else if (route == 2) {
            if (g == 0) {
                const int slot = wave_append(p.fb_count, true);
                p.fb_list[slot] = (int)pix;
            }
        } else if (g == 0) {
            double res = o.res;
            if (is_weighted(p)) res = weighted_mean(p, pix, x, o.pmin, o.pmax, o.nkept);
            write_result(p, pix, res, o.rl, o.rh);
            rl = o.rl;
            rh = o.rh;
        }
    }
    add_counts(p, rl, rh);
}

// ---------------------------------------------------------------- one lane per pixel, column in LDS
// SGPU_WZ=6: one pixel per lane (E = NP samples in VGPRs, G = 1: no
// cross-lane merge in the sort), the WHOLE sorted column written to LDS
// (lane-major rows of LS = N | 1 floats: lanes reading the same rank hit
// different banks), moments from the registers, then every round reads its
// ranks from LDS -- every rank is available (no stored-range fallbacks) and
// no rank record ever goes to HBM (traffic = the frames + the output).
struct ColStore {
    const float *base;                   // this lane's row: rank r at base[r]
    int kept;
    SG_HD bool fetch(int r, float &x) const {
        const bool ok = r >= 0 && r < kept;
        x = base[ok ? r : 0];
        return ok;
    }
};

// From the sorted column (ranks 0..N-1 in row[], missing samples +Inf at
// ranks >= kept) to the result: first median (median_win's rounding), the
// window moments about it in rank order (accumulator q takes ranks = q mod
// SGPU_NACC; ranks >= kept add 0), then every round on ColStore.  Shared by
// k_stack_wz1 (row in LDS) and the host simulation (tests/hostsim).
SG_HD int wz1_pixel(const float *row, int kept, int N, float sig0, float sig1, PixOut &o) {
    const int k2 = kept / 2;
    const float c0 = median_from(row[(kept & 1) ? k2 : k2 - 1], row[k2], kept);
    const double cd = (double)c0;
    double s1[SGPU_NACC], s2[SGPU_NACC];
#pragma unroll
    for (int q = 0; q < SGPU_NACC; q++) s1[q] = s2[q] = 0.0;
    const int el = (N + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
    for (int e = 0; e < el; e += SGPU_NACC) {
#pragma unroll
        for (int q = 0; q < SGPU_NACC; q++) {
            const int r = e + q;
            const float xe = r < kept ? row[r < N ? r : 0] : c0;
            const double y = (double)xe - cd;
            s1[q] += y;
            s2[q] = fma(y, y, s2[q]);
        }
    }
    double W1 = s1[0], W2 = s2[0];
#pragma unroll
    for (int q = 1; q < SGPU_NACC; q++) {
        W1 += s1[q];
        W2 += s2[q];
    }
    ColStore cs;
    cs.base = row;
    cs.kept = kept;
    return wz_finish(cs, kept, W1, W2, c0, el, sig0, sig1, o);
}

template <int NP, int XF, int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_wz1(KParams p, int LS) {
    extern __shared__ float s_col[];
    const int lane = (int)threadIdx.x;
    const long long pix = (long long)blockIdx.x * 64 + lane;
    const bool live = pix < p.npix;
    const int N = p.nframes;
    int rl = 0, rh = 0;
    int route = 2;
    PixOut o;
    int kept = 0, bad = 0;
    float *row = s_col + lane * LS;
    {
        // the column lives in VGPRs only for the gather and the sort; it
        // leaves for LDS right after (keeps the register peak at the sort's)
        float v[NP];
        // a dead lane gathers the block's first pixel (valid addresses) and
        // is discarded below; every lane runs the sort (wave-uniform code)
        const long long gp = live ? pix : (long long)blockIdx.x * 64;
        gather_column<XF, NP, 1, true>(p, v, gp, (int)(gp % p.W), 0, kept, bad);
        sort_col<NP, 1>(v, 0);
#if defined(__HIP_DEVICE_COMPILE__)
        // no scheduling of the stores into the sort network: interleaved,
        // they stretch the live ranges past the 256 VGPRs (66 spilled)
        __builtin_amdgcn_sched_barrier(0);
#endif
        // every slot is stored (no per-slot branches: they blew the register
        // allocation up); the padding slots e >= N all land on the row's
        // spare word row[N] (LS > N)
#pragma unroll
        for (int e = 0; e < NP; e++) row[e < N ? e : N] = v[e];
    }
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
    if (live) {
        route = (!bad && kept > 0) ? wz1_pixel(row, kept, N, p.sig0, p.sig1, o)
                                   : 2;   // NaN / Inf, or kept == 0: the exact kernel
        if (route == 1) {
            const int slot = wave_append(p.fb2_count, true);
            p.fb2_list[slot] = (int)pix;
        } else if (route == 2) {
            const int slot = wave_append(p.fb_count, true);
            p.fb_list[slot] = (int)pix;
        } else {
            double res = o.res;
            if (is_weighted(p)) res = weighted_mean(p, pix, (int)(pix % p.W), o.pmin, o.pmax, o.nkept);
            write_result(p, pix, res, o.rl, o.rh);
            rl = o.rl;
            rh = o.rh;
        }
    }
    add_counts(p, rl, rh);
}

// ---------------------------------------------------------------- two-kernel form
// The same path split where its needs split: k_stack_wz_prep (gather, sort,
// rank store, moments: the register-wide part, G lanes per pixel) writes a
// record per pixel to HBM -- ranks slot-major (lanes of a wave read
// neighbouring words), moments and packed bounds -- and k_stack_wz_rounds
// runs the latency-bound scalar rounds one lane per pixel at a few dozen
// VGPRs, so four times the pixels per SIMD are in flight.
// RSL: real-slot bound of the sort network (sort_col; the launch picks it
// with rs_pick, stack_sorted_rs*.hip instantiate the pruned variants)
template <int NP, int G, int XF, int W, int RSL = NP / G, int U16 = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_wz_prep(KParams p) {
    constexpr int E = NP / G;
    using RS = RankStore<NP, G>;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long loc = gid / G;
    const int g = (int)(gid % G);
    if (loc >= p.wz_cnt) return;              // group-uniform; no cross-wave work below
    const long long pix = p.wz_pix0 + loc;
    const int x = (int)(pix % p.W);
    int kept = 0, bad = 0;
    float v[E];
#ifndef SGPU_PREP_GATHER_RS
#define SGPU_PREP_GATHER_RS 0    // 1: the gather also bounded at RSL (A/B; the runtime gather stop already skips those loads)
#endif
    gather_column<XF, E, G, true, U16, SGPU_PREP_GATHER_RS ? RSL : E, false>(p, v, pix, x, g, kept, bad);
    bad = gsum_t<G>(bad);
    kept = gsum_t<G>(kept);
    int kmin = kept;
#pragma unroll
    for (int lm = 32; lm >= 1; lm >>= 1) kmin = min(kmin, __shfl_xor(kmin, lm, 64));
    kmin = __builtin_amdgcn_readfirstlane(kmin);
    RS rs;
    rs.base = p.wz_ranks;
    rs.stride = p.wz_cnt;
    rs.p = loc;
    double W1 = 0.0, W2 = 0.0;
    float c0 = 0.f;
#ifndef SGPU_WZ_GBUF
#define SGPU_WZ_GBUF 1          // 0: the record stored with per-rank predicates (RankStore::store; A/B)
#endif
    const int route = bad ? 2 : wz_prepare<NP, G, RSL, SGPU_WZ_GBUF != 0>(v, g, kept, kmin, p.nframes, rs, W1, W2, c0);
    if (g == 0) {
        p.wz_mom[loc] = W1;
        p.wz_mom[p.wz_cnt + loc] = W2;
        p.wz_mom[2 * p.wz_cnt + loc] = (double)c0;
        int4 m;
        m.x = route ? -1 : kept;
        m.y = rs.hi0;
        m.z = rs.mid0;
        m.w = rs.mid1;
        reinterpret_cast<int4 *>(p.wz_meta)[loc] = m;
    }
}

template <int NP, int W, int U16 = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_wz_rounds(KParams p) {
    using RS = RankStore<NP, 1>;
    const long long loc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int rl = 0, rh = 0;
    if (loc < p.wz_cnt) {
        const long long pix = p.wz_pix0 + loc;
        const int4 m = reinterpret_cast<const int4 *>(p.wz_meta)[loc];
        int route = 2;
        PixOut o;
        if (m.x > 0) {
            RS rs;
            rs.base = p.wz_ranks;
            rs.stride = p.wz_cnt;
            rs.p = loc;
            rs.kept = m.x;
            rs.hi0 = m.y;
            rs.mid0 = m.z;
            rs.mid1 = m.w;
            constexpr int G = NP / 64;         // the prep kernel's lanes per pixel (E = 64)
            const int N = p.nframes;
            const int el = (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
            route = wz_finish<U16>(rs, m.x, p.wz_mom[loc], p.wz_mom[p.wz_cnt + loc],
                                   (float)p.wz_mom[2 * p.wz_cnt + loc], G * el, p.sig0, p.sig1, o);
        }
        if (route == 1) {
            const int slot = wave_append(p.fb2_count, true);
            p.fb2_list[slot] = (int)pix;
        } else if (route == 2) {
            const int slot = wave_append(p.fb_count, true);
            p.fb_list[slot] = (int)pix;
        } else {
            double res = o.res;
            if (is_weighted(p)) res = weighted_mean<U16>(p, pix, (int)(pix % p.W), o.pmin, o.pmax, o.nkept);
            if constexpr (U16) write_result16(p, pix, res, o.rl, o.rh);
            else write_result(p, pix, res, o.rl, o.rh);
            rl = o.rl;
            rh = o.rh;
        }
    }
    add_counts(p, rl, rh);
}

// Round-wise rounds (SGPU_WZ_RW=100): one launch per rejection round.  The
// pixels of a wave take 1-6 rounds of 1-16 clamp iterations each; run as one
// loop nest, a wave pays the sum over rounds of its slowest pixel, with the
// finished pixels' lanes idle.  Here launch `pass` runs one round for every
// pixel still going (pass 0: all of the chunk) and appends the pixels that
// need another round to wz_list_out (one atomic per wave), their state to
// wz_state; the last pass (`last`) runs every remaining round.  A model of the
// bench data's round / iteration counts gives 0.65 active lanes per trip
// against 0.44 for the nest.
// (wave_append: stack_sorted_impl.h)

template <int NP, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_stack_wz_round(KParams p, int pass, int last) {
    using RS = RankStore<NP, 1>;
    constexpr int G = NP / 64;                 // the prep kernel's lanes per pixel (E = 64)
    const long long n = pass == 0 ? p.wz_cnt : (long long)p.wz_lcount[0];
    const long long stride = (long long)gridDim.x * blockDim.x;
    int rl = 0, rh = 0;
    // tiles of the launch: the loop trip count is wave-uniform (wave_append)
    for (long long t0 = (long long)blockIdx.x * blockDim.x; t0 < n; t0 += stride) {
        const long long i = t0 + threadIdx.x;
        const bool live = i < n;
        bool again = false;
        long long loc = 0;
        if (live) {
            loc = pass == 0 ? i : (long long)p.wz_list_in[i];
            const long long pix = p.wz_pix0 + loc;
            const int4 m = reinterpret_cast<const int4 *>(p.wz_meta)[loc];
            int route = 2;
            PixOut o;
            WzConst k;
            WzState st;
            if (m.x > 0) {
                RS rs;
                rs.base = p.wz_ranks;
                rs.stride = p.wz_cnt;
                rs.p = loc;
                rs.kept = m.x;
                rs.hi0 = m.y;
                rs.mid0 = m.z;
                rs.mid1 = m.w;
                const int N = p.nframes;
                const int el = (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
                const float c0 = (float)p.wz_mom[2 * p.wz_cnt + loc];
                if (pass == 0) {
                    route = wz_start(rs, m.x, p.wz_mom[loc], p.wz_mom[p.wz_cnt + loc], c0, G * el, p.sig0, p.sig1,
                                     k, st, o);
                } else {
                    float ymax, vmin;
                    route = wz_consts(rs, m.x, c0, G * el, p.sig0, p.sig1, k, ymax, vmin);
                    st = reinterpret_cast<const WzState *>(p.wz_state)[loc];
                    o.fallback = 0;
                }
                if (route == 3) {
                    route = 0;                 // kept == 1: o is the result
                } else if (route == 0) {
                    bool more = true;
                    do route = wz_round(rs, k, st, more);   // one call site: one inlined copy
                    while (last && more && !route);
                    if (!route && more) {
                        again = true;
                        reinterpret_cast<WzState *>(p.wz_state)[loc] = st;
                    } else if (!route) {
                        route = wz_final(rs, k, st, o);
                    }
                }
            }
            if (!again) {
                if (route == 1) {
                    const int slot = wave_append(p.fb2_count, true);
                    p.fb2_list[slot] = (int)pix;
                } else if (route == 2) {
                    const int slot = wave_append(p.fb_count, true);
                    p.fb_list[slot] = (int)pix;
                } else {
                    double res = o.res;
                    if (is_weighted(p)) res = weighted_mean(p, pix, (int)(pix % p.W), o.pmin, o.pmax, o.nkept);
                    write_result(p, pix, res, o.rl, o.rh);
                    rl += o.rl;
                    rh += o.rh;
                }
            }
        }
        const int slot = wave_append(p.wz_lcount + 1, again);
        if (again) p.wz_list_out[slot] = (int)loc;
    }
    add_counts(p, rl, rh);
}

// Rounds kernel with the rank records staged in LDS (default at N <= 128,
// SGPU_WZ_RW=64): one wave per block copies its 64 pixels' R rank slots
// (slot-major rows of the workspace: every copy instruction reads 256
// contiguous bytes) into LDS, so the dependent rank reads of the rounds
// (medians, tail walks, clip walks) are LDS round trips instead of L2 / HBM
// misses -- half of the global-read kernel's wave-cycles waited on them
// (profiles/r05q_pmc_rounds.json).  At R = 40 slots (KT = 16, KM = 8) a wave
// takes 10 KB: 16 waves per CU, the register-bound occupancy too.  (At the
// round-3 R = 64 the LDS held 10 waves per CU and the staging lost.)
template <int NP, int U16 = 0>
__global__ __launch_bounds__(64) void k_stack_wz_rounds_lds(KParams p) {
    using RS = RankStore<NP, 1>;
    __shared__ float s_rank[RS::R * 64];
    const int lane = (int)threadIdx.x;
    const long long loc = (long long)blockIdx.x * 64 + lane;
    const bool live = loc < p.wz_cnt;
    int4 m = make_int4(0, 0, 0, 0);
    if (live) m = reinterpret_cast<const int4 *>(p.wz_meta)[loc];
    {
        float t[RS::R];
#if defined(__HIP_DEVICE_COMPILE__)
        // one descriptor over the record (R * cnt * 4 bytes < 2^31: the
        // launcher's NP * ch * 4 <= 2^32 bound) and a 32-bit byte offset per
        // lane: slot j's uniform part goes to soffset (no 64-bit multiply per
        // slot); lanes past the chunk read zeros, discarded below
        const uint32_t S4 = (uint32_t)p.wz_cnt * 4u;
        const auto rr = __builtin_amdgcn_make_buffer_rsrc(p.wz_ranks, (short)0, (int)((uint32_t)RS::R * S4), 0x00020000);
        const int vo = live ? (int)((uint32_t)loc * 4u) : (int)((uint32_t)RS::R * S4);
#pragma unroll
        for (int j = 0; j < RS::R; j++)
            t[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, vo, (int)((uint32_t)j * S4), 0));
#else
#pragma unroll
        for (int j = 0; j < RS::R; j++) t[j] = live ? p.wz_ranks[(long long)j * p.wz_cnt + loc] : 0.f;
#endif
#pragma unroll
        for (int j = 0; j < RS::R; j++) s_rank[j * 64 + lane] = t[j];
    }
    __syncthreads();
    int rl = 0, rh = 0;
    if (live) {
        const long long pix = p.wz_pix0 + loc;
        int route = 2;
        PixOut o;
        if (m.x > 0) {
            RS rs;
            rs.base = s_rank;
            rs.stride = 64;
            rs.p = lane;
            rs.kept = m.x;
            rs.hi0 = m.y;
            rs.mid0 = m.z;
            rs.mid1 = m.w;
            constexpr int G = NP / 64;
            const int N = p.nframes;
            const int el = (((N + G - 1) / G) + SGPU_STOP_GRAN - 1) & ~(SGPU_STOP_GRAN - 1);
            route = wz_finish<U16>(rs, m.x, p.wz_mom[loc], p.wz_mom[p.wz_cnt + loc],
                                   (float)p.wz_mom[2 * p.wz_cnt + loc], G * el, p.sig0, p.sig1, o);
        }
        if (route == 1) {
            const int slot = wave_append(p.fb2_count, true);
            p.fb2_list[slot] = (int)pix;
        } else if (route == 2) {
            const int slot = wave_append(p.fb_count, true);
            p.fb_list[slot] = (int)pix;
        } else {
            double res = o.res;
            if (is_weighted(p)) res = weighted_mean<U16>(p, pix, (int)(pix % p.W), o.pmin, o.pmax, o.nkept);
            if constexpr (U16) write_result16(p, pix, res, o.rl, o.rh);
            else write_result(p, pix, res, o.rl, o.rh);
            rl = o.rl;
            rh = o.rh;
        }
    }
    add_counts(p, rl, rh);
}

}  // namespace sgpu
