// stack_sorted_inst.h -- one translation unit per column capacity NP
// instantiates the sorted-path kernels for every rejection type it supports;
// sgpu_capi.cpp picks the smallest NP >= N.  Each (NP, rejection) pair has
// its own lane-group width G (E = NP/G samples per lane) and occupancy
// target W (waves per SIMD the register allocator must allow): loop-heavy
// types with data-dependent trip counts (WINSORIZED) want more pixels per
// wave to be cheap (small E) but fewer of them diverging (G > 1); straight
// rejection types want G = 1 (no cross-lane reductions at all).
#pragma once
#include "stack_sorted_impl.h"

namespace sgpu {

template <int NP, int G, int RT, int W, int U16 = 0>
static int launch_one(const KParams &p, hipStream_t s) {
    const long long threads = p.npix * (long long)G;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    // 32-bit buffer offsets of the gather (gather_column)
    const unsigned long long es = U16 ? 2ull : 4ull;
    if ((unsigned long long)(G - 1) * (unsigned long long)p.frame_stride * es +
            (unsigned long long)p.npix * es >= 0xffffffffull)
        return 1;
    if (p.shiftx)   // host sets shiftx only when shifts / normalization are needed
        hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 1, W, U16>), grid, 256, 0, s, p);
    else
        hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 0, W, U16>), grid, 256, 0, s, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sgpu

#define SGPU_CASE(NP, RT, G, W) \
    case RT: return launch_one<NP, G, RT, W>(p, s);
// GW: a macro expanding to "G, W" (tuning knobs, see the np*.hip files)
#define SGPU_CASE_I(...) SGPU_CASE(__VA_ARGS__)
#define SGPU_CASEX(NP, RT, GW) SGPU_CASE_I(NP, RT, GW)

// 16-bit (DATA_USHORT) sorted path: every rejection type and the median stack
// (LINEARFIT / GESDT single-lane, N <= 128)
#define SGPU_CASE16(NP, RT, G, W) \
    case RT: return launch_one<NP, G, RT, W, 1>(p, s);
#define SGPU_CASE16_I(...) SGPU_CASE16(__VA_ARGS__)
#define SGPU_CASE16X(NP, RT, GW) SGPU_CASE16_I(NP, RT, GW)

// returns 0 launched, 1 not on the sorted path (exact kernel), -1 launch error
#define SGPU_DEFINE_SORTED_LAUNCHER(NP, CASES)                                 \
    namespace sgpu {                                                           \
    int launch_sorted_##NP(const KParams &p, hipStream_t s) {                  \
        switch (p.rtype) {                                                     \
            CASES                                                              \
            default:                                                           \
                return 1;                                                      \
        }                                                                      \
    }                                                                          \
    }

#define SGPU_DEFINE_SORTED16_LAUNCHER(NP, CASES)                              \
    namespace sgpu {                                                           \
    int launch_sorted16_##NP(const KParams &p, hipStream_t s) {                \
        switch (p.rtype) {                                                     \
            CASES                                                              \
            default:                                                           \
                return 1;                                                      \
        }                                                                      \
    }                                                                          \
    }
