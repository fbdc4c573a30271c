// stack_sorted_inst.h -- one translation unit per column capacity NP
// instantiates the sorted-path kernels (G lanes per pixel, E = NP/G samples
// per lane) for every rejection type it supports; sgpu_capi.cpp picks the
// smallest NP >= N.
#pragma once
#include "stack_sorted_impl.h"

#define SGPU_LAUNCH_CASE(NP, G, RT)                                                   \
    case RT:                                                                          \
        if (xf) hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 1>), grid, 256, 0, s, p); \
        else hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 0>), grid, 256, 0, s, p);    \
        break;

#define SGPU_DEFINE_SORTED_LAUNCHER(NP, G, EXTRA)                                     \
    namespace sgpu {                                                                  \
    int launch_sorted_##NP(const KParams &p, hipStream_t s) {                        \
        const long long threads = p.npix * (long long)(G);                           \
        const unsigned grid = (unsigned)((threads + 255) / 256);                     \
        const bool xf = (p.shiftx != nullptr);  /* host sets shiftx when XF needed */ \
        /* 32-bit buffer offsets of the gather (gather_column) */                    \
        if ((unsigned long long)((G) - 1) * (unsigned long long)p.frame_stride * 4ull +  \
                (unsigned long long)p.npix * 4ull >= 0xffffffffull)                   \
            return 1;                                                                 \
        switch (p.rtype) {                                                            \
            SGPU_LAUNCH_CASE(NP, G, PERCENTILE)                                       \
            SGPU_LAUNCH_CASE(NP, G, SIGMA)                                            \
            SGPU_LAUNCH_CASE(NP, G, SIGMEDIAN)                                        \
            SGPU_LAUNCH_CASE(NP, G, WINSORIZED)                                       \
            SGPU_LAUNCH_CASE(NP, G, KMEDIAN)                                          \
            EXTRA                                                                     \
            default:                                                                  \
                return 1; /* not on the sorted path: exact kernel for every pixel */ \
        }                                                                             \
        return hipGetLastError() == hipSuccess ? 0 : -1;                             \
    }                                                                                 \
    }
