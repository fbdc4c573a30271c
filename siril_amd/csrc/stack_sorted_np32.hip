// sorted-path kernels for N <= 32 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW32
#define SGPU_GW32 1, 4
#endif
#ifndef SGPU_GW32_LOOP
#define SGPU_GW32_LOOP 1, 4
#endif
SGPU_DEFINE_SORTED_LAUNCHER(32,
    SGPU_CASEX(32, PERCENTILE, SGPU_GW32)
    SGPU_CASEX(32, SIGMA, SGPU_GW32)
    SGPU_CASEX(32, SIGMEDIAN, SGPU_GW32_LOOP)
    SGPU_CASEX(32, WINSORIZED, SGPU_GW32_LOOP)
    SGPU_CASEX(32, MAD, SGPU_GW32_LOOP)
    SGPU_CASEX(32, KMEDIAN, SGPU_GW32)
    SGPU_CASE(32, LINEARFIT, 1, 4)
    SGPU_CASE(32, GESDT, 1, 4))
SGPU_DEFINE_SORTED16_LAUNCHER(32)
