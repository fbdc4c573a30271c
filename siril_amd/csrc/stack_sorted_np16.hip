// sorted-path kernels for N <= 16 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW16
#define SGPU_GW16 1, 4
#endif
#ifndef SGPU_GW16_LOOP
#define SGPU_GW16_LOOP 1, 4
#endif
SGPU_DEFINE_SORTED_LAUNCHER(16,
    SGPU_CASEX(16, PERCENTILE, SGPU_GW16)
    SGPU_CASEX(16, SIGMA, SGPU_GW16)
    SGPU_CASEX(16, SIGMEDIAN, SGPU_GW16_LOOP)
    SGPU_CASEX(16, WINSORIZED, SGPU_GW16_LOOP)
    SGPU_CASEX(16, MAD, SGPU_GW16_LOOP)
    SGPU_CASEX(16, KMEDIAN, SGPU_GW16)
    SGPU_CASE(16, LINEARFIT, 1, 4)
    SGPU_CASE(16, GESDT, 1, 4))
SGPU_DEFINE_SORTED16_LAUNCHER(16)
