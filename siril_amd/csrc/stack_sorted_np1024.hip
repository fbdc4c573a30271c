// sorted-path kernels for N <= 1024 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW1024
#define SGPU_GW1024 8, 2
#endif
#ifndef SGPU_GW1024_LOOP
#define SGPU_GW1024_LOOP 16, 3
#endif
SGPU_DEFINE_SORTED_LAUNCHER(1024,
    SGPU_CASEX(1024, PERCENTILE, SGPU_GW1024)
    SGPU_CASEX(1024, SIGMA, SGPU_GW1024)
    SGPU_CASEX(1024, SIGMEDIAN, SGPU_GW1024_LOOP)
    SGPU_CASEX(1024, WINSORIZED, SGPU_GW1024_LOOP)
    SGPU_CASEX(1024, MAD, SGPU_GW1024_LOOP)
    SGPU_CASEX(1024, KMEDIAN, SGPU_GW1024))
SGPU_DEFINE_SORTED16_LAUNCHER(1024)
