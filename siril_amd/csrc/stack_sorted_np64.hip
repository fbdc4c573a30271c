// sorted-path kernels for N <= 64 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW64
#define SGPU_GW64 1, 3
#endif
#ifndef SGPU_GW64_LOOP
#define SGPU_GW64_LOOP 1, 3
#endif
SGPU_DEFINE_SORTED_LAUNCHER(64,
    SGPU_CASEX(64, PERCENTILE, SGPU_GW64)
    SGPU_CASEX(64, SIGMA, SGPU_GW64)
    SGPU_CASEX(64, SIGMEDIAN, SGPU_GW64_LOOP)
    SGPU_CASEX(64, WINSORIZED, SGPU_GW64_LOOP)
    SGPU_CASEX(64, MAD, SGPU_GW64_LOOP)
    SGPU_CASEX(64, KMEDIAN, SGPU_GW64))
SGPU_DEFINE_SORTED16_LAUNCHER(64)
