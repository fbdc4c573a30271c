// sorted-path kernels for N <= 256 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW256
#define SGPU_GW256 2, 2
#endif
#ifndef SGPU_GW256_LOOP
#define SGPU_GW256_LOOP 4, 3
#endif
SGPU_DEFINE_SORTED_LAUNCHER(256,
    SGPU_CASEX(256, PERCENTILE, SGPU_GW256)
    SGPU_CASEX(256, SIGMA, SGPU_GW256)
    SGPU_CASEX(256, SIGMEDIAN, SGPU_GW256_LOOP)
    SGPU_CASEX(256, WINSORIZED, SGPU_GW256_LOOP)
    SGPU_CASEX(256, MAD, SGPU_GW256_LOOP)
    SGPU_CASEX(256, KMEDIAN, SGPU_GW256))
SGPU_DEFINE_SORTED16_LAUNCHER(256)
