// sorted-path kernels for N <= 512 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW512
#define SGPU_GW512 4, 3
#endif
#ifndef SGPU_GW512_LOOP
#define SGPU_GW512_LOOP 8, 3
#endif
SGPU_DEFINE_SORTED_LAUNCHER(512,
    SGPU_CASEX(512, PERCENTILE, SGPU_GW512)
    SGPU_CASEX(512, SIGMA, SGPU_GW512)
    SGPU_CASEX(512, SIGMEDIAN, SGPU_GW512_LOOP)
    SGPU_CASEX(512, WINSORIZED, SGPU_GW512_LOOP)
    SGPU_CASEX(512, MAD, SGPU_GW512_LOOP)
    SGPU_CASEX(512, KMEDIAN, SGPU_GW512))
SGPU_DEFINE_SORTED16_LAUNCHER(512)
