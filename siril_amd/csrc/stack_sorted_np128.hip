// sorted-path kernels for N <= 128 (see stack_sorted_inst.h).  Tuning knobs
// "G, W" per rejection family, overridable with -D for variant sweeps.
#include "stack_sorted_inst.h"
#ifndef SGPU_GW128
#define SGPU_GW128 1, 2
#endif
#ifndef SGPU_GW128_LOOP
#define SGPU_GW128_LOOP 2, 4
#endif
SGPU_DEFINE_SORTED_LAUNCHER(128,
    SGPU_CASEX(128, PERCENTILE, SGPU_GW128)
    SGPU_CASEX(128, SIGMA, SGPU_GW128)
    SGPU_CASEX(128, SIGMEDIAN, SGPU_GW128_LOOP)
    SGPU_CASEX(128, WINSORIZED, SGPU_GW128_LOOP)
    SGPU_CASEX(128, MAD, SGPU_GW128_LOOP)
    SGPU_CASEX(128, KMEDIAN, SGPU_GW128))
SGPU_DEFINE_SORTED16_LAUNCHER(128)
