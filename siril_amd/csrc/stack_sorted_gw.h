// stack_sorted_gw.h -- per column capacity NP, the lane-group width G and
// occupancy target W of the sorted-path kernels ("G, W"): straight rejection
// types (SGPU_GW<NP>) and loop types with data-dependent trip counts
// (SGPU_GW<NP>_LOOP; also the moment path's prep kernel).  Chosen by
// measurement (scripts/exp_variants.sh); -D overrides for variant sweeps.
#pragma once
#ifndef SGPU_GW16
#define SGPU_GW16 1, 4
#endif
#ifndef SGPU_GW16_LOOP
#define SGPU_GW16_LOOP 1, 4
#endif
#ifndef SGPU_GW32
#define SGPU_GW32 1, 4
#endif
#ifndef SGPU_GW32_LOOP
#define SGPU_GW32_LOOP 1, 4
#endif
#ifndef SGPU_GW64
#define SGPU_GW64 1, 3
#endif
#ifndef SGPU_GW64_LOOP
#define SGPU_GW64_LOOP 1, 3
#endif
#ifndef SGPU_GW128
#define SGPU_GW128 1, 2
#endif
#ifndef SGPU_GW128_LOOP
#define SGPU_GW128_LOOP 2, 4
#endif
#ifndef SGPU_GW256
#define SGPU_GW256 2, 2
#endif
#ifndef SGPU_GW256_LOOP
#define SGPU_GW256_LOOP 4, 3
#endif
#ifndef SGPU_GW512
#define SGPU_GW512 4, 3
#endif
#ifndef SGPU_GW512_LOOP
#define SGPU_GW512_LOOP 8, 3
#endif
#ifndef SGPU_GW1024
#define SGPU_GW1024 8, 2
#endif
#ifndef SGPU_GW1024_LOOP
#define SGPU_GW1024_LOOP 16, 3
#endif
// occupancy target of the moment path's prep kernel at NP = 128 (G = 2):
// waves per SIMD the register allocation must allow
#ifndef SGPU_WZ_PREP_W128
#define SGPU_WZ_PREP_W128 4
#endif
