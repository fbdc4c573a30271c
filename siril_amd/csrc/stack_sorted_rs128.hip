// stack_sorted_rs128.hip -- real-slot variants for N <= 128 (see
// stack_sorted_inst.h rs_kernel): the moment path's prep kernel (E = 64
// slots per lane, bounds 36..60 in steps of 4) and the float SIGMA,
// PERCENTILE and median kernels
// (E = 128, bounds 72..120 in steps of 8) whose sort networks leave out every comparator on a slot that
// only padding can occupy (oem_sort's RS).  Measured (profiles/r04q_ab_real_slots.txt):
// config 2 14.59 -> 13.69 ms, sigma400 43.56 -> 41.68 ms.
#include "stack_sorted_inst.h"
#include "stack_sorted_gw.h"

namespace sgpu {
namespace {
template <int NP, int G, int W, int RS>
KernelFn prep_rs(int xf, int rs) {
    if constexpr (RS >= NP / G) {
        return nullptr;
    } else {
        if (rs == RS) return xf ? &k_stack_wz_prep<NP, G, 1, W, RS> : &k_stack_wz_prep<NP, G, 0, W, RS>;
        return prep_rs<NP, G, W, RS + 4>(xf, rs);
    }
}
template <int NP, int RT, int G, int W, int RS>
KernelFn straight_rs(int xf, int rs) {
    constexpr int E = NP / G;
    if constexpr (RS >= E) {
        return nullptr;
    } else {
        if (rs == RS)
            return xf ? &k_stack_sorted<NP, G, RT, 1, W, 0, 0, RS> : &k_stack_sorted<NP, G, RT, 0, W, 0, 0, RS>;
        return straight_rs<NP, RT, G, W, RS + (E == 64 ? 4 : 8)>(xf, rs);
    }
}
}  // namespace

KernelFn rs_kernel_128(int kind, int xf, int rs) {
    switch (kind) {
        case 0: return prep_rs<128, 2, SGPU_WZ_PREP_W128, 36>(xf, rs);
        case SIGMA: return straight_rs<128, SIGMA, SGPU_GW128, 72>(xf, rs);
        case PERCENTILE: return straight_rs<128, PERCENTILE, SGPU_GW128, 72>(xf, rs);
        case KMEDIAN: return straight_rs<128, KMEDIAN, SGPU_GW128, 72>(xf, rs);
        default: return nullptr;
    }
}
}  // namespace sgpu
