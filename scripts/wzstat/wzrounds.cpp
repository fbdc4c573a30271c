// scripts/wzstat/wzrounds.cpp -- host statistics of the WINSORIZED moment
// path (stack_wz.h) per pixel: route, rounds, clamp iterations in total and
// per round (up to 16).  Tooling only; used by regroup_model.py.
//   hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -fPIC -shared
//         -ffp-contract=off -I siril_amd/csrc scripts/wzstat/wzrounds.cpp -o /tmp/wz/libwz2.so
#include <cstring>
static thread_local int g_ev[2];
static thread_local int g_it[16];
#define SGPU_WZ_TRACE(ev) do { if ((ev) == 0) g_ev[0]++; else { g_ev[1]++; if (g_ev[0] <= 16) g_it[g_ev[0]-1]++; } } while (0)
#include "stack_wz.h"
using namespace sgpu;
extern "C" void wz_stats2(const float *frames, int n, long long ncol, float sig0, float sig1, int *out) {
    constexpr int NP = 128;
    static float ranks[RankStore<NP, 1>::R * RankStore<NP, 1>::PW];
    for (long long j = 0; j < ncol; j++) {
        float v[NP];
        int kept = 0;
        for (int e = 0; e < NP; e++) {
            float val = f_inf();
            if (e < n) { val = frames[(long long)e * ncol + j]; if (val == 0.f) val = f_inf(); else kept++; }
            v[e] = val;
        }
        RankStore<NP, 1> rs; rs.base = ranks; rs.stride = RankStore<NP, 1>::PW; rs.p = 0;
        g_ev[0] = g_ev[1] = 0; for (int i = 0; i < 16; i++) g_it[i] = 0;
        double W1, W2; float c0;
        int route = wz_prepare<NP, 1>(v, 0, kept, kept, n, rs, W1, W2, c0) ? 2 : 0;
        PixOut o;
        if (!route) route = wz_finish(rs, kept, W1, W2, c0, (n + 3) & ~3, sig0, sig1, o);
        int *q = out + j * 20;
        q[0] = route; q[1] = g_ev[0]; q[2] = g_ev[1]; q[3] = kept;
        for (int i = 0; i < 16; i++) q[4 + i] = g_it[i];
    }
}
