// scripts/wzstat/wzstat.cpp -- host statistics of the WINSORIZED moment path
// (stack_wz.h) on a frame-major stack: per pixel the number of rejection
// rounds, clamp iterations and rank fetches, and per wave of 64 consecutive
// pixels (the rounds kernel's lanes) the maximum of each, which is what the
// wave pays.  Tooling only (not a test, not product code).
//
//   hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -fPIC -shared
//         -ffp-contract=off -I siril_amd/csrc scripts/wzstat/wzstat.cpp -o /tmp/libwzstat.so
#include <cstring>
static thread_local int g_ev[2];
#define SGPU_WZ_TRACE(ev) (g_ev[(ev)]++)
#include "stack_wz.h"

using namespace sgpu;

template <int NP>
struct CountRS : RankStore<NP, 1> {
    mutable int nf = 0;
    // deepest rank visited from each end and farthest from the middle (the
    // record sizes KT / KM that would have held every read of the pixel)
    mutable int lo_depth = -1, hi_depth = -1, mid_dev = -1;
    SG_HD bool fetch(int r, float &x) const {
        nf++;
        const int k = this->kept;
        const int dl = r, dh = k - 1 - r, dm = r - k / 2 >= 0 ? r - k / 2 : k / 2 - r;
        if (dl <= dh && dl < dm) lo_depth = dl > lo_depth ? dl : lo_depth;
        else if (dh < dl && dh < dm) hi_depth = dh > hi_depth ? dh : hi_depth;
        else mid_dev = dm > mid_dev ? dm : mid_dev;
        return RankStore<NP, 1>::fetch(r, x);
    }
};

// out[j*8 + 0..7] = route, rounds, clamp iterations, fetches, kept, deepest
// low rank, deepest high rank (from the top), farthest rank from the middle
extern "C" void wz_stats(const float *frames, int n, long long ncol, float sig0, float sig1, int *out) {
    constexpr int NP = 128;
    static float ranks[RankStore<NP, 1>::R * RankStore<NP, 1>::PW];
    for (long long j = 0; j < ncol; j++) {
        float v[NP];
        int kept = 0;
        for (int e = 0; e < NP; e++) {
            float val = f_inf();
            if (e < n) {
                val = frames[(long long)e * ncol + j];
                if (val == 0.f) val = f_inf();
                else kept++;
            }
            v[e] = val;
        }
        CountRS<NP> rs;
        rs.base = ranks;
        rs.stride = RankStore<NP, 1>::PW;
        rs.p = 0;
        g_ev[0] = g_ev[1] = 0;
        double W1, W2;
        float c0;
        int route = wz_prepare<NP, 1>(v, 0, kept, kept, n, rs, W1, W2, c0) ? 2 : 0;
        rs.nf = 0;
        rs.lo_depth = rs.hi_depth = rs.mid_dev = -1;
        PixOut o;
        if (!route) route = wz_finish(rs, kept, W1, W2, c0, (n + 3) & ~3, sig0, sig1, o);
        int *q = out + j * 8;
        q[0] = route;
        q[1] = g_ev[0];
        q[2] = g_ev[1];
        q[3] = rs.nf;
        q[4] = kept;
        q[5] = rs.lo_depth;
        q[6] = rs.hi_depth;
        q[7] = rs.mid_dev;
    }
}
