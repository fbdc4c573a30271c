// tests/hostsim/sim.hip -- TEST BUILD: runs the sorted-path per-pixel logic
// of siril_amd/csrc/stack_sorted_impl.h and the WINSORIZED moment path of
// stack_wz.h on the HOST (one lane per pixel, G == 1) so their algorithms can
// be checked against the oracle without a GPU.  The GPU kernels themselves
// are checked by the -m gpu tests.
#include <algorithm>
#include <cstring>
#include "stack_wz.h"

using namespace sgpu;

// WINSORIZED moment-path routes: [0] answered, [1] sorted path, [2] exact kernel
static long long sim_wz_route[3];
// 1: run the moment path the way the round-wise launches do (state saved and
// the constants rebuilt between rounds)
static int sim_roundwise = 0;
extern "C" void sim_set_roundwise(int on) { sim_roundwise = on; }
extern "C" void sim_wz_stats(long long *out) {
    for (int i = 0; i < 3; i++) out[i] = sim_wz_route[i];
}
extern "C" void sim_wz_stats_reset() {
    for (int i = 0; i < 3; i++) sim_wz_route[i] = 0;
}

template <int NP, int RT, int U16 = 0>
static int run(const float *col, int n, const PixCfg &c, double *res, int *rl, int *rh) {
    float v[NP];
    int kept = 0, bad = 0;
    for (int e = 0; e < NP; e++) {
        float val = f_inf();
        if (e < n) {
            val = col[e];
            if (!(val - val == 0.f)) bad = 1;
            if (RT != KMEDIAN) {
                if (val == 0.f) val = f_inf();
                else kept++;
            }
        }
        v[e] = val;
    }
    if (bad) return 1;
    if constexpr (RT == WINSORIZED && NP >= 128) {
        // the moment path, with the register-resident path as its fallback
        static float ranks[RankStore<NP, 1>::R * RankStore<NP, 1>::PW];
        RankStore<NP, 1> rs;
        rs.base = ranks;
        rs.stride = RankStore<NP, 1>::PW;
        rs.p = 0;
        float w[NP];
        for (int e = 0; e < NP; e++) w[e] = v[e];
        PixOut o;
        int route = 1;
        if (!sim_roundwise || U16) {
            route = wz_pixel<NP, 1, U16>(w, 0, kept, kept, c.nframes, c.sig0, c.sig1, rs, o);
        } else if constexpr (!U16) {
            // k_stack_wz_round's decomposition: pass 0 starts the pixel, every
            // later pass rebuilds the constants and resumes from the saved state
            double W1, W2;
            float c0;
            route = wz_prepare<NP, 1>(w, 0, kept, kept, c.nframes, rs, W1, W2, c0) ? 2 : 0;
            const int m = NP * 1;   // G * E of the hostsim's one-lane layout
            WzConst k;
            WzState st, saved;
            if (!route) {
                route = wz_start(rs, kept, W1, W2, c0, m, c.sig0, c.sig1, k, st, o);
                if (route == 3) {
                    route = 0;
                } else if (!route) {
                    bool more = true;
                    for (int pass = 0; !route && more; pass++) {
                        if (pass > 0) {
                            float ymax, vmin;
                            std::memcpy(&st, &saved, sizeof st);
                            WzConst k2;
                            route = wz_consts(rs, kept, c0, m, c.sig0, c.sig1, k2, ymax, vmin);
                            k = k2;
                            if (route) break;
                        }
                        route = wz_round(rs, k, st, more);
                        std::memcpy(&saved, &st, sizeof st);
                    }
                    if (!route) route = wz_final(rs, k, st, o);
                }
            }
        }
        sim_wz_route[route]++;
        if (route == 2) return 1;
        if (route == 0) {
            *res = o.res;
            *rl = o.rl;
            *rh = o.rh;
            return 0;
        }
    }
    sort_col<NP, 1>(v, 0);
    PixOut o = pixel_sorted<NP, 1, RT, U16>(v, 0, kept, c);
    *res = o.res;
    *rl = o.rl;
    *rh = o.rh;
    return o.fallback;
}

template <int NP, int U16 = 0>
static int run_np(int rt, const float *col, int n, const PixCfg &c, double *res, int *rl, int *rh) {
    switch (rt) {
        case PERCENTILE: return run<NP, PERCENTILE, U16>(col, n, c, res, rl, rh);
        case SIGMA: return run<NP, SIGMA, U16>(col, n, c, res, rl, rh);
        case MAD: return run<NP, MAD, U16>(col, n, c, res, rl, rh);
        case SIGMEDIAN: return run<NP, SIGMEDIAN, U16>(col, n, c, res, rl, rh);
        case WINSORIZED: return run<NP, WINSORIZED, U16>(col, n, c, res, rl, rh);
        case LINEARFIT: return run<NP, LINEARFIT, U16>(col, n, c, res, rl, rh);
        case GESDT: return run<NP, GESDT, U16>(col, n, c, res, rl, rh);
        case KMEDIAN: return run<NP, KMEDIAN, U16>(col, n, c, res, rl, rh);
        default: return -1;
    }
}

// returns: 0 = sorted / moment path result, 1 = deferred to the exact kernel, -1 = unsupported
extern "C" int sim_pixel(int rt, const float *col, int n, float sig0, float sig1,
                         const float *crit, float m_x, float m_dx2, double *res, int *rl, int *rh) {
    const int np = n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128;
    const int el = (n + 3) & ~3;   // G == 1: interleaved passes stop at ceil(n/4)*4
    PixCfg c{n, sig0, sig1, crit, m_x, m_dx2, el < np ? el : np};
    if (n <= 16) return run_np<16>(rt, col, n, c, res, rl, rh);
    if (n <= 32) return run_np<32>(rt, col, n, c, res, rl, rh);
    if (n <= 64) return run_np<64>(rt, col, n, c, res, rl, rh);
    if (n <= 128) return run_np<128>(rt, col, n, c, res, rl, rh);
    return -1;
}

// 16-bit columns (apply_rejection_ushort): samples are whole numbers held as
// floats; same return codes as sim_pixel
extern "C" int sim_pixel_u16(int rt, const float *col, int n, float sig0, float sig1,
                             const float *crit, float m_x, float m_dx2, double *res, int *rl, int *rh) {
    const int np = n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128;
    const int el = (n + 3) & ~3;
    PixCfg c{n, sig0, sig1, crit, m_x, m_dx2, el < np ? el : np};
    if (n <= 16) return run_np<16, 1>(rt, col, n, c, res, rl, rh);
    if (n <= 32) return run_np<32, 1>(rt, col, n, c, res, rl, rh);
    if (n <= 64) return run_np<64, 1>(rt, col, n, c, res, rl, rh);
    if (n <= 128) return run_np<128, 1>(rt, col, n, c, res, rl, rh);
    return -1;
}

// batch form: column j of frames [n][ncol] (frame-major, as the stack
// buffers); st[j] = sim_pixel's return code.  OpenMP-free: callers shard.
extern "C" void sim_pixels(int rt, const float *frames, int n, long long ncol, float sig0, float sig1,
                           const float *crit, float m_x, float m_dx2, double *res, int *rl, int *rh,
                           int *st) {
    float col[1024];
    for (long long j = 0; j < ncol; j++) {
        for (int f = 0; f < n; f++) col[f] = frames[(long long)f * ncol + j];
        st[j] = sim_pixel(rt, col, n, sig0, sig1, crit, m_x, m_dx2, res + j, rl + j, rh + j);
    }
}

// the one-lane-per-pixel fused form (k_stack_wz1, SGPU_WZ=6): the whole
// sorted column in a row (missing samples +Inf), wz1_pixel; st[j] = route
// (0 answered, 1 sorted kernel, 2 exact kernel)
extern "C" void sim_wz1_pixels(const float *frames, int n, long long ncol, float sig0, float sig1, double *res,
                               int *rl, int *rh, int *st) {
    float row[1025];
    for (long long j = 0; j < ncol; j++) {
        int kept = 0, bad = 0;
        for (int f = 0; f < n; f++) {
            float v = frames[(long long)f * ncol + j];
            if (!(v - v == 0.f)) bad = 1;
            if (v == 0.f) v = f_inf();
            else kept++;
            row[f] = v;
        }
        std::sort(row, row + n);
        PixOut o;
        const int route = (!bad && kept > 0) ? wz1_pixel(row, kept, n, sig0, sig1, o) : 2;
        st[j] = route;
        if (route == 0) {
            res[j] = o.res;
            rl[j] = o.rl;
            rh[j] = o.rh;
        }
    }
}

// real-slot sort networks (stack_sorted_impl.h oem_sort<E, RS>, rs_pick): the
// pruned network of bound rs on v (slots >= rs +Inf), into out
template <int E, int RS, int STEP>
static int sort_rs(float *v, int rs) {
    if constexpr (RS > E) {
        return -1;
    } else {
        if (rs != RS) return sort_rs<E, RS + STEP, STEP>(v, rs);
        float w[E];
        for (int e = 0; e < E; e++) w[e] = v[e];
        oem_sort<E, RS>(w);
        for (int e = 0; e < E; e++) v[e] = w[e];
        return 0;
    }
}
extern "C" int sim_sort_rs(float *v, int E, int rs) {
    if (E == 64) return sort_rs<64, 36, 4>(v, rs);
    if (E == 128) return sort_rs<128, 72, 8>(v, rs);
    return -1;
}
extern "C" int sim_rs_pick(int E, int G, int N) { return rs_pick(E, G, N); }
