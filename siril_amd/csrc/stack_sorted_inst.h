// stack_sorted_inst.h -- one translation unit per column capacity NP
// instantiates the sorted-path kernels for every rejection type it supports;
// sgpu_capi.cpp picks the smallest NP >= N.  Each (NP, rejection) pair has
// its own lane-group width G (E = NP/G samples per lane) and occupancy
// target W (waves per SIMD the register allocator must allow): loop-heavy
// types with data-dependent trip counts (WINSORIZED) want more pixels per
// wave to be cheap (small E) but fewer of them diverging (G > 1); straight
// rejection types want G = 1 (no cross-lane reductions at all).
#pragma once
#include "stack_sorted_impl.h"
#include "stack_wz.h"
#ifndef SGPU_WZ_RRW
#define SGPU_WZ_RRW 4      // occupancy of the round-wise rounds kernel
#endif

#include <algorithm>
#include <cstdlib>

#ifndef SGPU_WZ_MOMENTS
#define SGPU_WZ_MOMENTS 1        // 0: no moment-path kernels (WINSORIZED on the register-resident path only)
#endif
#ifndef SGPU_WZ_W128
#define SGPU_WZ_W128 4           // moment-path occupancy target (waves / SIMD), N <= 128
#endif
#ifndef SGPU_WZ_W
#define SGPU_WZ_W 3              // moment-path occupancy target, N > 128
#endif
#ifndef SGPU_WZ1_W
#define SGPU_WZ1_W 2             // one-lane-per-pixel single kernel (SGPU_WZ=5): waves / SIMD
#endif


namespace sgpu {

__global__ void k_stack_exact_lds(KParams p, int all_pixels);
__global__ void k_stack_exact_wave(KParams p, int all_pixels);

// total of the chunks' exact-kernel pixels (sgpu_last_exact_pixels)
template <int D>
__global__ void k_add_count(const int *src, int *dst) {
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(dst, *src * D);
}

// second stream and events of the overlapped moment path (SGPU_WZ=3), and
// the third stream of the per-chunk tails, per host thread and device
// (contexts on different threads never share them)
struct WzAux {
    hipStream_t s2 = nullptr, s3 = nullptr;
    hipEvent_t start, prep[2], rounds[2], tails;
};
inline int wz_aux(WzAux *&a) {
    thread_local WzAux tab[16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    a = &tab[dev & 15];
    if (!a->s2) {
        if (hipStreamCreateWithFlags(&a->s2, hipStreamNonBlocking) != hipSuccess) return -1;
        if (hipStreamCreateWithFlags(&a->s3, hipStreamNonBlocking) != hipSuccess) return -1;
        hipEvent_t *ev[6] = {&a->start, &a->prep[0], &a->prep[1], &a->rounds[0], &a->rounds[1], &a->tails};
        for (hipEvent_t *e : ev)
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return -1;
    }
    return 0;
}

// Real-slot variants (stack_sorted_rs*.hip): the moment path's prep kernel
// (kind 0) and the float SIGMA / PERCENTILE / median kernels (kind = the
// rejection type) with their sort networks
// pruned to the first rs slots of every lane (rs_pick), or null when this
// NP has none (the full network runs)
using KernelFn = void (*)(KParams);
KernelFn rs_kernel_128(int kind, int xf, int rs);
KernelFn rs_kernel_256(int kind, int xf, int rs);
KernelFn rs_kernel_512(int kind, int xf, int rs);
template <int NP> inline KernelFn rs_kernel(int kind, int xf, int rs) {
    if constexpr (NP == 128) return rs_kernel_128(kind, xf, rs);
    else if constexpr (NP == 256) return rs_kernel_256(kind, xf, rs);
    else if constexpr (NP == 512) return rs_kernel_512(kind, xf, rs);
    else return nullptr;
}
inline bool launch_fn(KernelFn f, unsigned grid, unsigned block, hipStream_t s, const KParams &p) {
    KParams k = p;
    void *args[] = {&k};
    return hipLaunchKernel((const void *)f, dim3(grid), dim3(block), args, 0, s) == hipSuccess;
}

// LDS scratch threads per block of the exact kernel (sgpu_capi.cpp exact_lds_block)
inline int wz_exact_block(int N) {
    const long long per = 24ll * N;
    int t = 64;
    while (t > 4 && (long long)t * per > 65536) t >>= 1;
    return (long long)t * per <= 65536 ? t : 0;
}

// overlapped moment path: the least number of chunks per launch, and the
// smallest chunk that rule may produce (SGPU_WZ_MINCH overrides the count).
// Off (1) by default: one 8-GPU rank's band of config 2 (500 rows, 3 M
// pixels) measured 1.94 ms as one chunk and 2.14 ms split in four
// (profiles/r05d_band*_winsorized100.json) -- the split's extra launches and
// tails cost more than the prep / rounds overlap it buys
constexpr int kWzMinChunks = 1;
constexpr long long kWzMinChunkPix = 1LL << 19;

template <int NP, int G, int RT, int W, int U16 = 0>
static int launch_one(const KParams &p, hipStream_t s) {
    const long long threads = p.npix * (long long)G;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    // sort network pruned to the slots that can hold samples (rs_pick)
    constexpr int E = NP / G;
    const int rs = rs_pick(E, G, p.nframes);
    // 32-bit buffer offsets of the gather (gather_column)
    const unsigned long long es = U16 ? 2ull : 4ull;
    if ((unsigned long long)(G - 1) * (unsigned long long)p.frame_stride * es +
            (unsigned long long)p.npix * es >= 0xffffffffull)
        return 1;
    // WINSORIZED columns of 65..1024 samples (float and, round 5, DATA_USHORT):
    // the moment path (stack_wz.h), then the register-resident kernel over
    // its fallbacks
    constexpr bool WZM = SGPU_WZ_MOMENTS && RT == WINSORIZED && NP >= 128;
    // (16-bit columns: the two-kernel form only; the single-kernel A/B forms
    // are float kernels)
    if constexpr (WZM) if (!U16 || (p.wz_mode >= 2 && p.wz_mode <= 4 && p.wz_ws)) {
        if (p.fb2_list && p.wz_mode >= 2 && p.wz_mode <= 4 && p.wz_ws) {
            // two-kernel form: chunks of pixels whose records fit the workspace.
            // Overlapped: the workspace is split in two and the prep of chunk
            // k + 1 runs on a second stream while the rounds of chunk k run on
            // this one (prep is latency / memory bound, the rounds VALU bound).
            // SGPU_WZ=2 (default): overlapped at NP <= 128 (config 2: 16.13 ->
            // 15.81 ms), one stream above (NP = 512: 52.4 vs 53.2 ms, twice
            // the chunks of 0.9 M pixels); 3: always overlapped; 4: never.
            const bool ovl = p.wz_mode == 3 || (p.wz_mode == 2 && NP <= 128);
            const int nbuf = ovl ? 2 : 1;
            constexpr int R = RankStore<NP, G>::R;
            // per pixel: ranks, moments, meta, round-wise state and two lists
            const long long per = (long long)R * 4 + 3 * 8 + 16 + (long long)sizeof(WzState) + 8;
            const long long wsb = (p.wz_ws_bytes / nbuf) & ~4095LL;
            static_assert(G == NP / 64 || NP < 128, "rounds kernels rebuild the prep kernel's G as NP / 64");
            long long ch = std::min<long long>(p.npix, ((wsb - 4096) / per) & ~255LL);
            // RankStore::fetch: umul24(slot, stride) -- stride < 2^24 and the
            // 32-bit product slot * stride < R * ch < 2^32
            ch = std::min<long long>(ch, (1LL << 23) - 256);
            ch = std::min<long long>(ch, (0xffffffffLL / R) & ~255LL);
            // RankStore::store_buf: NP * ch * 4 <= 2^32 (32-bit byte offsets
            // of the record's regions, negative slots down to -NP)
            ch = std::min<long long>(ch, ((1LL << 32) / (4LL * NP) - 256) & ~255LL);
            // overlapped form: at least kWzMinChunks chunks, so that a small
            // launch (one rank's row band at 8 GPUs: 3 M pixels of config 2,
            // one workspace-sized chunk) still hides the preps under the rounds
            static const int minch = std::getenv("SGPU_WZ_MINCH") ? std::atoi(std::getenv("SGPU_WZ_MINCH")) : kWzMinChunks;
            if (ovl && minch > 1 && p.npix > (long long)minch * kWzMinChunkPix)
                ch = std::min<long long>(ch, ((p.npix + minch - 1) / minch + 255) & ~255LL);
            if (p.wz_chunk > 0) ch = std::min<long long>(ch, (p.wz_chunk + 255) & ~255LL);
            if (ch <= 0) return 1;
            WzAux *aux = nullptr;
            hipStream_t sp = s;                      // the prep kernels' stream
            if (ovl) {
                if (wz_aux(aux)) return -1;
                sp = aux->s2;
                if (hipEventRecord(aux->start, s) != hipSuccess || hipStreamWaitEvent(sp, aux->start, 0) != hipSuccess)
                    return -1;
            }
            KParams q = p;
            int *lists[2], *cnts = nullptr;
            // per-chunk tails (KParams::wz_tcnt): each chunk's fallbacks (the
            // register-resident sorted kernel) and deferred pixels (the exact
            // kernel) run on a third stream right after the chunk's rounds,
            // under the next chunks' prep and rounds, from chunk-local lists
            const long long nch = (p.npix + ch - 1) / ch;
            const int et = wz_exact_block(p.nframes);
            // (16-bit: the tails run after the last chunk -- the LDS exact
            // kernel of the per-chunk form is the float one)
            const bool tails = !U16 && ovl && p.wz_tcnt && nch <= kWzMaxChunks && et > 0 && p.wz_rw != 100;
            auto place = [&](int b) {
                char *base = (char *)p.wz_ws + (long long)b * wsb;
                q.wz_ranks = (float *)base;
                q.wz_mom = (double *)(base + (((long long)R * 4 * ch + 255) & ~255LL));
                q.wz_meta = (int *)((char *)q.wz_mom + 3 * 8 * ch);
                q.wz_state = (void *)((char *)q.wz_meta + 16 * ch);
                lists[0] = (int *)((char *)q.wz_state + (long long)sizeof(WzState) * ch);
                lists[1] = lists[0] + ch;
                cnts = lists[1] + ch;                // 8 counters: pass k reads cnts[k], appends cnts[k + 1]
            };
            const KernelFn prep_rs = (!U16 && rs < E) ? rs_kernel<NP>(0, p.shiftx ? 1 : 0, rs) : nullptr;
            int k = 0;
            for (long long p0 = 0; p0 < p.npix; p0 += ch, k++) {
                const int b = k % nbuf;
                place(b);
                q.wz_pix0 = p0;
                q.wz_cnt = std::min(ch, p.npix - p0);
                if (tails) {
                    q.fb2_list = p.fb2_list + p0;
                    q.fb2_count = p.wz_tcnt + 2 * k;
                    q.fb_list = p.fb_list + p0;
                    q.fb_count = p.wz_tcnt + 2 * k + 1;
                }
                const unsigned g1 = (unsigned)((q.wz_cnt * G + 255) / 256), g2 = (unsigned)((q.wz_cnt + 255) / 256);
                // the buffer's previous chunk must be through its rounds
                if (ovl && k >= nbuf && hipStreamWaitEvent(sp, aux->rounds[b], 0) != hipSuccess) return -1;
                if (prep_rs) {
                    if (!launch_fn(prep_rs, g1, 256, sp, q)) return -1;
                } else if (p.shiftx) hipLaunchKernelGGL((k_stack_wz_prep<NP, G, 1, W, E, U16>), g1, 256, 0, sp, q);
                else hipLaunchKernelGGL((k_stack_wz_prep<NP, G, 0, W, E, U16>), g1, 256, 0, sp, q);
                if (ovl && (hipEventRecord(aux->prep[b], sp) != hipSuccess ||
                            hipStreamWaitEvent(s, aux->prep[b], 0) != hipSuccess))
                    return -1;
                if constexpr (U16 && NP <= 128) {
                    if (p.wz_rw == 64)
                        hipLaunchKernelGGL((k_stack_wz_rounds_lds<NP, 1>), dim3((unsigned)((q.wz_cnt + 63) / 64)), 64, 0,
                                           s, q);
                    else
                        hipLaunchKernelGGL((k_stack_wz_rounds<NP, 5, 1>), g2, 256, 0, s, q);
                } else if constexpr (U16) {
                    hipLaunchKernelGGL((k_stack_wz_rounds<NP, 5, 1>), g2, 256, 0, s, q);
                } else if (p.wz_rw == 100) {
                    // round-wise: rounds 1..kPasses-1 one launch each, then the rest
                    constexpr int kPasses = 3;
                    if (hipMemsetAsync(cnts, 0, 8 * sizeof(int), s) != hipSuccess) return -1;
                    for (int pass = 0; pass < kPasses; pass++) {
                        q.wz_list_in = lists[pass & 1];
                        q.wz_list_out = lists[(pass + 1) & 1];
                        q.wz_lcount = cnts + pass;
                        const unsigned gr = pass == 0 ? g2 : std::min<unsigned>(g2, 2048u);
                        hipLaunchKernelGGL((k_stack_wz_round<NP, SGPU_WZ_RRW>), gr, 256, 0, s, q, pass,
                                           pass == kPasses - 1 ? 1 : 0);
                    }
                } else {
                    switch (p.wz_rw) {
                        case 4: hipLaunchKernelGGL((k_stack_wz_rounds<NP, 4>), g2, 256, 0, s, q); break;
                        case 6: hipLaunchKernelGGL((k_stack_wz_rounds<NP, 6>), g2, 256, 0, s, q); break;
                        case 64:   // LDS-staged ranks (default; R = 40 slots at NP <= 128: 10 KB per wave)
                            if constexpr (NP <= 128)
                                hipLaunchKernelGGL((k_stack_wz_rounds_lds<NP>), dim3((unsigned)((q.wz_cnt + 63) / 64)),
                                                   64, 0, s, q);
                            else
                                hipLaunchKernelGGL((k_stack_wz_rounds<NP, 5>), g2, 256, 0, s, q);
                            break;
                        default: hipLaunchKernelGGL((k_stack_wz_rounds<NP, 5>), g2, 256, 0, s, q); break;
                    }
                }
                if (hipGetLastError() != hipSuccess) return -1;
                if (ovl && hipEventRecord(aux->rounds[b], s) != hipSuccess) return -1;
                if (tails) {
                    if (hipStreamWaitEvent(aux->s3, aux->rounds[b], 0) != hipSuccess) return -1;
                    const unsigned lg = (unsigned)std::min<long long>((q.wz_cnt * G + 255) / 256, 512);
                    if (p.shiftx) hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 1, W, U16, 1>), lg, 256, 0, aux->s3, q);
                    else hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 0, W, U16, 1>), lg, 256, 0, aux->s3, q);
                    // the chunk's deferred pixels: one wave each (stack_exact_wave.hip;
                    // SGPU_EXACT_WAVE=0: the one-thread LDS kernel)
                    static const bool wave = !std::getenv("SGPU_EXACT_WAVE") || std::atoi(std::getenv("SGPU_EXACT_WAVE")) != 0;
                    if (wave) {
                        const size_t lds = (size_t)5 * ((p.nframes + 1) & ~1) * sizeof(float);
                        const unsigned wb = (unsigned)std::max<long long>(1, std::min<long long>(q.wz_cnt, 1024));
                        hipLaunchKernelGGL(k_stack_exact_wave, dim3(wb), dim3(64), lds, aux->s3, q, 0);
                    } else {
                        const size_t lds = (size_t)et * 24ull * p.nframes;
                        const long long per_cu = std::max<long long>(1, (long long)((160ull << 10) / lds));
                        const long long eb = std::max<long long>(1, std::min<long long>((q.wz_cnt + et - 1) / et,
                                                                                        256 * per_cu));
                        hipLaunchKernelGGL(k_stack_exact_lds, dim3((unsigned)eb), dim3(et), lds, aux->s3, q, 0);
                    }
                    hipLaunchKernelGGL(k_add_count<1>, dim3(1), dim3(1), 0, aux->s3, (const int *)q.fb_count,
                                       p.wz_tcnt + 2 * kWzMaxChunks);
                    if (hipGetLastError() != hipSuccess) return -1;
                }
            }
            if (tails) {   // the launch ends when every chunk's tails have
                if (hipEventRecord(aux->tails, aux->s3) != hipSuccess ||
                    hipStreamWaitEvent(s, aux->tails, 0) != hipSuccess)
                    return -1;
                return 0;
            }
            // every prep was joined into s by its rounds; the list-mode kernel
            // below runs on s after all of them
        } else if (p.fb2_list && p.wz_mode == 1) {
            constexpr int WW = NP <= 128 ? SGPU_WZ_W128 : SGPU_WZ_W;
            if (p.shiftx) hipLaunchKernelGGL((k_stack_wz<NP, G, 1, WW>), grid, 256, 0, s, p);
            else hipLaunchKernelGGL((k_stack_wz<NP, G, 0, WW>), grid, 256, 0, s, p);
            if (hipGetLastError() != hipSuccess) return -1;
        } else if (p.fb2_list && p.wz_mode == 6) {
            // one kernel, one lane per pixel, the whole sorted column in LDS
            if constexpr (NP <= 128) {
                const int LS = (p.nframes + 1) | 1;          // odd row stride > N (spare word at N)
                const size_t lds = (size_t)64 * LS * sizeof(float);
                const unsigned g1 = (unsigned)((p.npix + 63) / 64);
                if (p.shiftx) hipLaunchKernelGGL((k_stack_wz1<NP, 1, SGPU_WZ1_W>), g1, 64, lds, s, p, LS);
                else hipLaunchKernelGGL((k_stack_wz1<NP, 0, SGPU_WZ1_W>), g1, 64, lds, s, p, LS);
                if (hipGetLastError() != hipSuccess) return -1;
            } else {
                return 1;
            }
        } else if (p.fb2_list && p.wz_mode == 5) {
            // one kernel, one lane per pixel (E = 128 samples in VGPRs): gather,
            // sort, rank store in LDS (64 KB per block) and the rounds from LDS
            // with every lane busy -- no rank records in HBM
            if constexpr (NP <= 128) {
                const unsigned g1 = (unsigned)((p.npix + 255) / 256);
                if (p.shiftx) hipLaunchKernelGGL((k_stack_wz<NP, 1, 1, SGPU_WZ1_W>), g1, 256, 0, s, p);
                else hipLaunchKernelGGL((k_stack_wz<NP, 1, 0, SGPU_WZ1_W>), g1, 256, 0, s, p);
                if (hipGetLastError() != hipSuccess) return -1;
            } else {
                if (p.shiftx) hipLaunchKernelGGL((k_stack_wz<NP, G, 1, SGPU_WZ_W>), grid, 256, 0, s, p);
                else hipLaunchKernelGGL((k_stack_wz<NP, G, 0, SGPU_WZ_W>), grid, 256, 0, s, p);
                if (hipGetLastError() != hipSuccess) return -1;
            }
        }
        if (p.fb2_list && (p.wz_mode == 1 || p.wz_mode == 5 || p.wz_mode == 6 ||
                           (p.wz_mode >= 2 && p.wz_mode <= 4 && p.wz_ws))) {
            // the register-resident kernel over the moment path's fallbacks:
            // enough groups to fill the chip, grid-stride over the list
            const unsigned lgrid = (unsigned)std::min<long long>(grid, 2048);
            if (p.shiftx) hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 1, W, U16, 1>), lgrid, 256, 0, s, p);
            else hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 0, W, U16, 1>), lgrid, 256, 0, s, p);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
    }
    if constexpr ((RT == SIGMA || RT == PERCENTILE || RT == KMEDIAN) && !U16) {
        if (rs < E) {
            if (const KernelFn f = rs_kernel<NP>(RT, p.shiftx ? 1 : 0, rs)) return launch_fn(f, grid, 256, s, p) ? 0 : -1;
        }
    }
    if (p.shiftx)   // host sets shiftx only when shifts / normalization are needed
        hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 1, W, U16>), grid, 256, 0, s, p);
    else
        hipLaunchKernelGGL((k_stack_sorted<NP, G, RT, 0, W, U16>), grid, 256, 0, s, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sgpu

#define SGPU_CASE(NP, RT, G, W) \
    case RT: return launch_one<NP, G, RT, W>(p, s);
// GW: a macro expanding to "G, W" (tuning knobs, see the np*.hip files)
#define SGPU_CASE_I(...) SGPU_CASE(__VA_ARGS__)
#define SGPU_CASEX(NP, RT, GW) SGPU_CASE_I(NP, RT, GW)

// 16-bit (DATA_USHORT) sorted path: every rejection type and the median stack
// (LINEARFIT / GESDT single-lane, N <= 128)
#define SGPU_CASE16(NP, RT, G, W) \
    case RT: return launch_one<NP, G, RT, W, 1>(p, s);
#define SGPU_CASE16_I(...) SGPU_CASE16(__VA_ARGS__)
#define SGPU_CASE16X(NP, RT, GW) SGPU_CASE16_I(NP, RT, GW)

// returns 0 launched, 1 not on the sorted path (exact kernel), -1 launch error
#define SGPU_DEFINE_SORTED_LAUNCHER(NP, CASES)                                 \
    namespace sgpu {                                                           \
    int launch_sorted_##NP(const KParams &p, hipStream_t s) {                  \
        switch (p.rtype) {                                                     \
            CASES                                                              \
            default:                                                           \
                return 1;                                                      \
        }                                                                      \
    }                                                                          \
    }

#define SGPU_DEFINE_SORTED16_LAUNCHER(NP, CASES)                              \
    namespace sgpu {                                                           \
    int launch_sorted16_##NP(const KParams &p, hipStream_t s) {                \
        switch (p.rtype) {                                                     \
            CASES                                                              \
            default:                                                           \
                return 1;                                                      \
        }                                                                      \
    }                                                                          \
    }
