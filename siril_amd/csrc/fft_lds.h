// fft_lds.h -- mixed-radix complex FFT of one row held in LDS (Stockham
// autosort, natural order in and out), for the DFT registration
// (registration/shift_methods.c:60-321) and the Richardson-Lucy FFT path.
//
// Sign convention of FFTW: forward X[k] = sum x[n] exp(-2 pi i k n / N),
// backward = +i, unnormalised.  Radices 10, 8, 5, 4, 3, 2 have dedicated
// butterflies; any other prime factor uses a generic R-point DFT through the
// twiddle table.  Twiddles come from a table w[k] = exp(-2 pi i k / N)
// computed on the host in double precision.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgpu {
namespace fft {

constexpr int kMaxFactors = 24;
constexpr int kMaxLen = 8192;       // 2 x N x 8 bytes of LDS (128 KiB at N = 8192)
#ifndef SGPU_FFT_THREADS
#define SGPU_FFT_THREADS 512
#endif
constexpr int kThreads = SGPU_FFT_THREADS;
#ifndef SGPU_FFT_TW_POW
#define SGPU_FFT_TW_POW 1
#endif

// compiled CFA pattern (get_compiled_pattern, algos/demosaicing.c:327-358):
// dim 2 (Bayer) or 6 (X-Trans), 0 = no CFA; values 0 R, 1 G, 2 B
struct Cfa {
    int dim;
    unsigned char c[36];
};

struct Plan {
    int n;                          // transform length
    int nf;                         // number of passes
    int radix[kMaxFactors];         // radices, in pass order
    const float2 *tw;               // w[k] = exp(-2 pi i k / n), k < n (device)
};

// radices 2, 3, 4, 5, 8, 10 only: the transform runs in place in one LDS buffer
// (run<S> below); a generic prime radix needs the second (scratch) buffer
inline __host__ __device__ bool plan_inplace(const Plan &pl) {
    for (int p = 0; p < pl.nf; p++)
        if (pl.radix[p] != 2 && pl.radix[p] != 3 && pl.radix[p] != 4 && pl.radix[p] != 5 && pl.radix[p] != 8 &&
            !(pl.radix[p] == 10 && pl.n / 10 <= kThreads))   // radix 10 in place: one butterfly per thread
            return false;
    return true;
}
// Kernels built with R10 = false (the RL FFTs: run<S, false>) have no
// radix-10 butterfly; their dispatch keeps the exact round-5 form (a device
// trap or an explicit radix-8 case there cost the RL column / row kernels
// 2-4 VGPRs and a wave per SIMD: config 5 62.5 -> 68.4 ms), so the contract
// is enforced where their plans are made: a plan holding a 10 must not reach
// them (rl_fft.hip make_plan refuses one).
inline __host__ __device__ bool plan_has_radix10(const Plan &pl) {
    for (int p = 0; p < pl.nf; p++)
        if (pl.radix[p] == 10) return true;
    return false;
}
// dynamic LDS of a kernel running one transform of the plan
inline size_t plan_lds_bytes(const Plan &pl) { return (plan_inplace(pl) ? 1 : 2) * (size_t)pl.n * 8; }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// z * (s*i), s = -1 forward, +1 backward
template <int S> __device__ __forceinline__ float2 rot(float2 z) { return make_float2(-S * z.y, S * z.x); }
template <int S> __device__ __forceinline__ float2 tw_get(const float2 *tw, int k) {
    const float2 w = tw[k];
    return S < 0 ? w : make_float2(w.x, -w.y);
}

template <int S> __device__ __forceinline__ void bfly2(float2 *v) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}
template <int S> __device__ __forceinline__ void bfly4(float2 *v) {
    const float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const float2 t2 = cadd(v[1], v[3]), t3 = rot<S>(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
}
template <int S> __device__ __forceinline__ void bfly8(float2 *v) {
    float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    bfly4<S>(e);
    bfly4<S>(o);
    const float r = 0.70710678118654752440f;
    const float2 w1 = make_float2(r, S * r), w3 = make_float2(-r, S * r);
    o[1] = cmul(o[1], w1);
    o[2] = rot<S>(o[2]);
    o[3] = cmul(o[3], w3);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = cadd(e[k], o[k]);
        v[k + 4] = csub(e[k], o[k]);
    }
}
template <int S> __device__ __forceinline__ void bfly3(float2 *v) {
    const float s3 = 0.86602540378443864676f;
    const float2 b = cadd(v[1], v[2]), d = csub(v[1], v[2]);
    const float2 a0 = v[0];
    v[0] = cadd(a0, b);
    const float2 t = csub(a0, cscale(b, 0.5f));
    const float2 u = rot<S>(cscale(d, s3));
    v[1] = cadd(t, u);
    v[2] = csub(t, u);
}
template <int S> __device__ __forceinline__ void bfly5(float2 *v) {
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const float2 a0 = v[0];
    const float2 b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]);
    const float2 d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
    v[0] = cadd(a0, cadd(b1, b2));
    const float2 t1 = cadd(a0, cadd(cscale(b1, c1), cscale(b2, c2)));
    const float2 t2 = cadd(a0, cadd(cscale(b1, c2), cscale(b2, c1)));
    const float2 u1 = rot<S>(cadd(cscale(d1, s1), cscale(d2, s2)));
    const float2 u2 = rot<S>(csub(cscale(d1, s2), cscale(d2, s1)));
    v[1] = cadd(t1, u1);
    v[4] = csub(t1, u1);
    v[2] = cadd(t2, u2);
    v[3] = csub(t2, u2);
}

// 10 = 2 x 5 (Cooley-Tukey): the DFT5s of the even and odd inputs, the odd
// one turned by w10^k, then the radix-2 step.  One pass instead of a 5 and
// half a 2 / 4 / 8: a 4000-point row runs 8, 10, 10, 5 (4 passes, 5
// butterfly rounds of 512 threads) instead of 8, 5, 5, 5, 4 (5 passes, 9)
template <int S> __device__ __forceinline__ void bfly10(float2 *v) {
    float2 e[5] = {v[0], v[2], v[4], v[6], v[8]}, o[5] = {v[1], v[3], v[5], v[7], v[9]};
    bfly5<S>(e);
    bfly5<S>(o);
    const float c1 = 0.80901699437494742410f, s1 = 0.58778525229247312917f;   // cos / sin 36 deg
    const float c2 = 0.30901699437494742410f, s2 = 0.95105651629515357212f;   // cos / sin 72 deg
    o[1] = cmul(o[1], make_float2(c1, S * s1));
    o[2] = cmul(o[2], make_float2(c2, S * s2));
    o[3] = cmul(o[3], make_float2(-c2, S * s2));
    o[4] = cmul(o[4], make_float2(-c1, S * s1));
#pragma unroll
    for (int k = 0; k < 5; k++) {
        v[k] = cadd(e[k], o[k]);
        v[k + 5] = csub(e[k], o[k]);
    }
}

// One Stockham pass of radix R over the LDS row `in` -> `out` (n points,
// Ns = product of the radices already applied).
template <int S, int R>
__device__ __forceinline__ void pass_fixed(const float2 *in, float2 *out, int n, int Ns, const float2 *tw) {
    const int nb = n / R;
    const int tstep = n / (Ns * R);             // twiddle index step
    for (int t = threadIdx.x; t < nb; t += blockDim.x) {
        const int j = t % Ns;
        float2 v[R];
#pragma unroll
        for (int q = 0; q < R; q++) v[q] = in[t + q * nb];
        if (Ns > 1) {
#if SGPU_FFT_TW_POW
            // one table read per butterfly, the other twiddles as its powers
            const float2 w1 = tw_get<S>(tw, j * tstep);
            float2 wq = w1;
#pragma unroll
            for (int q = 1; q < R; q++) {
                v[q] = cmul(v[q], wq);
                if (q + 1 < R) wq = cmul(wq, w1);
            }
#else
#pragma unroll
            for (int q = 1; q < R; q++) v[q] = cmul(v[q], tw_get<S>(tw, j * q * tstep));   // < n
#endif
        }
        if (R == 2) bfly2<S>(v);
        else if (R == 3) bfly3<S>(v);
        else if (R == 4) bfly4<S>(v);
        else if (R == 5) bfly5<S>(v);
        else if (R == 8) bfly8<S>(v);
        else if (R == 10) bfly10<S>(v);
        const int base = (t / Ns) * Ns * R + j;
#pragma unroll
        for (int q = 0; q < R; q++) out[base + q * Ns] = v[q];
    }
}

// generic radix (any other prime factor, through the twiddle table); each
// output re-reads its R inputs (rare radices: no register array)
template <int S>
__device__ __forceinline__ void pass_generic(const float2 *in, float2 *out, int n, int Ns, int R,
                                             const float2 *tw) {
    const int nb = n / R;
    const int tstep = n / (Ns * R);
    const int rstep = n / R;                    // w_R^1 = w_n^(n/R)
    for (int t = threadIdx.x; t < nb; t += blockDim.x) {
        const int j = t % Ns;
        const int base = (t / Ns) * Ns * R + j;
        for (int k = 0; k < R; k++) {
            float2 acc = in[t];
            for (int q = 1; q < R; q++) {
                float2 x = in[t + q * nb];
                if (Ns > 1) x = cmul(x, tw_get<S>(tw, j * q * tstep));
                acc = cadd(acc, cmul(x, tw_get<S>(tw, ((k * q) % R) * rstep)));
            }
            out[base + k * Ns] = acc;
        }
    }
}

// One Stockham pass in place: every thread first loads the inputs of all its
// butterflies into registers (at most MAXB per thread at the maximum length),
// the block synchronises, then writes the outputs over the same buffer.  Half
// the LDS of the ping-pong form, so 2-3x the blocks per CU on the long rows
// (the row kernels are LDS-latency bound).  Same arithmetic in the same
// order as pass_fixed: bit-identical results.  Needs blockDim.x == kThreads.
template <int S, int R>
__device__ __forceinline__ void pass_inplace(float2 *a, int n, int Ns, const float2 *tw) {
    // radix 10 runs in place only with at most one butterfly per thread
    // (plan_inplace): its 10 inputs then cost the registers of the radix-5
    // pass's 4 x 5, not twice that, and the row kernels keep their occupancy
    constexpr int MAXB = R == 10 ? 1 : (kMaxLen / R + kThreads - 1) / kThreads;
    const int nb = n / R;
    const int tstep = n / (Ns * R);
    float2 v[MAXB][R];
#pragma unroll
    for (int k = 0; k < MAXB; k++) {
        const int t = threadIdx.x + k * kThreads;
        if (t < nb) {
#pragma unroll
            for (int q = 0; q < R; q++) v[k][q] = a[t + q * nb];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MAXB; k++) {
        const int t = threadIdx.x + k * kThreads;
        if (t < nb) {
            const int j = t % Ns;
            if (Ns > 1) {
#if SGPU_FFT_TW_POW
                const float2 w1 = tw_get<S>(tw, j * tstep);
                float2 wq = w1;
#pragma unroll
                for (int q = 1; q < R; q++) {
                    v[k][q] = cmul(v[k][q], wq);
                    if (q + 1 < R) wq = cmul(wq, w1);
                }
#else
#pragma unroll
                for (int q = 1; q < R; q++) v[k][q] = cmul(v[k][q], tw_get<S>(tw, j * q * tstep));
#endif
            }
            if (R == 2) bfly2<S>(v[k]);
            else if (R == 3) bfly3<S>(v[k]);
            else if (R == 4) bfly4<S>(v[k]);
            else if (R == 5) bfly5<S>(v[k]);
            else if (R == 8) bfly8<S>(v[k]);
            else if (R == 10) bfly10<S>(v[k]);
            const int base = (t / Ns) * Ns * R + j;
#pragma unroll
            for (int q = 0; q < R; q++) a[base + q * Ns] = v[k][q];
        }
    }
    __syncthreads();
}

// Transform the row in LDS buffer a (scratch b); returns the buffer holding
// the result.  All threads of the block must call it.  R10: the kernel's plans
// may hold radix-10 passes (the DFT's); without it the radix-10 butterfly is
// not compiled in (its registers would lower the occupancy of every pass of
// the RL kernels, whose plans have no 10s: rl_fft.hip make_plan)
template <int S, bool R10 = false>
__device__ float2 *transform(float2 *a, float2 *b, const Plan &pl) {
    int Ns = 1;
    for (int p = 0; p < pl.nf; p++) {
        const int R = pl.radix[p];
        switch (R) {
            case 2: pass_fixed<S, 2>(a, b, pl.n, Ns, pl.tw); break;
            case 3: pass_fixed<S, 3>(a, b, pl.n, Ns, pl.tw); break;
            case 4: pass_fixed<S, 4>(a, b, pl.n, Ns, pl.tw); break;
            case 5: pass_fixed<S, 5>(a, b, pl.n, Ns, pl.tw); break;
            case 8: pass_fixed<S, 8>(a, b, pl.n, Ns, pl.tw); break;
            default:
                if constexpr (R10) {
                    if (R == 10) {
                        pass_fixed<S, 10>(a, b, pl.n, Ns, pl.tw);
                        break;
                    }
                }
                pass_generic<S>(a, b, pl.n, Ns, R, pl.tw);
                break;
        }
        __syncthreads();
        float2 *t = a;
        a = b;
        b = t;
        Ns *= R;
    }
    return a;
}

// The transform of a kernel's row: in place in `a` when the plan has only
// fixed radices (b may then be null), else ping-pong through b.  Returns the
// buffer holding the result.
template <int S, bool R10 = false>
__device__ float2 *run(float2 *a, float2 *b, const Plan &pl) {
    if (!plan_inplace(pl)) return transform<S, R10>(a, b, pl);
    int Ns = 1;
    for (int p = 0; p < pl.nf; p++) {
        switch (pl.radix[p]) {
            case 2: pass_inplace<S, 2>(a, pl.n, Ns, pl.tw); break;
            case 3: pass_inplace<S, 3>(a, pl.n, Ns, pl.tw); break;
            case 4: pass_inplace<S, 4>(a, pl.n, Ns, pl.tw); break;
            case 5: pass_inplace<S, 5>(a, pl.n, Ns, pl.tw); break;
            case 10:
                if constexpr (R10) {
                    pass_inplace<S, 10>(a, pl.n, Ns, pl.tw);
                    break;
                }
                [[fallthrough]];   // R10 = false: never reached -- see plan_has_radix10
            default: pass_inplace<S, 8>(a, pl.n, Ns, pl.tw); break;
        }
        Ns *= pl.radix[p];
    }
    return a;
}

}  // namespace fft
}  // namespace sgpu
