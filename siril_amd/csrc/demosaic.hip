// demosaic.hip -- CFA demosaic on the GPU for debayer_buffer_new_float
// (algos/demosaicing_rtp.cpp:228-390) and the super-pixel debayer
// (algos/demosaicing_siril.c:128-176).
//
// RCD (the default interpolation, librtprocess rcd_demosaic -- not vendored
// in the reference; restated in oracle/demosaic_ref.py from the published
// RCD 2.3 algorithm, parity with librtprocess unpinned).  One kernel per
// algorithm step over the whole image (every step is a small stencil, the
// pipeline is HBM-bound); the arithmetic follows the oracle operation for
// operation in f32 without contraction, so GPU == oracle bitwise.
// Siril's wrapper maps the CFA data to [0, 65535] with its min / max first
// and maps the result back with `v * invfactor + min`.
//
// The 16-bit wrapper debayer_buffer_new_ushort (demosaicing_rtp.cpp:74-224)
// hands RCD the raw WORD values converted to float, with no normalisation,
// and rounds the result with roundf_to_WORD (roundf_to_BYTE for 8-bit
// data, core/proto.h:256-261,341-346).  The same kernels run it with T =
// uint16_t input, O = uint16_t output and min / max pinned to 0 / 65535:
// (x - 0) * 1 and v * 1 + 0 are exact, so the arithmetic in between is
// exactly the unnormalised one.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

namespace sgpu {
namespace dm {

constexpr float EPS = 1e-5f;
constexpr float EPSSQ = 1e-10f;
constexpr float SCALE = 65536.f;
constexpr int BORDER = 6;           // border_interpolate margin (see oracle/demosaic_ref.py)

struct Img {
    int W, H;
    unsigned char cf[4];            // cfarray[row & 1][col & 1]: 0 R, 1 G, 2 B
    const unsigned *mm;             // ordered-uint min / max of the input
    int remap;                      // 1: XCD-contiguous tile order (DM_XY)
};

__device__ __forceinline__ unsigned f2ord(float v) {
    const unsigned b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// colour of (r, c): the 2x2 pattern packed in one 32-bit word (a dynamic
// index into the by-value kernel argument compiled to byte loads from the
// kernarg segment at every call)
__device__ __forceinline__ int fc(const Img &g, int r, int c) {
    const unsigned w = (unsigned)g.cf[0] | ((unsigned)g.cf[1] << 8) | ((unsigned)g.cf[2] << 16) |
                       ((unsigned)g.cf[3] << 24);
    return (int)((w >> (8 * (((r & 1) << 1) | (c & 1)))) & 0xffu);
}
__device__ __forceinline__ bool inr(const Img &g, int r, int c, int m) {
    return r >= m && r < g.H - m && c >= m && c < g.W - m;
}
// normalisation of the wrapper: (v - min) * factor, factor = 65535 / (max - min)
__device__ __forceinline__ void norm_consts(const Img &g, float &mn, float &factor) {
    mn = ord2f(g.mm[0]);
    const float mx = ord2f(g.mm[1]);
    factor = 65535.0f / (mx - mn);
}

// 64 x 4 pixel tiles.  remap: the dispatcher deals consecutive workgroups
// round-robin over the 8 XCDs (each with its own L2), so the tiles above and
// below a tile -- whose rows its stencils read -- ran on other XCDs and every
// tile fetched its halo rows from HBM (RCD moved ~64 planes of traffic for
// ~24 plane touches).  The tiles are renumbered so that each XCD walks one
// contiguous band of tile rows.
__device__ __forceinline__ void dm_tile(const Img &g, int &bx, int &by) {
    const unsigned total = gridDim.x * gridDim.y, L = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned w = (g.remap && total % 8u == 0u) ? (L % 8u) * (total / 8u) + L / 8u : L;
    bx = (int)(w % gridDim.x);
    by = (int)(w / gridDim.x);
}
#define DM_XY                                                        \
    int bx_, by_;                                                    \
    dm_tile(g, bx_, by_);                                            \
    const int x = bx_ * 64 + (threadIdx.x & 63);                     \
    const int y = by_ * 4 + (threadIdx.x >> 6);                      \
    if (x >= g.W || y >= g.H) return;                                \
    const long long p = (long long)y * g.W + x;                      \
    const long long W = g.W;

__global__ __launch_bounds__(1024) void k_minmax(const float *buf, long long n, unsigned *mm) {
    // 16-byte loads, four in flight per thread; one LDS block reduction and
    // one atomic pair per block, one 1024-thread block per CU (atomics on one
    // address serialise: per-wave atomics, 16 k of them, cost 0.38 ms, and
    // 2048 blocks' pairs 54 us against 38 us for 1024)
    unsigned lo = 0xffffffffu, hi = 0u;
    const long long n4 = ((reinterpret_cast<uintptr_t>(buf) & 15) == 0) ? n / 4 : 0;   // 16-B aligned
    const float4 *b4 = (const float4 *)buf;
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {        // four loads in flight per thread
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; u++) q[u] = b4[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            lo = min(lo, min(min(f2ord(q[u].x), f2ord(q[u].y)), min(f2ord(q[u].z), f2ord(q[u].w))));
            hi = max(hi, max(max(f2ord(q[u].x), f2ord(q[u].y)), max(f2ord(q[u].z), f2ord(q[u].w))));
        }
    }
    for (; i < n4; i += stride) {
        const float4 q = b4[i];
        lo = min(lo, min(min(f2ord(q.x), f2ord(q.y)), min(f2ord(q.z), f2ord(q.w))));
        hi = max(hi, max(max(f2ord(q.x), f2ord(q.y)), max(f2ord(q.z), f2ord(q.w))));
    }
    for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned o = f2ord(buf[i]);
        lo = min(lo, o);
        hi = max(hi, o);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, (unsigned)__shfl_xor((int)lo, off, 64));
        hi = max(hi, (unsigned)__shfl_xor((int)hi, off, 64));
    }
    __shared__ unsigned s_lo[16], s_hi[16];
    if ((threadIdx.x & 63) == 0) {
        s_lo[threadIdx.x >> 6] = lo;
        s_hi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
            lo = min(lo, s_lo[w]);
            hi = max(hi, s_hi[w]);
        }
        atomicMin(mm, lo);
        atomicMax(mm + 1, hi);
    }
}

__device__ __forceinline__ float ld(const float *b, long long i) { return b[i]; }
__device__ __forceinline__ float ld(const uint16_t *b, long long i) { return (float)b[i]; }
// the wrapper's output conversion: float as is; WORD / BYTE rounding
__device__ __forceinline__ void st(float *o, long long i, float v, int) { o[i] = v; }
__device__ __forceinline__ uint16_t to_word(float v, int byte) {
    const float top = byte ? 255.0f : 65535.0f;
    float f = v + 0.5f;
    f = f > top ? top : f;
    f = f < 0.0f ? 0.0f : f;
    return (uint16_t)f;
}
__device__ __forceinline__ void st(uint16_t *o, long long i, float v, int byte) { o[i] = to_word(v, byte); }

// cfa = LIM01(raw / 65536) of the normalised raw value
template <class T>
__global__ __launch_bounds__(256) void k_prep(Img g, const T *buf, float *cfa) {
    DM_XY
    float mn, factor;
    norm_consts(g, mn, factor);
    const float raw = (ld(buf, p) - mn) * factor;
    const float v = raw / SCALE;
    cfa[p] = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
}

__device__ __forceinline__ float hpf2(float m3, float m2, float m1, float c, float p1, float p2, float p3) {
    float t = ((m3 - m1) - p1) + p3;
    t = t - 3.0f * (m2 + p2);
    t = t + 6.0f * c;
    return t * t;
}

// step 1.1: squared vertical / horizontal high-pass
__global__ __launch_bounds__(256) void k_hv(Img g, const float *cfa, float *V, float *Hh) {
    DM_XY
    float v = 0.f, h = 0.f;
    if (y >= 3 && y < g.H - 3 && x >= 4 && x < g.W - 4)
        v = hpf2(cfa[p - 3 * W], cfa[p - 2 * W], cfa[p - W], cfa[p], cfa[p + W], cfa[p + 2 * W], cfa[p + 3 * W]);
    if (y >= 4 && y < g.H - 4 && x >= 3 && x < g.W - 3)
        h = hpf2(cfa[p - 3], cfa[p - 2], cfa[p - 1], cfa[p], cfa[p + 1], cfa[p + 2], cfa[p + 3]);
    V[p] = v;
    Hh[p] = h;
}

// step 1.2 VH_Dir; step 2 low pass; step 4.0 diagonal high-pass
__global__ __launch_bounds__(256) void k_dir(Img g, const float *cfa, const float *V, const float *Hh, float *VH,
                                             float *LP, float *P, float *Q) {
    DM_XY
    float vh = 0.f;
    if (inr(g, y, x, 4)) {
        const float vs = fmaxf(EPSSQ, (V[p - W] + V[p]) + V[p + W]);
        const float hs = fmaxf(EPSSQ, (Hh[p - 1] + Hh[p]) + Hh[p + 1]);
        vh = vs / (vs + hs);
    }
    VH[p] = vh;
    const bool ng = fc(g, y, x) != 1;
    float lp = 0.f, pp = 0.f, qq = 0.f;
    if (ng && inr(g, y, x, 2)) {
        lp = cfa[p] + 0.5f * (((cfa[p - W] + cfa[p + W]) + cfa[p - 1]) + cfa[p + 1]);
        lp = lp + 0.25f * (((cfa[p - W - 1] + cfa[p - W + 1]) + cfa[p + W - 1]) + cfa[p + W + 1]);
    }
    if (ng && inr(g, y, x, 3)) {
        pp = hpf2(cfa[p - 3 * W - 3], cfa[p - 2 * W - 2], cfa[p - W - 1], cfa[p], cfa[p + W + 1], cfa[p + 2 * W + 2],
                  cfa[p + 3 * W + 3]);
        qq = hpf2(cfa[p - 3 * W + 3], cfa[p - 2 * W + 2], cfa[p - W + 1], cfa[p], cfa[p + W - 1], cfa[p + 2 * W - 2],
                  cfa[p + 3 * W - 3]);
    }
    LP[p] = lp;
    P[p] = pp;
    Q[p] = qq;
}

// k_hv, k_dir and k_pq in one pass (round 6): VH_Dir from the six high-pass
// values it reads, recomputed from the CFA plane instead of stored in V / Hh
// and re-read, and the PQ ratio of step 4.1 from the six diagonal high-pass
// values instead of the P / Q planes -- 4 planes written (VH, LP, PQ) and 1 read
// (cfa) instead of 2 + 4 + 1 written and 1 + 3 + 2 read by the three kernels.
// Inside inr(4) every V / H / P / Q value the ratios read is in its own
// non-zero range (V: rows [3, H-3), H: columns [3, W-3), P / Q: red / blue
// sites in inr(3), and a red / blue site's diagonals are red / blue), so the
// recomputed values are the stored ones; where k_pq writes nothing the plane
// keeps the low-pass value, as k_pq's in-place buffer did.  Same
// expressions, same order: bitwise the three-kernel planes.
__global__ __launch_bounds__(256) void k_dir_pq(Img g, const float *cfa, float *VH, float *LP, float *PQ) {
    DM_XY
    auto vpf = [&](long long q) {
        return hpf2(cfa[q - 3 * W], cfa[q - 2 * W], cfa[q - W], cfa[q], cfa[q + W], cfa[q + 2 * W], cfa[q + 3 * W]);
    };
    auto hpf = [&](long long q) {
        return hpf2(cfa[q - 3], cfa[q - 2], cfa[q - 1], cfa[q], cfa[q + 1], cfa[q + 2], cfa[q + 3]);
    };
    const bool in4 = inr(g, y, x, 4);
    float vh = 0.f;
    if (in4) {
        const float vs = fmaxf(EPSSQ, (vpf(p - W) + vpf(p)) + vpf(p + W));
        const float hs = fmaxf(EPSSQ, (hpf(p - 1) + hpf(p)) + hpf(p + 1));
        vh = vs / (vs + hs);
    }
    VH[p] = vh;
    const bool ng = fc(g, y, x) != 1;
    float lp = 0.f;
    if (ng && inr(g, y, x, 2)) {
        lp = cfa[p] + 0.5f * (((cfa[p - W] + cfa[p + W]) + cfa[p - 1]) + cfa[p + 1]);
        lp = lp + 0.25f * (((cfa[p - W - 1] + cfa[p - W + 1]) + cfa[p + W - 1]) + cfa[p + W + 1]);
    }
    LP[p] = lp;
    float pq = lp;
    if (ng && in4) {
        auto ppf = [&](long long q) {
            return hpf2(cfa[q - 3 * W - 3], cfa[q - 2 * W - 2], cfa[q - W - 1], cfa[q], cfa[q + W + 1],
                        cfa[q + 2 * W + 2], cfa[q + 3 * W + 3]);
        };
        auto qpf = [&](long long q) {
            return hpf2(cfa[q - 3 * W + 3], cfa[q - 2 * W + 2], cfa[q - W + 1], cfa[q], cfa[q + W - 1],
                        cfa[q + 2 * W - 2], cfa[q + 3 * W - 3]);
        };
        const float ps = fmaxf(EPSSQ, (ppf(p - W - 1) + ppf(p)) + ppf(p + W + 1));
        const float qs = fmaxf(EPSSQ, (qpf(p - W + 1) + qpf(p)) + qpf(p + W - 1));
        pq = ps / (ps + qs);
    }
    PQ[p] = pq;
}

__device__ __forceinline__ float disc(float central, float nb) {
    return fabsf(0.5f - central) < fabsf(0.5f - nb) ? nb : central;
}

// step 3: green at red / blue sites
__global__ __launch_bounds__(256) void k_green(Img g, const float *cfa, const float *VH, const float *LP, float *G) {
    DM_XY
    const float c0 = cfa[p];
    if (fc(g, y, x) == 1) {
        G[p] = c0;
        return;
    }
    if (!inr(g, y, x, 4)) {
        G[p] = 0.f;
        return;
    }
    const float n1 = cfa[p - W], s1 = cfa[p + W], w1 = cfa[p - 1], e1 = cfa[p + 1];
    const float n2 = cfa[p - 2 * W], s2 = cfa[p + 2 * W], w2 = cfa[p - 2], e2 = cfa[p + 2];
    const float N_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - n2))) + (fabsf(n1 - cfa[p - 3 * W]) + fabsf(n2 - cfa[p - 4 * W]));
    const float S_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - s2))) + (fabsf(s1 - cfa[p + 3 * W]) + fabsf(s2 - cfa[p + 4 * W]));
    const float W_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - w2))) + (fabsf(w1 - cfa[p - 3]) + fabsf(w2 - cfa[p - 4]));
    const float E_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - e2))) + (fabsf(e1 - cfa[p + 3]) + fabsf(e2 - cfa[p + 4]));
    const float lpi = LP[p];
    const float l2 = lpi + lpi;
    const float N_Est = n1 * l2 / ((EPS + lpi) + LP[p - 2 * W]);
    const float S_Est = s1 * l2 / ((EPS + lpi) + LP[p + 2 * W]);
    const float W_Est = w1 * l2 / ((EPS + lpi) + LP[p - 2]);
    const float E_Est = e1 * l2 / ((EPS + lpi) + LP[p + 2]);
    const float V_Est = (S_Grad * N_Est + N_Grad * S_Est) / (N_Grad + S_Grad);
    const float H_Est = (W_Grad * E_Est + E_Grad * W_Est) / (E_Grad + W_Grad);
    const float nb = 0.25f * ((VH[p - W - 1] + VH[p - W + 1]) + (VH[p + W - 1] + VH[p + W + 1]));
    const float d = disc(VH[p], nb);
    G[p] = d * (H_Est - V_Est) + V_Est;
}

// step 4.1: PQ_Dir over the low-pass buffer (in place: reads only P / Q)
__global__ __launch_bounds__(256) void k_pq(Img g, const float *P, const float *Q, float *LPQ) {
    DM_XY
    if (fc(g, y, x) == 1 || !inr(g, y, x, 4)) return;
    const float ps = fmaxf(EPSSQ, (P[p - W - 1] + P[p]) + P[p + W + 1]);
    const float qs = fmaxf(EPSSQ, (Q[p - W + 1] + Q[p]) + Q[p + W - 1]);
    LPQ[p] = ps / (ps + qs);
}

// native value of colour c at (r, x), else 0 (rgb[c] before step 4.2)
__device__ __forceinline__ float nat(const Img &g, const float *cfa, long long q, int r, int x, int c) {
    return fc(g, r, x) == c ? cfa[q] : 0.f;
}

// step 4.2: red at blue sites, blue at red sites; native values elsewhere
__global__ __launch_bounds__(256) void k_rb_sites(Img g, const float *cfa, const float *G, const float *PQ, float *R,
                                                  float *B) {
    DM_XY
    const int col = fc(g, y, x);
    float r = col == 0 ? cfa[p] : 0.f, b = col == 2 ? cfa[p] : 0.f;
    if (col != 1 && inr(g, y, x, 4)) {
        const int c = 2 - col;              // the colour to interpolate (its sites are the diagonals)
        const float nb = 0.25f * (((PQ[p - W - 1] + PQ[p - W + 1]) + PQ[p + W - 1]) + PQ[p + W + 1]);
        const float d = disc(PQ[p], nb);
        const float NW = cfa[p - W - 1], NE = cfa[p - W + 1], SW = cfa[p + W - 1], SE = cfa[p + W + 1];
        const float g0 = G[p];
        const float NW_Grad = ((EPS + fabsf(NW - SE)) + fabsf(NW - cfa[p - 3 * W - 3])) + fabsf(g0 - G[p - 2 * W - 2]);
        const float NE_Grad = ((EPS + fabsf(NE - SW)) + fabsf(NE - cfa[p - 3 * W + 3])) + fabsf(g0 - G[p - 2 * W + 2]);
        const float SW_Grad = ((EPS + fabsf(NE - SW)) + fabsf(SW - cfa[p + 3 * W - 3])) + fabsf(g0 - G[p + 2 * W - 2]);
        const float SE_Grad = ((EPS + fabsf(NW - SE)) + fabsf(SE - cfa[p + 3 * W + 3])) + fabsf(g0 - G[p + 2 * W + 2]);
        const float NW_Est = NW - G[p - W - 1];
        const float NE_Est = NE - G[p - W + 1];
        const float SW_Est = SW - G[p + W - 1];
        const float SE_Est = SE - G[p + W + 1];
        const float P_Est = (NW_Grad * SE_Est + SE_Grad * NW_Est) / (NW_Grad + SE_Grad);
        const float Q_Est = (NE_Grad * SW_Est + SW_Grad * NE_Est) / (NE_Grad + SW_Grad);
        const float v = g0 + (d * (Q_Est - P_Est) + P_Est);
        if (c == 0) r = v;
        else b = v;
    }
    R[p] = r;
    B[p] = b;
}

// border_interpolate (3 x 3 same-colour mean) on the normalised raw data
template <class T>
__device__ void border(const Img &g, const T *buf, float mn, float factor, int y, int x, float out[3]) {
    float sm[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i1 = y - 1; i1 < y + 2; i1++)
        for (int j1 = x - 1; j1 < x + 2; j1++)
            if (i1 >= 0 && i1 < g.H && j1 >= 0 && j1 < g.W) {
                const int c = fc(g, i1, j1);
                sm[c] = sm[c] + (ld(buf, (long long)i1 * g.W + j1) - mn) * factor;
                sm[c + 3] = sm[c + 3] + 1.f;
            }
    const int c = fc(g, y, x);
    const float raw = (ld(buf, (long long)y * g.W + x) - mn) * factor;
    if (c == 1) {
        out[0] = sm[0] / sm[3];
        out[1] = raw;
        out[2] = sm[2] / sm[5];
    } else {
        out[1] = sm[1] / sm[4];
        out[0] = c == 0 ? raw : sm[0] / sm[3];
        out[2] = c == 0 ? sm[2] / sm[5] : raw;
    }
}

// step 4.3 (red / blue at green sites), border, and the wrapper's inverse
// mapping; writes the planar RGB output
template <class T, class O>
__global__ __launch_bounds__(256) void k_final(Img g, const T *buf, const float *G, const float *VH, const float *R,
                                               const float *B, O *rgb, int byte) {
    DM_XY
    float mn, factor;
    norm_consts(g, mn, factor);
    const float invfactor = (float)(1.0 / (double)factor);
    float o[3];
    if (!inr(g, y, x, BORDER)) {
        border(g, buf, mn, factor, y, x, o);
    } else {
        float r = R[p], b = B[p];
        const float g0 = G[p];
        if (fc(g, y, x) == 1) {
            const float nb = 0.25f * ((VH[p - W - 1] + VH[p - W + 1]) + (VH[p + W - 1] + VH[p + W + 1]));
            const float d = disc(VH[p], nb);
            const float N1 = EPS + fabsf(g0 - G[p - 2 * W]);
            const float S1 = EPS + fabsf(g0 - G[p + 2 * W]);
            const float W1 = EPS + fabsf(g0 - G[p - 2]);
            const float E1 = EPS + fabsf(g0 - G[p + 2]);
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const float *pl = k == 0 ? R : B;
                const float SNabs = fabsf(pl[p - W] - pl[p + W]);
                const float EWabs = fabsf(pl[p - 1] - pl[p + 1]);
                const float N_Grad = (N1 + SNabs) + fabsf(pl[p - W] - pl[p - 3 * W]);
                const float S_Grad = (S1 + SNabs) + fabsf(pl[p + W] - pl[p + 3 * W]);
                const float W_Grad = (W1 + EWabs) + fabsf(pl[p - 1] - pl[p - 3]);
                const float E_Grad = (E1 + EWabs) + fabsf(pl[p + 1] - pl[p + 3]);
                const float N_Est = pl[p - W] - G[p - W];
                const float S_Est = pl[p + W] - G[p + W];
                const float W_Est = pl[p - 1] - G[p - 1];
                const float E_Est = pl[p + 1] - G[p + 1];
                const float V_Est = (N_Grad * S_Est + S_Grad * N_Est) / (N_Grad + S_Grad);
                const float H_Est = (E_Grad * W_Est + W_Grad * E_Est) / (E_Grad + W_Grad);
                const float v = g0 + (d * (H_Est - V_Est) + V_Est);
                if (k == 0) r = v;
                else b = v;
            }
        }
        o[0] = fmaxf(0.f, r * SCALE);
        o[1] = fmaxf(0.f, g0 * SCALE);
        o[2] = fmaxf(0.f, b * SCALE);
    }
    const long long n = (long long)g.W * g.H;
#pragma unroll
    for (int k = 0; k < 3; k++) st(rgb, k * n + p, o[k] * invfactor + mn, byte);
}

// ---------------------------------------------------------------- bayerfast
// BAYER_BILINEAR: librtprocess bayerfast_demosaic (demosaicing_rtp.cpp:147-151,
// 318-323; RawTherapee fast_demosaic), restated in oracle/demosaic_ref.py
// (parity with librtprocess unpinned).  Two stencil passes in the
// reference's expression order, f32 without contraction:
//   k_bf_green: the green plane (raw at green sites, the gradient-weighted
//     mean of the four neighbours at red / blue sites, rows / columns
//     [3, -3): what the interior reads) -- the four reciprocals and the
//     division per red / blue site are done once;
//   k_bf_final: red / blue from the green plane (diagonal colour difference
//     at red / blue sites, cardinal at green sites, the diagonal one of the
//     neighbours recomputed from four green reads), the 5-pixel border
//     (border_interpolate), the wrapper's inverse map.
// (One pass recomputing every green it needs, 13 per pixel, was VALU-bound
// on the divisions: 2.03 ms per 6000 x 4000 frame, profiles/r05d_b_bayerfast.)
constexpr int BF_BORDER = 5;
constexpr float BF_CLIP = 4.f * 65535.f;   // clip_pt = 4 * 65535 * initGain, initGain = 1.0

template <class T>
struct BfSrc {
    const T *buf;
    int W;
    float mn, factor;
    __device__ __forceinline__ float raw(int y, int x) const { return (ld(buf, (long long)y * W + x) - mn) * factor; }
};
__device__ __forceinline__ float bf_min(float v) { return v < BF_CLIP ? v : BF_CLIP; }   // std::min(clip_pt, v)

template <class T>
__global__ __launch_bounds__(256) void k_bf_green(Img g, const T *buf, float *G) {
    DM_XY
    (void)W;
    float mn, factor;
    norm_consts(g, mn, factor);
    const BfSrc<T> b{buf, g.W, mn, factor};
    const float c = b.raw(y, x);
    if (fc(g, y, x) == 1 || !inr(g, y, x, BF_BORDER - 2)) {
        G[p] = c;                                  // outside [3, -3) nothing reads it as an estimate
        return;
    }
    const float n1 = b.raw(y - 1, x), s1 = b.raw(y + 1, x), w1 = b.raw(y, x - 1), e1 = b.raw(y, x + 1);
    float t;
    t = (1.f + fabsf(c - b.raw(y - 2, x))) + fabsf(n1 - s1);
    const float wtu = 1.f / (t * t);
    t = (1.f + fabsf(c - b.raw(y + 2, x))) + fabsf(s1 - n1);
    const float wtd = 1.f / (t * t);
    t = (1.f + fabsf(c - b.raw(y, x - 2))) + fabsf(w1 - e1);
    const float wtl = 1.f / (t * t);
    t = (1.f + fabsf(c - b.raw(y, x + 2))) + fabsf(e1 - w1);
    const float wtr = 1.f / (t * t);
    G[p] = (((wtu * n1 + wtd * s1) + wtl * w1) + wtr * e1) / (((wtu + wtd) + wtl) + wtr);
}

// colour k (0 red, 2 blue) at the red / blue site q = (y, x): native, or the
// colour difference of the four diagonals
template <class T>
__device__ __forceinline__ float bf_rb_site(const Img &g, const BfSrc<T> &b, const float *G, int y, int x, int k) {
    if (fc(g, y, x) == k) return b.raw(y, x);
    const long long W = g.W, q = (long long)y * W + x;
    const float gd = ((G[q - W - 1] + G[q - W + 1]) + G[q + W + 1]) + G[q + W - 1];
    const float rd = ((b.raw(y - 1, x - 1) + b.raw(y - 1, x + 1)) + b.raw(y + 1, x + 1)) + b.raw(y + 1, x - 1);
    return G[q] - 0.25f * (gd - bf_min(rd));
}

template <class T, class O>
__global__ __launch_bounds__(256) void k_bf_final(Img g, const T *buf, const float *G, O *rgb, int byte) {
    DM_XY
    float mn, factor;
    norm_consts(g, mn, factor);
    const float invfactor = (float)(1.0 / (double)factor);
    const BfSrc<T> b{buf, g.W, mn, factor};
    float o[3];
    if (!inr(g, y, x, BF_BORDER)) {
        border(g, buf, mn, factor, y, x, o);      // border_interpolate(bord = 5) on the normalised data
    } else {
        const float g0 = G[p];
        float r, bl;
        if (fc(g, y, x) != 1) {
            r = bf_rb_site(g, b, G, y, x, 0);
            bl = bf_rb_site(g, b, G, y, x, 2);
        } else {
            const float gN = G[p - W], gW = G[p - 1], gE = G[p + 1], gS = G[p + W];
            const float gsum = ((gN + gW) + gE) + gS;
            float v[2];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int k = 2 * q;
                const float xs = ((bf_rb_site(g, b, G, y - 1, x, k) + bf_rb_site(g, b, G, y, x - 1, k)) +
                                  bf_rb_site(g, b, G, y, x + 1, k)) +
                                 bf_rb_site(g, b, G, y + 1, x, k);
                v[q] = g0 - 0.25f * (gsum - bf_min(xs));
            }
            r = v[0];
            bl = v[1];
        }
        o[0] = fmaxf(0.f, r);
        o[1] = fmaxf(0.f, g0);
        o[2] = fmaxf(0.f, bl);
    }
    const long long n = (long long)g.W * g.H;
#pragma unroll
    for (int k = 0; k < 3; k++) st(rgb, k * n + p, o[k] * invfactor + mn, byte);
}

// One tiled pass (round 6): a workgroup owns a 64 x 32 tile of the output.
// It loads the normalised raw values of the tile and a 4-pixel halo into LDS
// (coalesced rows, each value converted once with the wrapper's (v - mn) *
// factor), computes the green plane of the tile and a 2-pixel halo into LDS
// with k_bf_green's expressions, then the three colours with k_bf_final's,
// reading G and raw from LDS: the green plane never reaches HBM (the
// two-pass form wrote and re-read it, and each thread fetched its ~20
// neighbours through L1).  Same expressions in the same order, so the
// result is bitwise the two-pass one.  The border (!inr(5)) keeps the global
// border_interpolate restatement.
constexpr int BFT_W = 64, BFT_H = 32;
constexpr int BFR_W = BFT_W + 8, BFR_H = BFT_H + 8;   // raw: halo 4
constexpr int BFG_W = BFT_W + 4, BFG_H = BFT_H + 4;   // green: halo 2

template <class T, class O>
__global__ __launch_bounds__(256) void k_bf_tiled(Img g, const T *buf, O *rgb, int byte) {
    __shared__ float s_raw[BFR_H * BFR_W];
    __shared__ float s_g[BFG_H * BFG_W];
    int bx, by;
    dm_tile(g, bx, by);
    const int x0 = bx * BFT_W, y0 = by * BFT_H;
    const int W = g.W, H = g.H;
    float mn, factor;
    norm_consts(g, mn, factor);
    // raw tile rows [y0 - 4, y0 + 20), columns [x0 - 4, x0 + 68); outside the
    // image: 0 (never read by an in-image estimate, see below)
    for (int i = threadIdx.x; i < BFR_H * BFR_W; i += 256) {
        const int ry = i / BFR_W, rx = i % BFR_W;
        const int yy = y0 - 4 + ry, xx = x0 - 4 + rx;
        s_raw[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? (ld(buf, (long long)yy * W + xx) - mn) * factor : 0.f;
    }
    __syncthreads();
    auto R = [&](int yy, int xx) { return s_raw[(yy - y0 + 4) * BFR_W + (xx - x0 + 4)]; };
    // green of the tile and a 2-pixel halo (k_bf_green): G at (yy, xx) reads
    // raw within 2 of it, inside the raw halo of 4
    for (int i = threadIdx.x; i < BFG_H * BFG_W; i += 256) {
        const int gy = i / BFG_W, gx = i % BFG_W;
        const int yy = y0 - 2 + gy, xx = x0 - 2 + gx;
        float v = 0.f;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const float c = R(yy, xx);
            if (fc(g, yy, xx) == 1 || !inr(g, yy, xx, BF_BORDER - 2)) {
                v = c;
            } else {
                const float n1 = R(yy - 1, xx), s1 = R(yy + 1, xx), w1 = R(yy, xx - 1), e1 = R(yy, xx + 1);
                float t;
                t = (1.f + fabsf(c - R(yy - 2, xx))) + fabsf(n1 - s1);
                const float wtu = 1.f / (t * t);
                t = (1.f + fabsf(c - R(yy + 2, xx))) + fabsf(s1 - n1);
                const float wtd = 1.f / (t * t);
                t = (1.f + fabsf(c - R(yy, xx - 2))) + fabsf(w1 - e1);
                const float wtl = 1.f / (t * t);
                t = (1.f + fabsf(c - R(yy, xx + 2))) + fabsf(e1 - w1);
                const float wtr = 1.f / (t * t);
                v = (((wtu * n1 + wtd * s1) + wtl * w1) + wtr * e1) / (((wtu + wtd) + wtl) + wtr);
            }
        }
        s_g[i] = v;
    }
    __syncthreads();
    auto Gg = [&](int yy, int xx) { return s_g[(yy - y0 + 2) * BFG_W + (xx - x0 + 2)]; };
    // bf_rb_site on the LDS planes
    auto rb_site = [&](int yy, int xx, int k) {
        if (fc(g, yy, xx) == k) return R(yy, xx);
        const float gd = ((Gg(yy - 1, xx - 1) + Gg(yy - 1, xx + 1)) + Gg(yy + 1, xx + 1)) + Gg(yy + 1, xx - 1);
        const float rd = ((R(yy - 1, xx - 1) + R(yy - 1, xx + 1)) + R(yy + 1, xx + 1)) + R(yy + 1, xx - 1);
        return Gg(yy, xx) - 0.25f * (gd - bf_min(rd));
    };
    const float invfactor = (float)(1.0 / (double)factor);
    const long long n = (long long)W * H;
    const int x = x0 + (int)(threadIdx.x & 63);
#pragma unroll
    for (int j = 0; j < BFT_H / 4; j++) {
        const int y = y0 + (int)(threadIdx.x >> 6) + 4 * j;
        if (x >= W || y >= H) continue;
        float o[3];
        if (!inr(g, y, x, BF_BORDER)) {
            border(g, buf, mn, factor, y, x, o);
        } else {
            const float g0 = Gg(y, x);
            float r, bl;
            if (fc(g, y, x) != 1) {
                r = rb_site(y, x, 0);
                bl = rb_site(y, x, 2);
            } else {
                const float gsum = ((Gg(y - 1, x) + Gg(y, x - 1)) + Gg(y, x + 1)) + Gg(y + 1, x);
                float v[2];
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const int k = 2 * q;
                    const float xs = ((rb_site(y - 1, x, k) + rb_site(y, x - 1, k)) + rb_site(y, x + 1, k)) +
                                     rb_site(y + 1, x, k);
                    v[q] = g0 - 0.25f * (gsum - bf_min(xs));
                }
                r = v[0];
                bl = v[1];
            }
            o[0] = fmaxf(0.f, r);
            o[1] = fmaxf(0.f, g0);
            o[2] = fmaxf(0.f, bl);
        }
        const long long p = (long long)y * W + x;
#pragma unroll
        for (int k = 0; k < 3; k++) st(rgb, k * n + p, o[k] * invfactor + mn, byte);
    }
}

// Site pairs (round 6, the default for Bayer patterns): the green sites of a
// Bayer CFA form a checkerboard, so every horizontal pair of columns (2i,
// 2i + 1) holds one green and one red / blue site.  k_bf_tiled gives one
// lane one pixel, so each wave ran the green-site branch and the red / blue
// branch one after the other (half its lanes masked in each), and a green
// site's red and blue recomputed the diagonal colour difference of each of
// its four neighbours (every such estimate was evaluated five times).  Here
// a lane owns one pair in every stage, so no branch diverges on the site
// colour, and the diagonal estimate of the red / blue site's missing colour
// is computed once into a third LDS plane D (one word per red / blue site,
// tile + 1-pixel halo) that the green sites read.  Same expressions in the
// same order (D holds the float rb_site returned), so the output is bitwise
// k_bf_tiled's.
constexpr int BFD_W = BFT_W / 2 + 1, BFD_H = BFT_H + 2;   // D: red / blue sites of the tile + halo 1

// Pair reads: a lane's pair (xx, xx + 1), xx even, sits at an even offset of
// every plane row (row widths and halos even), so the rows above, at and
// below a pair come in one ds_read_b64 each and a wave's 32-lane groups read
// contiguous 256 bytes (per-site b32 reads at a 2-word stride were 2-way
// bank conflicts: 12.8 M conflict cycles against 7.6 M LDS instructions,
// 0.165 ms against 0.156 ms).  Output: one 8-byte (float) / 4-byte (16-bit)
// store per plane and pair when aligned.
template <class O> struct Pair2;
template <> struct Pair2<float> {
    __device__ static void st2(float *o, long long i, float a, float b, int) {
        *reinterpret_cast<float2 *>(o + i) = make_float2(a, b);
    }
};
template <> struct Pair2<uint16_t> {
    __device__ static void st2(uint16_t *o, long long i, float a, float b, int byte) {
        *reinterpret_cast<unsigned *>(o + i) = (unsigned)to_word(a, byte) | ((unsigned)to_word(b, byte) << 16);
    }
};

template <class T, class O>
__global__ __launch_bounds__(256) void k_bf_pairs(Img g, const T *buf, O *rgb, int byte, int vec) {
    __shared__ __align__(16) float s_raw[BFR_H * BFR_W];
    __shared__ __align__(16) float s_g[BFG_H * BFG_W];
    __shared__ __align__(16) float s_d[BFD_H * BFD_W];
    int bx, by;
    dm_tile(g, bx, by);
    const int x0 = bx * BFT_W, y0 = by * BFT_H;   // x0 even
    const int W = g.W, H = g.H;
    float mn, factor;
    norm_consts(g, mn, factor);
    for (int i = threadIdx.x; i < BFR_H * BFR_W; i += 256) {
        const int ry = i / BFR_W, rx = i - ry * BFR_W;
        const int yy = y0 - 4 + ry, xx = x0 - 4 + rx;
        s_raw[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? (ld(buf, (long long)yy * W + xx) - mn) * factor : 0.f;
    }
    __syncthreads();
    // pair (xx, xx + 1) of row yy, xx even
    auto R2 = [&](int yy, int xx) {
        return *reinterpret_cast<const float2 *>(&s_raw[(yy - y0 + 4) * BFR_W + (xx - x0 + 4)]);
    };
    auto R = [&](int yy, int xx) { return s_raw[(yy - y0 + 4) * BFR_W + (xx - x0 + 4)]; };
    auto gpar = [&](int yy) { return fc(g, yy, 0) == 1 ? 0 : 1; };
    for (int i = threadIdx.x; i < BFG_H * (BFG_W / 2); i += 256) {
        const int gy = i / (BFG_W / 2), px = i - gy * (BFG_W / 2);
        const int yy = y0 - 2 + gy, xx = x0 - 2 + 2 * px;
        const int gp = gpar(yy), xg = xx + gp, xn = xx + 1 - gp;
        const bool row_in = yy >= 0 && yy < H;
        const float2 c2 = R2(yy, xx);
        float vg = 0.f, vn = 0.f;
        if (row_in && xg >= 0 && xg < W) vg = gp ? c2.y : c2.x;
        if (row_in && xn >= 0 && xn < W) {
            const float c = gp ? c2.x : c2.y;
            if (!inr(g, yy, xn, BF_BORDER - 2)) {
                vn = c;
            } else {
                const float2 a = R2(yy - 2, xx), b = R2(yy - 1, xx), d = R2(yy + 1, xx), e = R2(yy + 2, xx);
                const float2 l = R2(yy, xx - 2), r = R2(yy, xx + 2);
                const float n1 = gp ? b.x : b.y, s1 = gp ? d.x : d.y;
                const float w1 = gp ? l.y : c2.x, e1 = gp ? c2.y : r.x;
                const float nn = gp ? a.x : a.y, ss = gp ? e.x : e.y;
                const float ww = gp ? l.x : l.y, ee = gp ? r.x : r.y;
                float t;
                t = (1.f + fabsf(c - nn)) + fabsf(n1 - s1);
                const float wtu = 1.f / (t * t);
                t = (1.f + fabsf(c - ss)) + fabsf(s1 - n1);
                const float wtd = 1.f / (t * t);
                t = (1.f + fabsf(c - ww)) + fabsf(w1 - e1);
                const float wtl = 1.f / (t * t);
                t = (1.f + fabsf(c - ee)) + fabsf(e1 - w1);
                const float wtr = 1.f / (t * t);
                vn = (((wtu * n1 + wtd * s1) + wtl * w1) + wtr * e1) / (((wtu + wtd) + wtl) + wtr);
            }
        }
        *reinterpret_cast<float2 *>(&s_g[gy * BFG_W + 2 * px]) = gp ? make_float2(vn, vg) : make_float2(vg, vn);
    }
    __syncthreads();
    auto G2 = [&](int yy, int xx) {
        return *reinterpret_cast<const float2 *>(&s_g[(yy - y0 + 2) * BFG_W + (xx - x0 + 2)]);
    };
    auto Gg = [&](int yy, int xx) { return s_g[(yy - y0 + 2) * BFG_W + (xx - x0 + 2)]; };
    // D at the red / blue site x of row yy: its diagonals x - 1, x + 1 are
    // the same component of the pairs at (x - 1) & ~1 and (x + 1) & ~1
    for (int i = threadIdx.x; i < BFD_H * BFD_W; i += 256) {
        const int dy = i / BFD_W, dx = i - dy * BFD_W;
        const int yy = y0 - 1 + dy;
        const int gp = gpar(yy);
        const int x = x0 - (1 - gp) + 2 * dx;
        const int xl = (x - 1) & ~1, xr = xl + 2;
        const float2 gul = G2(yy - 1, xl), gur = G2(yy - 1, xr), gdl = G2(yy + 1, xl), gdr = G2(yy + 1, xr);
        const float2 rul = R2(yy - 1, xl), rur = R2(yy - 1, xr), rdl = R2(yy + 1, xl), rdr = R2(yy + 1, xr);
        const float2 gc = G2(yy, x & ~1);
        const bool hi = gp != 0;            // (x - 1) & 1 == gp
        const float gd = (((hi ? gul.y : gul.x) + (hi ? gur.y : gur.x)) + (hi ? gdr.y : gdr.x)) + (hi ? gdl.y : gdl.x);
        const float rd = (((hi ? rul.y : rul.x) + (hi ? rur.y : rur.x)) + (hi ? rdr.y : rdr.x)) + (hi ? rdl.y : rdl.x);
        s_d[i] = (hi ? gc.x : gc.y) - 0.25f * (gd - bf_min(rd));
    }
    __syncthreads();
    const float *Drow = s_d;
    const float invfactor = (float)(1.0 / (double)factor);
    const long long n = (long long)W * H;
    const int px = (int)(threadIdx.x & 31);
#pragma unroll
    for (int j = 0; j < BFT_H / 8; j++) {
        const int y = y0 + (int)(threadIdx.x >> 5) + 8 * j;
        if (y >= H) continue;
        const int xx = x0 + 2 * px;
        if (xx >= W) continue;
        const int gp = gpar(y), xg = xx + gp, xn = xx + 1 - gp;
        const int ch = fc(g, y, xn), cvv = fc(g, y + 1, xg);
        const float2 gu = G2(y - 1, xx), gc = G2(y, xx), gd = G2(y + 1, xx);
        const float2 ru = R2(y - 1, xx), rc = R2(y, xx), rd = R2(y + 1, xx);
        const float gside = Gg(y, gp ? xx + 2 : xx - 1), rside = R(y, gp ? xx + 2 : xx - 1);
        const float *dr = Drow + (y - y0 + 1) * BFD_W;
        const float dl = dr[px], drr = dr[px + 1];
        const float dup = dr[px + gp - BFD_W], ddn = dr[px + gp + BFD_W];
        float og[3] = {0.f, 0.f, 0.f}, on[3] = {0.f, 0.f, 0.f};
        // green site xg (outside the image at an odd width's last pair)
        if (xg >= W) {
        } else if (!inr(g, y, xg, BF_BORDER)) {
            border(g, buf, mn, factor, y, xg, og);
        } else {
            const float g0 = gp ? gc.y : gc.x;
            const float gsum = gp ? (((gu.y + gc.x) + gside) + gd.y) : (((gu.x + gside) + gc.y) + gd.x);
            const float uR = gp ? ru.y : ru.x, dR = gp ? rd.y : rd.x;
            const float lR = gp ? rc.x : rside, rR = gp ? rside : rc.y;
            float v[2];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int k = 2 * q;
                const float su = cvv == k ? uR : dup, sd = cvv == k ? dR : ddn;
                const float sl = ch == k ? lR : dl, sr = ch == k ? rR : drr;
                const float xs = ((su + sl) + sr) + sd;
                v[q] = g0 - 0.25f * (gsum - bf_min(xs));
            }
            og[0] = fmaxf(0.f, v[0]);
            og[1] = fmaxf(0.f, g0);
            og[2] = fmaxf(0.f, v[1]);
        }
        // red / blue site xn
        const bool xn_in = xn < W;
        if (xn_in) {
            if (!inr(g, y, xn, BF_BORDER)) {
                border(g, buf, mn, factor, y, xn, on);
            } else {
                const float nat = gp ? rc.x : rc.y, dn = gp ? dl : drr;
                on[0] = fmaxf(0.f, ch == 0 ? nat : dn);
                on[1] = fmaxf(0.f, gp ? gc.x : gc.y);
                on[2] = fmaxf(0.f, ch == 2 ? nat : dn);
            }
        }
        const long long p = (long long)y * W + xx;
        if (vec && xn_in) {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const float a = (gp ? on[k] : og[k]) * invfactor + mn, b = (gp ? og[k] : on[k]) * invfactor + mn;
                Pair2<O>::st2(rgb, k * n + p, a, b, byte);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (xg < W) st(rgb, k * n + y * (long long)W + xg, og[k] * invfactor + mn, byte);
                if (xn_in) st(rgb, k * n + y * (long long)W + xn, on[k] * invfactor + mn, byte);
            }
        }
    }
}

// Bayer: green on a checkerboard (the pair kernel's premise)
inline bool bayer_checkerboard(const Img &g) {
    return (g.cf[0] == 1) == (g.cf[3] == 1) && (g.cf[1] == 1) == (g.cf[2] == 1) && (g.cf[0] == 1) != (g.cf[1] == 1);
}

// ws: g.W * g.H floats (the green plane; the two-pass form only).
// SGPU_BF_TWOPASS=1 selects the two-pass form, SGPU_BF_TILED=1 the
// one-pixel-per-lane tiled pass (A/B).
template <class T, class O>
int launch_bayerfast(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s) {
    static const bool two = std::getenv("SGPU_BF_TWOPASS") && std::atoi(std::getenv("SGPU_BF_TWOPASS")) != 0;
    static const bool tiled = std::getenv("SGPU_BF_TILED") && std::atoi(std::getenv("SGPU_BF_TILED")) != 0;
    if (!two && !tiled && bayer_checkerboard(g)) {
        const dim3 grid((g.W + BFT_W - 1) / BFT_W, (g.H + BFT_H - 1) / BFT_H);
        // pair stores: even width and an output aligned to the pair size
        const int vec = (g.W % 2 == 0) && (reinterpret_cast<uintptr_t>(rgb) % (2 * sizeof(O)) == 0);
        hipLaunchKernelGGL((k_bf_pairs<T, O>), grid, dim3(256), 0, s, g, buf, rgb, byte, vec);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (!two) {
        const dim3 grid((g.W + BFT_W - 1) / BFT_W, (g.H + BFT_H - 1) / BFT_H);
        hipLaunchKernelGGL((k_bf_tiled<T, O>), grid, dim3(256), 0, s, g, buf, rgb, byte);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    const dim3 grid((g.W + 63) / 64, (g.H + 3) / 4);
    hipLaunchKernelGGL((k_bf_green<T>), grid, dim3(256), 0, s, g, buf, ws);
    hipLaunchKernelGGL((k_bf_final<T, O>), grid, dim3(256), 0, s, g, buf, (const float *)ws, rgb, byte);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
template int launch_bayerfast<float, float>(Img, const float *, float *, int, float *, hipStream_t);
template int launch_bayerfast<uint16_t, uint16_t>(Img, const uint16_t *, uint16_t *, int, float *, hipStream_t);

// ---------------------------------------------------------------- fused RCD
// The whole RCD pipeline (k_prep .. k_final above, same expressions in the
// same order, so the result is bitwise that of the multi-pass kernels) for a
// TX x TY output tile in one workgroup: every intermediate plane lives in LDS
// over the tile plus the halo the later steps read (cfa +10, V/H +7, VH +6,
// LP +7, P/Q +5, G +5, PQ +4, R/B +3), recomputed on the overlap instead of
// round-tripping 8 full planes through HBM.  HBM traffic: one read of the
// CFA frame (plus its halo) and one write of the three output planes.
struct Pl {
    float *d;
    int x0, y0, pw;   // global coordinates of element [0][0]; row pitch
    __device__ __forceinline__ float at(int x, int y) const { return d[(y - y0) * pw + (x - x0)]; }
};

template <int TX, int TY>
struct RcdLayout {
    static constexpr int CFA = 10, VHH = 7, VHD = 6, LPH = 7, PQH = 5, PQD = 4, GH = 5, RBH = 3;
    static constexpr int w(int h) { return TX + 2 * h; }
    static constexpr int h(int hh) { return TY + 2 * hh; }
    static constexpr int n(int hh) { return w(hh) * h(hh); }
    // LDS plan: [cfa][V -> P -> R][H -> Q -> B][VH][LP][PQ][G]
    static constexpr int o_cfa = 0;
    static constexpr int o_a = o_cfa + n(CFA);
    static constexpr int o_b = o_a + n(VHH);
    static constexpr int o_vh = o_b + n(VHH);
    static constexpr int o_lp = o_vh + n(VHD);
    static constexpr int o_pq = o_lp + n(LPH);
    static constexpr int o_g = o_pq + n(PQD);
    static constexpr int total = o_g + n(GH);
};

template <int TX, int TY>
size_t rcd_lds_bytes() { return sizeof(float) * RcdLayout<TX, TY>::total; }

#define RCD_REGION(HALO)                                                         \
    for (int i_ = threadIdx.x; i_ < L::n(HALO); i_ += blockDim.x) {              \
        const int ly_ = i_ / L::w(HALO), lx_ = i_ - ly_ * L::w(HALO);            \
        const int x = X0 - (HALO) + lx_, y = Y0 - (HALO) + ly_;                  \
        const bool in_img = x >= 0 && y >= 0 && x < g.W && y < g.H;

#define RCD_END }

template <int TX, int TY, class T, class O>
__global__ __launch_bounds__(512) void k_rcd_fused(Img g, const T *buf, O *rgb, int byte) {
    using L = RcdLayout<TX, TY>;
    extern __shared__ float lds[];
    const int X0 = blockIdx.x * TX, Y0 = blockIdx.y * TY;
    const int W = g.W;
    const Pl cfa{lds + L::o_cfa, X0 - L::CFA, Y0 - L::CFA, L::w(L::CFA)};
    const Pl V{lds + L::o_a, X0 - L::VHH, Y0 - L::VHH, L::w(L::VHH)};
    const Pl Hh{lds + L::o_b, X0 - L::VHH, Y0 - L::VHH, L::w(L::VHH)};
    const Pl VH{lds + L::o_vh, X0 - L::VHD, Y0 - L::VHD, L::w(L::VHD)};
    const Pl LP{lds + L::o_lp, X0 - L::LPH, Y0 - L::LPH, L::w(L::LPH)};
    const Pl P{lds + L::o_a, X0 - L::PQH, Y0 - L::PQH, L::w(L::PQH)};
    const Pl Q{lds + L::o_b, X0 - L::PQH, Y0 - L::PQH, L::w(L::PQH)};
    const Pl PQ{lds + L::o_pq, X0 - L::PQD, Y0 - L::PQD, L::w(L::PQD)};
    const Pl G{lds + L::o_g, X0 - L::GH, Y0 - L::GH, L::w(L::GH)};
    const Pl R{lds + L::o_a, X0 - L::RBH, Y0 - L::RBH, L::w(L::RBH)};
    const Pl B{lds + L::o_b, X0 - L::RBH, Y0 - L::RBH, L::w(L::RBH)};
    float mn, factor;
    norm_consts(g, mn, factor);

    // k_prep
    RCD_REGION(L::CFA)
        float v = 0.f;
        if (in_img) {
            const float raw = (ld(buf, (long long)y * W + x) - mn) * factor;
            const float t = raw / SCALE;
            v = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
        }
        cfa.d[i_] = v;
    RCD_END
    __syncthreads();
    // k_hv
    RCD_REGION(L::VHH)
        float v = 0.f, h = 0.f;
        if (in_img) {
            if (y >= 3 && y < g.H - 3 && x >= 4 && x < g.W - 4)
                v = hpf2(cfa.at(x, y - 3), cfa.at(x, y - 2), cfa.at(x, y - 1), cfa.at(x, y), cfa.at(x, y + 1),
                         cfa.at(x, y + 2), cfa.at(x, y + 3));
            if (y >= 4 && y < g.H - 4 && x >= 3 && x < g.W - 3)
                h = hpf2(cfa.at(x - 3, y), cfa.at(x - 2, y), cfa.at(x - 1, y), cfa.at(x, y), cfa.at(x + 1, y),
                         cfa.at(x + 2, y), cfa.at(x + 3, y));
        }
        V.d[i_] = v;
        Hh.d[i_] = h;
    RCD_END
    __syncthreads();
    // k_dir: VH_Dir, then (V / H dead) low pass and diagonal high-pass
    RCD_REGION(L::VHD)
        float vh = 0.f;
        if (in_img && inr(g, y, x, 4)) {
            const float vs = fmaxf(EPSSQ, (V.at(x, y - 1) + V.at(x, y)) + V.at(x, y + 1));
            const float hs = fmaxf(EPSSQ, (Hh.at(x - 1, y) + Hh.at(x, y)) + Hh.at(x + 1, y));
            vh = vs / (vs + hs);
        }
        VH.d[i_] = vh;
    RCD_END
    RCD_REGION(L::LPH)
        float lp = 0.f;
        if (in_img && fc(g, y, x) != 1 && inr(g, y, x, 2)) {
            lp = cfa.at(x, y) + 0.5f * (((cfa.at(x, y - 1) + cfa.at(x, y + 1)) + cfa.at(x - 1, y)) + cfa.at(x + 1, y));
            lp = lp + 0.25f * (((cfa.at(x - 1, y - 1) + cfa.at(x + 1, y - 1)) + cfa.at(x - 1, y + 1)) +
                               cfa.at(x + 1, y + 1));
        }
        LP.d[i_] = lp;
    RCD_END
    __syncthreads();
    RCD_REGION(L::PQH)
        float pp = 0.f, qq = 0.f;
        if (in_img && fc(g, y, x) != 1 && inr(g, y, x, 3)) {
            pp = hpf2(cfa.at(x - 3, y - 3), cfa.at(x - 2, y - 2), cfa.at(x - 1, y - 1), cfa.at(x, y),
                      cfa.at(x + 1, y + 1), cfa.at(x + 2, y + 2), cfa.at(x + 3, y + 3));
            qq = hpf2(cfa.at(x + 3, y - 3), cfa.at(x + 2, y - 2), cfa.at(x + 1, y - 1), cfa.at(x, y),
                      cfa.at(x - 1, y + 1), cfa.at(x - 2, y + 2), cfa.at(x - 3, y + 3));
        }
        P.d[i_] = pp;
        Q.d[i_] = qq;
    RCD_END
    __syncthreads();
    // k_green
    RCD_REGION(L::GH)
        float gv = 0.f;
        if (in_img) {
            const float c0 = cfa.at(x, y);
            if (fc(g, y, x) == 1) {
                gv = c0;
            } else if (inr(g, y, x, 4)) {
                const float n1 = cfa.at(x, y - 1), s1 = cfa.at(x, y + 1), w1 = cfa.at(x - 1, y), e1 = cfa.at(x + 1, y);
                const float n2 = cfa.at(x, y - 2), s2 = cfa.at(x, y + 2), w2 = cfa.at(x - 2, y), e2 = cfa.at(x + 2, y);
                const float N_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - n2))) +
                                     (fabsf(n1 - cfa.at(x, y - 3)) + fabsf(n2 - cfa.at(x, y - 4)));
                const float S_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - s2))) +
                                     (fabsf(s1 - cfa.at(x, y + 3)) + fabsf(s2 - cfa.at(x, y + 4)));
                const float W_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - w2))) +
                                     (fabsf(w1 - cfa.at(x - 3, y)) + fabsf(w2 - cfa.at(x - 4, y)));
                const float E_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - e2))) +
                                     (fabsf(e1 - cfa.at(x + 3, y)) + fabsf(e2 - cfa.at(x + 4, y)));
                const float lpi = LP.at(x, y);
                const float l2 = lpi + lpi;
                const float N_Est = n1 * l2 / ((EPS + lpi) + LP.at(x, y - 2));
                const float S_Est = s1 * l2 / ((EPS + lpi) + LP.at(x, y + 2));
                const float W_Est = w1 * l2 / ((EPS + lpi) + LP.at(x - 2, y));
                const float E_Est = e1 * l2 / ((EPS + lpi) + LP.at(x + 2, y));
                const float V_Est = (S_Grad * N_Est + N_Grad * S_Est) / (N_Grad + S_Grad);
                const float H_Est = (W_Grad * E_Est + E_Grad * W_Est) / (E_Grad + W_Grad);
                const float nb = 0.25f * ((VH.at(x - 1, y - 1) + VH.at(x + 1, y - 1)) +
                                          (VH.at(x - 1, y + 1) + VH.at(x + 1, y + 1)));
                const float d = disc(VH.at(x, y), nb);
                gv = d * (H_Est - V_Est) + V_Est;
            }
        }
        G.d[i_] = gv;
    RCD_END
    // k_pq writes the PQ ratio into the low-pass buffer only at non-green
    // interior sites: elsewhere that buffer still holds LP
    RCD_REGION(L::PQD)
        float v = 0.f;
        if (in_img) {
            if (fc(g, y, x) != 1 && inr(g, y, x, 4)) {
                const float ps = fmaxf(EPSSQ, (P.at(x - 1, y - 1) + P.at(x, y)) + P.at(x + 1, y + 1));
                const float qs = fmaxf(EPSSQ, (Q.at(x + 1, y - 1) + Q.at(x, y)) + Q.at(x - 1, y + 1));
                v = ps / (ps + qs);
            } else {
                v = LP.at(x, y);
            }
        }
        PQ.d[i_] = v;
    RCD_END
    __syncthreads();
    // k_rb_sites (P / Q dead: R / B take their buffers)
    RCD_REGION(L::RBH)
        float r = 0.f, b = 0.f;
        if (in_img) {
            const int col = fc(g, y, x);
            const float c0 = cfa.at(x, y);
            r = col == 0 ? c0 : 0.f;
            b = col == 2 ? c0 : 0.f;
            if (col != 1 && inr(g, y, x, 4)) {
                const float nb = 0.25f * (((PQ.at(x - 1, y - 1) + PQ.at(x + 1, y - 1)) + PQ.at(x - 1, y + 1)) +
                                          PQ.at(x + 1, y + 1));
                const float d = disc(PQ.at(x, y), nb);
                const float NW = cfa.at(x - 1, y - 1), NE = cfa.at(x + 1, y - 1), SW = cfa.at(x - 1, y + 1),
                            SE = cfa.at(x + 1, y + 1);
                const float g0 = G.at(x, y);
                const float NW_Grad = ((EPS + fabsf(NW - SE)) + fabsf(NW - cfa.at(x - 3, y - 3))) + fabsf(g0 - G.at(x - 2, y - 2));
                const float NE_Grad = ((EPS + fabsf(NE - SW)) + fabsf(NE - cfa.at(x + 3, y - 3))) + fabsf(g0 - G.at(x + 2, y - 2));
                const float SW_Grad = ((EPS + fabsf(NE - SW)) + fabsf(SW - cfa.at(x - 3, y + 3))) + fabsf(g0 - G.at(x - 2, y + 2));
                const float SE_Grad = ((EPS + fabsf(NW - SE)) + fabsf(SE - cfa.at(x + 3, y + 3))) + fabsf(g0 - G.at(x + 2, y + 2));
                const float NW_Est = NW - G.at(x - 1, y - 1);
                const float NE_Est = NE - G.at(x + 1, y - 1);
                const float SW_Est = SW - G.at(x - 1, y + 1);
                const float SE_Est = SE - G.at(x + 1, y + 1);
                const float P_Est = (NW_Grad * SE_Est + SE_Grad * NW_Est) / (NW_Grad + SE_Grad);
                const float Q_Est = (NE_Grad * SW_Est + SW_Grad * NE_Est) / (NE_Grad + SW_Grad);
                const float v = g0 + (d * (Q_Est - P_Est) + P_Est);
                if (col == 2) r = v;     // interpolating colour 2 - col
                else b = v;
            }
        }
        R.d[i_] = r;
        B.d[i_] = b;
    RCD_END
    __syncthreads();
    // k_final
    const float invfactor = (float)(1.0 / (double)factor);
    const long long n = (long long)g.W * g.H;
    RCD_REGION(0)
        if (!in_img) continue;
        float o[3];
        if (!inr(g, y, x, BORDER)) {
            border(g, buf, mn, factor, y, x, o);
        } else {
            float r = R.at(x, y), b = B.at(x, y);
            const float g0 = G.at(x, y);
            if (fc(g, y, x) == 1) {
                const float nb = 0.25f * ((VH.at(x - 1, y - 1) + VH.at(x + 1, y - 1)) +
                                          (VH.at(x - 1, y + 1) + VH.at(x + 1, y + 1)));
                const float d = disc(VH.at(x, y), nb);
                const float N1 = EPS + fabsf(g0 - G.at(x, y - 2));
                const float S1 = EPS + fabsf(g0 - G.at(x, y + 2));
                const float W1 = EPS + fabsf(g0 - G.at(x - 2, y));
                const float E1 = EPS + fabsf(g0 - G.at(x + 2, y));
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const Pl &pl = k == 0 ? R : B;
                    const float SNabs = fabsf(pl.at(x, y - 1) - pl.at(x, y + 1));
                    const float EWabs = fabsf(pl.at(x - 1, y) - pl.at(x + 1, y));
                    const float N_Grad = (N1 + SNabs) + fabsf(pl.at(x, y - 1) - pl.at(x, y - 3));
                    const float S_Grad = (S1 + SNabs) + fabsf(pl.at(x, y + 1) - pl.at(x, y + 3));
                    const float W_Grad = (W1 + EWabs) + fabsf(pl.at(x - 1, y) - pl.at(x - 3, y));
                    const float E_Grad = (E1 + EWabs) + fabsf(pl.at(x + 1, y) - pl.at(x + 3, y));
                    const float N_Est = pl.at(x, y - 1) - G.at(x, y - 1);
                    const float S_Est = pl.at(x, y + 1) - G.at(x, y + 1);
                    const float W_Est = pl.at(x - 1, y) - G.at(x - 1, y);
                    const float E_Est = pl.at(x + 1, y) - G.at(x + 1, y);
                    const float V_Est = (N_Grad * S_Est + S_Grad * N_Est) / (N_Grad + S_Grad);
                    const float H_Est = (E_Grad * W_Est + W_Grad * E_Est) / (E_Grad + W_Grad);
                    const float v = g0 + (d * (H_Est - V_Est) + V_Est);
                    if (k == 0) r = v;
                    else b = v;
                }
            }
            o[0] = fmaxf(0.f, r * SCALE);
            o[1] = fmaxf(0.f, g0 * SCALE);
            o[2] = fmaxf(0.f, b * SCALE);
        }
        const long long p = (long long)y * W + x;
#pragma unroll
        for (int k = 0; k < 3; k++) st(rgb, k * n + p, o[k] * invfactor + mn, byte);
    RCD_END
}

template <int TX, int TY, class T, class O>
int launch_rcd_fused(Img g, const T *buf, O *rgb, int byte, int threads, hipStream_t s) {
    const size_t lds = rcd_lds_bytes<TX, TY>();
    static bool configured = false;
    if (!configured) {
        if (hipFuncSetAttribute((const void *)k_rcd_fused<TX, TY, T, O>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds) != hipSuccess)
            return -1;
        configured = true;
    }
    const dim3 grid((g.W + TX - 1) / TX, (g.H + TY - 1) / TY);
    hipLaunchKernelGGL((k_rcd_fused<TX, TY, T, O>), grid, dim3(threads), lds, s, g, buf, rgb, byte);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------- two-kernel RCD
// The fused kernel's halo (cfa +10) and LDS plan (98 KB at 64 x 32: one
// workgroup per CU) cost more than the HBM round trips it saves.  Cut at the
// narrowest point instead: k_rcd_a computes steps 1-4.1 over the tile and
// writes G, VH and the PQ / LP plane (12 B/px); k_rcd_b reads them back with
// the halos steps 4.2-4.3 need and writes the output.  HBM per pixel: 4 (raw,
// each kernel) + 12 + 12 + 12 (output) = 44 B against the multi-pass
// pipeline's ~8 planes written and re-read.  Same expressions in the same
// order as k_prep .. k_final: bitwise the multi-pass result.
template <int TX, int TY>
struct RcdA {
    static constexpr int CFA = 6, VHH = 2, VHD = 1, LPH = 2, PQH = 1;
    static constexpr int w(int h) { return TX + 2 * h; }
    static constexpr int h(int hh) { return TY + 2 * hh; }
    static constexpr int n(int hh) { return w(hh) * h(hh); }
    // [cfa][V -> P][H -> Q][VH][LP]
    static constexpr int o_cfa = 0, o_a = n(CFA), o_b = o_a + n(VHH), o_vh = o_b + n(VHH), o_lp = o_vh + n(VHD);
    static constexpr int total = o_lp + n(LPH);
};
template <int TX, int TY>
struct RcdB {
    static constexpr int CFA = 6, GH = 5, PQD = 4, RBH = 3, VHD = 1;
    static constexpr int w(int h) { return TX + 2 * h; }
    static constexpr int h(int hh) { return TY + 2 * hh; }
    static constexpr int n(int hh) { return w(hh) * h(hh); }
    static constexpr int o_cfa = 0, o_g = n(CFA), o_pq = o_g + n(GH), o_vh = o_pq + n(PQD), o_r = o_vh + n(VHD),
                         o_b = o_r + n(RBH);
    static constexpr int total = o_b + n(RBH);
};

template <int TX, int TY, class T>
__global__ __launch_bounds__(256) void k_rcd_a(Img g, const T *buf, float *Gout, float *VHout, float *PQout) {
    using L = RcdA<TX, TY>;
    extern __shared__ float lds[];
    const int X0 = blockIdx.x * TX, Y0 = blockIdx.y * TY;
    const int W = g.W;
    const Pl cfa{lds + L::o_cfa, X0 - L::CFA, Y0 - L::CFA, L::w(L::CFA)};
    const Pl V{lds + L::o_a, X0 - L::VHH, Y0 - L::VHH, L::w(L::VHH)};
    const Pl Hh{lds + L::o_b, X0 - L::VHH, Y0 - L::VHH, L::w(L::VHH)};
    const Pl VH{lds + L::o_vh, X0 - L::VHD, Y0 - L::VHD, L::w(L::VHD)};
    const Pl LP{lds + L::o_lp, X0 - L::LPH, Y0 - L::LPH, L::w(L::LPH)};
    const Pl P{lds + L::o_a, X0 - L::PQH, Y0 - L::PQH, L::w(L::PQH)};
    const Pl Q{lds + L::o_b, X0 - L::PQH, Y0 - L::PQH, L::w(L::PQH)};
    float mn, factor;
    norm_consts(g, mn, factor);
    RCD_REGION(L::CFA)                                   // k_prep
        float v = 0.f;
        if (in_img) {
            const float raw = (ld(buf, (long long)y * W + x) - mn) * factor;
            const float t = raw / SCALE;
            v = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
        }
        cfa.d[i_] = v;
    RCD_END
    __syncthreads();
    RCD_REGION(L::VHH)                                   // k_hv
        float v = 0.f, h = 0.f;
        if (in_img) {
            if (y >= 3 && y < g.H - 3 && x >= 4 && x < g.W - 4)
                v = hpf2(cfa.at(x, y - 3), cfa.at(x, y - 2), cfa.at(x, y - 1), cfa.at(x, y), cfa.at(x, y + 1),
                         cfa.at(x, y + 2), cfa.at(x, y + 3));
            if (y >= 4 && y < g.H - 4 && x >= 3 && x < g.W - 3)
                h = hpf2(cfa.at(x - 3, y), cfa.at(x - 2, y), cfa.at(x - 1, y), cfa.at(x, y), cfa.at(x + 1, y),
                         cfa.at(x + 2, y), cfa.at(x + 3, y));
        }
        V.d[i_] = v;
        Hh.d[i_] = h;
    RCD_END
    __syncthreads();
    RCD_REGION(L::VHD)                                   // k_dir: VH_Dir
        float vh = 0.f;
        if (in_img && inr(g, y, x, 4)) {
            const float vs = fmaxf(EPSSQ, (V.at(x, y - 1) + V.at(x, y)) + V.at(x, y + 1));
            const float hs = fmaxf(EPSSQ, (Hh.at(x - 1, y) + Hh.at(x, y)) + Hh.at(x + 1, y));
            vh = vs / (vs + hs);
        }
        VH.d[i_] = vh;
    RCD_END
    RCD_REGION(L::LPH)                                   // low pass
        float lp = 0.f;
        if (in_img && fc(g, y, x) != 1 && inr(g, y, x, 2)) {
            lp = cfa.at(x, y) + 0.5f * (((cfa.at(x, y - 1) + cfa.at(x, y + 1)) + cfa.at(x - 1, y)) + cfa.at(x + 1, y));
            lp = lp + 0.25f * (((cfa.at(x - 1, y - 1) + cfa.at(x + 1, y - 1)) + cfa.at(x - 1, y + 1)) +
                               cfa.at(x + 1, y + 1));
        }
        LP.d[i_] = lp;
    RCD_END
    __syncthreads();
    RCD_REGION(L::PQH)                                   // diagonal high-pass (V / H dead)
        float pp = 0.f, qq = 0.f;
        if (in_img && fc(g, y, x) != 1 && inr(g, y, x, 3)) {
            pp = hpf2(cfa.at(x - 3, y - 3), cfa.at(x - 2, y - 2), cfa.at(x - 1, y - 1), cfa.at(x, y),
                      cfa.at(x + 1, y + 1), cfa.at(x + 2, y + 2), cfa.at(x + 3, y + 3));
            qq = hpf2(cfa.at(x + 3, y - 3), cfa.at(x + 2, y - 2), cfa.at(x + 1, y - 1), cfa.at(x, y),
                      cfa.at(x - 1, y + 1), cfa.at(x - 2, y + 2), cfa.at(x - 3, y + 3));
        }
        P.d[i_] = pp;
        Q.d[i_] = qq;
    RCD_END
    __syncthreads();
    RCD_REGION(0)                                        // k_green and k_pq over the tile
        if (!in_img) continue;
        float gv = 0.f;
        const float c0 = cfa.at(x, y);
        const bool green = fc(g, y, x) == 1;
        if (green) {
            gv = c0;
        } else if (inr(g, y, x, 4)) {
            const float n1 = cfa.at(x, y - 1), s1 = cfa.at(x, y + 1), w1 = cfa.at(x - 1, y), e1 = cfa.at(x + 1, y);
            const float n2 = cfa.at(x, y - 2), s2 = cfa.at(x, y + 2), w2 = cfa.at(x - 2, y), e2 = cfa.at(x + 2, y);
            const float N_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - n2))) +
                                 (fabsf(n1 - cfa.at(x, y - 3)) + fabsf(n2 - cfa.at(x, y - 4)));
            const float S_Grad = (EPS + (fabsf(n1 - s1) + fabsf(c0 - s2))) +
                                 (fabsf(s1 - cfa.at(x, y + 3)) + fabsf(s2 - cfa.at(x, y + 4)));
            const float W_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - w2))) +
                                 (fabsf(w1 - cfa.at(x - 3, y)) + fabsf(w2 - cfa.at(x - 4, y)));
            const float E_Grad = (EPS + (fabsf(w1 - e1) + fabsf(c0 - e2))) +
                                 (fabsf(e1 - cfa.at(x + 3, y)) + fabsf(e2 - cfa.at(x + 4, y)));
            const float lpi = LP.at(x, y);
            const float l2 = lpi + lpi;
            const float N_Est = n1 * l2 / ((EPS + lpi) + LP.at(x, y - 2));
            const float S_Est = s1 * l2 / ((EPS + lpi) + LP.at(x, y + 2));
            const float W_Est = w1 * l2 / ((EPS + lpi) + LP.at(x - 2, y));
            const float E_Est = e1 * l2 / ((EPS + lpi) + LP.at(x + 2, y));
            const float V_Est = (S_Grad * N_Est + N_Grad * S_Est) / (N_Grad + S_Grad);
            const float H_Est = (W_Grad * E_Est + E_Grad * W_Est) / (E_Grad + W_Grad);
            const float nb = 0.25f * ((VH.at(x - 1, y - 1) + VH.at(x + 1, y - 1)) +
                                      (VH.at(x - 1, y + 1) + VH.at(x + 1, y + 1)));
            const float d = disc(VH.at(x, y), nb);
            gv = d * (H_Est - V_Est) + V_Est;
        }
        float pq;
        if (!green && inr(g, y, x, 4)) {
            const float ps = fmaxf(EPSSQ, (P.at(x - 1, y - 1) + P.at(x, y)) + P.at(x + 1, y + 1));
            const float qs = fmaxf(EPSSQ, (Q.at(x + 1, y - 1) + Q.at(x, y)) + Q.at(x - 1, y + 1));
            pq = ps / (ps + qs);
        } else {
            pq = LP.at(x, y);
        }
        const long long p = (long long)y * W + x;
        Gout[p] = gv;
        VHout[p] = VH.at(x, y);
        PQout[p] = pq;
    RCD_END
}

template <int TX, int TY, class T, class O>
__global__ __launch_bounds__(256) void k_rcd_b(Img g, const T *buf, const float *Gin, const float *VHin,
                                               const float *PQin, O *rgb, int byte) {
    using L = RcdB<TX, TY>;
    extern __shared__ float lds[];
    const int X0 = blockIdx.x * TX, Y0 = blockIdx.y * TY;
    const int W = g.W;
    const Pl cfa{lds + L::o_cfa, X0 - L::CFA, Y0 - L::CFA, L::w(L::CFA)};
    const Pl G{lds + L::o_g, X0 - L::GH, Y0 - L::GH, L::w(L::GH)};
    const Pl PQ{lds + L::o_pq, X0 - L::PQD, Y0 - L::PQD, L::w(L::PQD)};
    const Pl VH{lds + L::o_vh, X0 - L::VHD, Y0 - L::VHD, L::w(L::VHD)};
    const Pl R{lds + L::o_r, X0 - L::RBH, Y0 - L::RBH, L::w(L::RBH)};
    const Pl B{lds + L::o_b, X0 - L::RBH, Y0 - L::RBH, L::w(L::RBH)};
    float mn, factor;
    norm_consts(g, mn, factor);
    RCD_REGION(L::CFA)
        float v = 0.f;
        if (in_img) {
            const float raw = (ld(buf, (long long)y * W + x) - mn) * factor;
            const float t = raw / SCALE;
            v = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
        }
        cfa.d[i_] = v;
    RCD_END
    RCD_REGION(L::GH)
        G.d[i_] = in_img ? Gin[(long long)y * W + x] : 0.f;
    RCD_END
    RCD_REGION(L::PQD)
        PQ.d[i_] = in_img ? PQin[(long long)y * W + x] : 0.f;
    RCD_END
    RCD_REGION(L::VHD)
        VH.d[i_] = in_img ? VHin[(long long)y * W + x] : 0.f;
    RCD_END
    __syncthreads();
    RCD_REGION(L::RBH)                                   // k_rb_sites
        float r = 0.f, b = 0.f;
        if (in_img) {
            const int col = fc(g, y, x);
            const float c0 = cfa.at(x, y);
            r = col == 0 ? c0 : 0.f;
            b = col == 2 ? c0 : 0.f;
            if (col != 1 && inr(g, y, x, 4)) {
                const float nb = 0.25f * (((PQ.at(x - 1, y - 1) + PQ.at(x + 1, y - 1)) + PQ.at(x - 1, y + 1)) +
                                          PQ.at(x + 1, y + 1));
                const float d = disc(PQ.at(x, y), nb);
                const float NW = cfa.at(x - 1, y - 1), NE = cfa.at(x + 1, y - 1), SW = cfa.at(x - 1, y + 1),
                            SE = cfa.at(x + 1, y + 1);
                const float g0 = G.at(x, y);
                const float NW_Grad = ((EPS + fabsf(NW - SE)) + fabsf(NW - cfa.at(x - 3, y - 3))) + fabsf(g0 - G.at(x - 2, y - 2));
                const float NE_Grad = ((EPS + fabsf(NE - SW)) + fabsf(NE - cfa.at(x + 3, y - 3))) + fabsf(g0 - G.at(x + 2, y - 2));
                const float SW_Grad = ((EPS + fabsf(NE - SW)) + fabsf(SW - cfa.at(x - 3, y + 3))) + fabsf(g0 - G.at(x - 2, y + 2));
                const float SE_Grad = ((EPS + fabsf(NW - SE)) + fabsf(SE - cfa.at(x + 3, y + 3))) + fabsf(g0 - G.at(x + 2, y + 2));
                const float NW_Est = NW - G.at(x - 1, y - 1);
                const float NE_Est = NE - G.at(x + 1, y - 1);
                const float SW_Est = SW - G.at(x - 1, y + 1);
                const float SE_Est = SE - G.at(x + 1, y + 1);
                const float P_Est = (NW_Grad * SE_Est + SE_Grad * NW_Est) / (NW_Grad + SE_Grad);
                const float Q_Est = (NE_Grad * SW_Est + SW_Grad * NE_Est) / (NE_Grad + SW_Grad);
                const float v = g0 + (d * (Q_Est - P_Est) + P_Est);
                if (col == 2) r = v;
                else b = v;
            }
        }
        R.d[i_] = r;
        B.d[i_] = b;
    RCD_END
    __syncthreads();
    const float invfactor = (float)(1.0 / (double)factor);
    const long long n = (long long)g.W * g.H;
    RCD_REGION(0)                                        // k_final
        if (!in_img) continue;
        float o[3];
        if (!inr(g, y, x, BORDER)) {
            border(g, buf, mn, factor, y, x, o);
        } else {
            float r = R.at(x, y), b = B.at(x, y);
            const float g0 = G.at(x, y);
            if (fc(g, y, x) == 1) {
                const float nb = 0.25f * ((VH.at(x - 1, y - 1) + VH.at(x + 1, y - 1)) +
                                          (VH.at(x - 1, y + 1) + VH.at(x + 1, y + 1)));
                const float d = disc(VH.at(x, y), nb);
                const float N1 = EPS + fabsf(g0 - G.at(x, y - 2));
                const float S1 = EPS + fabsf(g0 - G.at(x, y + 2));
                const float W1 = EPS + fabsf(g0 - G.at(x - 2, y));
                const float E1 = EPS + fabsf(g0 - G.at(x + 2, y));
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const Pl &pl = k == 0 ? R : B;
                    const float SNabs = fabsf(pl.at(x, y - 1) - pl.at(x, y + 1));
                    const float EWabs = fabsf(pl.at(x - 1, y) - pl.at(x + 1, y));
                    const float N_Grad = (N1 + SNabs) + fabsf(pl.at(x, y - 1) - pl.at(x, y - 3));
                    const float S_Grad = (S1 + SNabs) + fabsf(pl.at(x, y + 1) - pl.at(x, y + 3));
                    const float W_Grad = (W1 + EWabs) + fabsf(pl.at(x - 1, y) - pl.at(x - 3, y));
                    const float E_Grad = (E1 + EWabs) + fabsf(pl.at(x + 1, y) - pl.at(x + 3, y));
                    const float N_Est = pl.at(x, y - 1) - G.at(x, y - 1);
                    const float S_Est = pl.at(x, y + 1) - G.at(x, y + 1);
                    const float W_Est = pl.at(x - 1, y) - G.at(x - 1, y);
                    const float E_Est = pl.at(x + 1, y) - G.at(x + 1, y);
                    const float V_Est = (N_Grad * S_Est + S_Grad * N_Est) / (N_Grad + S_Grad);
                    const float H_Est = (E_Grad * W_Est + W_Grad * E_Est) / (E_Grad + W_Grad);
                    const float v = g0 + (d * (H_Est - V_Est) + V_Est);
                    if (k == 0) r = v;
                    else b = v;
                }
            }
            o[0] = fmaxf(0.f, r * SCALE);
            o[1] = fmaxf(0.f, g0 * SCALE);
            o[2] = fmaxf(0.f, b * SCALE);
        }
        const long long p = (long long)y * W + x;
#pragma unroll
        for (int k = 0; k < 3; k++) st(rgb, k * n + p, o[k] * invfactor + mn, byte);
    RCD_END
}

template <int TX, int TY, class T, class O>
int launch_rcd_split(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s) {
    const long long n = (long long)g.W * g.H;
    float *G = ws, *VH = ws + n, *PQ = ws + 2 * n;
    const size_t la = sizeof(float) * RcdA<TX, TY>::total, lb = sizeof(float) * RcdB<TX, TY>::total;
    static bool configured = false;
    if (!configured) {
        if (hipFuncSetAttribute((const void *)k_rcd_a<TX, TY, T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)la) != hipSuccess ||
            hipFuncSetAttribute((const void *)k_rcd_b<TX, TY, T, O>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lb) != hipSuccess)
            return -1;
        configured = true;
    }
    const dim3 grid((g.W + TX - 1) / TX, (g.H + TY - 1) / TY);
    hipLaunchKernelGGL((k_rcd_a<TX, TY, T>), grid, dim3(256), la, s, g, buf, G, VH, PQ);
    hipLaunchKernelGGL((k_rcd_b<TX, TY, T, O>), grid, dim3(256), lb, s, g, buf, G, VH, PQ, rgb, byte);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// tile variants (A/B knob SGPU_RCD_FUSED: 1 = 64x32 / 512 threads, 2 = 32x32 / 256)
template <class T, class O>
int launch_rcd(Img g, const T *buf, O *rgb, int byte, int variant, hipStream_t s) {
    if (variant == 1) return launch_rcd_fused<32, 32>(g, buf, rgb, byte, 256, s);
    return launch_rcd_fused<64, 32>(g, buf, rgb, byte, 512, s);
}

// the multi-pass pipeline (workspace: 8 planes of W x H floats)
template <class T, class O>
int launch_rcd_multipass(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s) {
    const long long n = (long long)g.W * g.H;
    float *cfa = ws, *V = ws + n, *Hh = ws + 2 * n, *VH = ws + 3 * n, *LP = ws + 4 * n, *P = ws + 5 * n,
          *Q = ws + 6 * n, *G = ws + 7 * n;
    const dim3 grid((g.W + 63) / 64, (g.H + 3) / 4), blk(256);
    hipLaunchKernelGGL(k_prep<T>, grid, blk, 0, s, g, buf, cfa);
    // SGPU_RCD_DIRPQ=0: the three-kernel form of steps 1.1-2 and 4.1 (A/B)
    static const bool dirpq = !std::getenv("SGPU_RCD_DIRPQ") || std::atoi(std::getenv("SGPU_RCD_DIRPQ")) != 0;
    if (dirpq) {
        // V / Hh hold the red / blue site planes, P the PQ ratio
        hipLaunchKernelGGL(k_dir_pq, grid, blk, 0, s, g, cfa, VH, LP, P);
        hipLaunchKernelGGL(k_green, grid, blk, 0, s, g, cfa, VH, LP, G);
        hipLaunchKernelGGL(k_rb_sites, grid, blk, 0, s, g, cfa, G, P, V, Hh);
        hipLaunchKernelGGL((k_final<T, O>), grid, blk, 0, s, g, buf, G, VH, V, Hh, rgb, byte);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL(k_hv, grid, blk, 0, s, g, cfa, V, Hh);
    hipLaunchKernelGGL(k_dir, grid, blk, 0, s, g, cfa, V, Hh, VH, LP, P, Q);
    hipLaunchKernelGGL(k_green, grid, blk, 0, s, g, cfa, VH, LP, G);
    hipLaunchKernelGGL(k_pq, grid, blk, 0, s, g, P, Q, LP);
    // V / Hh are dead after k_dir: they hold the red / blue site planes
    hipLaunchKernelGGL(k_rb_sites, grid, blk, 0, s, g, cfa, G, LP, V, Hh);
    hipLaunchKernelGGL((k_final<T, O>), grid, blk, 0, s, g, buf, G, VH, V, Hh, rgb, byte);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template int launch_rcd_split<64, 32, float, float>(Img, const float *, float *, int, float *, hipStream_t);
template int launch_rcd_split<64, 32, uint16_t, uint16_t>(Img, const uint16_t *, uint16_t *, int, float *, hipStream_t);
template int launch_rcd<float, float>(Img, const float *, float *, int, int, hipStream_t);
template int launch_rcd<uint16_t, uint16_t>(Img, const uint16_t *, uint16_t *, int, int, hipStream_t);
template int launch_rcd_multipass<float, float>(Img, const float *, float *, int, float *, hipStream_t);
template int launch_rcd_multipass<uint16_t, uint16_t>(Img, const uint16_t *, uint16_t *, int, float *, hipStream_t);

// super_pixel_float (demosaicing_siril.c:128-176): one thread per 2x2 cell,
// interleaved RGB output of (W/2 + W%2) x (H/2 + H%2); odd tail cells are 0
__global__ __launch_bounds__(256) void k_superpixel(const float *buf, int W, int H, int pattern, float *out) {
    const int cx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int cy = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int nw = W / 2 + W % 2, nh = H / 2 + H % 2;
    if (cx >= nw || cy >= nh) return;
    float *o = out + 3 * ((long long)cy * nw + cx);
    const int col = 2 * cx, row = 2 * cy;
    if (row >= H - 1 || col >= W - 1) {
        o[0] = o[1] = o[2] = 0.f;
        return;
    }
    const long long i = (long long)row * W + col;
    const float a = buf[i], b = buf[i + 1], c = buf[i + W], d = buf[i + W + 1];
    switch (pattern) {
        default:
        case 0: o[0] = a; o[1] = (b + c) * 0.5f; o[2] = d; break;          // RGGB
        case 1: o[2] = a; o[1] = (b + c) * 0.5f; o[0] = d; break;          // BGGR
        case 2: o[2] = b; o[0] = c; o[1] = (a + d) * 0.5f; break;          // GBRG
        case 3: o[0] = b; o[2] = c; o[1] = (a + d) * 0.5f; break;          // GRBG
    }
}

// Siril's own bilinear Bayer decoder, bayer_Bilinear (algos/demosaicing_siril.c
// :203-288, "OpenCV's Bayer decoding", the BAYER_BILINEAR of
// debayer_buffer_siril :737-790), as a per-pixel closed form of its paired
// row walk: output row y (1..H-2) starts with a green pixel when
// start_with_green ^ ((y - 1) & 1), its non-green pixels are blue when
// blue * (-1)^(y - 1) > 0 (tile: BGGR / GBRG start with blue = -1, GBRG /
// GRBG with green); a non-green pixel keeps its own colour, takes green from
// the cross (4 + 2) >> 2 and the other colour from the diagonals; a green
// pixel takes the vertical pair (+1 >> 1) for the colour of the rows above
// and below and the horizontal pair for its own row's colour.  The 1-pixel
// frame stays 0 (ClearBorders).  Output planar (the RGBRGB -> RRGGBB loop of
// debayer_ushort, demosaicing_siril.c:846-855), truncate_to_BYTE for 8-bit.
__global__ __launch_bounds__(256) void k_bilinear_siril(const uint16_t *bay, int W, int H, int tile, int byte,
                                                         uint16_t *rgb) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const long long n = (long long)W * H, i = (long long)y * W + x;
    unsigned r = 0, g = 0, b = 0;
    if (x >= 1 && x <= W - 2 && y >= 1 && y <= H - 2) {
        const int blue0 = (tile == 1 || tile == 2) ? -1 : 1;
        const int swg0 = (tile == 2 || tile == 3) ? 1 : 0;
        const int odd = (y - 1) & 1;
        const bool blue_row = (odd ? -blue0 : blue0) > 0;
        const bool green = ((x - 1) & 1) == ((swg0 ^ odd) ? 0 : 1);
        auto at = [&](int xx, int yy) { return (unsigned)bay[(long long)yy * W + xx]; };
        const unsigned c = at(x, y);
        if (green) {
            const unsigned vert = (at(x, y - 1) + at(x, y + 1) + 1) >> 1;
            const unsigned horz = (at(x - 1, y) + at(x + 1, y) + 1) >> 1;
            g = c;
            if (blue_row) { r = vert; b = horz; }
            else { r = horz; b = vert; }
        } else {
            const unsigned diag = (at(x - 1, y - 1) + at(x + 1, y - 1) + at(x - 1, y + 1) + at(x + 1, y + 1) + 2) >> 2;
            const unsigned cross = (at(x, y - 1) + at(x - 1, y) + at(x + 1, y) + at(x, y + 1) + 2) >> 2;
            g = cross;
            if (blue_row) { b = c; r = diag; }
            else { r = c; b = diag; }
        }
        if (byte) {
            r = r > 255u ? 255u : r;
            g = g > 255u ? 255u : g;
            b = b > 255u ? 255u : b;
        }
    }
    rgb[i] = (uint16_t)r;
    rgb[n + i] = (uint16_t)g;
    rgb[2 * n + i] = (uint16_t)b;
}

}  // namespace dm
}  // namespace sgpu
