// sgpu_dft.cpp -- C-ABI of the DFT cross-correlation registration
// (register_shift_dft, registration/shift_methods.c:60-321): plans, twiddle
// tables, workspace and the batched pipeline of dft_register.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fft_lds.h"
#include "sgpu_internal.h"

using sgpu::fft::Plan;
using sgpu_host::fail;

namespace sgpu {
namespace dft {
__global__ void k_nongreen(float *img, long long stride, int w, int h, sgpu::fft::Cfa cfa);
__global__ void k_rows_fwd(Plan pl, float2 *data, long long plane);
__global__ void k_rows_xpow_bwd(Plan pl, const float2 *fref, float2 *data, long long plane);
__global__ void k_cols_fwd_xpow_bwd(Plan pl, const float2 *fref, float2 *data, long long plane, int remap);
template <class T>
__global__ void k_rows_real2_fwd(Plan pl, const T *src, long long row_stride, long long frame_stride,
                                 float2 *dst, sgpu::fft::Cfa cfa);
extern template __global__ void k_rows_real2_fwd<float>(Plan, const float *, long long, long long, float2 *,
                                                        sgpu::fft::Cfa);
extern template __global__ void k_rows_real2_fwd<uint16_t>(Plan, const uint16_t *, long long, long long, float2 *,
                                                           sgpu::fft::Cfa);
__global__ void k_nongreen16(uint16_t *img, long long stride, int w, int h, sgpu::fft::Cfa cfa);
template <class T>
__global__ void k_nongreen_pass(const T *orig, long long so, const T *prev, T *out, int w, int h, sgpu::fft::Cfa cfa);
extern template __global__ void k_nongreen_pass<float>(const float *, long long, const float *, float *, int, int,
                                                       sgpu::fft::Cfa);
extern template __global__ void k_nongreen_pass<uint16_t>(const uint16_t *, long long, const uint16_t *, uint16_t *,
                                                          int, int, sgpu::fft::Cfa);
__global__ void k_rows_c2r2_argmax(Plan pl, const float2 *data, unsigned long long *best);
__global__ void k_rows_c2r2_argmax_t(Plan pl, const float2 *data, unsigned long long *best);
template <class T>
__global__ void k_rows_real2_fwd_t(Plan pl, const T *src, long long row_stride, long long frame_stride, float2 *dst,
                                   sgpu::fft::Cfa cfa);
extern template __global__ void k_rows_real2_fwd_t<float>(Plan, const float *, long long, long long, float2 *,
                                                          sgpu::fft::Cfa);
extern template __global__ void k_rows_real2_fwd_t<uint16_t>(Plan, const uint16_t *, long long, long long, float2 *,
                                                             sgpu::fft::Cfa);
__global__ void k_transpose_rect(const float2 *in, float2 *out, int rows, int cols);
__global__ void k_finalize(const unsigned long long *best, int nframes, int n, int *shifts, float *peak);
}  // namespace dft
}  // namespace sgpu

namespace {

// radix-10 passes (fft_lds.h bfly10); SGPU_DFT_R10=0 keeps the 8 / 5 / 4 plans (A/B)
bool r10_enabled() {
    static const bool on = !(std::getenv("SGPU_DFT_R10") && std::atoi(std::getenv("SGPU_DFT_R10")) == 0);
    return on;
}

// radices in pass order: 8s, 10s, 5s, then 4, 3, 2, then any other prime
bool factorize(int n, Plan &pl) {
    pl.n = n;
    pl.nf = 0;
    auto push = [&](int r) {
        if (pl.nf >= sgpu::fft::kMaxFactors) return false;
        pl.radix[pl.nf++] = r;
        return true;
    };
    // SGPU_DFT_PLAN="10,10,8,5": an explicit pass order (A/B of the plan
    // shape; used when its radices multiply to n and all have butterflies)
    if (const char *e = std::getenv("SGPU_DFT_PLAN")) {
        int prod = 1;
        for (const char *q = e; *q;) {
            const int r = std::atoi(q);
            if (r != 2 && r != 3 && r != 4 && r != 5 && r != 8 && r != 10) { prod = 0; break; }
            if (!push(r)) return false;
            prod *= r;
            while (*q && *q != ',') q++;
            if (*q == ',') q++;
        }
        if (prod == n) return true;
        pl.nf = 0;
    }
    int m = n;
    while (m % 8 == 0) { if (!push(8)) return false; m /= 8; }
    if (r10_enabled())
        while (m % 10 == 0) { if (!push(10)) return false; m /= 10; }
    while (m % 5 == 0) { if (!push(5)) return false; m /= 5; }
    while (m % 4 == 0) { if (!push(4)) return false; m /= 4; }
    while (m % 3 == 0) { if (!push(3)) return false; m /= 3; }
    while (m % 2 == 0) { if (!push(2)) return false; m /= 2; }
    for (int p = 7; m > 1 && p <= m; p += 2)
        while (m % p == 0) {
            if (p > 61) return false;          // large primes: not supported by the LDS kernel
            if (!push(p)) return false;
            m /= p;
        }
    if (m != 1) return false;
    // an odd radix first: the first pass writes its outputs R words apart
    // (Ns = 1), and an even R (8, 10) puts lanes 4-16 ways onto the same LDS
    // banks; 5 x 10 x 10 x 8 runs the 4000-point rows 5.7 % faster than
    // 8 x 10 x 10 x 5; every odd-first order measured alike (profiles/r05al_*,
    // r05am_*)
    for (int p = 0; p < pl.nf; p++)
        if (pl.radix[p] & 1) {
            const int r = pl.radix[p];
            for (int q = p; q > 0; q--) pl.radix[q] = pl.radix[q - 1];
            pl.radix[0] = r;
            break;
        }
    return true;
}

int ensure_plan(sgpu_context *c, int n, Plan &pl) {
    if (n < 2 || n > sgpu::fft::kMaxLen) return fail(SGPU_BAD_ARGUMENT, "DFT size must be in [2, 8192]");
    if (!factorize(n, pl)) return fail(SGPU_BAD_ARGUMENT, "DFT size has a prime factor > 61");
    int r;
    if ((r = c->dft_tw.ensure((size_t)n * sizeof(float2)))) return r;
    if (c->dft_n != n) {
        std::vector<float2> tw(n);
        for (int k = 0; k < n; k++) {
            const double a = 2.0 * M_PI * (double)k / (double)n;
            tw[k] = make_float2((float)std::cos(a), (float)-std::sin(a));
        }
        HIP_TRY(hipMemcpy(c->dft_tw.p, tw.data(), n * sizeof(float2), hipMemcpyHostToDevice));
        c->dft_n = n;
        const int lds = 2 * n * (int)sizeof(float2);
        for (const void *f : {(const void *)sgpu::dft::k_rows_fwd, (const void *)sgpu::dft::k_rows_xpow_bwd,
                              (const void *)sgpu::dft::k_rows_real2_fwd<float>,
                              (const void *)sgpu::dft::k_rows_real2_fwd_t<float>,
                              (const void *)sgpu::dft::k_rows_real2_fwd_t<uint16_t>,
                              (const void *)sgpu::dft::k_rows_c2r2_argmax_t,
                              (const void *)sgpu::dft::k_rows_real2_fwd<uint16_t>,
                              (const void *)sgpu::dft::k_rows_c2r2_argmax,
                              (const void *)sgpu::dft::k_cols_fwd_xpow_bwd})
            HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    }
    pl.tw = (const float2 *)c->dft_tw.p;
    return SGPU_OK;
}

// The half spectra go to the column pass in the column-major layout: written
// there directly by the row kernel (default; 16-byte stores per row pair and
// column, XCD-grouped row pairs) or through the rectangular transpose kernel
// (SGPU_DFT_TRANSPOSE=1, A/B)
inline bool dft_transpose_kernel() {
    static const bool t = std::getenv("SGPU_DFT_TRANSPOSE") && std::atoi(std::getenv("SGPU_DFT_TRANSPOSE")) != 0;
    return t;
}

// forward 2-D half spectrum (kx in [0, n/2]), stored transposed as nh rows
// of n: real row pairs -> (transposed store) -> column FFTs (cols = 0: the
// column transforms are left to the caller's fused column pass)
template <class T>
int spectrum_half_T(sgpu_context *c, const Plan &pl, const T *src, long long row_stride,
                    long long frame_stride, int batch, float2 *t1, float2 *out, const sgpu::fft::Cfa &cfa,
                    int cols = 1) {
    const int n = pl.n, nh = n / 2 + 1;
    const size_t lds = sgpu::fft::plan_lds_bytes(pl);
    hipStream_t s = c->stream;
    if (dft_transpose_kernel()) {
        hipLaunchKernelGGL(sgpu::dft::k_rows_real2_fwd<T>, dim3((n + 1) / 2, batch), dim3(sgpu::fft::kThreads), lds,
                           s, pl, src, row_stride, frame_stride, t1, cfa);
        hipLaunchKernelGGL(sgpu::dft::k_transpose_rect, dim3((nh + 31) / 32, (n + 31) / 32, batch), dim3(256), 0, s,
                           t1, out, n, nh);
    } else {
        hipLaunchKernelGGL(sgpu::dft::k_rows_real2_fwd_t<T>, dim3((n + 1) / 2, batch), dim3(sgpu::fft::kThreads),
                           lds, s, pl, src, row_stride, frame_stride, out, cfa);
    }
    if (cols)
        hipLaunchKernelGGL(sgpu::dft::k_rows_fwd, dim3(nh, batch), dim3(sgpu::fft::kThreads), lds, s, pl, out,
                           (long long)nh * n);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "DFT spectrum launch failed");
}

// X-Trans (dim 6): the reference tests a neighbour with FC_array(nx, ny)
// (column first).  Where that transposed test calls a non-green pixel green,
// the in-place raster loop (image_format_fits.c:4319-4381) reads a value it
// may already have rewritten: a raster-order dependency.  xtrans_depth: the
// longest chain of such reads on the 6x6 torus (0: the pattern never reads a
// rewritten pixel, as XTRANS_1 from an origin with x = y mod 3; -1: a cycle,
// chains as long as the image); the engine then runs depth + 1 Jacobi passes
// (k_nongreen_pass) before the transform, which reproduce the sequential
// loop exactly.
int xtrans_depth(const unsigned char *c) {
    // edges: non-green site -> earlier non-green neighbour the transposed test calls green
    int depth[36], state[36];
    for (int i = 0; i < 36; i++) depth[i] = 0, state[i] = 0;
    // iterative DFS over 36 nodes (recursion is fine at this size)
    struct Dfs {
        const unsigned char *c;
        int *depth, *state;
        int go(int u) {
            if (state[u] == 1) return -1;
            if (state[u] == 2) return depth[u];
            state[u] = 1;
            int d = 0;
            const int r = u / 6, q = u % 6;
            if (c[u] != 1)
                for (int dy = -1; dy <= 0; dy++)
                    for (int dx = -1; dx <= 1; dx++) {
                        if (dy == 0 && dx >= 0) continue;             // raster-earlier neighbours only
                        const int ny = (r + dy + 6) % 6, nx = (q + dx + 6) % 6;
                        if (c[nx * 6 + ny] == 1 && c[ny * 6 + nx] != 1) {
                            const int e = go(ny * 6 + nx);
                            if (e < 0) return -1;
                            d = d > e + 1 ? d : e + 1;
                        }
                    }
            state[u] = 2;
            depth[u] = d;
            return d;
        }
    } dfs{c, depth, state};
    int m = 0;
    for (int u = 0; u < 36; u++) {
        const int d = dfs.go(u);
        if (d < 0) return -1;
        m = d > m ? d : m;
    }
    return m;
}

// passes: 0 = the per-pixel stencil (fused into the transform), k > 0 = k
// Jacobi passes of k_nongreen_pass first
int make_cfa(const unsigned char *pattern, int dim, sgpu::fft::Cfa &cfa, int *passes = nullptr) {
    std::memset(&cfa, 0, sizeof cfa);
    if (passes) *passes = 0;
    if (!pattern || dim == 0) return SGPU_OK;
    if (dim != 2 && dim != 6) return fail(SGPU_BAD_ARGUMENT, "CFA patterns are 2x2 (Bayer) or 6x6 (X-Trans)");
    cfa.dim = dim;
    std::memcpy(cfa.c, pattern, (size_t)dim * dim);
    if (dim == 6) {
        // any transposed-green non-green neighbour, earlier or later, makes the
        // in-place per-pixel kernel racy: those patterns take the passes
        bool reads_non_green = false;
        for (int u = 0; u < 36; u++) {
            if (pattern[u] == 1) continue;
            const int r = u / 6, q = u % 6;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    if (!dx && !dy) continue;
                    const int ny = (r + dy + 6) % 6, nx = (q + dx + 6) % 6;
                    if (pattern[nx * 6 + ny] == 1 && pattern[ny * 6 + nx] != 1) reads_non_green = true;
                }
        }
        if (reads_non_green) {
            const int d = xtrans_depth(pattern);
            if (d < 0) return fail(SGPU_BAD_ARGUMENT, "X-Trans pattern with unbounded in-place dependency chains");
            if (!passes) return fail(SGPU_BAD_ARGUMENT, "X-Trans pattern needs the multi-pass interpolation");
            *passes = d + 1;
        }
    }
    return SGPU_OK;
}

// interpolate_nongreen of nb frames (src[f * fstride + y * stride + x], w x h)
// into dst (contiguous w x h frames) by `passes` Jacobi passes; tmp holds
// one w x h frame of T
template <class T>
int nongreen_passes(hipStream_t s, const T *src, long long stride, long long fstride, int nb, int w, int h,
                    const sgpu::fft::Cfa &cfa, int passes, T *dst, T *tmp) {
    const dim3 grid((w + 63) / 64, (h + 3) / 4), blk(256);
    for (int f = 0; f < nb; f++) {
        const T *o = src + (long long)f * fstride;
        T *out = dst + (long long)f * w * h;
        // ping-pong so that the last pass lands in `out`
        T *a = (passes % 2) ? out : tmp, *b = (passes % 2) ? tmp : out;
        const T *prev = nullptr;
        for (int k = 0; k < passes; k++) {
            T *cur = (k % 2 == 0) ? a : b;
            hipLaunchKernelGGL(sgpu::dft::k_nongreen_pass<T>, grid, blk, 0, s, o, stride, prev, cur, w, h, cfa);
            prev = cur;
        }
    }
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "nongreen pass launch failed");
}

// the standalone in-place interpolation by passes: result staged, copied back
template <class T>
int nongreen_in_place(sgpu_context *c, T *img, int w, int h, long stride, const sgpu::fft::Cfa &cfa, int passes) {
    const long long px = (long long)w * h;
    if (int r = c->cfa_tmp.ensure((size_t)2 * px * sizeof(T))) return r;
    T *dst = (T *)c->cfa_tmp.p;
    if (int r = nongreen_passes<T>(c->stream, img, stride, 0, 1, w, h, cfa, passes, dst, dst + px)) return r;
    HIP_TRY(hipMemcpy2DAsync(img, (size_t)stride * sizeof(T), dst, (size_t)w * sizeof(T), (size_t)w * sizeof(T), h,
                             hipMemcpyDeviceToDevice, c->stream));
    return SGPU_OK;
}

}  // namespace

namespace {
// the batched pipeline for float or WORD selections
template <class T>
int dft_register(sgpu_context *c, const T *d_ref, long ref_row_stride, const T *d_frames, long row_stride,
                 long frame_stride, int nframes, int size, const unsigned char *cfa_pattern, int cfa_dim,
                 int *d_shifts, float *d_peaks) {
    if (!c || !d_ref || !d_frames || !d_shifts) return fail(SGPU_BAD_ARGUMENT, "null argument");
    sgpu::fft::Cfa cfa;
    int passes = 0;
    if (int e = make_cfa(cfa_pattern, cfa_dim, cfa, &passes)) return e;
    if (nframes < 1) return fail(SGPU_BAD_ARGUMENT, "nframes < 1");
    if (ref_row_stride < size || row_stride < size) return fail(SGPU_BAD_ARGUMENT, "row stride < size");
    HIP_TRY(hipSetDevice(c->device));
    Plan pl;
    int r = ensure_plan(c, size, pl);
    if (r) return r;
    const int n = size, nh = n / 2 + 1;
    const size_t plane = (size_t)nh * n * sizeof(float2);   // half spectrum
    // frames per batch: two complex planes each, within ~4 GiB
    int batch = (int)std::max<size_t>(1, (4ull << 30) / (2 * plane));
    batch = std::min(batch, nframes);
    if ((r = c->dft_ref.ensure(plane)) || (r = c->dft_t1.ensure(plane * batch)) ||
        (r = c->dft_t2.ensure(plane * batch)) || (r = c->dft_best.ensure(nframes * sizeof(unsigned long long))))
        return r;
    hipStream_t s = c->stream;
    float2 *fref = (float2 *)c->dft_ref.p, *t1 = (float2 *)c->dft_t1.p, *t2 = (float2 *)c->dft_t2.p;
    unsigned long long *best = (unsigned long long *)c->dft_best.p;
    // timing group [pipeline start, stop, -, -] (sgpu_last_timing ms[0])
    c->ev_used = 0;
    sgpu_host::mark(c);
    HIP_TRY(hipMemsetAsync(best, 0, nframes * sizeof(unsigned long long), s));
    // X-Trans with in-place dependencies: the selections are interpolated by
    // Jacobi passes into a staging buffer first, then transformed as plain
    // images ((passes: make_cfa)
    const T *ref_src = d_ref;
    long ref_stride = ref_row_stride;
    sgpu::fft::Cfa cfa_t = cfa;
    T *stage = nullptr;
    const long long sel = (long long)n * n;
    if (passes) {
        if ((r = c->cfa_tmp.ensure((size_t)(batch + 1) * sel * sizeof(T)))) return r;
        stage = (T *)c->cfa_tmp.p;
        T *tmp = stage + (long long)batch * sel;
        if ((r = nongreen_passes<T>(c->stream, d_ref, ref_row_stride, 0, 1, n, n, cfa, passes, stage, tmp))) return r;
        ref_src = stage;
        ref_stride = n;
        cfa_t.dim = 0;
    }
    // reference spectrum (shift_methods.c:165-178)
    if ((r = spectrum_half_T(c, pl, ref_src, ref_stride, 0, 1, t1, fref, cfa_t))) return r;
    const size_t lds = sgpu::fft::plan_lds_bytes(pl);
    const char *fz = std::getenv("SGPU_DFT_FUSED");          // "0": separate column passes (A/B knob)
    const bool fused = !(fz && fz[0] == '0');
    const char *rm = std::getenv("SGPU_DFT_REMAP");          // "1": frame-fastest XCD-contiguous order (A/B)
    const int remap = (rm && rm[0] == '1') ? 1 : 0;
    for (int f0 = 0; f0 < nframes; f0 += batch) {
        const int nb = std::min(batch, nframes - f0);
        if (passes) {
            // (the reference spectrum is done: the staging buffer is reused)
            if ((r = nongreen_passes<T>(s, d_frames + (long long)f0 * frame_stride, row_stride, frame_stride, nb, n, n,
                                        cfa, passes, stage, stage + (long long)batch * sel)))
                return r;
            r = spectrum_half_T(c, pl, (const T *)stage, n, sel, nb, t1, t2, cfa_t, fused ? 0 : 1);
        } else {
            r = spectrum_half_T(c, pl, d_frames + (long long)f0 * frame_stride, row_stride, frame_stride, nb, t1, t2,
                                cfa, fused ? 0 : 1);
        }
        if (r) return r;
        if (fused) {
            // forward columns, cross power, inverse columns in one LDS pass
            hipLaunchKernelGGL(sgpu::dft::k_cols_fwd_xpow_bwd, dim3(nh, nb), dim3(sgpu::fft::kThreads), lds, s, pl,
                               fref, t2, (long long)nh * n, remap);
        } else {
            // cross-power spectrum fused into the first inverse pass (columns)
            hipLaunchKernelGGL(sgpu::dft::k_rows_xpow_bwd, dim3(nh, nb), dim3(sgpu::fft::kThreads), lds, s, pl,
                               fref, t2, (long long)nh * n);
        }
        // inverse rows (two real rows per complex transform) + argmax
        if (dft_transpose_kernel()) {
            hipLaunchKernelGGL(sgpu::dft::k_transpose_rect, dim3((n + 31) / 32, (nh + 31) / 32, nb), dim3(256), 0, s,
                               t2, t1, nh, n);
            hipLaunchKernelGGL(sgpu::dft::k_rows_c2r2_argmax, dim3((n + 1) / 2, nb), dim3(sgpu::fft::kThreads), lds,
                               s, pl, t1, best + f0);
        } else {
            hipLaunchKernelGGL(sgpu::dft::k_rows_c2r2_argmax_t, dim3((n + 1) / 2, nb), dim3(sgpu::fft::kThreads), lds,
                               s, pl, t2, best + f0);
        }
        if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "DFT launch failed");
    }
    hipLaunchKernelGGL(sgpu::dft::k_finalize, dim3((nframes + 255) / 256), dim3(256), 0, s, best, nframes, n,
                       d_shifts, d_peaks);
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "DFT finalize failed");
}
}  // namespace

extern "C" int sgpu_dft_register_cfa_device(sgpu_context *c, const float *d_ref, long ref_row_stride,
                                            const float *d_frames, long row_stride, long frame_stride,
                                            int nframes, int size, const unsigned char *cfa_pattern,
                                            int cfa_dim, int *d_shifts, float *d_peaks) {
    return dft_register(c, d_ref, ref_row_stride, d_frames, row_stride, frame_stride, nframes, size, cfa_pattern,
                        cfa_dim, d_shifts, d_peaks);
}

extern "C" int sgpu_dft_register_u16_device(sgpu_context *c, const uint16_t *d_ref, long ref_row_stride,
                                            const uint16_t *d_frames, long row_stride, long frame_stride,
                                            int nframes, int size, const unsigned char *cfa_pattern,
                                            int cfa_dim, int *d_shifts, float *d_peaks) {
    return dft_register(c, d_ref, ref_row_stride, d_frames, row_stride, frame_stride, nframes, size, cfa_pattern,
                        cfa_dim, d_shifts, d_peaks);
}

extern "C" int sgpu_interpolate_nongreen_u16_device(sgpu_context *c, uint16_t *d_img, int width, int height,
                                                    long row_stride, const unsigned char *cfa_pattern,
                                                    int cfa_dim) {
    if (!c || !d_img || !cfa_pattern) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (width < 1 || height < 1 || row_stride < width) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    sgpu::fft::Cfa cfa;
    int passes = 0;
    if (int e = make_cfa(cfa_pattern, cfa_dim, cfa, &passes)) return e;
    HIP_TRY(hipSetDevice(c->device));
    if (passes) return nongreen_in_place(c, d_img, width, height, row_stride, cfa, passes);
    dim3 grid((width + 63) / 64, (height + 3) / 4);
    hipLaunchKernelGGL(sgpu::dft::k_nongreen16, grid, dim3(256), 0, c->stream, d_img, (long long)row_stride, width,
                       height, cfa);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "nongreen launch failed");
}

extern "C" int sgpu_dft_shifts_u16(sgpu_context *c, const uint16_t *ref, const uint16_t *const *frames, int nframes,
                                   int size, const unsigned char *cfa_pattern, int cfa_dim, int *shiftx,
                                   int *shifty) {
    if (!c || !ref || !frames || !shiftx || !shifty) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (nframes < 1) return fail(SGPU_BAD_ARGUMENT, "nframes < 1");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t fbytes = (size_t)size * size * sizeof(uint16_t);
    int r;
    if ((r = c->dft_frames.ensure(fbytes * (nframes + 1))) ||
        (r = c->dft_shifts.ensure(2 * nframes * sizeof(int))))
        return r;
    uint16_t *d = (uint16_t *)c->dft_frames.p;
    HIP_TRY(hipMemcpyAsync(d, ref, fbytes, hipMemcpyHostToDevice, s));
    for (int f = 0; f < nframes; f++)
        HIP_TRY(hipMemcpyAsync(d + (size_t)(f + 1) * size * size, frames[f], fbytes, hipMemcpyHostToDevice, s));
    r = sgpu_dft_register_u16_device(c, d, size, d + (size_t)size * size, size, (long)size * size, nframes, size,
                                     cfa_pattern, cfa_dim, (int *)c->dft_shifts.p, nullptr);
    if (r) return r;
    std::vector<int> h(2 * nframes);
    HIP_TRY(hipMemcpyAsync(h.data(), c->dft_shifts.p, 2 * nframes * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int f = 0; f < nframes; f++) {
        shiftx[f] = h[2 * f];
        shifty[f] = h[2 * f + 1];
    }
    return SGPU_OK;
}

extern "C" int sgpu_dft_register_device(sgpu_context *c, const float *d_ref, long ref_row_stride,
                                        const float *d_frames, long row_stride, long frame_stride,
                                        int nframes, int size, int *d_shifts, float *d_peaks) {
    return sgpu_dft_register_cfa_device(c, d_ref, ref_row_stride, d_frames, row_stride, frame_stride, nframes,
                                        size, nullptr, 0, d_shifts, d_peaks);
}

extern "C" int sgpu_interpolate_nongreen_device(sgpu_context *c, float *d_img, int width, int height,
                                                long row_stride, const unsigned char *cfa_pattern, int cfa_dim) {
    if (!c || !d_img || !cfa_pattern) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (width < 1 || height < 1 || row_stride < width) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    sgpu::fft::Cfa cfa;
    int passes = 0;
    if (int e = make_cfa(cfa_pattern, cfa_dim, cfa, &passes)) return e;
    HIP_TRY(hipSetDevice(c->device));
    if (passes) return nongreen_in_place(c, d_img, width, height, row_stride, cfa, passes);
    dim3 grid((width + 63) / 64, (height + 3) / 4);
    hipLaunchKernelGGL(sgpu::dft::k_nongreen, grid, dim3(256), 0, c->stream, d_img, (long long)row_stride, width,
                       height, cfa);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "nongreen launch failed");
}

extern "C" int sgpu_dft_shifts_cfa(sgpu_context *c, const float *ref, const float *const *frames, int nframes,
                                   int size, const unsigned char *cfa_pattern, int cfa_dim, int *shiftx,
                                   int *shifty);

extern "C" int sgpu_dft_shifts(sgpu_context *c, const float *ref, const float *const *frames, int nframes,
                               int size, int *shiftx, int *shifty) {
    return sgpu_dft_shifts_cfa(c, ref, frames, nframes, size, nullptr, 0, shiftx, shifty);
}

extern "C" int sgpu_dft_shifts_cfa(sgpu_context *c, const float *ref, const float *const *frames, int nframes,
                                   int size, const unsigned char *cfa_pattern, int cfa_dim, int *shiftx,
                                   int *shifty) {
    if (!c || !ref || !frames || !shiftx || !shifty) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (nframes < 1) return fail(SGPU_BAD_ARGUMENT, "nframes < 1");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t fbytes = (size_t)size * size * sizeof(float);
    int r;
    if ((r = c->dft_frames.ensure(fbytes * (nframes + 1))) ||
        (r = c->dft_shifts.ensure(2 * nframes * sizeof(int))))
        return r;
    float *d = (float *)c->dft_frames.p;
    HIP_TRY(hipMemcpyAsync(d, ref, fbytes, hipMemcpyHostToDevice, s));
    for (int f = 0; f < nframes; f++)
        HIP_TRY(hipMemcpyAsync(d + (size_t)(f + 1) * size * size, frames[f], fbytes, hipMemcpyHostToDevice, s));
    r = sgpu_dft_register_cfa_device(c, d, size, d + (size_t)size * size, size, (long)size * size, nframes, size,
                                     cfa_pattern, cfa_dim, (int *)c->dft_shifts.p, nullptr);
    if (r) return r;
    std::vector<int> h(2 * nframes);
    HIP_TRY(hipMemcpyAsync(h.data(), c->dft_shifts.p, 2 * nframes * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int f = 0; f < nframes; f++) {
        shiftx[f] = h[2 * f];
        shifty[f] = h[2 * f + 1];
    }
    return SGPU_OK;
}
