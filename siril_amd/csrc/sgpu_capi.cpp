// sgpu_capi.cpp -- C-ABI of libsirilgpu.so (include/sirilgpu.h): contexts,
// device workspace, parameter marshalling and kernel selection for the
// rejection / median stack.  Host code, built by hipcc for gfx950.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sirilgpu.h"
#include "sgpu_internal.h"
#include "sgpu_kparams.h"

namespace sgpu {
int launch_sorted_16(const KParams &, hipStream_t);
int launch_sorted_32(const KParams &, hipStream_t);
int launch_sorted_64(const KParams &, hipStream_t);
int launch_sorted_128(const KParams &, hipStream_t);
int launch_sorted_256(const KParams &, hipStream_t);
int launch_sorted_512(const KParams &, hipStream_t);
int launch_sorted_1024(const KParams &, hipStream_t);
int launch_sorted16_16(const KParams &, hipStream_t);
int launch_sorted16_32(const KParams &, hipStream_t);
int launch_sorted16_64(const KParams &, hipStream_t);
int launch_sorted16_128(const KParams &, hipStream_t);
int launch_sorted16_256(const KParams &, hipStream_t);
int launch_sorted16_512(const KParams &, hipStream_t);
int launch_sorted16_1024(const KParams &, hipStream_t);
int launch_stack_mean(const KParams &, hipStream_t);
__global__ void k_stack_exact(KParams p, int all_pixels);
__global__ void k_stack_exact16(KParams p, int all_pixels);
__global__ void k_stack_exact_lds(KParams p, int all_pixels);
__global__ void k_stack_exact_wave(KParams p, int all_pixels);
template <int NW>
__global__ void k_stack_exact_small(KParams p, int all_pixels);
template <int NW>
__global__ void k_stack_exact16_small(KParams p, int all_pixels);
__global__ void k_fold_counts(const unsigned long long *stripes, unsigned long long *counts);
__global__ void k_stack_exact16_lds(KParams p, int all_pixels);
}  // namespace sgpu

using sgpu::KParams;

namespace sgpu_host {
hipEvent_t next_event(sgpu_context *c) {
    if (c->ev_used == c->ev.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev.push_back(e);
    }
    return c->ev[c->ev_used++];
}
void mark(sgpu_context *c) {
    if (!c->timing) return;
    hipEvent_t e = next_event(c);
    if (e) (void)hipEventRecord(e, c->stream);
}

}  // namespace sgpu_host

namespace sgpu_host {
thread_local std::string g_err;
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace sgpu_host

using sgpu_host::DevBuf;
using sgpu_host::fail;
using sgpu_host::g_err;

namespace {
constexpr long long kMaxLaunchPixels = 1LL << 28;   // 32-bit byte offsets in the kernels
// Threads of the exact sequential kernel.  Every thread owns 6*N floats of
// scratch; measured on MI355X (r02): an all-exact launch is fastest at 64K
// threads (more only thrashes the L2/MALL with scratch: PERCENTILE N=100
// u16 179 -> 360 ms at 512K), while the deferred-pixel pass after the sorted
// path wants more threads to hide its irregular gathers (WINSORIZED N=12,
// 6.6M deferred pixels: 92.7 -> 23.1 ms at 128K).  Both are capped so the
// scratch stays within the 256 MB MALL.
constexpr int kExactThreadsMax = 1 << 16;
constexpr int kDeferThreads = 1 << 17;
constexpr size_t kScratchCap = 256ull << 20;

long long exact_threads(long long npix, int N, bool all_exact) {
    long long threads = std::min<long long>(npix, all_exact ? kExactThreadsMax : kDeferThreads);
    threads = ((threads + 63) / 64) * 64;
    const size_t per_thread = 6ull * (size_t)N * sizeof(float);
    // halve until the scratch fits, staying a multiple of the 64-thread block
    // (the launch is threads / 64 blocks and scratch_threads = threads)
    while (threads > 64 && (size_t)threads * per_thread > kScratchCap)
        threads = std::max(64LL, (threads / 2) / 64 * 64);
    return threads;
}
// The sequential kernels with their scratch in LDS (k_stack_exact_lds):
// threads per block (a power of two <= 64) whose 6 * N words fit 64 KB, 0
// when fewer than 4 would (N > 682: global scratch).  SGPU_EXACT_LDS=0 forces
// the global-scratch kernels (A/B).
int exact_lds_block(int N) {
    static const int env = [] {
        const char *e = std::getenv("SGPU_EXACT_LDS");
        return e ? std::atoi(e) : 1;
    }();
    if (!env) return 0;
    const size_t per = 24ull * (size_t)N;
    int t = 64;
    while (t > 4 && (size_t)t * per > 65536) t >>= 1;
    return (size_t)t * per <= 65536 ? t : 0;
}

// rejection types the small-column kernels run (k_stack_exact_small)
inline bool small_type(int rt) {
    return rt == SGPU_SIGMA || rt == SGPU_WINSORIZED || rt == SGPU_PERCENTILE || rt == SGPU_SIGMEDIAN;
}
// the largest N whose every pixel goes to the small-column kernel instead of
// the sorted one: SGPU_SMALL_ALL (A/B), default 0 = never.  Before the rejection
// totals were striped (kCountStripes) every sorted launch had a ~9 ms
// same-address-atomics floor and the small-column kernel won at N <= 16 / 32
// (profiles/r04i_ab_small_all.txt); without that floor the sorted kernel wins
// everywhere measured: sigma12 0.85 vs 2.65 ms, winsorized12 5.14 vs 9.80 ms,
// sigma24 1.63 vs 6.25 ms (profiles/r04n_ab_small_all.txt).  The small-column
// kernel keeps the sorted path's deferred pixels.
inline int small_all_limit(int) {
    static const int env = std::getenv("SGPU_SMALL_ALL") ? std::atoi(std::getenv("SGPU_SMALL_ALL")) : 0;
    return env;
}

// Launch the sequential kernel over the deferred list (or every pixel).
int launch_exact(sgpu_context *c, KParams k, bool all, bool u16) {
    hipStream_t s = c->stream;
    const int N = k.nframes;
    // deferred float SIGMA / WINSORIZED / PERCENTILE / median columns of
    // 33..1024 samples: one wave per pixel (stack_exact_wave.hip) -- the
    // pixels are few and each one's sequential loops are the tail's latency.
    // exact_only == 2 sends every pixel there (tests).  SGPU_EXACT_WAVE=0: A/B
    static const bool wave_on = !std::getenv("SGPU_EXACT_WAVE") || std::atoi(std::getenv("SGPU_EXACT_WAVE")) != 0;
    const bool wave_type = k.rtype == SGPU_SIGMA || k.rtype == SGPU_WINSORIZED || k.rtype == SGPU_PERCENTILE ||
                           k.rtype == sgpu::KMEDIAN;
    if (!u16 && wave_type && N >= 33 && N <= 1024 && ((wave_on && !all) || c->exact_only == 2)) {
        const size_t lds = (size_t)5 * ((N + 1) & ~1) * sizeof(float);
        const long long blocks = all ? std::min<long long>(k.npix, 8192) : std::min<long long>(k.npix, 2048);
        hipLaunchKernelGGL(sgpu::k_stack_exact_wave, dim3((unsigned)std::max<long long>(blocks, 1)), dim3(64), lds, s,
                           k, all ? 1 : 0);
        if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "exact (wave) kernel launch failed");
        return SGPU_OK;
    }
    // small SIGMA / WINSORIZED columns: the stack alone in LDS, w_stack in
    // registers (k_stack_exact_small); SGPU_EXACT_SMALL=0 for A/B
    static const bool small_on = !std::getenv("SGPU_EXACT_SMALL") || std::atoi(std::getenv("SGPU_EXACT_SMALL")) != 0;
    if (small_on && N <= 32 && small_type(k.rtype)) {
        const size_t lds = (size_t)64 * N * sizeof(float);
        const long long blocks = std::max<long long>(1, std::min<long long>((k.npix + 63) / 64, 256LL * 32));
        const dim3 g((unsigned)blocks), b(64);
        if (u16 && N <= 16) hipLaunchKernelGGL(sgpu::k_stack_exact16_small<16>, g, b, lds, s, k, all ? 1 : 0);
        else if (u16) hipLaunchKernelGGL(sgpu::k_stack_exact16_small<32>, g, b, lds, s, k, all ? 1 : 0);
        else if (N <= 16) hipLaunchKernelGGL(sgpu::k_stack_exact_small<16>, g, b, lds, s, k, all ? 1 : 0);
        else hipLaunchKernelGGL(sgpu::k_stack_exact_small<32>, g, b, lds, s, k, all ? 1 : 0);
        if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "exact (small) kernel launch failed");
        return SGPU_OK;
    }
    const int t = exact_lds_block(N);
    if (t) {
        // LDS-resident: as many blocks as the 160 KB of LDS per CU holds on
        // all 256 CUs (the deferred list is on the device: surplus blocks
        // find no pixel and exit)
        const size_t lds = (size_t)t * 24ull * N;
        const long long per_cu = std::max<long long>(1, (long long)((160ull << 10) / lds));
        const long long blocks = std::max<long long>(1, std::min<long long>((k.npix + t - 1) / t, 256 * per_cu));
        if (u16)
            hipLaunchKernelGGL(sgpu::k_stack_exact16_lds, dim3((unsigned)blocks), dim3(t), lds, s, k, all ? 1 : 0);
        else
            hipLaunchKernelGGL(sgpu::k_stack_exact_lds, dim3((unsigned)blocks), dim3(t), lds, s, k, all ? 1 : 0);
        if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "exact (LDS) kernel launch failed");
        return SGPU_OK;
    }
    const long long threads = exact_threads(k.npix, N, all);
    const size_t per_thread = 6ull * (size_t)N * sizeof(float);
    int r;
    if ((r = c->scratch.ensure(threads * per_thread))) return r;
    k.scratch = (float *)c->scratch.p;
    k.scratch_threads = threads;
    if (u16)
        hipLaunchKernelGGL(sgpu::k_stack_exact16, dim3((unsigned)(threads / 64)), dim3(64), 0, s, k, all ? 1 : 0);
    else
        hipLaunchKernelGGL(sgpu::k_stack_exact, dim3((unsigned)(threads / 64)), dim3(64), 0, s, k, all ? 1 : 0);
    if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "exact kernel launch failed");
    return SGPU_OK;
}
}  // namespace

extern "C" {

int sgpu_abi_version(void) { return SGPU_ABI_VERSION; }

int sgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *sgpu_last_error(void) { return g_err.c_str(); }

int sgpu_init(int device, sgpu_context **out) {
    if (!out) return fail(SGPU_BAD_ARGUMENT, "null context pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(SGPU_NO_DEVICE, "no HIP device available");
    if (device < 0 || device >= n) return fail(SGPU_BAD_ARGUMENT, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    auto *c = new sgpu_context();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(SGPU_NO_DEVICE, "hipStreamCreate failed");
    }
    c->stream = c->own;
    *out = c;
    return SGPU_OK;
}

void sgpu_release(sgpu_context *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->release_all();
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int sgpu_set_stream(sgpu_context *c, void *s) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    // NULL is the device's null (default) stream, as hipStream_t 0 is for
    // every HIP API: a caller working on the default stream (torch's current
    // stream is often 0) must be ordered with it, not with the context's own
    // non-blocking stream
    c->stream = (hipStream_t)s;
    return SGPU_OK;
}

int sgpu_synchronize(sgpu_context *c) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SGPU_OK;
}

int sgpu_set_exact_only(sgpu_context *c, int on) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    c->exact_only = on == 2 ? 2 : (on ? 1 : 0);
    return SGPU_OK;
}

int sgpu_set_input_bitpix(sgpu_context *c, int bitpix) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    if (bitpix != 0 && bitpix != 8 && bitpix != 16 && bitpix != -32)
        return fail(SGPU_BAD_ARGUMENT, "bitpix: 0, 8, 16 or -32");
    c->in_bitpix = bitpix;
    return SGPU_OK;
}

int sgpu_set_timing(sgpu_context *c, int on) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    c->timing = on ? 1 : 0;
    return SGPU_OK;
}

int sgpu_last_timing(sgpu_context *c, float ms[2]) {
    if (!c || !ms) return fail(SGPU_BAD_ARGUMENT, "null argument");
    ms[0] = ms[1] = 0.f;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (size_t i = 0; i + 3 < c->ev_used; i += 4) {   // [start main, stop main, start exact, stop exact]
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, c->ev[i], c->ev[i + 1]));
        HIP_TRY(hipEventElapsedTime(&b, c->ev[i + 2], c->ev[i + 3]));
        ms[0] += a;
        ms[1] += b;
    }
    return SGPU_OK;
}

long sgpu_last_exact_pixels(sgpu_context *c) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    if (hipStreamSynchronize(c->stream) != hipSuccess) return SGPU_NO_DEVICE;
    if (c->last_all_exact) return (long)c->last_npix;
    int n = 0;
    if (!c->fb_count.p) return 0;
    if (hipMemcpy(&n, c->fb_count.p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return SGPU_NO_DEVICE;
    if (c->wz_cnt.p) {   // the moment path's per-chunk exact pixels (stack_sorted_inst.h)
        int t = 0;
        if (hipMemcpy(&t, (int *)c->wz_cnt.p + 2 * sgpu::kWzMaxChunks, sizeof(int), hipMemcpyDeviceToHost) !=
            hipSuccess)
            return SGPU_NO_DEVICE;
        n += t;
    }
    return n;
}

long sgpu_last_order_sensitive(sgpu_context *c, int *idx, long cap) {
    if (!c) return fail(SGPU_BAD_ARGUMENT, "null context");
    if (hipStreamSynchronize(c->stream) != hipSuccess) return SGPU_NO_DEVICE;
    if (!c->last_mean || !c->fb2_count.p) return 0;
    int n = 0;
    if (hipMemcpy(&n, c->fb2_count.p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return SGPU_NO_DEVICE;
    if (idx && cap > 0 && n > 0 &&
        hipMemcpy(idx, c->fb2_list.p, (size_t)std::min<long>(cap, n) * sizeof(int), hipMemcpyDeviceToHost) !=
            hipSuccess)
        return SGPU_NO_DEVICE;
    return n;
}

}  // extern "C"

namespace {

// LINEARFIT constants, median_and_mean.c:1487-1500 (float arithmetic, no FMA)
void linear_fit_constants(int n, float *m_x, float *m_dx2) {
    float mx = (n - 1) * 0.5f, md = 0.f;
    for (int j = 0; j < n; ++j) {
        const float dx = j - mx;
        const float xf = 1.f / (j + 1);
        md += (dx * dx - md) * xf;
    }
    *m_x = mx;
    *m_dx2 = 1.f / md;
}

int sorted_capacity(int n) {
    for (int np : {16, 32, 64, 128, 256, 512, 1024})
        if (n <= np) return np;
    return 0;
}

int launch_sorted(int np, const KParams &p, hipStream_t s) {
    switch (np) {
        case 16: return sgpu::launch_sorted_16(p, s);
        case 32: return sgpu::launch_sorted_32(p, s);
        case 64: return sgpu::launch_sorted_64(p, s);
        case 128: return sgpu::launch_sorted_128(p, s);
        case 256: return sgpu::launch_sorted_256(p, s);
        case 512: return sgpu::launch_sorted_512(p, s);
        case 1024: return sgpu::launch_sorted_1024(p, s);
        default: return 1;
    }
}

int launch_sorted16(int np, const KParams &p, hipStream_t s) {
    switch (np) {
        case 16: return sgpu::launch_sorted16_16(p, s);
        case 32: return sgpu::launch_sorted16_32(p, s);
        case 64: return sgpu::launch_sorted16_64(p, s);
        case 128: return sgpu::launch_sorted16_128(p, s);
        case 256: return sgpu::launch_sorted16_256(p, s);
        case 512: return sgpu::launch_sorted16_512(p, s);
        case 1024: return sgpu::launch_sorted16_1024(p, s);
        default: return 1;
    }
}

// Upload the per-frame tables and fill the parameter block (everything but
// frames/out/rej/npix).
int prepare(sgpu_context *c, int N, long W, const sgpu_stack_params *P, KParams &k, bool &xf) {
    if (N < 1) return fail(SGPU_BAD_ARGUMENT, "nframes < 1");
    if (P->method != SGPU_METHOD_MEAN && P->method != SGPU_METHOD_MEDIAN)
        return fail(SGPU_BAD_ARGUMENT, "unknown method");
    if (P->method == SGPU_METHOD_MEAN &&
        (P->type_of_rejection < SGPU_NO_REJEC || P->type_of_rejection > SGPU_GESDT))
        return fail(SGPU_BAD_ARGUMENT, "unknown rejection type");
    std::memset(&k, 0, sizeof k);
    k.nframes = N;
    k.W = (int)W;
    k.rtype = (P->method == SGPU_METHOD_MEDIAN) ? sgpu::KMEDIAN : P->type_of_rejection;
    k.sig0 = P->sig[0];
    k.sig1 = P->sig[1];
    k.norm = P->normalize;
    k.output_norm = P->output_norm;
    // normalize_to16bit (median_and_mean.c:547-555, applied at :1729-1732 when
    // output_norm): 8-bit sources scaled to the 16-bit range before rounding
    k.out16_mul = (c->in_bitpix == 8 && P->output_norm) ? 65535.0 / 255.0 : 1.0;
    hipStream_t s = c->stream;

    // normalization tables, one formula on the device (stack_sorted_impl.h)
    const bool add = (P->normalize == SGPU_ADDITIVE || P->normalize == SGPU_ADDITIVE_SCALING);
    const bool mulm = (P->normalize == SGPU_MULTIPLICATIVE || P->normalize == SGPU_MULTIPLICATIVE_SCALING);
    xf = add || mulm || P->shiftx != nullptr;
    // the copies below outlive the async uploads (previous call's transfers
    // are ordered before them on the same stream)
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<double> &sc = c->h_scale, &of = c->h_offset, &mu = c->h_mul;
    sc.assign(N, 1.0);
    of.assign(N, 0.0);
    mu.assign(N, 1.0);
    if (add || mulm) {
        for (int f = 0; f < N; f++) {
            if (P->scale) sc[f] = P->scale[f];
            if (add && P->offset) of[f] = P->offset[f];
            if (mulm && P->mul) mu[f] = P->mul[f];
        }
    }
    std::vector<int> &sh = c->h_shift;
    sh.assign(N, 0);
    if (P->shiftx) std::memcpy(sh.data(), P->shiftx, N * sizeof(int));
    int r;
    if ((r = c->scale.ensure(N * sizeof(double))) || (r = c->offset.ensure(N * sizeof(double))) ||
        (r = c->mul.ensure(N * sizeof(double))) || (r = c->shiftx.ensure(N * sizeof(int))))
        return r;
    HIP_TRY(hipMemcpyAsync(c->scale.p, sc.data(), N * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->offset.p, of.data(), N * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->mul.p, mu.data(), N * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->shiftx.p, sh.data(), N * sizeof(int), hipMemcpyHostToDevice, s));
    k.scale = (const double *)c->scale.p;
    k.offset = (const double *)c->offset.p;
    k.mul = (const double *)c->mul.p;
    k.shiftx = xf ? (const int *)c->shiftx.p : nullptr;

    if (P->weights && P->method == SGPU_METHOD_MEAN) {
        if ((r = c->weights.ensure(N * sizeof(double)))) return r;
        c->h_weights.assign(P->weights, P->weights + N);
        HIP_TRY(hipMemcpyAsync(c->weights.p, c->h_weights.data(), N * sizeof(double), hipMemcpyHostToDevice, s));
        k.weights = (const double *)c->weights.p;
    }
    if (k.rtype == SGPU_GESDT) {
        const int max_out = (int)std::floor((float)N * P->sig[0]);
        if (max_out > 0 && !P->critical_value)
            return fail(SGPU_BAD_ARGUMENT, "GESDT needs critical_value[floor(nframes*sig[0])]");
        const int nc = std::max(max_out, 1);
        std::vector<float> &cv = c->h_crit;
        cv.assign(nc, 0.f);
        if (max_out > 0) std::memcpy(cv.data(), P->critical_value, max_out * sizeof(float));
        if ((r = c->crit.ensure(nc * sizeof(float)))) return r;
        HIP_TRY(hipMemcpyAsync(c->crit.p, cv.data(), nc * sizeof(float), hipMemcpyHostToDevice, s));
        k.crit = (const float *)c->crit.p;
    }
    if (k.rtype == SGPU_LINEARFIT) linear_fit_constants(N, &k.m_x, &k.m_dx2);
    return SGPU_OK;
}

void mark(sgpu_context *c) { sgpu_host::mark(c); }

// Queue one launch over npix pixels (npix <= kMaxLaunchPixels).
int run_launch_body(sgpu_context *c, KParams k, bool has_shift);

// one launch with striped rejection totals (sgpu_kparams.h kCountStripes):
// zeroed before, folded into k.counts after every kernel of the launch
int run_launch(sgpu_context *c, KParams k, bool has_shift) {
    hipStream_t s = c->stream;
    static const bool striped = !std::getenv("SGPU_COUNT_STRIPES") || std::atoi(std::getenv("SGPU_COUNT_STRIPES")) != 0;
    const size_t sb = (size_t)sgpu::kCountStripes * 8 * sizeof(unsigned long long);
    k.cstripe = nullptr;
    if (striped && k.counts && c->cstripe.ensure(sb) == SGPU_OK) {
        k.cstripe = (unsigned long long *)c->cstripe.p;
        HIP_TRY(hipMemsetAsync(k.cstripe, 0, sb, s));
    }
    if (int r = run_launch_body(c, k, has_shift)) return r;
    if (k.cstripe) {
        hipLaunchKernelGGL(sgpu::k_fold_counts, dim3(1), dim3(256), 0, s, (const unsigned long long *)k.cstripe,
                           k.counts);
        if (hipGetLastError() != hipSuccess) return fail(SGPU_NO_DEVICE, "count fold launch failed");
    }
    return SGPU_OK;
}

int run_launch_body(sgpu_context *c, KParams k, bool has_shift) {
    hipStream_t s = c->stream;
    const int N = k.nframes;
    int r;
    if ((r = c->fb_list.ensure(k.npix * sizeof(int))) || (r = c->fb_count.ensure(sizeof(int))))
        return r;
    k.fb_list = (int *)c->fb_list.p;
    k.fb_count = (int *)c->fb_count.p;
    HIP_TRY(hipMemsetAsync(k.fb_count, 0, sizeof(int), s));
    if (c->wz_cnt.p) HIP_TRY(hipMemsetAsync((int *)c->wz_cnt.p + 2 * sgpu::kWzMaxChunks, 0, sizeof(int), s));
    // the WINSORIZED moment path's fallback list and record workspace
    // (stack_wz.h); SGPU_WZ=0 / 1 / 2 (default) / 3 / 4: off / one kernel /
    // two kernels (prep and rounds overlapped on two streams at N <= 128) /
    // always overlapped / never; SGPU_WZ_RW: the rounds kernel's form (A/B)
    static const int wz_mode = std::getenv("SGPU_WZ") ? std::atoi(std::getenv("SGPU_WZ")) : 2;
    static const int wz_rw = std::getenv("SGPU_WZ_RW") ? std::atoi(std::getenv("SGPU_WZ_RW")) : 64;
    k.wz_mode = wz_mode;
    k.wz_rw = wz_rw;
    // NO_REJEC mean (stack_mean.hip): fb2_list collects the pixels whose float
    // mean the kernel cannot prove independent of the summation order
    if (!k.frames16 && k.rtype == SGPU_NO_REJEC) {
        if ((r = c->fb2_list.ensure(k.npix * sizeof(int))) || (r = c->fb2_count.ensure(sizeof(int)))) return r;
        k.fb2_list = (int *)c->fb2_list.p;
        k.fb2_count = (int *)c->fb2_count.p;
        HIP_TRY(hipMemsetAsync(k.fb2_count, 0, sizeof(int), s));
    }
    c->last_mean = k.rtype == SGPU_NO_REJEC && !k.frames16;
    if (k.rtype == SGPU_WINSORIZED && wz_mode) {
        if ((r = c->fb2_list.ensure(k.npix * sizeof(int))) || (r = c->fb2_count.ensure(sizeof(int)))) return r;
        k.fb2_list = (int *)c->fb2_list.p;
        k.fb2_count = (int *)c->fb2_count.p;
        HIP_TRY(hipMemsetAsync(k.fb2_count, 0, sizeof(int), s));
        // workspace: two buffers of rank records (R slots + moments, meta,
        // round state, lists per pixel; stack_sorted_inst.h), at most 2 GiB
        // and no more than this launch's pixels need
        const int npw = sorted_capacity(N);
        const long long R = npw <= 128 ? 64 : npw / 2 + 16;
        const size_t need = (size_t)(2 * k.npix * (R * 4 + 96) + (1 << 20));
        const size_t ws = std::min(need, (size_t)2 << 30);
        static const long long chunk = std::getenv("SGPU_WZ_CHUNK") ? std::atoll(std::getenv("SGPU_WZ_CHUNK")) : 0;
        k.wz_chunk = chunk;
        // per-chunk tails (fallback sorted + exact kernels of a chunk on a third
        // stream, under the next chunks' work): counters zeroed per launch
        static const bool tails = !std::getenv("SGPU_WZ_TAILS") || std::atoi(std::getenv("SGPU_WZ_TAILS")) != 0;
        if (tails && c->wz_cnt.ensure((2 * sgpu::kWzMaxChunks + 1) * sizeof(int)) == SGPU_OK) {
            k.wz_tcnt = (int *)c->wz_cnt.p;
            HIP_TRY(hipMemsetAsync(k.wz_tcnt, 0, (2 * sgpu::kWzMaxChunks + 1) * sizeof(int), s));
        }
        if (c->wz_ws.ensure(ws) == SGPU_OK) {
            k.wz_ws = c->wz_ws.p;
            k.wz_ws_bytes = (long long)ws;
        }
    }

    if (k.frames16) {
        // 16-bit sequences: the 16-bit sorted kernels for every rejection type
        // and the median, normalized (round_to_WORD in the gather), weighted
        // and with weight planes; the sequential exact kernel for the pixels
        // they defer and for rejection at N > 1024.  The plain mean (no
        // weight planes) runs on the streaming kernel up to N = 65536, so the
        // sorted path's capacity does not bound it.
        const int np16 = sorted_capacity(N);
        const bool mean16 = k.rtype == SGPU_NO_REJEC && !k.drizz && !k.mask && N <= 65536;
        bool all16 = c->exact_only != 0 || (np16 == 0 && !mean16);
        if (N <= small_all_limit(k.rtype) && N <= 32 && small_type(k.rtype)) all16 = true;
        mark(c);
        if (!all16 && mean16) {
            KParams t = k;
            if (!has_shift) t.shiftx = nullptr;   // lets stack_mean use 16-byte loads
            if (sgpu::launch_stack_mean(t, s)) return fail(SGPU_NO_DEVICE, "stack_mean launch failed");
        } else if (!all16) {
            const int lr = launch_sorted16(np16, k, s);
            if (lr < 0) return fail(SGPU_NO_DEVICE, "16-bit sorted-path launch failed");
            if (lr == 1) all16 = true;
        }
        mark(c);
        mark(c);
        if ((r = launch_exact(c, k, all16, true))) return r;
        mark(c);
        c->last_all_exact = all16;
        c->last_npix = k.npix;
        return SGPU_OK;
    }
    bool all_exact = c->exact_only != 0;
    const int np = sorted_capacity(N);
    // small columns straight to the sequential small-column kernel (exact by
    // construction, no deferral), up to small_all_limit
    if (N <= small_all_limit(k.rtype) && N <= 32 && small_type(k.rtype)) all_exact = true;
    mark(c);
    // no-rejection mean with per-sample planes: the drizzle nulls change the
    // kept set the streaming kernel counts, so the exact kernel takes it
    if (k.rtype == SGPU_NO_REJEC && (k.drizz || k.mask)) all_exact = true;
    if (!all_exact) {
        if (k.rtype == SGPU_NO_REJEC) {
            KParams t = k;
            if (!has_shift) t.shiftx = nullptr;   // lets stack_mean use 16-byte loads
            if (sgpu::launch_stack_mean(t, s)) return fail(SGPU_NO_DEVICE, "stack_mean launch failed");
        } else if ((k.rtype == SGPU_LINEARFIT || k.rtype == SGPU_GESDT) && np > 128) {
            all_exact = true;   // sorted path for these is single-lane (N <= 128)
        } else if (np == 0) {
            all_exact = true;   // N > 1024
        } else {
            // diagnostic: SGPU_PROF=1 with a -DSGPU_PROF=1 build prints the
            // sorted kernel's per-section lane-cycles (stack_sorted_impl.h)
            static unsigned long long *d_prof = nullptr;
            static const bool prof = std::getenv("SGPU_PROF") != nullptr;
            if (prof && !d_prof && hipMalloc((void **)&d_prof, 16 * sizeof(unsigned long long)) != hipSuccess)
                d_prof = nullptr;
            if (prof && d_prof) {
                HIP_TRY(hipMemsetAsync(d_prof, 0, 16 * sizeof(unsigned long long), s));
                k.prof = d_prof;
            }
            const int lr = launch_sorted(np, k, s);
            if (lr < 0) return fail(SGPU_NO_DEVICE, "sorted-path launch failed");
            if (lr == 1) all_exact = true;   // no sorted instantiation
            if (prof && d_prof) {
                unsigned long long h[16];
                HIP_TRY(hipMemcpyAsync(h, d_prof, sizeof h, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                std::fprintf(stderr, "SGPU_PROF");
                for (int q = 0; q < 12; q++) std::fprintf(stderr, " %llu", h[q]);
                std::fprintf(stderr, "\n");
                k.prof = nullptr;
            }
        }
    }
    // exact sequential kernel: deferred pixels (or every pixel)
    mark(c);
    mark(c);
    if ((r = launch_exact(c, k, all_exact, false))) return r;
    mark(c);
    c->last_all_exact = all_exact;
    c->last_npix = k.npix;
    return SGPU_OK;
}

}  // namespace

namespace {
int stack_rows_device_impl(sgpu_context *c, const float *d_frames, const float *d_drizz, const float *d_mask,
                           int N, long W, long rows, long frame_stride, const sgpu_stack_params *P, float *d_out,
                           uint16_t *d_rej_lo, uint16_t *d_rej_hi, uint64_t *d_counts);
}

extern "C" int sgpu_stack_rows_device(sgpu_context *c, const float *d_frames, int N, long W,
                                      long rows, long frame_stride, const sgpu_stack_params *P,
                                      float *d_out, uint16_t *d_rej_lo, uint16_t *d_rej_hi,
                                      uint64_t *d_counts) {
    return stack_rows_device_impl(c, d_frames, nullptr, nullptr, N, W, rows, frame_stride, P, d_out, d_rej_lo,
                                  d_rej_hi, d_counts);
}

extern "C" int sgpu_stack_rows_planes_device(sgpu_context *c, const float *d_frames, const float *d_drizz,
                                             const float *d_mask, int N, long W, long rows, long frame_stride,
                                             const sgpu_stack_params *P, float *d_out, uint16_t *d_rej_lo,
                                             uint16_t *d_rej_hi, uint64_t *d_counts) {
    return stack_rows_device_impl(c, d_frames, d_drizz, d_mask, N, W, rows, frame_stride, P, d_out, d_rej_lo,
                                  d_rej_hi, d_counts);
}

namespace {
int stack_rows_device_impl(sgpu_context *c, const float *d_frames, const float *d_drizz, const float *d_mask,
                           int N, long W, long rows, long frame_stride, const sgpu_stack_params *P, float *d_out,
                           uint16_t *d_rej_lo, uint16_t *d_rej_hi, uint64_t *d_counts) {
    if (!c || !P || !d_frames || !d_out || !d_counts) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    if (W > (1L << 30)) return fail(SGPU_BAD_ARGUMENT, "width too large");
    HIP_TRY(hipSetDevice(c->device));
    KParams k;
    bool xf;
    c->ev_used = 0;
    int r = prepare(c, N, W, P, k, xf);
    if (r) return r;
    k.counts = (unsigned long long *)d_counts;
    const bool planes = (d_drizz || d_mask) && P->method == SGPU_METHOD_MEAN;
    // the per-sample planes are read by the gather's shift path (XF = 1)
    if (planes) k.shiftx = (const int *)c->shiftx.p;
    const long rows_per = std::max(1L, (long)(kMaxLaunchPixels / W));
    for (long y0 = 0; y0 < rows; y0 += rows_per) {
        const long nr = std::min(rows_per, rows - y0);
        KParams kk = k;
        kk.frames = d_frames + y0 * W;
        kk.frame_stride = frame_stride;
        kk.npix = (long long)nr * W;
        kk.out = d_out + y0 * W;
        kk.rej_lo = d_rej_lo ? d_rej_lo + y0 * W : nullptr;
        kk.rej_hi = d_rej_hi ? d_rej_hi + y0 * W : nullptr;
        kk.drizz = (planes && d_drizz) ? d_drizz + y0 * W : nullptr;
        kk.mask = (planes && d_mask) ? d_mask + y0 * W : nullptr;
        if ((r = run_launch(c, kk, P->shiftx != nullptr || planes))) return r;
    }
    return SGPU_OK;
}
}  // namespace

extern "C" int sgpu_stack_rows_planes(sgpu_context *c, const float *frames, const float *drizz,
                                      const float *mask, int N, long W, long rows, long frame_stride,
                                      const sgpu_stack_params *P, float *out, uint16_t *rej_lo, uint16_t *rej_hi,
                                      uint64_t counts[2]);

extern "C" int sgpu_stack_rows(sgpu_context *c, const float *frames, int N, long W, long rows,
                               long frame_stride, const sgpu_stack_params *P, float *out,
                               uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]) {
    return sgpu_stack_rows_planes(c, frames, nullptr, nullptr, N, W, rows, frame_stride, P, out, rej_lo, rej_hi,
                                  counts);
}

extern "C" int sgpu_stack_rows_planes(sgpu_context *c, const float *frames, const float *drizz,
                                      const float *mask, int N, long W, long rows, long frame_stride,
                                      const sgpu_stack_params *P, float *out, uint16_t *rej_lo, uint16_t *rej_hi,
                                      uint64_t counts[2]) {
    if (!c || !P || !frames || !out) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    // row chunks bounded by a device staging budget (frames of the chunk)
    const size_t budget = 8ull << 30;
    const int nplanes = 1 + (drizz ? 1 : 0) + (mask ? 1 : 0);
    long chunk = std::max(1L, (long)(budget / ((size_t)nplanes * N * W * sizeof(float))));
    chunk = std::min(chunk, rows);
    int r;
    if ((r = c->frames.ensure((size_t)N * chunk * W * sizeof(float))) ||
        (r = c->out.ensure((size_t)chunk * W * sizeof(float))) ||
        (r = c->counts.ensure(2 * sizeof(uint64_t))))
        return r;
    if (rej_lo && (r = c->rej_lo.ensure((size_t)chunk * W * sizeof(uint16_t)))) return r;
    if (drizz && (r = c->pl_drizz.ensure((size_t)N * chunk * W * sizeof(float)))) return r;
    if (mask && (r = c->pl_mask.ensure((size_t)N * chunk * W * sizeof(float)))) return r;
    if (rej_hi && (r = c->rej_hi.ensure((size_t)chunk * W * sizeof(uint16_t)))) return r;
    HIP_TRY(hipMemsetAsync(c->counts.p, 0, 2 * sizeof(uint64_t), s));
    for (long y0 = 0; y0 < rows; y0 += chunk) {
        const long nr = std::min(chunk, rows - y0);
        const size_t rowbytes = (size_t)nr * W * sizeof(float);
        HIP_TRY(hipMemcpy2DAsync(c->frames.p, rowbytes, frames + y0 * W, frame_stride * sizeof(float),
                                 rowbytes, N, hipMemcpyHostToDevice, s));
        if (drizz)
            HIP_TRY(hipMemcpy2DAsync(c->pl_drizz.p, rowbytes, drizz + y0 * W, frame_stride * sizeof(float),
                                     rowbytes, N, hipMemcpyHostToDevice, s));
        if (mask)
            HIP_TRY(hipMemcpy2DAsync(c->pl_mask.p, rowbytes, mask + y0 * W, frame_stride * sizeof(float),
                                     rowbytes, N, hipMemcpyHostToDevice, s));
        r = stack_rows_device_impl(c, (const float *)c->frames.p, drizz ? (const float *)c->pl_drizz.p : nullptr,
                                   mask ? (const float *)c->pl_mask.p : nullptr, N, W, nr, nr * W, P,
                                   (float *)c->out.p, rej_lo ? (uint16_t *)c->rej_lo.p : nullptr,
                                   rej_hi ? (uint16_t *)c->rej_hi.p : nullptr, (uint64_t *)c->counts.p);
        if (r) return r;
        HIP_TRY(hipMemcpyAsync(out + y0 * W, c->out.p, rowbytes, hipMemcpyDeviceToHost, s));
        if (rej_lo)
            HIP_TRY(hipMemcpyAsync(rej_lo + y0 * W, c->rej_lo.p, (size_t)nr * W * 2, hipMemcpyDeviceToHost, s));
        if (rej_hi)
            HIP_TRY(hipMemcpyAsync(rej_hi + y0 * W, c->rej_hi.p, (size_t)nr * W * 2, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    uint64_t hc[2] = {0, 0};
    HIP_TRY(hipMemcpy(hc, c->counts.p, sizeof hc, hipMemcpyDeviceToHost));
    if (counts) {
        counts[0] += hc[0];
        counts[1] += hc[1];
    }
    return SGPU_OK;
}

extern "C" int sgpu_stack_rows_u16_planes_device(sgpu_context *c, const uint16_t *d_frames, const float *d_drizz,
                                                 const float *d_mask, int N, long W, long rows,
                                                 long frame_stride, const sgpu_stack_params *P, float *d_out_f32,
                                                 uint16_t *d_out_u16, uint16_t *d_rej_lo, uint16_t *d_rej_hi,
                                                 uint64_t *d_counts);

extern "C" int sgpu_stack_rows_u16_device(sgpu_context *c, const uint16_t *d_frames, int N, long W,
                                          long rows, long frame_stride, const sgpu_stack_params *P,
                                          float *d_out_f32, uint16_t *d_out_u16, uint16_t *d_rej_lo,
                                          uint16_t *d_rej_hi, uint64_t *d_counts) {
    return sgpu_stack_rows_u16_planes_device(c, d_frames, nullptr, nullptr, N, W, rows, frame_stride, P, d_out_f32,
                                             d_out_u16, d_rej_lo, d_rej_hi, d_counts);
}

extern "C" int sgpu_stack_rows_u16_planes_device(sgpu_context *c, const uint16_t *d_frames, const float *d_drizz,
                                                 const float *d_mask, int N, long W, long rows,
                                                 long frame_stride, const sgpu_stack_params *P, float *d_out_f32,
                                                 uint16_t *d_out_u16, uint16_t *d_rej_lo, uint16_t *d_rej_hi,
                                                 uint64_t *d_counts) {
    if (!c || !P || !d_frames || !d_counts || (!d_out_f32 && !d_out_u16))
        return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    HIP_TRY(hipSetDevice(c->device));
    KParams k;
    bool xf;
    c->ev_used = 0;
    int r = prepare(c, N, W, P, k, xf);
    if (r) return r;
    k.counts = (unsigned long long *)d_counts;
    const bool planes = (d_drizz || d_mask) && P->method == SGPU_METHOD_MEAN;
    // the gather's XF path carries the shift, the WORD normalization and the
    // per-sample planes
    k.shiftx = (xf || planes) ? (const int *)c->shiftx.p : nullptr;
    const long rows_per = std::max(1L, (long)(kMaxLaunchPixels / W));
    for (long y0 = 0; y0 < rows; y0 += rows_per) {
        const long nr = std::min(rows_per, rows - y0);
        KParams kk = k;
        kk.frames16 = d_frames + y0 * W;
        kk.frame_stride = frame_stride;
        kk.npix = (long long)nr * W;
        kk.out = d_out_f32 ? d_out_f32 + y0 * W : nullptr;
        kk.out_f32 = d_out_f32 != nullptr;
        kk.out16 = d_out_u16 ? d_out_u16 + y0 * W : nullptr;
        kk.rej_lo = d_rej_lo ? d_rej_lo + y0 * W : nullptr;
        kk.rej_hi = d_rej_hi ? d_rej_hi + y0 * W : nullptr;
        kk.drizz = (planes && d_drizz) ? d_drizz + y0 * W : nullptr;
        kk.mask = (planes && d_mask) ? d_mask + y0 * W : nullptr;
        if ((r = run_launch(c, kk, P->shiftx != nullptr))) return r;
    }
    return SGPU_OK;
}

extern "C" int sgpu_stack_rows_u16(sgpu_context *c, const uint16_t *frames, int N, long W, long rows,
                                   long frame_stride, const sgpu_stack_params *P, float *out_f32,
                                   uint16_t *out_u16, uint16_t *rej_lo, uint16_t *rej_hi,
                                   uint64_t counts[2]) {
    if (!c || !P || !frames || (!out_f32 && !out_u16)) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t budget = 8ull << 30;
    long chunk = std::max(1L, (long)(budget / ((size_t)N * W * sizeof(uint16_t))));
    chunk = std::min(chunk, rows);
    int r;
    if ((r = c->frames.ensure((size_t)N * chunk * W * sizeof(uint16_t))) ||
        (r = c->counts.ensure(2 * sizeof(uint64_t))))
        return r;
    if (out_f32 && (r = c->out.ensure((size_t)chunk * W * sizeof(float)))) return r;
    if (out_u16 && (r = c->out16.ensure((size_t)chunk * W * sizeof(uint16_t)))) return r;
    if (rej_lo && (r = c->rej_lo.ensure((size_t)chunk * W * sizeof(uint16_t)))) return r;
    if (rej_hi && (r = c->rej_hi.ensure((size_t)chunk * W * sizeof(uint16_t)))) return r;
    HIP_TRY(hipMemsetAsync(c->counts.p, 0, 2 * sizeof(uint64_t), s));
    for (long y0 = 0; y0 < rows; y0 += chunk) {
        const long nr = std::min(chunk, rows - y0);
        const size_t rowbytes = (size_t)nr * W * sizeof(uint16_t);
        HIP_TRY(hipMemcpy2DAsync(c->frames.p, rowbytes, frames + y0 * W, frame_stride * sizeof(uint16_t),
                                 rowbytes, N, hipMemcpyHostToDevice, s));
        r = sgpu_stack_rows_u16_device(c, (const uint16_t *)c->frames.p, N, W, nr, nr * W, P,
                                       out_f32 ? (float *)c->out.p : nullptr,
                                       out_u16 ? (uint16_t *)c->out16.p : nullptr,
                                       rej_lo ? (uint16_t *)c->rej_lo.p : nullptr,
                                       rej_hi ? (uint16_t *)c->rej_hi.p : nullptr, (uint64_t *)c->counts.p);
        if (r) return r;
        if (out_f32)
            HIP_TRY(hipMemcpyAsync(out_f32 + y0 * W, c->out.p, (size_t)nr * W * 4, hipMemcpyDeviceToHost, s));
        if (out_u16)
            HIP_TRY(hipMemcpyAsync(out_u16 + y0 * W, c->out16.p, (size_t)nr * W * 2, hipMemcpyDeviceToHost, s));
        if (rej_lo)
            HIP_TRY(hipMemcpyAsync(rej_lo + y0 * W, c->rej_lo.p, (size_t)nr * W * 2, hipMemcpyDeviceToHost, s));
        if (rej_hi)
            HIP_TRY(hipMemcpyAsync(rej_hi + y0 * W, c->rej_hi.p, (size_t)nr * W * 2, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    uint64_t hc[2] = {0, 0};
    HIP_TRY(hipMemcpy(hc, c->counts.p, sizeof hc, hipMemcpyDeviceToHost));
    if (counts) {
        counts[0] += hc[0];
        counts[1] += hc[1];
    }
    return SGPU_OK;
}

// ---------------------------------------------------------------- multi-GPU
// Several devices of one node behind one handle: the pixel rows of a block
// are split into contiguous balanced bands (the exact decomposition, SURVEY
// 8e: every output pixel depends on its own column only; Siril's own OpenMP
// decomposition is by rows too, median_and_mean.c:295-356), each band is
// stacked by its own context on its own device from a host thread of its
// own, and the host gathers the bands by writing them straight into the
// caller's output rows.  Counters are summed on the host.
struct sgpu_multi {
    std::vector<sgpu_context *> ctx;
};

extern "C" int sgpu_row_bands(long rows, int nparts, long *starts) {
    if (rows < 0 || nparts < 1 || !starts) return fail(SGPU_BAD_ARGUMENT, "bad argument");
    const long base = rows / nparts, extra = rows % nparts;
    long y = 0;
    for (int r = 0; r < nparts; r++) {
        starts[r] = y;
        y += base + (r < extra ? 1 : 0);
    }
    starts[nparts] = y;
    return SGPU_OK;
}

extern "C" int sgpu_multi_init(const int *devices, int ndevices, sgpu_multi **out) {
    if (!out || !devices || ndevices < 1) return fail(SGPU_BAD_ARGUMENT, "bad argument");
    *out = nullptr;
    auto *m = new sgpu_multi();
    for (int i = 0; i < ndevices; i++) {
        sgpu_context *c = nullptr;
        const int r = sgpu_init(devices[i], &c);
        if (r) {
            for (sgpu_context *o : m->ctx) sgpu_release(o);
            delete m;
            return r;
        }
        m->ctx.push_back(c);
    }
    *out = m;
    return SGPU_OK;
}

extern "C" void sgpu_multi_release(sgpu_multi *m) {
    if (!m) return;
    for (sgpu_context *c : m->ctx) sgpu_release(c);
    delete m;
}

extern "C" int sgpu_multi_size(const sgpu_multi *m) { return m ? (int)m->ctx.size() : 0; }

extern "C" sgpu_context *sgpu_multi_context(sgpu_multi *m, int i) {
    return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[i] : nullptr;
}

namespace {
template <typename T, typename F>
int multi_bands(sgpu_multi *m, long W, long rows, F &&band_call, uint64_t counts[2]) {
    const int nd = (int)m->ctx.size();
    std::vector<long> st(nd + 1);
    sgpu_row_bands(rows, nd, st.data());
    std::vector<int> rc(nd, SGPU_OK);
    std::vector<std::string> msg(nd);
    std::vector<uint64_t> cnt(2 * nd, 0);
    auto work = [&](int d) {
        const long y0 = st[d], nr = st[d + 1] - st[d];
        if (nr <= 0) return;
        rc[d] = band_call(m->ctx[d], y0, nr, &cnt[2 * d]);
        if (rc[d]) msg[d] = g_err;          // thread-local message of that thread
    };
    std::vector<std::thread> th;
    for (int d = 1; d < nd; d++) th.emplace_back(work, d);
    work(0);
    for (std::thread &t : th) t.join();
    for (int d = 0; d < nd; d++)
        if (rc[d]) return fail(rc[d], "device " + std::to_string(d) + ": " + msg[d]);
    if (counts) {
        for (int d = 0; d < nd; d++) {
            counts[0] += cnt[2 * d];
            counts[1] += cnt[2 * d + 1];
        }
    }
    (void)W;
    return SGPU_OK;
}
}  // namespace

extern "C" int sgpu_multi_stack_rows(sgpu_multi *m, const float *frames, int N, long W, long rows,
                                     long frame_stride, const sgpu_stack_params *P, float *out,
                                     uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]) {
    if (!m || m->ctx.empty() || !frames || !out || !P) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    return multi_bands<float>(m, W, rows, [&](sgpu_context *c, long y0, long nr, uint64_t *cn) {
        return sgpu_stack_rows(c, frames + y0 * W, N, W, nr, frame_stride, P, out + y0 * W,
                               rej_lo ? rej_lo + y0 * W : nullptr, rej_hi ? rej_hi + y0 * W : nullptr, cn);
    }, counts);
}

extern "C" int sgpu_multi_stack_rows_u16(sgpu_multi *m, const uint16_t *frames, int N, long W, long rows,
                                         long frame_stride, const sgpu_stack_params *P, float *out_f32,
                                         uint16_t *out_u16, uint16_t *rej_lo, uint16_t *rej_hi,
                                         uint64_t counts[2]) {
    if (!m || m->ctx.empty() || !frames || (!out_f32 && !out_u16) || !P)
        return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (W <= 0 || rows <= 0 || N < 1) return fail(SGPU_BAD_ARGUMENT, "empty block");
    if (frame_stride < W * rows) return fail(SGPU_BAD_ARGUMENT, "frame_stride < width*rows");
    return multi_bands<uint16_t>(m, W, rows, [&](sgpu_context *c, long y0, long nr, uint64_t *cn) {
        return sgpu_stack_rows_u16(c, frames + y0 * W, N, W, nr, frame_stride, P,
                                   out_f32 ? out_f32 + y0 * W : nullptr, out_u16 ? out_u16 + y0 * W : nullptr,
                                   rej_lo ? rej_lo + y0 * W : nullptr, rej_hi ? rej_hi + y0 * W : nullptr, cn);
    }, counts);
}

namespace sgpu_host {
// parameter marshalling shared with the other stack entry points (stack_partial.hip)
int prepare_params(sgpu_context *c, int N, long W, const sgpu_stack_params *P, KParams &k, bool &xf) {
    return prepare(c, N, W, P, k, xf);
}
}  // namespace sgpu_host
