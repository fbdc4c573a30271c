// sgpu_demosaic.cpp -- C-ABI of the debayer entry points over the kernels of
// demosaic.hip (RCD and BAYER_BILINEAR = librtprocess bayerfast):
// debayer_buffer_new_float (algos/demosaicing_rtp.cpp:228-390),
// debayer_buffer_new_ushort (:74-224) and debayer_buffer_superpixel_float
// (algos/demosaicing_siril.c:806-820).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "sgpu_internal.h"

using sgpu_host::fail;

namespace sgpu {
namespace dm {
struct Img {
    int W, H;
    unsigned char cf[4];
    const unsigned *mm;
    int remap;
};
__global__ void k_minmax(const float *buf, long long n, unsigned *mm);
__global__ void k_superpixel(const float *buf, int W, int H, int pattern, float *out);
__global__ void k_bilinear_siril(const uint16_t *bay, int W, int H, int tile, int byte, uint16_t *rgb);
template <class T, class O>
int launch_rcd(Img g, const T *buf, O *rgb, int byte, int variant, hipStream_t s);
template <class T, class O>
int launch_rcd_multipass(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s);
template <int TX, int TY, class T, class O>
int launch_rcd_split(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s);
template <class T, class O>
int launch_bayerfast(Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s);
}  // namespace dm
}  // namespace sgpu

namespace {

// interpolation_method / sensor_pattern (core/settings.h:54-80)
enum { BAYER_BILINEAR = 0, BAYER_RCD = 8, XTRANS = 9 };
enum { BAYER_FILTER_RGGB = 0, BAYER_FILTER_GRBG = 3 };

// pattern_to_cfarray (algos/demosaicing_rtp.cpp:20-41)
const unsigned char kCfarray[4][4] = {{0, 1, 1, 2}, {2, 1, 1, 0}, {1, 2, 0, 1}, {1, 0, 2, 1}};

// the librtprocess switch (demosaicing_rtp.cpp:141-160, 312-330): BAYER_BILINEAR
// -> bayerfast_demosaic, BAYER_RCD and unknown values (`default: case
// BAYER_RCD`) -> rcd_demosaic; VNG / AHD / AMaZE / DCB / HPHD / IGV / LMMSE
// are not built
bool is_bilinear(int interpolation) { return interpolation == BAYER_BILINEAR; }
int check_rcd_args(int width, int height, int interpolation, int pattern) {
    if (width < 1 || height < 1) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    const bool rcd = interpolation == BAYER_RCD || interpolation < BAYER_BILINEAR || interpolation > XTRANS;
    if (!rcd && !is_bilinear(interpolation))
        return fail(SGPU_BAD_ARGUMENT, "only the RCD and BAYER_BILINEAR (bayerfast) interpolations are implemented");
    if (pattern < BAYER_FILTER_RGGB || pattern > BAYER_FILTER_GRBG)
        return fail(SGPU_BAD_ARGUMENT, "only 2x2 Bayer patterns are supported");
    return SGPU_OK;
}

float ord2f(unsigned o) {
    const unsigned b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    float v;
    std::memcpy(&v, &b, 4);
    return v;
}

}  // namespace

namespace {
// SGPU_RCD_FUSED: unset / "0" the step-per-kernel pipeline (default: 1.10 ms
// per 6000x4000 frame with seven passes, 0.90 ms with steps 1.1-2 and 4.1 in
// one pass, k_dir_pq), "3" the two-kernel split (steps
// 1-4.1 and 4.2-4.3 with LDS halos, 2.75x the traffic floor instead of ~16x,
// but 1.32 ms: round 4), "1" one LDS-tiled kernel (64 x 32 tiles, 1.26 ms),
// "2" the same with 32 x 32 tiles; all are bitwise identical
int rcd_mode() {
    const char *e = std::getenv("SGPU_RCD_FUSED");
    if (!e || !*e) return 0;
    return std::atoi(e);
}
template <class T, class O>
int run_rcd(int mode, sgpu::dm::Img g, const T *buf, O *rgb, int byte, float *ws, hipStream_t s) {
    if (mode == 1 || mode == 2) return sgpu::dm::launch_rcd(g, buf, rgb, byte, mode == 2 ? 1 : 0, s);
    if (mode == 0) return sgpu::dm::launch_rcd_multipass(g, buf, rgb, byte, ws, s);
    return sgpu::dm::launch_rcd_split<64, 32>(g, buf, rgb, byte, ws, s);
}
}  // namespace

// XCD-contiguous tile order of the stencil kernels (demosaic.hip DM_XY);
// SGPU_DM_REMAP=0: the dispatcher's order (A/B)
static int dm_remap() {
    static const int r = !std::getenv("SGPU_DM_REMAP") || std::atoi(std::getenv("SGPU_DM_REMAP")) != 0;
    return r;
}

extern "C" int sgpu_debayer_device(sgpu_context *c, const float *d_buf, int width, int height, int interpolation,
                                   int pattern, float *d_rgb) {
    if (!c || !d_buf || !d_rgb) return fail(SGPU_BAD_ARGUMENT, "null argument");
    int r = check_rcd_args(width, height, interpolation, pattern);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const long long n = (long long)width * height;
    const int mode = rcd_mode();
    if (((mode != 1 && mode != 2) || is_bilinear(interpolation)) &&
        (r = c->dm_ws.ensure((size_t)n * 8 * sizeof(float))))
        return r;
    if ((r = c->dm_mm.ensure(64))) return r;
    float *ws = (float *)c->dm_ws.p;
    unsigned *mm = (unsigned *)c->dm_mm.p;
    const unsigned init[2] = {0xffffffffu, 0u};
    c->ev_used = 0;
    sgpu_host::mark(c);
    HIP_TRY(hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, s));
    long long blocks = std::min<long long>(256, (n / 16 + 1023) / 1024 + 1);   // one per CU
    hipLaunchKernelGGL(sgpu::dm::k_minmax, dim3((unsigned)blocks), dim3(1024), 0, s, d_buf, n, mm);
    // the min == max test reads the range back after the demosaic launch, so
    // the kernels follow k_minmax with no host round trip between them (the
    // kernels read the range on the device); with min == max their output is
    // discarded (unspecified contents, the call fails as the reference's
    // NULL return).  The read-back is enqueued only once every launch has
    // succeeded and is waited for right away: no return path leaves a copy
    // into this frame's h_mm in flight.
    sgpu::dm::Img g;
    g.W = width;
    g.H = height;
    std::memcpy(g.cf, kCfarray[pattern], 4);
    g.mm = mm;
    g.remap = dm_remap();
    r = is_bilinear(interpolation) ? sgpu::dm::launch_bayerfast(g, d_buf, d_rgb, 0, ws, s)
                                   : run_rcd(mode, g, d_buf, d_rgb, 0, ws, s);
    if (r) return fail(SGPU_NO_DEVICE, "debayer launch failed");
    unsigned h_mm[2];
    HIP_TRY(hipMemcpyAsync(h_mm, mm, sizeof h_mm, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ord2f(h_mm[0]) == ord2f(h_mm[1]))   // range == 0: the reference returns NULL
        return fail(SGPU_GENERIC_ERROR, "debayer normalisation: min == max");
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "debayer launch failed");
}

extern "C" int sgpu_debayer_u16_device(sgpu_context *c, const uint16_t *d_buf, int width, int height,
                                       int interpolation, int pattern, int bit_depth, uint16_t *d_rgb) {
    if (!c || !d_buf || !d_rgb) return fail(SGPU_BAD_ARGUMENT, "null argument");
    int r = check_rcd_args(width, height, interpolation, pattern);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const long long n = (long long)width * height;
    const int mode = rcd_mode();
    if (((mode != 1 && mode != 2) || is_bilinear(interpolation)) &&
        (r = c->dm_ws.ensure((size_t)n * 8 * sizeof(float))))
        return r;
    if ((r = c->dm_mm.ensure(64))) return r;
    // no normalisation in the 16-bit wrapper: min / max pinned to 0 / 65535
    // make the kernels' (x - min) * factor and v * invfactor + min exact
    // identities (factor = 65535 / 65535 = 1)
    const unsigned pin[2] = {0x80000000u, 0x80000000u | 0x477fff00u};   // ordered 0.0f, 65535.0f
    unsigned *mm = (unsigned *)c->dm_mm.p;
    c->ev_used = 0;
    sgpu_host::mark(c);
    HIP_TRY(hipMemcpyAsync(mm, pin, sizeof pin, hipMemcpyHostToDevice, s));
    sgpu::dm::Img g;
    g.W = width;
    g.H = height;
    std::memcpy(g.cf, kCfarray[pattern], 4);
    g.mm = mm;
    g.remap = dm_remap();
    const int byte = bit_depth == 8;         // BYTE_IMG: roundf_to_BYTE (demosaicing_rtp.cpp:206-210)
    r = is_bilinear(interpolation) ? sgpu::dm::launch_bayerfast(g, d_buf, d_rgb, byte, (float *)c->dm_ws.p, s)
                                   : run_rcd(mode, g, d_buf, d_rgb, byte, (float *)c->dm_ws.p, s);
    if (r) return fail(SGPU_NO_DEVICE, "debayer launch failed");
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    sgpu_host::mark(c);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "debayer launch failed");
}

extern "C" int sgpu_superpixel_device(sgpu_context *c, const float *d_buf, int width, int height, int pattern,
                                      float *d_out) {
    if (!c || !d_buf || !d_out) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (width < 1 || height < 1) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    HIP_TRY(hipSetDevice(c->device));
    const int nw = width / 2 + width % 2, nh = height / 2 + height % 2;
    hipLaunchKernelGGL(sgpu::dm::k_superpixel, dim3((nw + 63) / 64, (nh + 3) / 4), dim3(256), 0, c->stream, d_buf,
                       width, height, pattern, d_out);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "superpixel launch failed");
}

namespace {
sgpu_context *g_dm_ctx = nullptr;
sgpu_context *dm_context() {
    if (!g_dm_ctx && sgpu_init(0, &g_dm_ctx) != SGPU_OK) g_dm_ctx = nullptr;
    return g_dm_ctx;
}
}  // namespace

// Reference signature (algos/demosaicing.h): returns a malloc'd planar RGB
// buffer the caller frees, or NULL.  Unlike the reference, `buf` is left
// unmodified (the reference normalises it in place and never restores it).
extern "C" float *sgpu_debayer_buffer_new_float(float *buf, int *width, int *height, int interpolation,
                                                int pattern, unsigned int xtrans[6][6]) {
    (void)xtrans;
    if (!buf || !width || !height) {
        fail(SGPU_BAD_ARGUMENT, "null argument");
        return nullptr;
    }
    sgpu_context *c = dm_context();
    if (!c) return nullptr;
    const long long n = (long long)*width * *height;
    if (check_rcd_args(*width, *height, interpolation, pattern)) return nullptr;
    if (c->dm_io.ensure((size_t)n * 4 * sizeof(float))) return nullptr;
    float *d_in = (float *)c->dm_io.p, *d_rgb = d_in + n;
    float *out = (float *)std::malloc((size_t)n * 3 * sizeof(float));
    if (!out) {
        fail(SGPU_ALLOC_ERROR, "malloc failed");
        return nullptr;
    }
    if (hipMemcpyAsync(d_in, buf, (size_t)n * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        sgpu_debayer_device(c, d_in, *width, *height, interpolation, pattern, d_rgb) != SGPU_OK ||
        hipMemcpyAsync(out, d_rgb, (size_t)n * 12, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(out);
        return nullptr;
    }
    return out;
}

// Reference signature (algos/demosaicing.h): WORD input, malloc'd planar RGB
// WORD output the caller frees, or NULL; bit_depth 8 (BYTE_IMG) rounds to
// BYTE range.
extern "C" uint16_t *sgpu_debayer_buffer_new_ushort(uint16_t *buf, int *width, int *height, int interpolation,
                                                    int pattern, unsigned int xtrans[6][6], int bit_depth) {
    (void)xtrans;
    if (!buf || !width || !height) {
        fail(SGPU_BAD_ARGUMENT, "null argument");
        return nullptr;
    }
    sgpu_context *c = dm_context();
    if (!c) return nullptr;
    const long long n = (long long)*width * *height;
    if (check_rcd_args(*width, *height, interpolation, pattern)) return nullptr;
    if (c->dm_io.ensure((size_t)n * 4 * sizeof(uint16_t))) return nullptr;
    uint16_t *d_in = (uint16_t *)c->dm_io.p, *d_rgb = d_in + n;
    uint16_t *out = (uint16_t *)std::malloc((size_t)n * 3 * sizeof(uint16_t));
    if (!out) {
        fail(SGPU_ALLOC_ERROR, "malloc failed");
        return nullptr;
    }
    if (hipMemcpyAsync(d_in, buf, (size_t)n * 2, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        sgpu_debayer_u16_device(c, d_in, *width, *height, interpolation, pattern, bit_depth, d_rgb) != SGPU_OK ||
        hipMemcpyAsync(out, d_rgb, (size_t)n * 6, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(out);
        return nullptr;
    }
    return out;
}

extern "C" int sgpu_debayer_siril_u16_device(sgpu_context *c, const uint16_t *d_buf, int width, int height,
                                             int interpolation, int pattern, int bit_depth, uint16_t *d_rgb) {
    if (!c || !d_buf || !d_rgb) return fail(SGPU_BAD_ARGUMENT, "null argument");
    if (width < 3 || height < 3) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    if (interpolation != BAYER_BILINEAR)
        return fail(SGPU_BAD_ARGUMENT, "debayer_buffer_siril: only BAYER_BILINEAR is implemented");
    if (pattern < BAYER_FILTER_RGGB || pattern > BAYER_FILTER_GRBG)
        return fail(SGPU_BAD_ARGUMENT, "only 2x2 Bayer patterns are supported");
    HIP_TRY(hipSetDevice(c->device));
    dim3 grid((width + 63) / 64, (height + 3) / 4);
    hipLaunchKernelGGL(sgpu::dm::k_bilinear_siril, grid, dim3(256), 0, c->stream, d_buf, width, height, pattern,
                       bit_depth == 8 ? 1 : 0, d_rgb);
    return hipGetLastError() == hipSuccess ? SGPU_OK : fail(SGPU_NO_DEVICE, "bilinear launch failed");
}

extern "C" uint16_t *sgpu_debayer_buffer_siril_ushort(uint16_t *buf, int *width, int *height, int interpolation,
                                                      int pattern, int bit_depth) {
    if (!buf || !width || !height) {
        fail(SGPU_BAD_ARGUMENT, "null argument");
        return nullptr;
    }
    sgpu_context *c = dm_context();
    if (!c) return nullptr;
    const long long n = (long long)*width * *height;
    if (c->dm_io.ensure((size_t)n * 4 * sizeof(uint16_t))) return nullptr;
    uint16_t *d_in = (uint16_t *)c->dm_io.p, *d_rgb = d_in + n;
    uint16_t *out = (uint16_t *)std::malloc((size_t)n * 3 * sizeof(uint16_t));
    if (!out) {
        fail(SGPU_ALLOC_ERROR, "malloc failed");
        return nullptr;
    }
    if (hipMemcpyAsync(d_in, buf, (size_t)n * 2, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        sgpu_debayer_siril_u16_device(c, d_in, *width, *height, interpolation, pattern, bit_depth, d_rgb) != SGPU_OK ||
        hipMemcpyAsync(out, d_rgb, (size_t)n * 6, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(out);
        return nullptr;
    }
    return out;
}

extern "C" float *sgpu_debayer_buffer_superpixel_float(float *buf, int *width, int *height, int pattern) {
    if (!buf || !width || !height) {
        fail(SGPU_BAD_ARGUMENT, "null argument");
        return nullptr;
    }
    sgpu_context *c = dm_context();
    if (!c) return nullptr;
    const int w = *width, h = *height;
    const int nw = w / 2 + w % 2, nh = h / 2 + h % 2;
    const size_t nin = (size_t)w * h, nout = (size_t)nw * nh * 3;
    if (c->dm_io.ensure((nin + nout) * sizeof(float))) return nullptr;
    float *d_in = (float *)c->dm_io.p, *d_out = d_in + nin;
    float *out = (float *)std::malloc(nout * sizeof(float));
    if (!out) {
        fail(SGPU_ALLOC_ERROR, "malloc failed");
        return nullptr;
    }
    if (hipMemcpyAsync(d_in, buf, nin * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        sgpu_superpixel_device(c, d_in, w, h, pattern, d_out) != SGPU_OK ||
        hipMemcpyAsync(out, d_out, nout * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(out);
        return nullptr;
    }
    *width = nw;
    *height = nh;
    return out;
}

extern "C" void sgpu_free(void *p) { std::free(p); }
