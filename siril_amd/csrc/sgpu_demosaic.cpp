// sgpu_demosaic.cpp -- C-ABI of the float debayer (debayer_buffer_new_float,
// algos/demosaicing_rtp.cpp:228-390; debayer_buffer_superpixel_float,
// algos/demosaicing_siril.c:806-820) over the kernels of demosaic.hip.
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
};
__global__ void k_minmax(const float *buf, long long n, unsigned *mm);
__global__ void k_prep(Img g, const float *buf, float *cfa);
__global__ void k_hv(Img g, const float *cfa, float *V, float *Hh);
__global__ void k_dir(Img g, const float *cfa, const float *V, const float *Hh, float *VH, float *LP, float *P,
                      float *Q);
__global__ void k_green(Img g, const float *cfa, const float *VH, const float *LP, float *G);
__global__ void k_pq(Img g, const float *P, const float *Q, float *LPQ);
__global__ void k_rb_sites(Img g, const float *cfa, const float *G, const float *PQ, float *R, float *B);
__global__ void k_final(Img g, const float *buf, const float *G, const float *VH, const float *R, const float *B,
                        float *rgb);
__global__ void k_superpixel(const float *buf, int W, int H, int pattern, float *out);
int launch_rcd(Img g, const float *buf, float *rgb, int variant, hipStream_t s);
}  // namespace dm
}  // namespace sgpu

namespace {

// interpolation_method / sensor_pattern (core/settings.h:54-80)
enum { BAYER_BILINEAR = 0, BAYER_RCD = 8, XTRANS = 9 };
enum { BAYER_FILTER_RGGB = 0, BAYER_FILTER_GRBG = 3 };

// pattern_to_cfarray (algos/demosaicing_rtp.cpp:20-41)
const unsigned char kCfarray[4][4] = {{0, 1, 1, 2}, {2, 1, 1, 0}, {1, 2, 0, 1}, {1, 0, 2, 1}};

int check_rcd_args(int width, int height, int interpolation, int pattern) {
    if (width < 1 || height < 1) return fail(SGPU_BAD_ARGUMENT, "bad image size");
    // the reference's switch sends unknown values to RCD (`default: case BAYER_RCD`)
    const bool rcd = interpolation == BAYER_RCD || interpolation < BAYER_BILINEAR || interpolation > XTRANS;
    if (!rcd) return fail(SGPU_BAD_ARGUMENT, "only the RCD interpolation is implemented");
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

extern "C" int sgpu_debayer_device(sgpu_context *c, const float *d_buf, int width, int height, int interpolation,
                                   int pattern, float *d_rgb) {
    if (!c || !d_buf || !d_rgb) return fail(SGPU_BAD_ARGUMENT, "null argument");
    int r = check_rcd_args(width, height, interpolation, pattern);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const long long n = (long long)width * height;
    const char *fz0 = std::getenv("SGPU_RCD_FUSED");
    const bool multipass = !(fz0 && (fz0[0] == '1' || fz0[0] == '2'));
    if ((multipass && (r = c->dm_ws.ensure((size_t)n * 8 * sizeof(float)))) || (r = c->dm_mm.ensure(64))) return r;
    float *ws = (float *)c->dm_ws.p;
    float *cfa = ws, *V = ws + n, *Hh = ws + 2 * n, *VH = ws + 3 * n, *LP = ws + 4 * n, *P = ws + 5 * n,
          *Q = ws + 6 * n, *G = ws + 7 * n;
    unsigned *mm = (unsigned *)c->dm_mm.p;
    const unsigned init[2] = {0xffffffffu, 0u};
    c->ev_used = 0;
    sgpu_host::mark(c);
    HIP_TRY(hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, s));
    long long blocks = std::min<long long>(1024, (n / 4 + 255) / 256 + 1);   // 4 per CU
    hipLaunchKernelGGL(sgpu::dm::k_minmax, dim3((unsigned)blocks), dim3(256), 0, s, d_buf, n, mm);
    unsigned h_mm[2];
    HIP_TRY(hipMemcpyAsync(h_mm, mm, sizeof h_mm, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ord2f(h_mm[0]) == ord2f(h_mm[1]))   // range == 0: the reference returns NULL
        return fail(SGPU_GENERIC_ERROR, "debayer normalisation: min == max");
    sgpu::dm::Img g;
    g.W = width;
    g.H = height;
    std::memcpy(g.cf, kCfarray[pattern], 4);
    g.mm = mm;
    // SGPU_RCD_FUSED: unset / "0" the step-per-kernel pipeline (default:
    // measured faster, 1.09 vs 1.26 ms per 6000x4000 frame), "1" one LDS-tiled
    // kernel (64 x 32 tiles), "2" the same with 32 x 32 tiles; all three are
    // bitwise identical
    const char *fz = std::getenv("SGPU_RCD_FUSED");
    const int mode = (fz && fz[0] == '1') ? 1 : (fz && fz[0] == '2') ? 2 : 0;
    if (mode != 0) {
        if (sgpu::dm::launch_rcd(g, d_buf, d_rgb, mode == 2 ? 1 : 0, s))
            return fail(SGPU_NO_DEVICE, "debayer launch failed");
    } else {
        const dim3 grid((width + 63) / 64, (height + 3) / 4), blk(256);
        hipLaunchKernelGGL(sgpu::dm::k_prep, grid, blk, 0, s, g, d_buf, cfa);
        hipLaunchKernelGGL(sgpu::dm::k_hv, grid, blk, 0, s, g, cfa, V, Hh);
        hipLaunchKernelGGL(sgpu::dm::k_dir, grid, blk, 0, s, g, cfa, V, Hh, VH, LP, P, Q);
        hipLaunchKernelGGL(sgpu::dm::k_green, grid, blk, 0, s, g, cfa, VH, LP, G);
        hipLaunchKernelGGL(sgpu::dm::k_pq, grid, blk, 0, s, g, P, Q, LP);
        // V / Hh are dead after k_dir: they hold the red / blue site planes
        hipLaunchKernelGGL(sgpu::dm::k_rb_sites, grid, blk, 0, s, g, cfa, G, LP, V, Hh);
        hipLaunchKernelGGL(sgpu::dm::k_final, grid, blk, 0, s, g, d_buf, G, VH, V, Hh, d_rgb);
    }
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
