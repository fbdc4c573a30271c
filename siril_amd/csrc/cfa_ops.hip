// cfa_ops.hip -- frame-level data movement either side of the stack (SURVEY
// 8f ranks 3 and 4), pure index arithmetic on HBM-resident frames:
//
//   * apply_reg with interpolation "none" (registration/applyreg.c:653-660 ->
//     shift_fit_from_reg, registration/registration.c:322-370): every frame
//     translated by integer (shiftx, shifty) = round_to_int of its homography
//     relative to the reference (cvTransfH, opencv/opencv.cpp:385-396; for
//     translations h02_img - h02_ref and -(h12_img - h12_ref)), zero fill,
//     dest[x + sx, y + sy] = src[x, y] in Siril's bottom-up row order (which
//     is FITS row order);
//   * extract_CFA_buffer_float (algos/demosaicing.c:936-975): the samples of
//     one colour of a 2x2 (Bayer) or 6x6 (X-Trans) compiled pattern, in
//     raster order, compacted -- the output index of a matching sample is a
//     closed form of (x, y), so one thread per input sample writes it;
//   * split_cfa_float / split_cfa_ushort (algos/extraction.c:914-1050) and
//     merge_cfa (algos/demosaicing.c:757-840): the four 2x2 sub-planes.
// HBM-bound streaming kernels: one read and one write of every sample.
#include <hip/hip_runtime.h>

#include <vector>

#include <algorithm>
#include <cstring>

#include "sgpu_internal.h"

namespace sgpu {

template <typename T>
__global__ __launch_bounds__(256) void k_shift_frames(const T *in, T *out, int W, int H, long long fstride,
                                                      const int *sx, const int *sy) {
    const int f = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    // gather form of the reference's scatter: dest (x, y) <- src (x - sx, y - sy)
    const int xs = x - sx[f], ys = y - sy[f];
    T v = (T)0;
    if (xs >= 0 && xs < W && ys >= 0 && ys < H) v = in[(long long)f * fstride + (long long)ys * W + xs];
    out[(long long)f * fstride + (long long)y * W + x] = v;
}

struct CfaPat {
    unsigned char p[36];
    int size;
    int rowcnt[6];        // matching samples per pattern row over one period of columns
    int colpre[6][7];     // matching samples of pattern row r among columns [0, c)
    int rowpre[7];        // samples per pattern-row period prefix: rows [0, r) of a period
};

template <typename T>
__global__ __launch_bounds__(256) void k_extract_cfa(const T *in, T *out, int W, int H, CfaPat P, int layer,
                                                     long long per_row_period) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)W * H) return;
    const int y = (int)(i / W), x = (int)(i % W);
    const int ps = P.size, ry = y % ps, rx = x % ps;
    if (P.p[ry * ps + rx] != layer) return;
    // samples per full row of pattern row r: (W / ps) * rowcnt[r] + colpre[r][W % ps]
    const int wq = W / ps, wr = W % ps;
    long long j = (long long)(y / ps) * per_row_period;
    for (int r = 0; r < ry; r++) j += (long long)wq * P.rowcnt[r] + P.colpre[r][wr];
    j += (long long)(x / ps) * P.rowcnt[ry] + P.colpre[ry][rx];
    out[j] = in[i];
}

template <typename T>
__global__ __launch_bounds__(256) void k_split_cfa(const T *in, T *o0, T *o1, T *o2, T *o3, int W, int w2, int h2) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (long long)w2 * h2) return;
    const int r = (int)(j / w2), c = (int)(j % w2);
    const long long a = (long long)(2 * r) * W + 2 * c;
    o0[j] = in[a];
    o1[j] = in[a + 1];
    o2[j] = in[a + W];
    o3[j] = in[a + W + 1];
}

template <typename T>
__global__ __launch_bounds__(256) void k_merge_cfa(const T *c0, const T *c1, const T *c2, const T *c3, T *out, int w2,
                                                   int h2) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (long long)w2 * h2) return;
    const int r = (int)(j / w2), c = (int)(j % w2);
    const long long W = 2LL * w2;
    const long long a = (long long)(2 * r) * W + 2 * c;
    out[a] = c0[j];
    out[a + 1] = c1[j];
    out[a + W] = c2[j];
    out[a + W + 1] = c3[j];
}

}  // namespace sgpu

using sgpu_host::fail;

namespace {
int check_es(int es) { return (es == 2 || es == 4) ? SGPU_OK : fail(SGPU_BAD_ARGUMENT, "element size must be 2 or 4"); }
}  // namespace

extern "C" int sgpu_apply_reg_shifts(int nframes, const double *h02, const double *h12, int ref_index, int *shiftx,
                                     int *shifty) {
    if (nframes < 1 || !h02 || !h12 || !shiftx || !shifty || ref_index < 0 || ref_index >= nframes)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    auto round_to_int = [](double x) {   // core/proto.h:208-213
        x = std::min(x, 2147483647.0 - 0.5);
        x = std::max(x, -2147483648.0 + 0.5);
        return (int)(x + (x >= 0.0 ? 0.5 : -0.5));
    };
    for (int i = 0; i < nframes; i++) {
        // H = Htransf^-1 * Himg for translations: (h02 - h02_ref, h12 - h12_ref);
        // translation_from_H: dx = h02, dy = -h12 (registration.c:301-304)
        const double dx = h02[i] - h02[ref_index];
        const double dy = -(h12[i] - h12[ref_index]);
        shiftx[i] = round_to_int(dx);
        shifty[i] = round_to_int(dy);
    }
    return SGPU_OK;
}

extern "C" int sgpu_shift_frames_device(sgpu_context *c, const void *d_in, void *d_out, int elem_size, int nframes,
                                        int width, int height, long frame_stride, const int *shiftx,
                                        const int *shifty) {
    if (!c || !d_in || !d_out || !shiftx || !shifty || nframes < 1 || width < 1 || height < 1 ||
        frame_stride < (long)width * height || nframes > 65535)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (d_in == d_out) return fail(SGPU_BAD_ARGUMENT, "in place shift is not supported");
    if (int r = check_es(elem_size)) return r;
    HIP_TRY(hipSetDevice(c->device));
    if (int r = c->shiftx.ensure(2 * (size_t)nframes * sizeof(int))) return r;
    c->h_shift.assign(shiftx, shiftx + nframes);
    c->h_shift.insert(c->h_shift.end(), shifty, shifty + nframes);
    HIP_TRY(hipMemcpyAsync(c->shiftx.p, c->h_shift.data(), 2 * (size_t)nframes * sizeof(int), hipMemcpyHostToDevice,
                           c->stream));
    const int *dsx = (const int *)c->shiftx.p, *dsy = dsx + nframes;
    dim3 grid((unsigned)((width + 63) / 64), (unsigned)((height + 3) / 4), (unsigned)nframes);
    if (elem_size == 4)
        hipLaunchKernelGGL(sgpu::k_shift_frames<float>, grid, dim3(256), 0, c->stream, (const float *)d_in,
                           (float *)d_out, width, height, (long long)frame_stride, dsx, dsy);
    else
        hipLaunchKernelGGL(sgpu::k_shift_frames<uint16_t>, grid, dim3(256), 0, c->stream, (const uint16_t *)d_in,
                           (uint16_t *)d_out, width, height, (long long)frame_stride, dsx, dsy);
    HIP_TRY(hipGetLastError());
    // the shift table must outlive the async copy: synchronise before returning
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SGPU_OK;
}

// apply_reg_image_hook (registration/applyreg.c:388-660) on the translations
// REG_DFT produces, at scale 1 with FRAMING_CURRENT: H = Htransf^-1 * Himg
// (cvTransfH, opencv.cpp:385-396; Htransf = the reference image's H), then
//   * interpolation OPENCV_NONE (5): shift_fit_from_reg (registration.c:322-370),
//     round_to_int of the translation;
//   * OPENCV_NEAREST .. OPENCV_LANCZOS4 (0-4): cvTransformImage
//     (opencv.cpp:520-560) = warpPerspective(H', BORDER_TRANSPARENT) with H'
//     the y-flipped H (cvPrepareH).  For an INTEGER translation every OpenCV
//     kernel samples at fractional offset 0, where its coefficient table is
//     exactly (1, 0, ...): the output is the source pixel itself (the zero
//     taps of partially outside neighbourhoods read reflected pixels and add
//     0), destination pixels whose source is outside keep the zero fill, and
//     the Lanczos / cubic clamp compares against an INTER_AREA warp that is
//     the same shift (no pixel changes).  So the result is the integer shift.
// Non-translation homographies and sub-pixel translations under an OpenCV
// interpolation (star-alignment registrations, -scale) are refused: REG_DFT
// never produces them.  H: 9 doubles per frame (h00 h01 h02 h10 .. h22).
extern "C" int sgpu_apply_reg_device(sgpu_context *c, const void *d_in, void *d_out, int elem_size, int nframes,
                                     int width, int height, long frame_stride, const double *H, int ref_index,
                                     int interpolation) {
    if (!c || !H || nframes < 1 || ref_index < 0 || ref_index >= nframes)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (interpolation < 0 || interpolation > 5) return fail(SGPU_BAD_ARGUMENT, "interpolation: OPENCV_NEAREST..NONE");
    std::vector<double> h02(nframes), h12(nframes);
    for (int i = 0; i < nframes; i++) {
        const double *m = H + 9 * (size_t)i;
        if (m[0] != 1.0 || m[1] != 0.0 || m[3] != 0.0 || m[4] != 1.0 || m[6] != 0.0 || m[7] != 0.0 || m[8] != 1.0)
            return fail(SGPU_BAD_ARGUMENT, "apply_reg: only translation registrations (REG_DFT) are supported");
        h02[i] = m[2];
        h12[i] = m[5];
    }
    std::vector<int> sx(nframes), sy(nframes);
    if (int r = sgpu_apply_reg_shifts(nframes, h02.data(), h12.data(), ref_index, sx.data(), sy.data())) return r;
    if (interpolation <= 4)
        for (int i = 0; i < nframes; i++) {
            const double dx = h02[i] - h02[ref_index], dy = -(h12[i] - h12[ref_index]);
            if (dx != (double)sx[i] || dy != (double)sy[i])
                return fail(SGPU_BAD_ARGUMENT, "apply_reg: sub-pixel translations need OpenCV resampling (not built)");
        }
    return sgpu_shift_frames_device(c, d_in, d_out, elem_size, nframes, width, height, frame_stride, sx.data(),
                                    sy.data());
}

extern "C" long sgpu_cfa_count(int width, int height, const unsigned char *pattern, int pattern_size, int layer) {
    if (width < 1 || height < 1 || !pattern || (pattern_size != 2 && pattern_size != 6)) return -1;
    long n = 0;
    for (int r = 0; r < pattern_size; r++) {
        long rowcnt = 0, pre = 0;
        for (int c = 0; c < pattern_size; c++) rowcnt += pattern[r * pattern_size + c] == layer;
        for (int c = 0; c < width % pattern_size; c++) pre += pattern[r * pattern_size + c] == layer;
        const long rows = height / pattern_size + (r < height % pattern_size ? 1 : 0);
        n += rows * ((long)(width / pattern_size) * rowcnt + pre);
    }
    return n;
}

extern "C" int sgpu_extract_cfa_device(sgpu_context *c, const void *d_in, int elem_size, int width, int height,
                                       const unsigned char *pattern, int pattern_size, int layer, void *d_out,
                                       long *newsize) {
    if (!c || !d_in || !d_out || !pattern || width < 1 || height < 1 || (pattern_size != 2 && pattern_size != 6))
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (int r = check_es(elem_size)) return r;
    sgpu::CfaPat P;
    std::memset(&P, 0, sizeof P);
    P.size = pattern_size;
    std::memcpy(P.p, pattern, (size_t)pattern_size * pattern_size);
    long long per_period = 0;
    const int wq = width / pattern_size, wr = width % pattern_size;
    for (int r = 0; r < pattern_size; r++) {
        P.colpre[r][0] = 0;
        for (int cc = 0; cc < pattern_size; cc++) P.colpre[r][cc + 1] = P.colpre[r][cc] + (pattern[r * pattern_size + cc] == layer);
        P.rowcnt[r] = P.colpre[r][pattern_size];
        per_period += (long long)wq * P.rowcnt[r] + P.colpre[r][wr];
    }
    HIP_TRY(hipSetDevice(c->device));
    const long long n = (long long)width * height;
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (elem_size == 4)
        hipLaunchKernelGGL(sgpu::k_extract_cfa<float>, dim3(grid), dim3(256), 0, c->stream, (const float *)d_in,
                           (float *)d_out, width, height, P, layer, per_period);
    else
        hipLaunchKernelGGL(sgpu::k_extract_cfa<uint16_t>, dim3(grid), dim3(256), 0, c->stream, (const uint16_t *)d_in,
                           (uint16_t *)d_out, width, height, P, layer, per_period);
    HIP_TRY(hipGetLastError());
    if (newsize) *newsize = sgpu_cfa_count(width, height, pattern, pattern_size, layer);
    return SGPU_OK;
}

extern "C" int sgpu_split_cfa_device(sgpu_context *c, const void *d_in, int elem_size, int width, int height,
                                     void *d_cfa0, void *d_cfa1, void *d_cfa2, void *d_cfa3) {
    if (!c || !d_in || !d_cfa0 || !d_cfa1 || !d_cfa2 || !d_cfa3 || width < 2 || height < 2)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (int r = check_es(elem_size)) return r;
    HIP_TRY(hipSetDevice(c->device));
    const int w2 = width / 2, h2 = height / 2;
    const unsigned grid = (unsigned)(((long long)w2 * h2 + 255) / 256);
    if (elem_size == 4)
        hipLaunchKernelGGL(sgpu::k_split_cfa<float>, dim3(grid), dim3(256), 0, c->stream, (const float *)d_in,
                           (float *)d_cfa0, (float *)d_cfa1, (float *)d_cfa2, (float *)d_cfa3, width, w2, h2);
    else
        hipLaunchKernelGGL(sgpu::k_split_cfa<uint16_t>, dim3(grid), dim3(256), 0, c->stream, (const uint16_t *)d_in,
                           (uint16_t *)d_cfa0, (uint16_t *)d_cfa1, (uint16_t *)d_cfa2, (uint16_t *)d_cfa3, width, w2,
                           h2);
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}

extern "C" int sgpu_merge_cfa_device(sgpu_context *c, const void *d_cfa0, const void *d_cfa1, const void *d_cfa2,
                                     const void *d_cfa3, int elem_size, int width2, int height2, void *d_out) {
    if (!c || !d_out || !d_cfa0 || !d_cfa1 || !d_cfa2 || !d_cfa3 || width2 < 1 || height2 < 1)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    if (int r = check_es(elem_size)) return r;
    HIP_TRY(hipSetDevice(c->device));
    const unsigned grid = (unsigned)(((long long)width2 * height2 + 255) / 256);
    if (elem_size == 4)
        hipLaunchKernelGGL(sgpu::k_merge_cfa<float>, dim3(grid), dim3(256), 0, c->stream, (const float *)d_cfa0,
                           (const float *)d_cfa1, (const float *)d_cfa2, (const float *)d_cfa3, (float *)d_out, width2,
                           height2);
    else
        hipLaunchKernelGGL(sgpu::k_merge_cfa<uint16_t>, dim3(grid), dim3(256), 0, c->stream, (const uint16_t *)d_cfa0,
                           (const uint16_t *)d_cfa1, (const uint16_t *)d_cfa2, (const uint16_t *)d_cfa3,
                           (uint16_t *)d_out, width2, height2);
    HIP_TRY(hipGetLastError());
    return SGPU_OK;
}
