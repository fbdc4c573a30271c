// rl_conv.h -- device-side pieces of the Richardson-Lucy path shared by
// rl_conv.hip (kernels) and sgpu_rl.cpp (host orchestration).
#pragma once
#include <hip/hip_runtime.h>

namespace sgpu {
namespace rl {

enum Epi : int {
    EPI_STORE = 0,        // out = c
    EPI_RATIO = 1,        // out = f / sanitize(c)          (deconvolve.hpp:131-132, image.hpp:1337-1346)
    EPI_RATIO_NAIVE = 2,  // out = max(1e-9, f / c)         (deconvolve.hpp:229-230)
    EPI_MULT = 3,         // out = c * est                  (REG_NONE_MULT, deconvolve.hpp:145)
    EPI_GRAD = 4,         // out = est + dt * (-1 + c)      (REG_NONE_GRAD, deconvolve.hpp:155)
    EPI_TAPER = 5,        // out = w*in + (1. - w)*c        (edgetaper.hpp:95-99)
    EPI_MULT_REG = 6,     // out = c * est * (1 / (1 - rl * w))    (REG_TV/FH_MULT, deconvolve.hpp:146-149)
    EPI_GRAD_REG = 7,     // out = est + dt * ((-1 + rl * w) + c)  (REG_TV/FH_GRAD, deconvolve.hpp:154-156)
};

// regulariser weight w of one iteration (deconvolve.hpp:104-126 FFT path,
// :199-222 naive path)
enum Reg : int {
    REG_W_FFT_TV = 0,     // divergence(grad / (|grad| + eps)), expression edge rules
    REG_W_FFT_FH = 1,     // sqrt(gxx^2 + gyy^2 + 2 gxy^2), sanitized
    REG_W_NAIVE_TV = 2,   // img_t path: sanitized gradients, img_t::divergence
    REG_W_NAIVE_FH = 3,   // img_t path: max(1e-9, g)^2 terms; also stores gxy
};

struct ConvArgs {
    const float *in;      // H x W input (the convolved image)
    float *out;           // H x W output; must not alias `in`
    int W, H;
    const float *taps;    // ks x ks, [row][col] = K(x = col, y = row); convolution (not correlation)
    int ks;               // odd
    int wrap;             // 1 circular (FFT path), 0 zero outside (naive path)
    const float *f;       // EPI_RATIO*: numerator image
    const float *est;     // EPI_MULT/GRAD: current estimate (may alias out)
    float dt;             // EPI_GRAD step
    const float *wy, *wx; // EPI_TAPER separable weights (H and W entries)
    double *stop_acc;     // optional: += sum |new - ref| / |ref| (EPI_MULT/GRAD[_REG])
    const float *stop_ref;// reference image of the stop measure (null: the old estimate)
    const float *w;       // EPI_*_REG: regulariser weight
    float rlam;           // EPI_*_REG: reallambda
};

// geometry of one slice (image.hpp:404-492), in padded-image coordinates
struct SliceGeom {
    int x0, y0;           // origin of the slice's own (non-overlap) region
    int aw, ah;           // size of that region
    int pl, pt;           // overlap on the left / top
    int sw, sh;           // full slice size including overlap
};

// The RL point-wise step applied to one convolution output c at pixel
// (ox, oy) = flat index p of the W x H slice (shared by the direct MFMA
// convolution and the FFT convolution).
__device__ __forceinline__ float rl_epilogue(const ConvArgs &a, int epi, long long p, int ox, int oy, float c,
                                             double &stop_part) {
    float o;
    switch (epi) {
        default:
        case EPI_STORE:
            o = c;
            break;
        case EPI_RATIO: {
            const float d = (c != c || c == 0.f) ? 1.e-9f : c;
            o = a.f[p] / d;
            break;
        }
        case EPI_RATIO_NAIVE: {
            const float q = a.f[p] / c;
            o = (1.e-9f < q) ? q : 1.e-9f;
            break;
        }
        case EPI_MULT:
        case EPI_GRAD:
        case EPI_MULT_REG:
        case EPI_GRAD_REG: {
            const float e = a.est[p];
            float nv;
            if (epi == EPI_MULT) nv = c * e;
            else if (epi == EPI_GRAD) nv = e + a.dt * (-1.f + c);
            else if (epi == EPI_MULT_REG) nv = (c * e) * (1.f / (1.f - a.rlam * a.w[p]));
            else nv = e + a.dt * ((-1.f + a.rlam * a.w[p]) + c);
            o = nv;
            if (a.stop_acc) {
                const float r = a.stop_ref ? a.stop_ref[p] : e;
                stop_part += (double)(fabsf(nv - r) / fabsf(r));
            }
            break;
        }
        case EPI_TAPER: {
            const float w = a.wy[oy] * a.wx[ox];
            o = (float)((double)(w * a.in[p]) + (1. - (double)w) * (double)c);
            break;
        }
    }
    a.out[p] = o;
    return o;
}

size_t conv_lds_bytes(int ks);
int max_conv_ks();
int launch_conv(const ConvArgs &a, int epi, hipStream_t s);

// FFT convolution (rl_fft.hip): the slice's circular convolution as a linear
// convolution of its periodic extension (h = ks/2 on every side) with FFT
// lengths n1 >= W + 3h (rows) and n2 >= H + 3h (columns), 2-3-5-smooth and
// <= 8192; the taps' spectrum (scaled by 1/(n1 n2)) is computed once per slice.
struct FftConv {
    int n1, n2, nh1;          // FFT lengths, half-spectrum width
    int W, H, h;              // slice size, half kernel
    const float2 *tw1, *tw2;  // twiddle tables (device)
    float2 *t1, *t2;          // work planes, nh1 x n2 complex each
};
int fft_smooth_len(int need);   // 0 when no 2-3-5-smooth length <= 8192 exists
int fft_conv_setup(FftConv &fc, hipStream_t s);   // LDS attributes
// spectrum of the ks x ks taps, laid out as the column pass reads it
int fft_conv_taps(const FftConv &fc, const float *taps, int ks, float2 *khat, hipStream_t s);
int fft_conv(const FftConv &fc, const ConvArgs &a, const float2 *khat, int epi, hipStream_t s);
// The same convolution inside an iteration chain: `have`: t1 already holds
// the forward half spectra of a.in (left by the previous call); `next`: also
// leave the forward half spectra of this call's output in t1 (the inverse row
// pass transforms its output rows straight back: no forward row pass and no
// re-read of the image in the next convolution).
int fft_conv_chain(const FftConv &fc, const ConvArgs &a, const float2 *khat, int epi, bool have, bool next,
                   hipStream_t s);
// w (and gxy for REG_W_NAIVE_FH) from the estimate e, all W x H
int launch_reg(const float *e, float *w, float *gxy, int W, int H, int mode, hipStream_t s);
// max of a channel into *bits (ordered-uint encoding; *bits zeroed by the caller)
int launch_chan_max(const float *f, long long n, unsigned *bits, hipStream_t s);
float decode_max(unsigned bits);
// slice pixel = f[mirror(reflect(...))] (/ mx when div): add_padding (utils.hpp:71-112)
// followed by the slice extraction of process_in_slices (image.hpp:430-455)
int launch_extract(const float *f, int rx, int ry, int pad, int Wp, int Hp, SliceGeom g, float mx, int div,
                   float *out, hipStream_t s);
// own region of a slice -> channel output, remove_padding + (* mx when mul)
int launch_store(const float *x, int rx, int ry, int pad, SliceGeom g, float mx, int mul, float *u,
                 hipStream_t s);

}  // namespace rl
}  // namespace sgpu
