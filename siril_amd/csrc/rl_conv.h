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

size_t conv_lds_bytes(int ks);
int max_conv_ks();
int launch_conv(const ConvArgs &a, int epi, hipStream_t s);
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
