// sgpu_rl.cpp -- C-ABI of Richardson-Lucy deconvolution
// (filters/deconvolution/deconvolve.cpp:56-114, deconvolve.hpp:78-261):
// per-channel normalisation, padding, slice geometry, edge taper and the RL
// iteration loop, with every pixel pass on the GPU (rl_conv.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rl_conv.h"
#include "sgpu_internal.h"

using sgpu::rl::ConvArgs;
using sgpu::rl::SliceGeom;
using sgpu_host::fail;

namespace {

// regtype_t, filters/deconvolution/deconvolution.h:39
enum { REG_TV_GRAD = 0, REG_FH_GRAD, REG_NONE_GRAD, REG_TV_MULT, REG_FH_MULT, REG_NONE_MULT };

const int kGoodSizes[] = {256,  320,  384,  400,  512,  640,  768,  800,  1024, 1280, 1536, 1600,
                          1920, 2048, 2560, 3072, 3200, 3840, 4096, 5120, 6144, 6400, 7680, 8192};

struct Size2 {
    int w, h;
};

// calculate_slice_memory (image.hpp:298-303)
size_t slice_mem(int w, int h, int K, int N) { return (size_t)N * (w + 2 * K) * (h + 2 * K) * sizeof(float); }

// smallest_number_of_slices (image.hpp:305-320)
Size2 smallest(int W, int H, size_t M, int K, int N) {
    int w = W, h = H;
    while (slice_mem(w, h, K, N) > M) {
        if (w > h) w = (w + 1) / 2;
        else h = (h + 1) / 2;
    }
    return {w, h};
}

// optimum_fftw3_speed (image.hpp:322-345)
Size2 fastest(int W, int H, size_t M, int K, int N) {
    Size2 best{0, 0};
    size_t area = 0;
    for (int w : kGoodSizes)
        for (int h : kGoodSizes)
            if (slice_mem(w, h, K, N) <= M && (size_t)w * h > area) {
                best = {w, h};
                area = (size_t)w * h;
            }
    return best.w ? best : smallest(W, H, M, K, N);
}

int next_good(int s) {
    for (int g : kGoodSizes)
        if (g >= s) return g;
    return kGoodSizes[sizeof(kGoodSizes) / sizeof(int) - 1];
}

// best_compromise (image.hpp:353-401), max_slice_size preference at its
// default (32769, settings.c:252: no clamp)
Size2 best_compromise(int W, int H, size_t M, int K, int N) {
    const Size2 sm = smallest(W, H, M, K, N), fa = fastest(W, H, M, K, N);
    Size2 best;
    if ((double)(fa.w * fa.h) < 0.8 * sm.w * sm.h) {
        best = sm;
        double best_score = 0;
        for (int w : kGoodSizes)
            for (int h : kGoodSizes)
                if (slice_mem(w, h, K, N) <= M) {
                    const double score = std::min((double)(w * h) / (sm.w * sm.h), 1.0);
                    if (score > best_score) {
                        best = {w, h};
                        best_score = score;
                    }
                }
    } else {
        best = fa;
    }
    if (best.w <= W && best.h <= H) return best;
    const int nw = next_good(W), nh = next_good(H);
    best.w = ((float)nw / W < 1.1f) ? nw : W;
    best.h = ((float)nh / H < 1.1f) ? nh : H;
    return best;
}

// process_in_slices (image.hpp:404-492)
std::vector<SliceGeom> make_slices(int W, int H, size_t M, int overlap, int N) {
    const Size2 b = best_compromise(W, H, M, overlap, N);
    const int sw = b.w - 2 * overlap, sh = b.h - 2 * overlap;
    std::vector<SliceGeom> out;
    if (sw < 1 || sh < 1) return out;
    for (int sy = 0; sy < (H + sh - 1) / sh; sy++)
        for (int sx = 0; sx < (W + sw - 1) / sw; sx++) {
            SliceGeom g;
            g.x0 = sx * sw;
            g.y0 = sy * sh;
            const int x1 = std::min(g.x0 + sw, W), y1 = std::min(g.y0 + sh, H);
            g.aw = x1 - g.x0;
            g.ah = y1 - g.y0;
            g.pl = std::min(overlap, g.x0);
            g.pt = std::min(overlap, g.y0);
            g.sw = g.aw + g.pl + std::min(overlap, W - x1);
            g.sh = g.ah + g.pt + std::min(overlap, H - y1);
            out.push_back(g);
        }
    return out;
}

// img_t::sum: sequential float fold
float fsum(const std::vector<float> &v) {
    float s = 0.f;
    for (float x : v) s += x;
    return s;
}

// img_t::flip (image.hpp:717-730): swaps (x, y) <-> (w-1-x, h-1-y) for
// x < w/2 only, so an odd kernel's middle column is left unflipped
void flip_quirk(std::vector<float> &K, int ks) {
    for (int y = 0; y < ks; y++)
        for (int x = 0; x < ks / 2; x++) std::swap(K[y * ks + x], K[(ks - 1 - y) * ks + ks - 1 - x]);
}

std::vector<float> flip_full(const std::vector<float> &K, int ks) {
    std::vector<float> o(K.size());
    for (int y = 0; y < ks; y++)
        for (int x = 0; x < ks; x++) o[y * ks + x] = K[(ks - 1 - y) * ks + ks - 1 - x];
    return o;
}

// edgetaper weights (edgetaper.hpp:40-58): double sin^2 stored as float
void taper_weights(int n, int kn, float *w) {
    for (int y = 0; y < n; y++) {
        float v = 1.f;
        if (y < kn) v = (float)std::pow(std::sin(y * M_PI / (kn * 2 - 1)), 2.);
        else if (y > n - kn) v = (float)std::pow(std::sin((n - 1 - y) * M_PI / (kn * 2 - 1)), 2.);
        w[y] = v;
    }
}

int conv(sgpu_context *c, const float *in, float *out, int W, int H, const float *taps, int ks, int wrap, int epi,
         const float *f = nullptr, const float *est = nullptr, float dt = 0.f, const float *wy = nullptr,
         const float *wx = nullptr, double *stop = nullptr, const float *wreg = nullptr, float rlam = 0.f,
         const float *stop_ref = nullptr) {
    ConvArgs a;
    a.in = in;
    a.out = out;
    a.W = W;
    a.H = H;
    a.taps = taps;
    a.ks = ks;
    a.wrap = wrap;
    a.f = f;
    a.est = est;
    a.dt = dt;
    a.wy = wy;
    a.wx = wx;
    a.stop_acc = stop;
    a.stop_ref = stop_ref;
    a.w = wreg;
    a.rlam = rlam;
    if (sgpu::rl::launch_conv(a, epi, c->stream)) return fail(SGPU_NO_DEVICE, "convolution launch failed");
    c->rl_conv_launches++;
    return SGPU_OK;
}

// FFT convolution of the current slice (the FFT path's circular convolution)
int fconv(sgpu_context *c, const sgpu::rl::FftConv &fc, const float2 *khat, const float *in, float *out, int W,
          int H, int ks, int epi, const float *f = nullptr, const float *est = nullptr, float dt = 0.f,
          const float *wy = nullptr, const float *wx = nullptr, double *stop = nullptr,
          const float *wreg = nullptr, float rlam = 0.f, const float *stop_ref = nullptr, int chain = -1) {
    // chain < 0: a standalone convolution; else bit 0 = t1 already holds the
    // input's spectrum, bit 1 = leave the output's spectrum for the next call
    ConvArgs a;
    a.in = in;
    a.out = out;
    a.W = W;
    a.H = H;
    a.taps = nullptr;
    a.ks = ks;
    a.wrap = 1;
    a.f = f;
    a.est = est;
    a.dt = dt;
    a.wy = wy;
    a.wx = wx;
    a.stop_acc = stop;
    a.stop_ref = stop_ref;
    a.w = wreg;
    a.rlam = rlam;
    if (chain < 0) {
        if (sgpu::rl::fft_conv(fc, a, khat, epi, c->stream))
            return fail(SGPU_NO_DEVICE, "FFT convolution launch failed");
    } else if (sgpu::rl::fft_conv_chain(fc, a, khat, epi, (chain & 1) != 0, (chain & 2) != 0, c->stream)) {
        return fail(SGPU_NO_DEVICE, "FFT convolution launch failed");
    }
    c->rl_fft_convs++;
    return SGPU_OK;
}

// twiddle table w[k] = exp(-2 pi i k / n) in double, stored float
int upload_twiddles(sgpu_context *c, sgpu_host::DevBuf &buf, int n) {
    if (int r = buf.ensure((size_t)n * sizeof(float2))) return r;
    std::vector<float2> tw((size_t)n);
    for (int k = 0; k < n; k++) {
        const double a = 2.0 * M_PI * (double)k / (double)n;
        tw[(size_t)k] = make_float2((float)std::cos(a), (float)-std::sin(a));
    }
    HIP_TRY(hipMemcpy(buf.p, tw.data(), (size_t)n * sizeof(float2), hipMemcpyHostToDevice));
    return SGPU_OK;
}

// FFT-convolution plan of a W x H slice with a ks x ks kernel, or fc.n1 = 0
// when the direct convolution is used (SGPU_RL_DIRECT=1, or no smooth
// length <= 8192 covers the extended slice)
int fft_plan(sgpu_context *c, int W, int H, int ks, sgpu::rl::FftConv &fc) {
    fc.n1 = 0;
    const char *ev = std::getenv("SGPU_RL_DIRECT");
    if (ev && ev[0] == '1') return SGPU_OK;
    const int h = ks / 2;
    const int n1 = sgpu::rl::fft_smooth_len(W + 3 * h), n2 = sgpu::rl::fft_smooth_len(H + 3 * h);
    if (!n1 || !n2) return SGPU_OK;
    const int nh1 = n1 / 2 + 1;
    const size_t plane = (size_t)nh1 * n2 * sizeof(float2);
    int r;
    if ((r = c->rlf_t1.ensure(plane)) || (r = c->rlf_t2.ensure(plane)) || (r = c->rlf_ka.ensure(plane)) ||
        (r = c->rlf_kb.ensure(plane)) || (r = c->rlf_kt.ensure(plane)))
        return r;
    if (c->rlf_n1 != n1) {
        if ((r = upload_twiddles(c, c->rlf_tw1, n1))) return r;
        c->rlf_n1 = n1;
    }
    if (c->rlf_n2 != n2) {
        if ((r = upload_twiddles(c, c->rlf_tw2, n2))) return r;
        c->rlf_n2 = n2;
    }
    fc.n1 = n1;
    fc.n2 = n2;
    fc.nh1 = nh1;
    fc.W = W;
    fc.H = H;
    fc.h = h;
    fc.tw1 = (const float2 *)c->rlf_tw1.p;
    fc.tw2 = (const float2 *)c->rlf_tw2.p;
    fc.t1 = (float2 *)c->rlf_t1.p;
    fc.t2 = (float2 *)c->rlf_t2.p;
    if (sgpu::rl::fft_conv_setup(fc, c->stream)) return fail(SGPU_NO_DEVICE, "FFT convolution setup failed");
    return SGPU_OK;
}

struct RlArgs {
    int ks, maxiter, regtype, stop_active, naive;
    float stepsize, stopcriterion;
    float lambda;        // the entry point's lambda (deconvolve.cpp:56,86)
};

// one channel, device resident: d_f (rx x ry) -> d_u (rx x ry)
int rl_channel(sgpu_context *c, const float *d_f, float *d_u, int rx, int ry, std::vector<float> &K,
               const RlArgs &ra, int *ret) {
    hipStream_t s = c->stream;
    const int ks = ra.ks, hk = ks / 2;
    int r;
    // K /= K.sum()  (deconvolve.cpp:65, float division)
    {
        const float sum = fsum(K);
        for (float &v : K) v = v / sum;
    }
    // max (deconvolve.cpp:66-70)
    unsigned *d_bits = (unsigned *)c->rl_small.p;
    HIP_TRY(hipMemsetAsync(d_bits, 0, sizeof(unsigned), s));
    if (sgpu::rl::launch_chan_max(d_f, (long long)rx * ry, d_bits, s)) return fail(SGPU_NO_DEVICE, "max launch failed");
    unsigned bits = 0;
    HIP_TRY(hipMemcpyAsync(&bits, d_bits, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const float mx = bits ? sgpu::rl::decode_max(bits) : 0.f;
    if (mx == 0.0f) {
        *ret = 1;
        return SGPU_OK;
    }
    const int scale = (mx != 1.0f);
    // add_padding: ks/2 (FFT path, utils.hpp:114-124 via K) or 2*ks (naive path)
    const int pad = ra.naive ? 2 * ks : hk;
    const int Wp = rx + 2 * pad, Hp = ry + 2 * pad;
    const int ncopies = ra.naive ? 7 : ((ra.regtype == REG_TV_GRAD || ra.regtype == REG_TV_MULT) ? 12 : 10);
    const std::vector<SliceGeom> sl = make_slices(Wp, Hp, c->rl_memory, hk, ncopies);
    if (sl.empty()) return fail(SGPU_BAD_ARGUMENT, "slice geometry is empty (memory budget too small)");
    size_t maxpix = 0;
    int maxw = 0, maxh = 0;
    for (const SliceGeom &g : sl) {
        maxpix = std::max(maxpix, (size_t)g.sw * g.sh);
        maxw = std::max(maxw, g.sw);
        maxh = std::max(maxh, g.sh);
    }
    const bool tv = ra.regtype == REG_TV_GRAD || ra.regtype == REG_TV_MULT;
    const bool fh = ra.regtype == REG_FH_GRAD || ra.regtype == REG_FH_MULT;
    if ((r = c->rl_e.ensure(maxpix * 4)) || (r = c->rl_f.ensure(maxpix * 4)) || (r = c->rl_r.ensure(maxpix * 4)) ||
        (r = c->rl_w.ensure((size_t)(maxw + maxh) * 4)) || (r = c->rl_taps.ensure((size_t)3 * ks * ks * 4)))
        return r;
    if ((tv || fh) && (r = c->rl_reg.ensure(maxpix * 4))) return r;
    if (fh && ra.naive && (r = c->rl_gxy.ensure(maxpix * 4))) return r;
    float *Wreg = (tv || fh) ? (float *)c->rl_reg.p : nullptr;
    float *Gxy = (fh && ra.naive) ? (float *)c->rl_gxy.p : nullptr;
    // reallambda = 1 / (2 / lambda) in float (deconvolve.cpp:72,102 -> deconvolve.hpp:100,194)
    const float rlam = 1.f / (2.f / ra.lambda);
    const int reg_mode = tv ? (ra.naive ? sgpu::rl::REG_W_NAIVE_TV : sgpu::rl::REG_W_FFT_TV)
                            : (ra.naive ? sgpu::rl::REG_W_NAIVE_FH : sgpu::rl::REG_W_FFT_FH);
    float *E = (float *)c->rl_e.p, *F = (float *)c->rl_f.p, *R = (float *)c->rl_r.p;
    float *wts = (float *)c->rl_w.p;
    float *t_taper = (float *)c->rl_taps.p, *t_a = t_taper + ks * ks, *t_b = t_a + ks * ks;
    double *stop = (double *)((char *)c->rl_small.p + 64);
    std::vector<float> h_taps(3 * ks * ks), h_w;

    for (const SliceGeom &g : sl) {
        // host staging buffers are rewritten below: previous uploads must be done
        HIP_TRY(hipStreamSynchronize(s));
        // edge-taper weights for this slice (edgetaper.hpp:40-58)
        h_w.assign(g.sh + g.sw, 1.f);
        taper_weights(g.sh, ks, h_w.data());
        taper_weights(g.sw, ks, h_w.data() + g.sh);
        // taps: taper = K as is; FFT: K_otf = K/sum (pre-flip), Kflip_otf = flip(K)/sum,
        // K stays flipped for the next slice (deconvolve.hpp:84-96)
        std::memcpy(h_taps.data(), K.data(), ks * ks * 4);
        std::vector<float> ka, kb;
        if (!ra.naive) {
            const float r1 = 1.0f / fsum(K);
            ka = K;
            for (float &v : ka) v *= r1;
            flip_quirk(K, ks);
            const float r2 = 1.0f / fsum(K);
            kb = K;
            for (float &v : kb) v *= r2;
        } else {
            // conv2 is a correlation (image.hpp:498-600): correlation with K =
            // convolution with flip(K); the second pass correlates with flip(K)
            ka = flip_full(K, ks);
            kb = K;
        }
        std::memcpy(h_taps.data() + ks * ks, ka.data(), ks * ks * 4);
        std::memcpy(h_taps.data() + 2 * ks * ks, kb.data(), ks * ks * 4);
        HIP_TRY(hipMemcpyAsync(t_taper, h_taps.data(), h_taps.size() * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(wts, h_w.data(), h_w.size() * 4, hipMemcpyHostToDevice, s));
        const float *wy = wts, *wx = wts + g.sh;
        const int W = g.sw, H = g.sh;
        // FFT path: the taps' spectra of this slice (K flips between slices)
        sgpu::rl::FftConv fc;
        fc.n1 = 0;
        if (!ra.naive) {
            if ((r = fft_plan(c, W, H, ks, fc))) return r;
            if (fc.n1 && (sgpu::rl::fft_conv_taps(fc, t_taper, ks, (float2 *)c->rlf_kt.p, s) ||
                          sgpu::rl::fft_conv_taps(fc, t_a, ks, (float2 *)c->rlf_ka.p, s) ||
                          sgpu::rl::fft_conv_taps(fc, t_b, ks, (float2 *)c->rlf_kb.p, s)))
                return fail(SGPU_NO_DEVICE, "taps spectrum launch failed");
        }
        const bool use_fft = fc.n1 != 0;
        const float2 *k_t = (const float2 *)c->rlf_kt.p, *k_a = (const float2 *)c->rlf_ka.p,
                     *k_b = (const float2 *)c->rlf_kb.p;

        // timing groups: [iterations start, stop, extract+taper start, stop]
        sgpu_host::mark(c);
        sgpu_host::mark(c);
        sgpu_host::mark(c);
        if (sgpu::rl::launch_extract(d_f, rx, ry, pad, Wp, Hp, g, mx, scale, E, s))
            return fail(SGPU_NO_DEVICE, "slice extract failed");
        // edgetaper(slice, slice, K, 3): E -> F -> E -> F
        if (use_fft) {
            if ((r = fconv(c, fc, k_t, E, F, W, H, ks, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)) ||
                (r = fconv(c, fc, k_t, F, E, W, H, ks, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)) ||
                (r = fconv(c, fc, k_t, E, F, W, H, ks, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)))
                return r;
        } else if ((r = conv(c, E, F, W, H, t_taper, ks, 1, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)) ||
                   (r = conv(c, F, E, W, H, t_taper, ks, 1, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)) ||
                   (r = conv(c, E, F, W, H, t_taper, ks, 1, sgpu::rl::EPI_TAPER, nullptr, nullptr, 0.f, wy, wx)))
            return r;
        HIP_TRY(hipMemcpyAsync(E, F, (size_t)W * H * 4, hipMemcpyDeviceToDevice, s));
        sgpu_host::mark(c);
        // re-record the group's first two events around the iteration loop
        hipEvent_t ev_it0 = nullptr, ev_it1 = nullptr;
        if (c->timing && c->ev_used >= 4) {
            ev_it0 = c->ev[c->ev_used - 4];
            ev_it1 = c->ev[c->ev_used - 3];
            HIP_TRY(hipEventRecord(ev_it0, s));
        }

        const int wrap = ra.naive ? 0 : 1;
        const int epi_ratio = ra.naive ? sgpu::rl::EPI_RATIO_NAIVE : sgpu::rl::EPI_RATIO;
        const bool mult = ra.regtype == REG_NONE_MULT || ra.regtype == REG_TV_MULT || ra.regtype == REG_FH_MULT;
        const int epi_upd = Wreg ? (mult ? sgpu::rl::EPI_MULT_REG : sgpu::rl::EPI_GRAD_REG)
                                 : (mult ? sgpu::rl::EPI_MULT : sgpu::rl::EPI_GRAD);
        const float dt = mult ? 1.f : ra.stepsize;
        // the naive path's stop measure divides by gxy (deconvolve.hpp:250-251),
        // which only the FH regulariser writes: with TV or none it is the
        // zero-initialised image and the measure never fires
        const bool use_stop = ra.stop_active == 1 && (!ra.naive || Gxy);
        // SGPU_RL_CHAIN=1: chain the spectra through the iteration (fused
        // inverse + forward row pass; bit-identical, measured slower: the
        // fused kernel's registers halve its occupancy, 195 us against
        // 91 + 51 us for the two passes) -- A/B knob, off by default
        const char *cev = std::getenv("SGPU_RL_CHAIN");
        const bool chain_off = !(cev && cev[0] == '1');
        bool have = false;                                  // t1 holds E's spectrum
        for (int it = 0; it < ra.maxiter; it++) {
            if (use_stop) HIP_TRY(hipMemsetAsync(stop, 0, sizeof(double), s));
            if (Wreg && sgpu::rl::launch_reg(E, Wreg, Gxy, W, H, reg_mode, s))
                return fail(SGPU_NO_DEVICE, "regulariser launch failed");
            c->rl_iter_flops += 2.0 * 2.0 * ks * ks * (double)W * H;
            if (use_fft) {
                // algorithmic bytes per convolution: the slice read, the half
                // spectrum plane (n2 x nh1 complex) written by the rows, read
                // + written by each transpose, read + written + the taps
                // spectrum read by the column pass, read by the inverse rows
                // (9 planes), the epilogue's read and write
                const double half = 8.0 * fc.nh1 * fc.n2, pix = 4.0 * W * H;
                c->rl_iter_bytes += 2.0 * (9.0 * half + 3.0 * pix);
                // with the chain on, the ratio's inverse row pass leaves R's
                // spectrum for the second convolution and the update's leaves
                // E's for the next iteration
                const bool more = it + 1 < ra.maxiter && !chain_off;
                if ((r = fconv(c, fc, k_a, E, R, W, H, ks, epi_ratio, F, nullptr, 0.f, nullptr, nullptr, nullptr,
                               nullptr, 0.f, nullptr, chain_off ? -1 : ((have ? 1 : 0) | 2))) ||
                    (r = fconv(c, fc, k_b, R, E, W, H, ks, epi_upd, nullptr, E, dt, nullptr, nullptr,
                               use_stop ? stop : nullptr, Wreg, rlam, Gxy, chain_off ? -1 : (1 | (more ? 2 : 0)))))
                    return r;
                have = more;
            } else if ((r = conv(c, E, R, W, H, t_a, ks, wrap, epi_ratio, ra.naive ? E : F)) ||
                       (r = conv(c, R, E, W, H, t_b, ks, wrap, epi_upd, nullptr, E, dt, nullptr, nullptr,
                                 use_stop ? stop : nullptr, Wreg, rlam, Gxy)))
                // naive: rl_deconvolve_naive(slice, slice, ...) aliases x and f
                // (deconvolve.cpp:103), so its numerator is the current estimate
                return r;
            if (use_stop) {
                double acc = 0;
                HIP_TRY(hipMemcpyAsync(&acc, stop, sizeof(double), hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                if ((float)(acc / ((double)W * H)) < ra.stopcriterion) break;
            }
        }
        if (ev_it1) HIP_TRY(hipEventRecord(ev_it1, s));
        if (sgpu::rl::launch_store(E, rx, ry, pad, g, mx, scale, d_u, s))
            return fail(SGPU_NO_DEVICE, "slice store failed");
    }
    HIP_TRY(hipStreamSynchronize(s));
    *ret = 0;
    return SGPU_OK;
}

int check_args(unsigned rx, unsigned ry, int ks, int regtype, int naive) {
    if (ks < 1 || !(ks & 1)) return fail(SGPU_BAD_ARGUMENT, "PSF size must be odd");
    if (ks > sgpu::rl::max_conv_ks()) return fail(SGPU_BAD_ARGUMENT, "PSF larger than the direct-convolution tile");
    if (regtype < REG_TV_GRAD || regtype > REG_NONE_MULT) return fail(SGPU_BAD_ARGUMENT, "unknown regtype");
    const unsigned pad = naive ? 2u * ks : (unsigned)ks / 2;
    if (rx <= pad || ry <= pad || rx < (unsigned)ks || ry < (unsigned)ks)
        return fail(SGPU_BAD_ARGUMENT, "image smaller than the padding / PSF");
    return SGPU_OK;
}

int rl_device(sgpu_context *c, float *d_fdata, unsigned rx, unsigned ry, unsigned nchans, const float *kernel,
              int ks, unsigned kchans, float lambda, int maxiter, float stopcriterion, int regtype, float stepsize,
              int stop_active, int naive) {
    if (!c || !d_fdata || !kernel) return fail(SGPU_BAD_ARGUMENT, "null argument");
    int r = check_args(rx, ry, ks, regtype, naive);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    const size_t npix = (size_t)rx * ry;
    if ((r = c->rl_u.ensure(npix * 4)) || (r = c->rl_small.ensure(256))) return r;
    // any lambda is accepted: reallambda = 1.f / (2.f / lambda) follows IEEE as
    // the reference does (deconvolve.cpp:73, deconvolve.hpp:100): lambda 0
    // gives an unregularised update, lambda inf (-alpha=0) an infinite one
    RlArgs ra{ks, maxiter, regtype, stop_active, naive, stepsize, stopcriterion, lambda};
    c->rl_conv_launches = 0;
    c->ev_used = 0;
    c->rl_iter_flops = 0.0;
    c->rl_iter_bytes = 0.0;
    c->rl_fft_convs = 0;
    for (unsigned ch = 0; ch < nchans; ch++) {
        const unsigned kc = ch < kchans ? ch : 0;
        std::vector<float> K(kernel + (size_t)kc * ks * ks, kernel + (size_t)(kc + 1) * ks * ks);
        float *d_f = d_fdata + ch * npix;
        int ret = 0;
        if ((r = rl_channel(c, d_f, (float *)c->rl_u.p, (int)rx, (int)ry, K, ra, &ret))) return r;
        if (ret) return 1;
        HIP_TRY(hipMemcpyAsync(d_f, c->rl_u.p, npix * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int rl_host(sgpu_context *c, float *fdata, unsigned rx, unsigned ry, unsigned nchans, const float *kernel, int ks,
            unsigned kchans, float lambda, int maxiter, float stopcriterion, int regtype, float stepsize,
            int stop_active, int naive) {
    if (!c || !fdata || !kernel) return fail(SGPU_BAD_ARGUMENT, "null argument");
    int r = check_args(rx, ry, ks, regtype, naive);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = (size_t)rx * ry * nchans * 4;
    if ((r = c->rl_io.ensure(bytes))) return r;
    HIP_TRY(hipMemcpyAsync(c->rl_io.p, fdata, bytes, hipMemcpyHostToDevice, c->stream));
    int ret = rl_device(c, (float *)c->rl_io.p, rx, ry, nchans, kernel, ks, kchans, lambda, maxiter, stopcriterion,
                        regtype, stepsize, stop_active, naive);
    if (ret < 0) return ret;
    // channels before a max == 0 channel are written, as in the reference
    HIP_TRY(hipMemcpyAsync(fdata, c->rl_io.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ret;
}

sgpu_context *g_default = nullptr;

sgpu_context *default_context() {
    if (!g_default && sgpu_init(0, &g_default) != SGPU_OK) g_default = nullptr;
    return g_default;
}

}  // namespace

extern "C" int sgpu_rl_set_memory(sgpu_context *c, size_t bytes) {
    if (!c || bytes == 0) return fail(SGPU_BAD_ARGUMENT, "bad memory budget");
    c->rl_memory = bytes;
    return SGPU_OK;
}

extern "C" int sgpu_rl_fft_device(sgpu_context *c, float *d_fdata, unsigned rx, unsigned ry, unsigned nchans,
                                  const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter,
                                  float stopcriterion, int regtype, float stepsize, int stopcriterion_active) {
    return rl_device(c, d_fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion, regtype,
                     stepsize, stopcriterion_active, 0);
}

extern "C" int sgpu_rl_naive_device(sgpu_context *c, float *d_fdata, unsigned rx, unsigned ry, unsigned nchans,
                                    const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter,
                                    float stopcriterion, int regtype, float stepsize, int stopcriterion_active) {
    return rl_device(c, d_fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion, regtype,
                     stepsize, stopcriterion_active, 1);
}

extern "C" int sgpu_rl_fft(sgpu_context *c, float *fdata, unsigned rx, unsigned ry, unsigned nchans,
                           const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter,
                           float stopcriterion, int regtype, float stepsize, int stopcriterion_active) {
    return rl_host(c, fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion, regtype,
                   stepsize, stopcriterion_active, 0);
}

extern "C" int sgpu_rl_naive(sgpu_context *c, float *fdata, unsigned rx, unsigned ry, unsigned nchans,
                             const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter,
                             float stopcriterion, int regtype, float stepsize, int stopcriterion_active) {
    return rl_host(c, fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion, regtype,
                   stepsize, stopcriterion_active, 1);
}

// Reference signatures (filters/deconvolution/deconvolution.h:138-139) on a
// process-wide context bound to device 0.  `max_threads` sizes the
// reference's CPU thread pool and has no meaning here.
extern "C" int sgpu_fft_richardson_lucy(float *fdata, unsigned rx, unsigned ry, unsigned nchans, float *kernel,
                                        int kernelsize, unsigned kchans, float lambda, int maxiter,
                                        float stopcriterion, int max_threads, int regtype, float stepsize,
                                        int stopcriterion_active) {
    (void)max_threads;
    sgpu_context *c = default_context();
    if (!c) return SGPU_NO_DEVICE;
    return sgpu_rl_fft(c, fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion, regtype,
                       stepsize, stopcriterion_active);
}

extern "C" int sgpu_naive_richardson_lucy(float *fdata, unsigned rx, unsigned ry, unsigned nchans, float *kernel,
                                          int kernelsize, unsigned kchans, float lambda, int maxiter,
                                          float stopcriterion, int max_threads, int regtype, float stepsize,
                                          int stopcriterion_active) {
    (void)max_threads;
    sgpu_context *c = default_context();
    if (!c) return SGPU_NO_DEVICE;
    return sgpu_rl_naive(c, fdata, rx, ry, nchans, kernel, kernelsize, kchans, lambda, maxiter, stopcriterion,
                         regtype, stepsize, stopcriterion_active);
}

extern "C" long sgpu_rl_last_conv_launches(sgpu_context *c) { return c ? c->rl_conv_launches : -1; }

extern "C" double sgpu_rl_last_iter_flops(sgpu_context *c) { return c ? c->rl_iter_flops : -1.0; }
extern "C" double sgpu_rl_last_iter_bytes(sgpu_context *c) { return c ? c->rl_iter_bytes : -1.0; }
extern "C" long sgpu_rl_last_fft_convs(sgpu_context *c) { return c ? c->rl_fft_convs : -1; }
