// sgpu_internal.h -- host-side internals shared by the C-ABI translation
// units: error reporting, growable device buffers, the context object.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/sirilgpu.h"

namespace sgpu_host {

int fail(int code, const std::string &msg);

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return sgpu_host::fail(SGPU_NO_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// device buffer that only grows
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SGPU_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, (size_t)256);
        if (hipMalloc(&p, want) != hipSuccess) return fail(SGPU_ALLOC_ERROR, "hipMalloc failed");
        cap = want;
        return SGPU_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// page-locked host buffer, grow-only (sequence block staging)
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SGPU_OK;
        release();
        const size_t want = std::max(bytes, (size_t)256);
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return fail(SGPU_ALLOC_ERROR, "hipHostMalloc failed");
        }
        cap = want;
        return SGPU_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace sgpu_host

struct sgpu_context;
namespace sgpu_host {
// record a timing event on the context stream when timing is on
// (consumed in groups of four by sgpu_last_timing)
void mark(sgpu_context *c);
}  // namespace sgpu_host

struct sgpu_context {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int exact_only = 0;
    int timing = 0;
    int in_bitpix = 0;            // sample type of the source files (8: BYTE_IMG, normalize_to16bit)
    std::vector<hipEvent_t> ev;   // per launch: start main, stop main, start exact, stop exact
    size_t ev_used = 0;
    long long last_npix = 0;
    int last_all_exact = 0;
    int last_mean = 0;          // last launch was the float NO_REJEC mean (fb2_list = order-sensitive pixels)
    int seq_readers = 0;        // sequence stacks: block reader threads (0: OMP_NUM_THREADS, else 8)
    double seq_stats[12] = {};  // last sequence stack (sgpu_last_seq_stats)
    // sequence stacks: pinned block buffers, device block / output buffers
    // (kept across calls: page-locking 2 x 512 MB costs more than a small stack)
    sgpu_host::HostBuf seq_pin[2], seq_res;
    sgpu_host::DevBuf seq_in[2], seq_out, seq_lo, seq_hi, seq_cnt;
    // stacking workspace
    sgpu_host::DevBuf fb_list, fb_count, fb2_list, fb2_count, wz_ws, counts, scratch;
    sgpu_host::DevBuf wz_cnt;             // moment path: per-chunk deferral counters + their total
    sgpu_host::DevBuf scale, offset, mul, shiftx, weights, crit;
    // host-API staging
    sgpu_host::DevBuf frames, out, rej_lo, rej_hi, out16, pl_drizz, pl_mask;
    // host copies of the per-frame tables (outlive the async uploads)
    std::vector<double> h_scale, h_offset, h_mul, h_weights;
    std::vector<int> h_shift;
    std::vector<float> h_crit;
    // DFT registration workspace
    int dft_n = 0;
    sgpu_host::DevBuf dft_tw, dft_ref, dft_t1, dft_t2, dft_best, dft_shifts, dft_frames;
    // Richardson-Lucy workspace
    sgpu_host::DevBuf rl_u, rl_e, rl_f, rl_r, rl_w, rl_taps, rl_small, rl_io, rl_reg, rl_gxy;
    // Richardson-Lucy FFT convolution: work planes, taps spectra, twiddles
    sgpu_host::DevBuf rlf_t1, rlf_t2, rlf_ka, rlf_kb, rlf_kt, rlf_tw1, rlf_tw2;
    int rlf_n1 = 0, rlf_n2 = 0;           // lengths the twiddle tables hold
    long rl_fft_convs = 0;                // FFT convolutions of the last call
    double rl_iter_bytes = 0.0;           // algorithmic HBM bytes of the iteration convolutions
    size_t rl_memory = (size_t)1 << 40;   // slicing budget (get_available_memory() in the reference)
    long rl_conv_launches = 0;
    double rl_iter_flops = 0.0;           // algorithmic flops of the RL iteration convolutions
    // demosaic workspace
    sgpu_host::DevBuf dm_ws, dm_mm, dm_io;
    // normalization statistics workspace
    sgpu_host::DevBuf ns_state, ns_hist, ns_part, ns_io;
    sgpu_host::DevBuf bn_rows;            // background noise: per-row estimates
    sgpu_host::DevBuf fe_tab, fe_dt;      // feather masks: resize tables / distance-transform planes
    sgpu_host::DevBuf cfa_tmp;            // X-Trans interpolation passes (staged selections)
    sgpu_host::DevBuf cstripe;            // striped rejection totals of one launch
    // registration quality workspace
    sgpu_host::DevBuf qe_buf, qe_part, qe_io;
    // output normalization (norm_to_0_1_range) min/max keys
    sgpu_host::DevBuf onorm;
    // overlap normalization: packed pair samples and the pair table
    sgpu_host::DevBuf ov_ws, ov_tab;

    void release_all() {
        for (sgpu_host::DevBuf *b : {&fb_list, &fb_count, &counts, &scratch, &scale, &offset, &mul,
                                     &shiftx, &weights, &crit, &frames, &out, &rej_lo, &rej_hi, &out16, &pl_drizz, &pl_mask,
                                     &dft_tw, &dft_ref, &dft_t1, &dft_t2, &dft_best, &dft_shifts,
                                     &dft_frames, &rl_u, &rl_e, &rl_f, &rl_r, &rl_w, &rl_taps, &rl_small,
                                     &rl_io, &rl_reg, &rl_gxy, &rlf_t1, &rlf_t2, &rlf_ka, &rlf_kb, &rlf_kt, &rlf_tw1, &rlf_tw2, &dm_ws, &dm_mm, &dm_io, &ns_state, &ns_hist, &ns_part, &ns_io, &bn_rows, &qe_buf, &qe_part, &qe_io, &onorm, &ov_ws, &ov_tab,
                                     &fb2_list, &fb2_count, &wz_ws, &wz_cnt, &fe_tab, &fe_dt, &cfa_tmp, &cstripe,
                                     &seq_in[0], &seq_in[1], &seq_out, &seq_lo, &seq_hi, &seq_cnt})
            b->release();
        seq_pin[0].release();
        seq_pin[1].release();
        seq_res.release();
    }
};
