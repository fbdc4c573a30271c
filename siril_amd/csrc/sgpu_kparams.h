// sgpu_kparams.h -- kernel parameter block shared by the host C-ABI layer
// (sgpu_capi.cpp) and the HIP kernels.  Plain data, device pointers only.
#pragma once
#include <stdint.h>

namespace sgpu {

// rejection enum, reference core/settings.h:43-52
enum Rejection : int {
    NO_REJEC = 0, PERCENTILE = 1, SIGMA = 2, MAD = 3, SIGMEDIAN = 4,
    WINSORIZED = 5, LINEARFIT = 6, GESDT = 7,
    KMEDIAN = 16   // pseudo type: stack_median (median_and_mean.c:1711-1715)
};
// normalization enum, reference core/settings.h:34-40
enum Normalization : int {
    NO_NORM = 0, ADDITIVE = 1, MULTIPLICATIVE = 2, ADDITIVE_SCALING = 3,
    MULTIPLICATIVE_SCALING = 4
};

struct KParams {
    const float *frames;        // frame-major block: frames[f*frame_stride + y*W + x]
    long long frame_stride;     // elements between frames
    long long npix;             // rows * W output pixels
    int W;                      // row length
    int nframes;                // N (nb_images_to_stack)
    int rtype;                  // Rejection (or KMEDIAN)
    float sig0, sig1;           // args->sig[0..1]
    int norm;                   // Normalization
    const double *scale, *offset, *mul;   // per-frame coefficients (device) or null
    const int *shiftx;          // per-frame integer x shift (device) or null
    const double *weights;      // per-frame weights (device) or null
    const float *drizz;         // per-sample drizzle weights, layout of frames (args->drizzle), or null
    const float *mask;          // per-sample feather-mask weights, layout of frames (masking), or null
    const float *crit;          // GESD critical values (device) or null
    float m_x, m_dx2;           // LINEARFIT constants (median_and_mean.c:1487-1500)
    int output_norm;            // 0 -> clamp result to [0,1]
    float *out;                 // rows*W
    uint16_t *rej_lo, *rej_hi;  // rows*W each, or null
    unsigned long long *counts; // [2] low/high rejection totals (accumulated)
    unsigned long long *cstripe;  // striped per-wave partial totals (kCountStripes x 8, reduced into counts) or null
    int *fb_list;               // pixels deferred to the exact sequential kernel
    int *fb_count;              // number of entries in fb_list
    int *fb2_list;              // WINSORIZED moment path: pixels for the register-resident sorted kernel
    int *fb2_count;             // number of entries in fb2_list
    // WINSORIZED two-kernel moment path (stack_wz.h): pixels [wz_pix0,
    // wz_pix0 + wz_cnt) of this launch, their rank records (slot-major,
    // stride wz_cnt), window moments [2][wz_cnt] and packed bounds / routes
    long long wz_pix0, wz_cnt;
    float *wz_ranks;
    double *wz_mom;
    int *wz_meta;
    void *wz_state;             // round-wise rounds: WzState per pixel of the chunk
    int *wz_list_in, *wz_list_out;   // pixels (chunk-local) entering / leaving the round
    int *wz_lcount;             // [0]: pixels in wz_list_in, [1]: appended to wz_list_out
    void *wz_ws;                // workspace the launcher carves these from (two-kernel form), or null
    long long wz_ws_bytes;
    long long wz_chunk;         // two-kernel form: at most this many pixels per chunk (0: as the workspace allows)
    int *wz_tcnt;               // overlapped form: 2 counters per chunk (fb2, fb) + [kWzMaxChunks*2] the total
                                // of the chunks' exact-kernel pixels, or null (tails after the last chunk)
    int wz_mode;                // 0 register-resident kernel only, 1 moment path in one kernel (LDS), 2 two kernels
    int wz_rw;                  // two-kernel form: rounds kernel -- 64 ranks staged in LDS (default, N <= 128), 4 / 5 / 6 global reads at that occupancy, 100 round-wise
    float *scratch;             // fallback kernel scratch
    long long scratch_threads;  // number of fallback threads the scratch covers
    // DATA_USHORT sequences (apply_rejection_ushort path)
    const uint16_t *frames16;   // non-null: 16-bit input (frames ignored)
    uint16_t *out16;            // 16-bit output (round_to_WORD), or null
    int out_f32;                // 16-bit input: write the float output (double_ushort_to_float_range)
    double out16_mul;           // 16-bit output: result x this before round_to_WORD (normalize_to16bit:
                                // 65535/255 for BYTE_IMG input with output_norm, else 1)
    unsigned long long *prof;   // diagnostic builds (-DSGPU_PROF=1): per-section lane-cycles [16], or null
};

// most chunks of one launch whose tails run per chunk (KParams::wz_tcnt)
constexpr int kWzMaxChunks = 256;
// rejection totals: one wave per pixel group ends with one pair of atomics;
// on one address those serialise across the XCDs (hundreds of thousands of
// waves per launch), so waves add into kCountStripes pairs 64 B apart and a
// one-block kernel folds them into `counts` at the end of the launch
constexpr int kCountStripes = 1024;

}  // namespace sgpu
