/*
 * sirilgpu.h -- C-ABI of the MI355X stacking engine (libsirilgpu.so).
 *
 * Drop-in boundary for Siril's per-pixel rejection / median stack
 * (lock042/siril 1.5.0-dev).  Plain C types only: caller-owned buffers,
 * pointers + sizes, ST_*-compatible return codes.  Each entry point names
 * the reference interface it replaces; INTEGRATION.md shows the Siril-side
 * call sites.
 *
 * Threading: a context owns one HIP stream and its device workspace; calls on
 * one context must be serialised by the caller (Siril calls from its single
 * processing thread).  Different contexts may be used concurrently.
 */
#ifndef SIRILGPU_H
#define SIRILGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes: identical values to Siril's ST_* (stacking/stacking.h:18-24)
 * plus engine-specific ones below -20. */
#define SGPU_OK               0
#define SGPU_GENERIC_ERROR   (-1)   /* ST_GENERIC_ERROR */
#define SGPU_SEQUENCE_ERROR  (-2)   /* ST_SEQUENCE_ERROR */
#define SGPU_CANCEL          (-9)   /* ST_CANCEL */
#define SGPU_ALLOC_ERROR     (-10)  /* ST_ALLOC_ERROR */
#define SGPU_NO_DEVICE       (-20)  /* no HIP device / HIP runtime error */
#define SGPU_BAD_ARGUMENT    (-21)

/* rejection enum, core/settings.h:43-52 */
enum sgpu_rejection {
	SGPU_NO_REJEC = 0, SGPU_PERCENTILE = 1, SGPU_SIGMA = 2, SGPU_MAD = 3,
	SGPU_SIGMEDIAN = 4, SGPU_WINSORIZED = 5, SGPU_LINEARFIT = 6, SGPU_GESDT = 7
};
/* normalization enum, core/settings.h:34-40 */
enum sgpu_normalization {
	SGPU_NO_NORM = 0, SGPU_ADDITIVE = 1, SGPU_MULTIPLICATIVE = 2,
	SGPU_ADDITIVE_SCALING = 3, SGPU_MULTIPLICATIVE_SCALING = 4
};
/* stack methods: stack_mean_with_rejection / stack_median
 * (stacking/median_and_mean.c:1103-1109) */
enum sgpu_method { SGPU_METHOD_MEAN = 0, SGPU_METHOD_MEDIAN = 1 };

/* ABI version of this header.  Bumped whenever an existing entry point's
 * signature or a struct layout changes (3: sgpu_rl_fft / sgpu_rl_naive and
 * their _device variants take `lambda` before maxiter, as the reference's
 * fft_richardson_lucy does).  A caller compiled against this header checks
 * sgpu_abi_version() == SGPU_ABI_VERSION before its first call. */
#define SGPU_ABI_VERSION 4
int sgpu_abi_version(void);

typedef struct sgpu_context sgpu_context;

/* Parameters of one stack call: the fields of struct stacking_args
 * (stacking/stacking.h:65-117) the per-pixel loop reads. */
typedef struct {
	int method;                 /* enum sgpu_method */
	int type_of_rejection;      /* enum sgpu_rejection (args->type_of_rejection) */
	float sig[2];               /* args->sig: low/high sigma, percentiles, or GESD (max outlier fraction, alpha) */
	int normalize;              /* enum sgpu_normalization (args->normalize) */
	const double *scale;        /* args->coeff.pscale[layer], nframes entries, or NULL */
	const double *offset;       /* args->coeff.poffset[layer], or NULL */
	const double *mul;          /* args->coeff.pmul[layer], or NULL */
	const int *shiftx;          /* per-frame x shift round_to_int(dx*scale) (median_and_mean.c:1618-1622), or NULL */
	const double *weights;      /* args->weights + layer*nframes, or NULL (unweighted) */
	const float *critical_value;/* GESD critical values, floor(nframes*sig[0]) entries (median_and_mean.c:1477-1484) */
	int output_norm;            /* args->output_norm: 0 -> clamp result to [0,1] */
} sgpu_stack_params;

/* ---- context ------------------------------------------------------------ */

/* Number of HIP devices visible (0 when none). */
int sgpu_device_count(void);

/* Create a context on `device` with its own HIP stream. */
int sgpu_init(int device, sgpu_context **ctx);

/* Destroy a context (frees its device workspace and stream). */
void sgpu_release(sgpu_context *ctx);

/* Use an external HIP stream (hipStream_t cast to void*) for subsequent
 * calls; NULL is the device's null (default) stream.  Until the first call
 * the context works on its own non-blocking stream. */
int sgpu_set_stream(sgpu_context *ctx, void *hip_stream);

/* Wait for all work queued on the context's stream. */
int sgpu_synchronize(sgpu_context *ctx);

/* Human-readable description of the last error on this thread. */
const char *sgpu_last_error(void);

/* ---- rejection / median stack ------------------------------------------- */

/* Host-buffer drop-in for the per-pixel loop of stack_mean_or_median
 * (stacking/median_and_mean.c:1592-1737) over one block of rows: replaces
 * the OpenMP block loop at :1551-1760 for DATA_FLOAT sequences.
 *   frames[f*frame_stride + y*width + x], f < nframes, y < rows (host memory,
 *   y-shift and zero fill already applied by the block reader, as
 *   stack_read_block_data does);
 *   out[y*width + x]: mean_and_reject() (method MEAN) or quickmedian_float()
 *   (method MEDIAN), clamped to [0,1] unless output_norm;
 *   rej_lo/rej_hi (may be NULL): per-pixel rejection counts, truncated to u16;
 *   counts[2] (may be NULL): low/high rejection totals, accumulated.
 * Rows are returned in input order (the caller writes row y at H-1-y as :1597
 * does).  Synchronous. */
int sgpu_stack_rows(sgpu_context *ctx, const float *frames, int nframes, long width,
		long rows, long frame_stride, const sgpu_stack_params *params, float *out,
		uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]);

/* Same computation with every array already resident in device memory
 * (frames, out, rej_lo, rej_hi, d_counts: device pointers; d_counts is two
 * uint64 accumulated on the device).  The per-frame arrays in `params` are
 * HOST pointers (copied internally).  Asynchronous on the context stream. */
int sgpu_stack_rows_device(sgpu_context *ctx, const float *d_frames, int nframes, long width,
		long rows, long frame_stride, const sgpu_stack_params *params, float *d_out,
		uint16_t *d_rej_lo, uint16_t *d_rej_hi, uint64_t *d_counts);

/* DATA_USHORT sequences (16-bit FITS/SER): apply_rejection_ushort and the
 * ushort branch of mean_and_reject (median_and_mean.c:703-1036), the 16-bit
 * twin of the float path.  frames16[f*frame_stride + y*width + x].
 * use_32bit_output != 0: out_f32 receives (float)result/65535 clamped to
 * [0,1] unless output_norm (double_ushort_to_float_range, :1720-1723);
 * otherwise out_u16 receives round_to_WORD(result) (:1729-1733).  Either
 * output pointer may be NULL.  Synchronous. */
int sgpu_stack_rows_u16(sgpu_context *ctx, const uint16_t *frames16, int nframes, long width,
		long rows, long frame_stride, const sgpu_stack_params *params, float *out_f32,
		uint16_t *out_u16, uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]);

/* Device-resident variant of sgpu_stack_rows_u16 (asynchronous). */
int sgpu_stack_rows_u16_device(sgpu_context *ctx, const uint16_t *d_frames16, int nframes,
		long width, long rows, long frame_stride, const sgpu_stack_params *params,
		float *d_out_f32, uint16_t *d_out_u16, uint16_t *d_rej_lo, uint16_t *d_rej_hi,
		uint64_t *d_counts);

/* Per-sample weight planes of the block (the rest of the per-pixel loop's
 * inputs, median_and_mean.c:1687-1692): drizz = data->drizz (args->drizzle,
 * the drizzle weights read with the frames), mask = data->mask (feather
 * masking, args->feather_dist > 0, the ramped mask values), both frame-major
 * with the frames' layout and stride, either may be NULL.  A sample whose
 * drizzle weight is 0 is removed like a null pixel (rejection_float.c:117-126,
 * median_and_mean.c:716-731), and the mean is the weighted branch of
 * mean_and_reject with n = drizzle * mask * frame weight (:1043-1082, the
 * ushort twin :967-1021).  Ignored by the median stack.  The reference's
 * readers of the weight files (drizztmp / .msk caches) stay on the host. */
int sgpu_stack_rows_planes(sgpu_context *ctx, const float *frames, const float *drizz, const float *mask,
		int nframes, long width, long rows, long frame_stride, const sgpu_stack_params *params, float *out,
		uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]);
int sgpu_stack_rows_planes_device(sgpu_context *ctx, const float *d_frames, const float *d_drizz,
		const float *d_mask, int nframes, long width, long rows, long frame_stride,
		const sgpu_stack_params *params, float *d_out, uint16_t *d_rej_lo, uint16_t *d_rej_hi,
		uint64_t *d_counts);
int sgpu_stack_rows_u16_planes_device(sgpu_context *ctx, const uint16_t *d_frames16, const float *d_drizz,
		const float *d_mask, int nframes, long width, long rows, long frame_stride,
		const sgpu_stack_params *params, float *d_out_f32, uint16_t *d_out_u16, uint16_t *d_rej_lo,
		uint16_t *d_rej_hi, uint64_t *d_counts);

/* Feathering masks (`stack ... -feather=<dist>`).
 *
 * sgpu_stack_blocks: Siril's row-block plan, stack_compute_parallel_blocks
 * (stacking/median_and_mean.c:295-356, refine_blocks_candidate :261-283):
 * nb_threads threads, max_rows rows of all frames in memory, an image of
 * `height` rows and `channels` layers.  *nb_blocks receives the block count
 * (also when cap is too small: SGPU_BAD_ARGUMENT); start_row / block_height /
 * channel (cap entries each) the blocks in the reference's internal row order
 * (row s is FITS row height - 1 - s); *largest (may be NULL) the tallest.
 * Host code, no device needed.
 *
 * sgpu_feather_mask_size: (int)(0.1 w) x (int)(0.1 h), the downscaled mask
 * (compute_downscaled_mask_size, blending.c:52-59).
 *
 * sgpu_feather_masks_device: compute_mask_image_hook + cvDownscaleBlendMask
 * (blending.c:131-191, opencv/opencv.cpp:587-609) for nframes frames of one
 * layer (the green layer of colour frames, else the only one), float
 * (elem_size 4: non-zero samples) or uint16 (2: samples > 0), FITS row order,
 * d_frames[f*frame_stride + y*width + x]: d_masks[f][mh][mw] receives the
 * distances to black of the 7x7-closed, linearly downscaled 0/255 image (the
 * .msk cache file's content, FITS row order).  Synchronous.
 *
 * sgpu_feather_block_area: for one frame and one block (start_row,
 * block_height in the reference's internal rows), the area logic of
 * stack_read_block_data (:406-446, 483-499) with the frame's y shift
 * (area.y = start_row + shifty; registered = 0: no registration data):
 * *plane_row = first block row written (the reader's offset), *area_h rows
 * from downscaled rows [*mask_row, *mask_row + *mask_h) (0 rows: the frame
 * contributes zeros).  Host code.
 *
 * sgpu_feather_block_device: the block's mask planes, data->mask of
 * stack_read_block_data: per frame cvUpscaleBlendMask (opencv.cpp:611-616,
 * float INTER_LINEAR to area_h x width, vertical flip) of the area's
 * downscaled rows, zero outside the area, then `d > feather ? 1 :
 * ramp(d / feather)` for d != 0 (init_ramp, blending.c:34-50).  shifty: the
 * reference's per-frame y shifts (NULL: no registration); placex: canvas
 * column of each frame's column 0 (-maximize, rearrange_block_data; NULL: 0);
 * d_planes[f*plane_stride + r*canvas_width + x], r in FITS order
 * (fits_order = 1: block row r is the reference's internal row
 * block_height - 1 - r) or in the reference's internal order (0).
 * Synchronous.  The planes feed sgpu_stack_rows*_planes_device as `mask`.
 *
 * The upscaled rows of a frame depend on where its blocks start and end:
 * a stack matches Siril's only over the same block plan.  Resize and
 * distance-transform arithmetic restates OpenCV's generic code (OpenCV is
 * not available here: parity with Siril's binary is unpinned). */
int sgpu_stack_blocks(long max_rows, long height, long channels, int nb_threads, int cap,
		long *start_row, long *block_height, int *channel, int *nb_blocks, long *largest);
void sgpu_feather_mask_size(long width, long height, long *mask_width, long *mask_height);
int sgpu_feather_masks_device(sgpu_context *ctx, const void *d_frames, int elem_size, int nframes,
		long width, long height, long frame_stride, float *d_masks);
int sgpu_feather_block_area(long width, long height, long start_row, long block_height, int shifty,
		int registered, int *plane_row, int *area_h, int *mask_row, int *mask_h);
int sgpu_feather_block_device(sgpu_context *ctx, const float *d_masks, int nframes, long width,
		long height, long start_row, long block_height, const int *shifty, const int *placex,
		long canvas_width, float feather, int fits_order, float *d_planes, long plane_stride);

/* Sample type of the sequence's files (seq->bitpix / stack_open_all_files'
 * bitpix): 8 = BYTE_IMG, 16, -32, 0 = unknown (default).  With 8 and
 * params->output_norm, the 16-bit outputs (out_u16) of the DATA_USHORT stack
 * calls are scaled by 65535/255 before round_to_WORD, as normalize_to16bit
 * does (stacking/median_and_mean.c:547-555, 1729-1732). */
int sgpu_set_input_bitpix(sgpu_context *ctx, int bitpix);

/* Diagnostics of the last stack call on this context: number of pixels that
 * were resolved by the exact sequential kernel (order-dependent cutoff,
 * NaN/Inf columns, kept==0, MAD, or N beyond the sorted-path capacity).
 * Synchronises the context stream. */
long sgpu_last_exact_pixels(sgpu_context *ctx);

/* Float NO_REJEC mean (last launch of the last stack call, <= 2^28 pixels):
 * the number of pixels whose float mean the kernel could not prove to be
 * independent of the summation order.  The reference sums kept >= 16 samples
 * with `#pragma omp simd reduction(+:sum)` (stacking/median_and_mean.c:
 * 1083-1090), an order fixed by its build; every other pixel's mean is the
 * same float in every order (exact f64 sum, or float-stable against the
 * order-error bound).  The listed pixels carry the sequential order's value
 * (the scalar branch, :1091-1094).  Copies up to `cap` launch-relative pixel
 * indices into `idx` (may be NULL).  Synchronises the context stream. */
long sgpu_last_order_sensitive(sgpu_context *ctx, int *idx, long cap);

/* Force every pixel through the exact sequential kernels (1), through the
 * one-wave-per-pixel exact kernel where it applies (2: float SIGMA,
 * WINSORIZED, PERCENTILE and median stacks of 33..1024 frames; the others as
 * 1), or use the sorted fast path with exact fallback (0, default).  The
 * deferred pixels of those types already take the wave kernel.  Test hook. */
int sgpu_set_exact_only(sgpu_context *ctx, int on);

/* ---- several GPUs of one node ------------------------------------------- */

/* A handle over contexts on several devices (devices[i] may repeat).  Replaces
 * the OpenMP block loop of stack_mean_or_median (median_and_mean.c:1551-1760)
 * for a whole block of rows at once: the rows are split into contiguous
 * balanced bands (sgpu_row_bands), band d is stacked on devices[d] by its own
 * host thread (sgpu_stack_rows), written straight into the caller's out /
 * rej_lo / rej_hi rows (host gather) and the counters are summed.  Same
 * arguments and results as sgpu_stack_rows / sgpu_stack_rows_u16.
 * Synchronous.  For frames already resident in HBM on each device use the
 * per-device contexts (sgpu_multi_context) and RCCL (siril_amd.distributed). */
typedef struct sgpu_multi sgpu_multi;
int sgpu_multi_init(const int *devices, int ndevices, sgpu_multi **multi);
void sgpu_multi_release(sgpu_multi *multi);
int sgpu_multi_size(const sgpu_multi *multi);
sgpu_context *sgpu_multi_context(sgpu_multi *multi, int index);
int sgpu_multi_stack_rows(sgpu_multi *multi, const float *frames, int nframes, long width, long rows,
		long frame_stride, const sgpu_stack_params *params, float *out, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2]);
int sgpu_multi_stack_rows_u16(sgpu_multi *multi, const uint16_t *frames16, int nframes, long width,
		long rows, long frame_stride, const sgpu_stack_params *params, float *out_f32,
		uint16_t *out_u16, uint16_t *rej_lo, uint16_t *rej_hi, uint64_t counts[2]);
/* Frame-sharded no-rejection mean (the north star's "partial-sum /
 * partial-count" multi-GPU split; exact for the unweighted NO_REJEC mean,
 * median_and_mean.c:1083-1097): each rank accumulates, in frame order, the
 * f64 sum and the count of the present (non-zero) samples of its frames
 * (d_frames[f*frame_stride + y*width + x], f < nframes, params' per-frame
 * arrays for those frames) INTO d_sum / d_count (rows*width each); after an
 * all-reduce of both, sgpu_mean_finish_device writes sum/count (0 where no
 * sample is present, Siril's quickmedian of an all-zero column), clamped to
 * [0, 1] unless output_norm.  Bit-identical to the single-device mean
 * whenever the f64 sums are exact (samples within a 2^29 dynamic range).
 * Rejection and the median need whole columns: frame-sharded input goes
 * through an all-to-all transpose to row bands instead
 * (siril_amd.distributed.stack_frame_sharded).  Asynchronous. */
int sgpu_mean_partial_device(sgpu_context *ctx, const float *d_frames, int nframes, long width, long rows,
		long frame_stride, const sgpu_stack_params *params, double *d_sum, int *d_count);
int sgpu_mean_finish_device(sgpu_context *ctx, const double *d_sum, const int *d_count, long npix,
		float *d_out, int output_norm);
/* The guarded forms: the partial pass also folds min |x| and max |x| of the
 * present samples into d_amin / d_amax (initialise to +inf / 0; all-reduce
 * with MIN / MAX across ranks), and the finish writes d_flag[i] = 1 where the
 * f64 sums are not provably exact in every order (ceil(log2 count) +
 * e(max|x|) - e(min|x|) + 24 > 53): those pixels' means depend on the
 * summation order, and the caller recomputes them in frame order from their
 * columns (sgpu_gather_columns_device + an all-gather), as
 * siril_amd.distributed.stack_frame_sharded does.  Asynchronous. */
int sgpu_mean_partial_guard_device(sgpu_context *ctx, const float *d_frames, int nframes, long width, long rows,
		long frame_stride, const sgpu_stack_params *params, double *d_sum, int *d_count, float *d_amin,
		float *d_amax);
int sgpu_mean_finish_guard_device(sgpu_context *ctx, const double *d_sum, const int *d_count,
		const float *d_amin, const float *d_amax, long npix, float *d_out, int output_norm,
		unsigned char *d_flag);
/* The shifted, normalized samples (as the stack gathers them,
 * median_and_mean.c:1615-1686) of the k pixels d_idx[j] of the block:
 * d_out[f*k + j], f < nframes.  Asynchronous. */
int sgpu_gather_columns_device(sgpu_context *ctx, const float *d_frames, int nframes, long width, long rows,
		long frame_stride, const sgpu_stack_params *params, const long long *d_idx, long long k,
		float *d_out);
/* Band partition: starts[0..nparts], band r = rows [starts[r], starts[r+1]);
 * the first rows % nparts bands get one extra row.  Host only. */
int sgpu_row_bands(long rows, int nparts, long *starts);

/* ---- DFT cross-correlation registration -------------------------------- */

/* register_shift_dft (registration/shift_methods.c:60-321) on square S x S
 * selections: for every frame, the integer translation maximising the
 * (unnormalised) cross-correlation with the reference, computed as
 * IFFT2(FFT2(ref) . conj(FFT2(img))), first strict maximum of the real part in
 * row-major order, wrapped to (-S/2, S/2] (:259-273).  The caller turns
 * (shiftx, shifty) into the registration matrix with set_shifts()
 * (io/sequence.c:1863-1868).  S in [2, 8192] with prime factors <= 61.
 *   ref, frames[f]: host arrays of S*S floats (the selection, row-major). */
int sgpu_dft_shifts(sgpu_context *ctx, const float *ref, const float *const *frames, int nframes,
		int size, int *shiftx, int *shifty);

/* Device-resident variant: the selection of frame f starts at
 * d_frames + f*frame_stride, rows row_stride floats apart (so a centred
 * window of full frames in HBM needs no copy).  d_shifts receives
 * (shiftx, shifty) pairs; d_peaks (may be NULL) the correlation maxima.
 * Asynchronous on the context stream. */
int sgpu_dft_register_device(sgpu_context *ctx, const float *d_ref, long ref_row_stride,
		const float *d_frames, long row_stride, long frame_stride, int nframes, int size,
		int *d_shifts, float *d_peaks);

/* Frame quality of register_shift_dft (registration/shift_methods.c:176,234):
 * QualityEstimate_float (algos/quality_float.c:41-147) of each width x height
 * float image (the S x S selection; frame f at d_frames + f*frame_stride,
 * rows row_stride apart).  quality[f] = sqrt(sum over levels), unnormalised;
 * the f64 gradient sums are reduced in a fixed order of their own (the
 * reference's is row-major), so results agree to rounding.  Synchronous. */
int sgpu_quality_estimate_device(sgpu_context *ctx, const float *d_frames, int nframes, int width,
		int height, long row_stride, long frame_stride, double *quality);
int sgpu_quality_estimate(sgpu_context *ctx, const float *frames, int nframes, int width, int height,
		double *quality);
/* DATA_USHORT frames: QualityEstimate_ushort (algos/quality.c:49-276, the
 * branch QualityEstimate takes for 16-bit fits, :39-45): WORD subsample,
 * the running top-6 histogram stretch, integer smoothing, THRESHOLD_USHRT;
 * bit-exact gradient sums (integers).  Synchronous. */
int sgpu_quality_estimate_u16_device(sgpu_context *ctx, const uint16_t *d_frames, int nframes, int width,
		int height, long row_stride, long frame_stride, double *quality);
int sgpu_quality_estimate_u16(sgpu_context *ctx, const uint16_t *frames, int nframes, int width, int height,
		double *quality);
/* normalizeQualityData (shift_methods.c:36-54), in place. */
void sgpu_normalize_quality(double *quality, int n, double q_min, double q_max);

/* ---- Richardson-Lucy deconvolution -------------------------------------- */

/* Drop-in for fft_richardson_lucy / naive_richardson_lucy
 * (filters/deconvolution/deconvolution.h:138-139, deconvolve.cpp:56-114), same
 * arguments and return values: planar fdata (nchans planes of rx*ry floats)
 * deconvolved in place with the ks x ks (odd) kernel plane min(c, kchans-1);
 * returns 0, or 1 if a channel's maximum is 0 (earlier channels are already
 * written, as in the reference).  Runs on a process-wide context on device 0.
 * regtype: any regtype_t (deconvolution.h:39): REG_TV_GRAD 0, REG_FH_GRAD 1,
 * REG_NONE_GRAD 2, REG_TV_MULT 3, REG_FH_MULT 4, REG_NONE_MULT 5; the TV / FH
 * weights (deconvolve.hpp:104-126, 199-222) use reallambda = 1 / (2 / lambda)
 * as deconvolve.cpp passes it.  The FFT path's blur is the reference's
 * circular convolution over each slice, computed as the linear convolution of
 * the slice's periodic extension through the engine's own LDS FFTs on
 * 2-3-5-smooth lengths (rl_fft.hip; equal up to rounding; SGPU_RL_DIRECT=1
 * selects a direct convolution on the matrix cores instead); the naive path
 * keeps the reference's zero-border correlation (direct, on the matrix
 * cores). */
int sgpu_fft_richardson_lucy(float *fdata, unsigned rx, unsigned ry, unsigned nchans, float *kernel,
		int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int max_threads, int regtype, float stepsize, int stopcriterion_active);
int sgpu_naive_richardson_lucy(float *fdata, unsigned rx, unsigned ry, unsigned nchans, float *kernel,
		int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int max_threads, int regtype, float stepsize, int stopcriterion_active);

/* Same on an explicit context; host buffers (copied to and from HBM). */
int sgpu_rl_fft(sgpu_context *ctx, float *fdata, unsigned rx, unsigned ry, unsigned nchans,
		const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int regtype, float stepsize, int stopcriterion_active);
int sgpu_rl_naive(sgpu_context *ctx, float *fdata, unsigned rx, unsigned ry, unsigned nchans,
		const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int regtype, float stepsize, int stopcriterion_active);

/* Device-resident variants: d_fdata in HBM (kernel stays a host array).
 * Synchronous (returns when the result is in d_fdata). */
int sgpu_rl_fft_device(sgpu_context *ctx, float *d_fdata, unsigned rx, unsigned ry, unsigned nchans,
		const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int regtype, float stepsize, int stopcriterion_active);
int sgpu_rl_naive_device(sgpu_context *ctx, float *d_fdata, unsigned rx, unsigned ry, unsigned nchans,
		const float *kernel, int kernelsize, unsigned kchans, float lambda, int maxiter, float stopcriterion,
		int regtype, float stepsize, int stopcriterion_active);

/* Memory budget M of the slice geometry (process_in_slices(M, ...),
 * image.hpp:404-421; the reference passes get_available_memory()).
 * Default 2^40 bytes: the large-RAM geometry. */
int sgpu_rl_set_memory(sgpu_context *ctx, size_t bytes);

/* Benchmarks: number of direct-convolution launches of the last RL call,
 * the algorithmic flops (2 * ks^2 per pixel per convolution) of its
 * iteration loops, its FFT convolutions and their algorithmic HBM bytes
 * (the FFT path convolves through rl_fft.hip unless SGPU_RL_DIRECT=1 or the
 * extended slice exceeds 8192 samples a side; the naive path is always
 * direct).  With sgpu_set_timing on, sgpu_last_timing() returns ms[0] = time
 * of the iteration loops, ms[1] = slice extraction + edge taper. */
long sgpu_rl_last_conv_launches(sgpu_context *ctx);
double sgpu_rl_last_iter_flops(sgpu_context *ctx);
long sgpu_rl_last_fft_convs(sgpu_context *ctx);
double sgpu_rl_last_iter_bytes(sgpu_context *ctx);

/* CFA sequences (nb_layers == 1): register_shift_dft first runs
 * interpolate_nongreen on each selection (shift_methods.c:115-117,214-215;
 * io/image_format_fits.c:4319-4349).  Same as above with the compiled CFA
 * pattern of the selection (get_compiled_pattern, algos/demosaicing.c:327:
 * cfa_dim 2 (Bayer; X-Trans is refused), cfa_pattern[4] with 0 = R, 1 = G, 2 = B); the
 * interpolation is fused into the first FFT pass (frames are not modified).
 * cfa_pattern NULL / cfa_dim 0 = no CFA. */
int sgpu_dft_shifts_cfa(sgpu_context *ctx, const float *ref, const float *const *frames, int nframes,
		int size, const unsigned char *cfa_pattern, int cfa_dim, int *shiftx, int *shifty);
int sgpu_dft_register_cfa_device(sgpu_context *ctx, const float *d_ref, long ref_row_stride,
		const float *d_frames, long row_stride, long frame_stride, int nframes, int size,
		const unsigned char *cfa_pattern, int cfa_dim, int *d_shifts, float *d_peaks);

/* DATA_USHORT sequences: register_shift_dft reads WORD selections, runs
 * interpolate_nongreen_ushort on CFA frames (io/image_format_fits.c:4351-4381:
 * the float weighted mean stored back with roundf_to_WORD) and transforms
 * (float)data (shift_methods.c:166-169).  Same shifts contract as the float
 * entry points; WORD selections (d_ref / d_frames: uint16_t). */
int sgpu_dft_register_u16_device(sgpu_context *ctx, const uint16_t *d_ref, long ref_row_stride,
		const uint16_t *d_frames, long row_stride, long frame_stride, int nframes, int size,
		const unsigned char *cfa_pattern, int cfa_dim, int *d_shifts, float *d_peaks);
int sgpu_dft_shifts_u16(sgpu_context *ctx, const uint16_t *ref, const uint16_t *const *frames, int nframes,
		int size, const unsigned char *cfa_pattern, int cfa_dim, int *shiftx, int *shifty);
/* interpolate_nongreen_ushort in place on a device WORD image (the CFA
 * frame QualityEstimate then reads).  Asynchronous. */
int sgpu_interpolate_nongreen_u16_device(sgpu_context *ctx, uint16_t *d_img, int width, int height,
		long row_stride, const unsigned char *cfa_pattern, int cfa_dim);

/* interpolate_nongreen_float (io/image_format_fits.c:4319-4349) in place on a
 * device image (width x height, rows row_stride floats apart). Asynchronous. */
int sgpu_interpolate_nongreen_device(sgpu_context *ctx, float *d_img, int width, int height,
		long row_stride, const unsigned char *cfa_pattern, int cfa_dim);

/* ---- applying the registration ------------------------ */

/* Integer shifts of apply_reg with interpolation "none" (applyreg.c:653-660 ->
 * shift_fit_from_reg, registration.c:322-370) from the layer's homographies:
 * H = Href^-1 * Himg (cvTransfH, opencv.cpp:385-396), for translations
 * shiftx = round_to_int(h02 - h02[ref]), shifty = round_to_int(-(h12 - h12[ref])).
 * Host only. */
int sgpu_apply_reg_shifts(int nframes, const double *h02, const double *h12, int ref_index, int *shiftx,
		int *shifty);
/* shift_fit_from_reg on nframes device frames (elem_size 4: float, 2: WORD),
 * frame f at d_in + f*frame_stride elements, rows in Siril's (bottom-up =
 * FITS) order: out[x + shiftx[f], y + shifty[f]] = in[x, y], zero elsewhere.
 * d_out must not alias d_in.  shiftx/shifty are host arrays.  Synchronous. */
int sgpu_shift_frames_device(sgpu_context *ctx, const void *d_in, void *d_out, int elem_size, int nframes,
		int width, int height, long frame_stride, const int *shiftx, const int *shifty);

/* apply_reg_image_hook (registration/applyreg.c:388-660) for the translation
 * registrations REG_DFT stores, scale 1, FRAMING_CURRENT: H (9 doubles per
 * frame, h00..h22) composed with the reference image's (cvTransfH); the
 * interpolation (OPENCV_NEAREST 0, LINEAR 1, CUBIC 2, AREA 3, LANCZOS4 4,
 * NONE 5; core/siril.h:333-340) -- NONE: shift_fit_from_reg's rounded
 * shift; 0-4: cvTransformImage, which for an integer translation samples
 * every kernel at phase 0, i.e. the same exact shift.  Homographies other
 * than translations, and sub-pixel translations with 0-4, return
 * SGPU_BAD_ARGUMENT.  Frames as sgpu_shift_frames_device.  Synchronous. */
int sgpu_apply_reg_device(sgpu_context *ctx, const void *d_in, void *d_out, int elem_size, int nframes,
		int width, int height, long frame_stride, const double *H, int ref_index, int interpolation);

/* ---- CFA helpers -------------------------------------- */

/* extract_CFA_buffer_float (algos/demosaicing.c:936-975) on a device image:
 * the samples whose compiled-pattern colour (get_compiled_pattern: pattern
 * [pattern_size * pattern_size], 0 = R, 1 = G, 2 = B; pattern_size 2 Bayer or
 * 6 X-Trans) equals `layer`, in raster order, compacted into d_out
 * (sgpu_cfa_count elements, returned in *newsize).  elem_size 4 (float) or 2
 * (WORD, extract_CFA_buffer_ushort).  Asynchronous. */
int sgpu_extract_cfa_device(sgpu_context *ctx, const void *d_in, int elem_size, int width, int height,
		const unsigned char *pattern, int pattern_size, int layer, void *d_out, long *newsize);
/* Number of samples extract_CFA_buffer returns; -1 on bad arguments.  Host only. */
long sgpu_cfa_count(int width, int height, const unsigned char *pattern, int pattern_size, int layer);
/* split_cfa_float / split_cfa_ushort (algos/extraction.c:914-1050): the four
 * (width/2) x (height/2) sub-planes CFA0..CFA3 = (0,0), (1,0), (0,1), (1,1) of
 * every 2x2 cell.  Asynchronous. */
int sgpu_split_cfa_device(sgpu_context *ctx, const void *d_in, int elem_size, int width, int height,
		void *d_cfa0, void *d_cfa1, void *d_cfa2, void *d_cfa3);
/* merge_cfa (algos/demosaicing.c:757-840): the inverse, a (2*width2) x
 * (2*height2) mosaic from the four sub-planes.  Asynchronous. */
int sgpu_merge_cfa_device(sgpu_context *ctx, const void *d_cfa0, const void *d_cfa1, const void *d_cfa2,
		const void *d_cfa3, int elem_size, int width2, int height2, void *d_out);

/* ---- CFA demosaic ------------------------------------------------------- */

/* Drop-in for debayer_buffer_new_float (algos/demosaicing.h,
 * demosaicing_rtp.cpp:228-390): min/max normalisation of the mono CFA buffer
 * to [0, 65535], demosaic, `v * invfactor + min` back; returns a malloc'd
 * planar RGB buffer (3 * width * height floats, free() it) or NULL (min == max,
 * unsupported method).  interpolation: interpolation_method
 * (core/settings.h:68-79): BAYER_RCD (8, and unknown values, as the
 * reference's `default:`) -> rcd_demosaic, restated from the published RCD
 * 2.3 algorithm; BAYER_BILINEAR (0) -> bayerfast_demosaic (:147-151,
 * 318-323; what io/ser.c:1177-1182 forces for every colour SER frame),
 * restated from RawTherapee's fast_demosaic (librtprocess is not vendored:
 * parity with it is unpinned for both; oracle/demosaic_ref.py).
 * pattern: sensor_pattern 0..3 (RGGB, BGGR, GBRG, GRBG); xtrans is ignored.
 * `buf` is not modified (the reference leaves it normalised). */
float *sgpu_debayer_buffer_new_float(float *buf, int *width, int *height, int interpolation,
		int pattern, unsigned int xtrans[6][6]);

/* Drop-in for debayer_buffer_new_ushort (algos/demosaicing.h,
 * demosaicing_rtp.cpp:74-224): the raw WORD values go to the demosaic as
 * float without normalisation and every output sample is rounded with
 * roundf_to_WORD (roundf_to_BYTE when bit_depth == 8, BYTE_IMG; core/proto.h
 * :256-261,341-346).  Returns a malloc'd planar RGB buffer of 3 * width *
 * height WORDs (free() it) or NULL.  Same interpolation / pattern rules as
 * the float variant. */
uint16_t *sgpu_debayer_buffer_new_ushort(uint16_t *buf, int *width, int *height, int interpolation,
		int pattern, unsigned int xtrans[6][6], int bit_depth);

/* Siril's own bayer_Bilinear (algos/demosaicing_siril.c:203-288, OpenCV's
 * integer Bayer decoder, used by debayer_buffer_siril :737-790 only when
 * USE_SIRIL_DEBAYER, which the shipped build leaves off: the shipped
 * BAYER_BILINEAR is bayerfast, through sgpu_debayer_buffer_new_float /
 * _ushort above).  This restates it, bit for bit, for DATA_USHORT
 * CFA frames: planar WORD RGB (debayer_ushort's RGBRGB -> RRGGBB loop,
 * :846-855, truncate_to_BYTE when bit_depth == 8), the 1-pixel frame 0.
 * interpolation must be BAYER_BILINEAR (0).  Returns a malloc'd buffer of
 * 3 * width * height WORDs (free() it) or NULL. */
uint16_t *sgpu_debayer_buffer_siril_ushort(uint16_t *buf, int *width, int *height, int interpolation,
		int pattern, int bit_depth);
int sgpu_debayer_siril_u16_device(sgpu_context *ctx, const uint16_t *d_buf, int width, int height,
		int interpolation, int pattern, int bit_depth, uint16_t *d_rgb);

/* debayer_buffer_superpixel_float (algos/demosaicing_siril.c:806-820):
 * interleaved RGB of (w/2 + w%2) x (h/2 + h%2), width/height updated. */
float *sgpu_debayer_buffer_superpixel_float(float *buf, int *width, int *height, int pattern);

/* Device variants: d_rgb is planar 3 x height x width; the super-pixel output
 * interleaved.  sgpu_debayer_device synchronises once, after the demosaic
 * launch (the min == max test), and returns SGPU_GENERIC_ERROR when min ==
 * max (d_rgb's contents are then unspecified). */
int sgpu_debayer_device(sgpu_context *ctx, const float *d_buf, int width, int height,
		int interpolation, int pattern, float *d_rgb);
int sgpu_superpixel_device(sgpu_context *ctx, const float *d_buf, int width, int height,
		int pattern, float *d_out);
/* 16-bit variant (no synchronisation, no min == max failure: the 16-bit
 * wrapper does not normalise); d_rgb is planar 3 x height x width WORDs. */
int sgpu_debayer_u16_device(sgpu_context *ctx, const uint16_t *d_buf, int width, int height,
		int interpolation, int pattern, int bit_depth, uint16_t *d_rgb);

/* free() for buffers returned by this library. */
void sgpu_free(void *p);

/* Kernel timing (benchmarks): when on, the context records HIP events on its
 * stream around the main stack kernel (sorted / mean path) and the exact
 * kernel of every launch; sgpu_last_timing() synchronises and returns the
 * summed milliseconds of the last stack call: ms[0] main kernel(s),
 * ms[1] exact kernel(s). */
int sgpu_set_timing(sgpu_context *ctx, int on);
int sgpu_last_timing(sgpu_context *ctx, float ms[2]);

/* ---- headless sequence stacking (scripting path) ------------------------ */

/* `stack <seq> ...`: replaces stack_one_seq -> main_stack ->
 * stack_mean_or_median (command.c:11729, stacking.c:76, median_and_mean.c:1261)
 * including its block reader stack_read_block_data (:382-545).  Reads the .seq
 * file (io/seqfile.c:84-500; S, T, L, I and R<layer> lines) of a regular FITS
 * sequence (<name><%0{fixed}d>.fit), a FITSEQ (TF: every image HDU of
 * <name>.fit) or a SER file (TS: <name>.ser; 8/16-bit, mono, CFA read as mono,
 * RGB/BGR), frames of 1 or 3 layers (FITS BITPIX -32; 16 or 8 -> the
 * DATA_USHORT path).  Float FITS holding ADU values are brought to [0, 1] as
 * Siril's partial reader does.  The registration of the first layer with
 * data (dx = h02 on the device, dy = -h12 in the reader, zero fill) is applied
 * when use_registration; row blocks of at most max_block_bytes (<= 0: 512 MiB)
 * per buffer are stacked on the GPU per layer while the next block is read;
 * out_path gets BITPIX -32 (float input or use_32bit_output; then
 * norm_to_0_1_range when params->output_norm) or 16, NAXIS3 = layers.
 * params->shiftx, when set, overrides the registration x shifts.
 * counts[2] (may be NULL) receives the rejection totals of all layers.
 * sgpu_stack_seq, _ex and _ex2 stack the .seq's INCLUDED frames (the
 * -filter-incl selection of sgpu_stack_seq_opts), so per-frame arrays in
 * params (weights, scale/offset/mul, shiftx, GESD critical values) are sized
 * for that count; sgpu_stack_seq_opts without filter_included stacks every
 * frame, as the reference's `stack` command does.
 * Returns ST_*. */
int sgpu_stack_seq(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
		int use_registration, int use_32bit_output, const char *out_path, uint64_t counts[2],
		long max_block_bytes);
/* sgpu_stack_seq with the -fastnorm flag (args->lite_norm): when
 * params->normalize != SGPU_NO_NORM and params carries no scale/offset/mul
 * arrays, the coefficients are computed first, per layer, as do_normalization
 * does (stacking/normalization.c:44-78): per-frame estimators on the GPU
 * (sgpu_norm_stats, STATS_NORM or, with lite_norm, STATS_LITENORM) and
 * sgpu_norm_factors relative to the sequence's reference image
 * (sequence_find_refimage, io/sequence.c:1791-1846).  sgpu_stack_seq ==
 * lite_norm 0. */
int sgpu_stack_seq_ex(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
		int use_registration, int use_32bit_output, const char *out_path, uint64_t counts[2],
		long max_block_bytes, int lite_norm);
/* ... and the -rejmap (rejmaps 1: one "<out>_low+high_rejmap.fit") or -rejmaps
 * (2: "<out>_low_rejmap.fit" and "<out>_high_rejmap.fit") outputs of
 * command.c:11592-11602,11778-11803: per-pixel rejection counts * (1.0f / N)
 * as float images (ignored without rejection, as the reference does). */
int sgpu_stack_seq_ex2(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
		int use_registration, int use_32bit_output, const char *out_path, uint64_t counts[2],
		long max_block_bytes, int lite_norm, int rejmaps);

/* weightingType (stacking/stacking.h:47-53) */
enum { SGPU_NO_WEIGHT = 0, SGPU_NBSTARS_WEIGHT = 1, SGPU_WFWHM_WEIGHT = 2, SGPU_NOISE_WEIGHT = 3,
	SGPU_NBSTACK_WEIGHT = 4 };

/* The rest of the `stack` command line (command.c:11493-11614) as
 * stack_one_seq applies it (:11626-11730).  Frames: every image of the
 * sequence that passes the filters (no filter = seq_filter_all; filter_included
 * = -filter-incl, the .seq's included images), at least two
 * (core/sequence_filtering.c:219-355); a filtered-out reference image is
 * replaced by the first selected one.  f_<name> is a literal threshold,
 * f_<name>_p a percentage (or, with f_<name>_k, a k-sigma clip) of the
 * sequence's registration values (struct seq_filter_config,
 * sequence_filtering.h:36-40).  weighting: -weight= (wfwhm / nbstars from the
 * registration data, nbstack from each frame's STACKCNT, noise from each
 * frame's bgnoise and normalization scale; noise is ignored without
 * normalization or with overlap_norm, as the reference does).  equalize_rgb:
 * -rgb_equal (normalization.c:157-159).  maximize: -maximize framing of a
 * registered mean stack (the canvas is the union of the shifted frames,
 * median_and_mean.c:160-190).  overlap_norm: with maximize, the coefficients
 * come from the pairs' overlaps (normalization.c:666-906); without it the
 * request is dropped (command.c:11696-11699).  feather > 0 (mean stacks):
 * the feathering masks of compute_masks and the per-block mask planes of
 * stack_read_block_data (sgpu_feather_*), over Siril's block plan for
 * block_threads (com.max_thread; <= 0: 1) and block_max_rows
 * (stack_get_max_number_of_rows; <= 0: the whole image), which the mask
 * upscale depends on.  Registration shifts are taken relative to the
 * reference image's own shift truncated to int (args->offset,
 * median_and_mean.c:190-194) for FITS sequences. */
typedef struct {
	int lite_norm;                /* -fastnorm */
	int rejmaps;                  /* 0, 1 (-rejmap), 2 (-rejmaps) */
	int equalize_rgb;             /* -rgb_equal */
	int weighting;                /* SGPU_*_WEIGHT */
	float f_fwhm, f_fwhm_p, f_wfwhm, f_wfwhm_p, f_round, f_round_p, f_quality, f_quality_p,
		f_bkg, f_bkg_p, f_nbstars, f_nbstars_p;
	int f_fwhm_k, f_wfwhm_k, f_round_k, f_quality_k, f_bkg_k, f_nbstars_k;
	int filter_included;          /* -filter-incl */
	int maximize;                 /* -maximize */
	int overlap_norm;             /* -overlap_norm */
	int feather;                  /* -feather= distance */
	long max_block_bytes;         /* reader block budget (<= 0: 512 MiB) */
	int block_threads;            /* feather: the block plan's thread count */
	long block_max_rows;          /* feather: the block plan's row budget */
} sgpu_stack_seq_options;
int sgpu_stack_seq_opts(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
		int use_registration, int use_32bit_output, const char *out_path, uint64_t counts[2],
		const sgpu_stack_seq_options *opts);
/* The frames sgpu_stack_seq_opts would stack (sequence indices, ascending;
 * the first cap of them written to indices), their number and the stack's
 * reference image: lets a caller size per-frame inputs (GESD critical values,
 * weights) before the stack. */
int sgpu_stack_seq_frames(const char *seq_path, const sgpu_stack_seq_options *opts, int *indices,
		int cap, int *nframes, int *ref_image);

/* Sequence stacks read Siril's row blocks (stack_read_block_data,
 * median_and_mean.c:382-545) with a pool of host threads into two
 * page-locked buffers; each block's H2D copy runs on its own stream while
 * the next block is read, and the stack waits for it (the overlapped block
 * loop of :1551-1760).  readers: threads per block read (0: OMP_NUM_THREADS,
 * else 8; at most 64). */
int sgpu_set_seq_readers(sgpu_context *ctx, int readers);
/* Memory a sequence stack keeps in the context for the next one: two
 * page-locked block buffers (up to 2 x 512 MB of host RAM), a page-locked
 * result image (W x H x layers x 4 bytes) and, on the device, two block
 * buffers plus the result / rejection-map bands.  They are reused by the
 * next sgpu_stack_seq* call on this context and freed by sgpu_release; this
 * frees them now (a caller stacking one sequence and keeping the context for
 * other work).  Never call it while a stack on this context is running. */
int sgpu_release_seq_buffers(sgpu_context *ctx);
/* Measurements of the last sequence stack on this context (non-feathered
 * path): out[0] blocks, [1] readers' wall seconds summed over blocks, [2]
 * H2D milliseconds (HIP events on the copy stream), [3] H2D bytes, [4] stack
 * kernel milliseconds (events around each block's stack), [5] wall seconds
 * of the block loop, [6] 1 when the block buffers were page-locked, [7]
 * reader threads, [8] seconds from the call to the block loop (sequence,
 * headers, selection, normalization), [9] seconds writing the result FITS,
 * [10] seconds of the whole call up to that write, [11] reserved. */
int sgpu_last_seq_stats(sgpu_context *ctx, double out[12]);

/* Per-frame normalization estimators, DATA_FLOAT planes (normValue 1).
 * Replaces the statistics pass of compute_normalization
 * (stacking/normalization.c:107-146,249-294) -> statistics_internal_float
 * with STATS_NORM / STATS_LITENORM (algos/statistics_float.c:281-480):
 * stats[4*f + 0..3] = median, mad, location, scale of frame f (location and
 * scale 0 when lite).  status[f] = 1 where the reference returns NULL stats
 * (no non-zero pixel, IKSS kept == 0, MAD == 0): the caller fails the
 * normalization as the reference does.  The _device variant reads frames in
 * HBM (frame f at d_frames + f*frame_stride) and synchronises once at the
 * end; sgpu_norm_stats stages host frames in 1 GiB batches. */
int sgpu_norm_stats_device(sgpu_context *ctx, const float *d_frames, int nframes, long npix,
		long frame_stride, int lite, double *stats, long *ngood, int *status);
int sgpu_norm_stats(sgpu_context *ctx, const float *frames, int nframes, long npix,
		long frame_stride, int lite, double *stats, long *ngood, int *status);
/* DATA_USHORT twins: statistics_internal_ushort (algos/statistics.c:231-449):
 * median = histogram_median and mad = siril_stats_ushort_mad (exact order
 * statistics of the samples > 0), IKSS on the [0,1]-scaled floats, location
 * and scale returned in 16-bit units (x 65535.0), as Siril caches them. */
int sgpu_norm_stats_u16_device(sgpu_context *ctx, const uint16_t *d_frames, int nframes, long npix,
		long frame_stride, int lite, double *stats, long *ngood, int *status);
int sgpu_norm_stats_u16(sgpu_context *ctx, const uint16_t *frames, int nframes, long npix,
		long frame_stride, int lite, double *stats, long *ngood, int *status);
/* Background noise of each frame (imstats bgnoise: siril_fits_img_stats_*
 * -> FnNoise1_float / FnNoise1_ushort, algos/quantize.c:1202-1488): per row
 * the 5-sigma-clipped RMS of first-order differences of valid pixels, the
 * median over rows x 0.70710678; float frames in their own units, 16-bit in
 * ADU.  The estimator of -weight=noise (median_and_mean.c:1111-1135).
 * Frames are width x height, frame_stride samples apart; noise[nframes].
 * The _device variants take HBM frames; all synchronise once. */
int sgpu_bgnoise_device(sgpu_context *ctx, const float *d_frames, int nframes, int width, int height,
		long frame_stride, double *noise);
int sgpu_bgnoise_u16_device(sgpu_context *ctx, const uint16_t *d_frames, int nframes, int width, int height,
		long frame_stride, double *noise);
int sgpu_bgnoise(sgpu_context *ctx, const float *frames, int nframes, int width, int height,
		long frame_stride, double *noise);
int sgpu_bgnoise_u16(sgpu_context *ctx, const uint16_t *frames, int nframes, int width, int height,
		long frame_stride, double *noise);
/* compute_factors_from_estimators (stacking/normalization.c:150-185) for one
 * layer: estimators picked as _compute_estimators_for_image does (:119-141:
 * location or median, scale or 1.5*mad when lite), factors relative to
 * frame ref_index of ref_stats (NULL = stats; the reflayer's stats for
 * equalizeRGB).  Outputs are coeff.poffset / pmul / pscale of the layer. */
int sgpu_norm_factors(int normalize, int lite, int nframes, int ref_index, const double *stats,
		const double *ref_stats, double *offset, double *mul, double *scale);

/* Overlap normalization (`stack ... -overlap_norm`, stacking/normalization.c:
 * 296-938; replaces _compute_estimators_for_images :458-598 and
 * solve_overlap_coeffs :296-355 of compute_normalization_overlaps :666-906).
 *
 * sgpu_overlap_rect: compute_overlap (:420-456) for two frames of one size
 * from their translation_from_H shifts (dx = H.h02, dy = -H.h12):
 * area = {x, y, w, h} on each frame, *npix = w * h (0: no overlap).
 *
 * sgpu_overlap_stats[_u16]_device: for every pair i < j of the nframes frames
 * in HBM (frame f at d_frames + f*frame_stride, width x height, plane of one
 * layer; h02/h12 = per-frame registration of the reglayer), the samples
 * non-zero in both frames of the overlap (16-bit as (float)x/USHRT_MAX) and,
 * when there are more than 3: per side the float median / MAD
 * (histogram_median_float, siril_stats_float_mad) and, unless lite, the
 * IKSSlite location / scale (0 / 1 where IKSSlite returns early).  Pair p =
 * get_ijth_pair_index(nframes, i, j) (:412-414); nij[p] = sample count (0 when
 * <= 3 or no overlap), stats[8p + 0..7] = medij, medji, madij, madji, locij,
 * locji, scaij, scaji.  Samples that are NaN are skipped (the reference keeps
 * them).  Synchronous.
 *
 * sgpu_overlap_factors: the coefficients of one layer from that table
 * (:804-906): scales from the scale estimators (ADDITIVE_SCALING,
 * MULTIPLICATIVE_SCALING), offsets from the rescaled locations (ADDITIVE,
 * ADDITIVE_SCALING), multipliers (MULTIPLICATIVE), each an LU solve with
 * partial pivoting relative to frame ref_index; lite selects median / MAD. */
int sgpu_overlap_rect(int width, int height, double dxi, double dyi, double dxj, double dyj,
		int *area_i, int *area_j, long *npix);
int sgpu_overlap_stats_device(sgpu_context *ctx, const float *d_frames, int nframes, long width, long height,
		long frame_stride, const double *h02, const double *h12, int lite, long *nij, double *stats);
int sgpu_overlap_stats_u16_device(sgpu_context *ctx, const uint16_t *d_frames, int nframes, long width,
		long height, long frame_stride, const double *h02, const double *h12, int lite, long *nij,
		double *stats);
int sgpu_overlap_factors(int normalize, int lite, int nframes, int ref_index, const long *nij,
		const double *stats, double *offset, double *mul, double *scale);

/* norm_to_0_1_range (stacking/median_and_mean.c:557-582): the post-pass of a
 * 32-bit stack with args->output_norm (:1774-1775) on a device image of n
 * floats: min / max of the non-zero samples of indices 1..n-1, then
 * (x - min) / (max - min) in float, zeros kept.  Asynchronous. */
int sgpu_norm_to_0_1_range_device(sgpu_context *ctx, float *d_img, long n);

/* FITS helpers of the headless path (BITPIX -32, 16 with BZERO 32768 or
 * signed, 8).  Rows are in FITS order; rows outside the image read as zero;
 * `out` holds float (BITPIX -32) or uint16 (BITPIX 16 / 8) samples of plane 0. */
int sgpu_fits_info(const char *path, long *width, long *height, int *bitpix);
int sgpu_fits_read_rows(const char *path, long row0, long nrows, void *out);
/* Same with Siril's [0, 1] conversion of float data: mode 0 raw, 1 as the
 * stack's block reader (internal_read_partial_fits, image_format_fits.c:
 * 994-1007: DATAMAX, or the 3-sample diagonal probe of the rows read, > 10 ->
 * x * INV_USHRT_MAX_SINGLE), 2 as readfits for whole frames (:906-910: the
 * file's max unless written by Siril, then DATAMAX). */
int sgpu_fits_read_rows_ex(const char *path, long row0, long nrows, void *out, int mode);
/* Number of planes (NAXIS3, 1 or 3) of a FITS image. */
int sgpu_fits_layers(const char *path);
/* Rows of frame `frame`, layer `layer` of a FITS file (frame 0), a FITSEQ
 * file (frame = image HDU index) or a SER file (path ending in .ser), in FITS
 * row order (SER rows are stored top-down: FITS-order row q is SER row h-1-q),
 * as the block reader sees them (mode as above). */
int sgpu_image_read_rows(const char *path, int frame, int layer, long row0, long nrows, void *out, int mode);
int sgpu_fits_write(const char *path, const void *data, long width, long height, int bitpix);
/* nlayers planes (1 or 3) of width x height, plane-major. */
int sgpu_fits_write_planes(const char *path, const void *data, long width, long height, int nlayers,
		int bitpix);
/* SER files (io/ser.c): a writer for sequences and fixtures -- frames as
 * [nframes][height][width][planes] uint16 samples in the file's top-down
 * row order, color_id (0 mono, 8-11 Bayer, 100 RGB, 101 BGR), bit_depth 1-16
 * (8 bits and below: 1 byte per sample), endian_flag as Siril reads it
 * (ser.h: 0 little-endian, 1 big-endian), optional per-frame UTC seconds
 * (timestamp trailer, date_time_to_ser_timestamp), observer and date_utc --
 * and the header / trailer reader (ser_read_header, ser_read_timestamp,
 * io/ser.c:106-382): returns the number of timestamps stored in unix_seconds
 * (at most max_ts), or an error code. */
int sgpu_ser_write(const char *path, const void *frames, int nframes, int width, int height, int color_id,
		int bit_depth, int endian_flag, const int64_t *unix_seconds, const char *observer, uint64_t date_utc);
int sgpu_ser_info(const char *path, int *width, int *height, int *frame_count, int *color_id, int *bit_depth,
		int *endian_flag, char observer[40], uint64_t *date_utc, int64_t *unix_seconds, int max_ts);

#ifdef __cplusplus
}
#endif
#endif /* SIRILGPU_H */
