/* tests/capi_c/capi_check.c -- TEST PROGRAM: a plain C99 caller of
 * include/sirilgpu.h, compiled with gcc and linked against libsirilgpu.so the
 * way Siril's C host would (stacking.h:16 stack_method, deconvolution.h:138
 * fft_richardson_lucy, demosaicing.h debayer_buffer_new_float,
 * registration.h:15 REG_DFT).  It pins the header's struct layout and calling
 * conventions independently of the ctypes mirror in siril_amd/_lib.py.
 *
 *   capi_check layout            print sizeof / offsetof of the ABI structs
 *   capi_check run <dir>         read the <dir>/NAME.in.bin inputs, call the entry points,
 *                                write <dir>/NAME.out.bin (tests/test_capi_c.py
 *                                compares them with the oracle)
 *
 * Exit codes: 0 ok, 77 no HIP device, 1 failure. */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sirilgpu.h"

/* fixed problem sizes (tests/test_capi_c.py writes inputs of these shapes) */
enum { ST_N = 24, ST_ROWS = 16, ST_W = 40 };          /* Winsorized 3/3 stack */
enum { DFT_S = 64, DFT_NF = 3 };                      /* REG_DFT selections */
enum { RL_W = 80, RL_H = 64, RL_KS = 15, RL_IT = 4 }; /* fft_richardson_lucy */
enum { DM_W = 40, DM_H = 32 };                        /* debayer RGGB */

static int read_file(const char *dir, const char *name, void *buf, size_t bytes) {
	char path[1024];
	FILE *f;
	size_t got;
	snprintf(path, sizeof path, "%s/%s", dir, name);
	f = fopen(path, "rb");
	if (!f) {
		fprintf(stderr, "cannot open %s\n", path);
		return 1;
	}
	got = fread(buf, 1, bytes, f);
	fclose(f);
	if (got != bytes) {
		fprintf(stderr, "%s: %zu of %zu bytes\n", path, got, bytes);
		return 1;
	}
	return 0;
}

static int write_file(const char *dir, const char *name, const void *buf, size_t bytes) {
	char path[1024];
	FILE *f;
	snprintf(path, sizeof path, "%s/%s", dir, name);
	f = fopen(path, "wb");
	if (!f || fwrite(buf, 1, bytes, f) != bytes) {
		fprintf(stderr, "cannot write %s\n", path);
		if (f) fclose(f);
		return 1;
	}
	return fclose(f) != 0;
}

static void layout(void) {
	printf("abi %d\n", SGPU_ABI_VERSION);
	printf("sgpu_stack_params.size %zu\n", sizeof(sgpu_stack_params));
#define OFF(f) printf("sgpu_stack_params.%s %zu\n", #f, offsetof(sgpu_stack_params, f))
	OFF(method);
	OFF(type_of_rejection);
	OFF(sig);
	OFF(normalize);
	OFF(scale);
	OFF(offset);
	OFF(mul);
	OFF(shiftx);
	OFF(weights);
	OFF(critical_value);
	OFF(output_norm);
#undef OFF
	printf("sgpu_stack_seq_options.size %zu\n", sizeof(sgpu_stack_seq_options));
	printf("sgpu_stack_seq_options.filter_included %zu\n", offsetof(sgpu_stack_seq_options, filter_included));
	printf("sgpu_stack_seq_options.max_block_bytes %zu\n", offsetof(sgpu_stack_seq_options, max_block_bytes));
}

static int run_stack(sgpu_context *ctx, const char *dir) {
	static float frames[ST_N * ST_ROWS * ST_W], out[ST_ROWS * ST_W];
	static uint16_t rl[ST_ROWS * ST_W], rh[ST_ROWS * ST_W];
	uint64_t counts[2] = {0, 0};
	sgpu_stack_params p;
	int r;
	if (read_file(dir, "stack_frames.in.bin", frames, sizeof frames)) return 1;
	memset(&p, 0, sizeof p);
	p.method = SGPU_METHOD_MEAN;
	p.type_of_rejection = SGPU_WINSORIZED;
	p.sig[0] = 3.0f;
	p.sig[1] = 3.0f;
	p.normalize = SGPU_NO_NORM;
	r = sgpu_stack_rows(ctx, frames, ST_N, ST_W, ST_ROWS, (long)ST_ROWS * ST_W, &p, out, rl, rh, counts);
	if (r != SGPU_OK) {
		fprintf(stderr, "sgpu_stack_rows: %d %s\n", r, sgpu_last_error());
		return 1;
	}
	return write_file(dir, "stack_out.out.bin", out, sizeof out) || write_file(dir, "stack_rl.out.bin", rl, sizeof rl) ||
	       write_file(dir, "stack_rh.out.bin", rh, sizeof rh) ||
	       write_file(dir, "stack_counts.out.bin", counts, sizeof counts);
}

static int run_dft(sgpu_context *ctx, const char *dir) {
	static float ref[DFT_S * DFT_S], fr[DFT_NF][DFT_S * DFT_S];
	const float *frames[DFT_NF];
	int sx[DFT_NF], sy[DFT_NF], shifts[2 * DFT_NF], f, r;
	if (read_file(dir, "dft_ref.in.bin", ref, sizeof ref) || read_file(dir, "dft_frames.in.bin", fr, sizeof fr))
		return 1;
	for (f = 0; f < DFT_NF; f++) frames[f] = fr[f];
	r = sgpu_dft_shifts(ctx, ref, frames, DFT_NF, DFT_S, sx, sy);
	if (r != SGPU_OK) {
		fprintf(stderr, "sgpu_dft_shifts: %d %s\n", r, sgpu_last_error());
		return 1;
	}
	for (f = 0; f < DFT_NF; f++) {
		shifts[2 * f] = sx[f];
		shifts[2 * f + 1] = sy[f];
	}
	return write_file(dir, "dft_shifts.out.bin", shifts, sizeof shifts);
}

static int run_rl(const char *dir) {
	static float img[RL_W * RL_H], k[RL_KS * RL_KS];
	int r;
	if (read_file(dir, "rl_img.in.bin", img, sizeof img) || read_file(dir, "rl_psf.in.bin", k, sizeof k)) return 1;
	/* the reference's argument list (deconvolution.h:138): lambda is passed
	 * as 2 / alpha, regtype REG_NONE_GRAD (2), stepsize 0.0003 */
	r = sgpu_fft_richardson_lucy(img, RL_W, RL_H, 1, k, RL_KS, 1, 2.0f / 0.001f, RL_IT, 0.002f, 8, 2, 0.0003f, 0);
	if (r != 0) {
		fprintf(stderr, "sgpu_fft_richardson_lucy: %d %s\n", r, sgpu_last_error());
		return 1;
	}
	return write_file(dir, "rl_img.out.bin", img, sizeof img);
}

static int run_debayer(const char *dir) {
	static float cfa[DM_W * DM_H];
	int w = DM_W, h = DM_H, r;
	float *rgb;
	if (read_file(dir, "dm_cfa.in.bin", cfa, sizeof cfa)) return 1;
	/* BAYER_RCD (8), RGGB (0); xtrans unused for Bayer patterns */
	rgb = sgpu_debayer_buffer_new_float(cfa, &w, &h, 8, 0, NULL);
	if (!rgb || w != DM_W || h != DM_H) {
		fprintf(stderr, "sgpu_debayer_buffer_new_float failed: %s\n", sgpu_last_error());
		free(rgb);
		return 1;
	}
	r = write_file(dir, "dm_rgb.out.bin", rgb, sizeof(float) * 3 * DM_W * DM_H);
	free(rgb);
	return r;
}

int main(int argc, char **argv) {
	sgpu_context *ctx = NULL;
	int r;
	if (argc >= 2 && strcmp(argv[1], "layout") == 0) {
		layout();
		return 0;
	}
	if (argc < 3 || strcmp(argv[1], "run") != 0) {
		fprintf(stderr, "usage: capi_check layout | run <dir>\n");
		return 1;
	}
	if (sgpu_abi_version() != SGPU_ABI_VERSION) {
		fprintf(stderr, "ABI mismatch: library %d, header %d\n", sgpu_abi_version(), SGPU_ABI_VERSION);
		return 1;
	}
	if (sgpu_device_count() <= 0) return 77;
	if (sgpu_init(0, &ctx) != SGPU_OK) {
		fprintf(stderr, "sgpu_init: %s\n", sgpu_last_error());
		return 1;
	}
	r = run_stack(ctx, argv[2]) || run_dft(ctx, argv[2]) || run_rl(argv[2]) || run_debayer(argv[2]);
	sgpu_release(ctx);
	if (!r) printf("capi_check ok\n");
	return r ? 1 : 0;
}
