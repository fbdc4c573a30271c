/*
 * oracle/stack_ref.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, sequential CPU restatement of Siril's per-pixel rejection stack
 * (the data-parallel hot path this repository accelerates on MI355X).  It is
 * the CHECKER for the HIP kernels in siril_amd/csrc and the `cpu_baseline`
 * leg of bench.py.  Nothing in the product (libsirilgpu.so, siril_amd Python modules)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * lock042/siril, 1.5.0-dev).  The restatement keeps the reference's control
 * flow, element visiting order, in-place permutations (Lomuto quickselect,
 * the n<9 sorting networks, quicksort/insertion sort) and float/double
 * typing, because the `N - r <= 4` cutoff of the SIGMA/MAD/WINSORIZED/
 * LINEARFIT loops makes the result depend on element order
 * (rejection_float.c:188,239,279).
 *
 * Pinning: the reference itself cannot be compiled here without stand-in
 * glib/gsl/cfitsio headers (not allowed), so this restatement is pinned by
 * the reference's own known-answer tests (src/tests/rejection_test.c:96-230:
 * GESDT, PERCENTILE, LINEARFIT) and by the quickmedian-vs-sort property of
 * src/tests/sorting.c:58-110, run on the float quickmedian and on both WORD
 * helpers of that test (quickmedian and histogram_median, sizes 1-400, the
 * sortnet cases 1-9 included) -- see tests/test_oracle.py.  SIGMA, MAD,
 * SIGMEDIAN and WINSORIZED have no reference fixture: parity for those is
 * pinned only by this restatement ("Oracle").
 *
 * Build: oracle/Makefile -> oracle/liboracle_stack.so  (gcc -O2 -fopenmp,
 * -ffp-contract=off to mirror x86-64 gcc without FMA).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* rejection enum, core/settings.h:43-52 */
enum { OR_NO_REJEC = 0, OR_PERCENTILE, OR_SIGMA, OR_MAD, OR_SIGMEDIAN,
       OR_WINSORIZED, OR_LINEARFIT, OR_GESDT };
/* normalization enum, core/settings.h:34-40 */
enum { OR_NO_NORM = 0, OR_ADDITIVE, OR_MULTIPLICATIVE, OR_ADDITIVE_SCALING,
       OR_MULTIPLICATIVE_SCALING };

/* ------------------------------------------------------------------ sorting */

/* insertionSort_f, sorting.c:90-103 */
static void or_insertion_sort_f(float *a, size_t n) {
	for (long i = 1; i < (long)n; i++) {
		const float v = a[i];
		long j = i - 1;
		while (j >= 0 && a[j] > v) {
			a[j + 1] = a[j];
			--j;
		}
		a[j + 1] = v;
	}
}

/* quicksort_f, sorting.c:110-135 (insertion sort below 33 elements,
 * middle-element pivot, two converging pointers) */
void or_quicksort_f(float *a, size_t n) {
	if (n <= 32) {
		or_insertion_sort_f(a, n);
		return;
	}
	const float pivot = a[n / 2];
	float *lo = a, *hi = a + n - 1;
	while (lo <= hi) {
		if (*lo < pivot) { lo++; continue; }
		if (*hi > pivot) { hi--; continue; }
		float t = *lo;
		*lo++ = *hi;
		*hi-- = t;
	}
	or_quicksort_f(a, hi - a + 1);
	or_quicksort_f(lo, a + n - lo);
}

/* Comparator lists of sortnet_median_float, sorting.c:468-513.  Each pair
 * (i,j) swaps a[i],a[j] when a[i] > a[j]. */
static const unsigned char net2[] = {0,1};
static const unsigned char net3[] = {0,1, 1,2, 0,1};
static const unsigned char net4[] = {0,1, 2,3, 0,2, 1,3, 1,2};
static const unsigned char net5[] = {0,1, 2,3, 1,3, 2,4, 0,2, 1,4, 1,2, 3,4, 2,3};
static const unsigned char net6[] = {0,1, 2,3, 4,5, 0,2, 3,5, 1,4, 0,1, 2,3, 4,5,
				     1,2, 3,4, 2,3};
static const unsigned char net7[] = {1,2, 3,4, 5,6, 0,2, 4,6, 3,5, 2,6, 1,5, 0,4,
				     2,5, 0,3, 2,4, 1,3, 0,1, 2,3, 4,5};
static const unsigned char net8[] = {0,1, 2,3, 4,5, 6,7, 0,2, 1,3, 4,6, 5,7, 1,2,
				     5,6, 0,4, 1,5, 2,6, 3,7, 2,4, 3,5, 1,2, 3,4, 5,6};
static const unsigned char *const nets[9] = {0, 0, net2, net3, net4, net5, net6, net7, net8};
static const int net_len[9] = {0, 0, sizeof net2 / 2, sizeof net3 / 2, sizeof net4 / 2,
			       sizeof net5 / 2, sizeof net6 / 2, sizeof net7 / 2, sizeof net8 / 2};

/* sortnet_median_float, sorting.c:468-513: NOTE the even-size result adds
 * the two middle elements in float before the double division (:512). */
double or_sortnet_median_f(float *a, size_t n) {
	size_t k = n / 2;
	if (n == 1) return a[0];
	if (n < 2 || n > 8) return 0.0;	/* default branch of the switch */
	const unsigned char *p = nets[n];
	for (int c = 0; c < net_len[n]; c++) {
		int i = p[2 * c], j = p[2 * c + 1];
		if (a[i] > a[j]) { float t = a[i]; a[i] = a[j]; a[j] = t; }
	}
	return (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
}

/* quickmedian_float, sorting.c:240-273: Lomuto quickselect, pivot at the
 * middle index, swapped to the right end; permutes `a` in place. */
double or_quickmedian_f(float *a, size_t n) {
	if (n < 9) return or_sortnet_median_f(a, n);
	size_t k = n / 2, left = 0, right = n - 1;
	while (left < right) {
		size_t p = (left + right) / 2;
		float pivot = a[p];
		a[p] = a[right];
		a[right] = pivot;
		p = left;
		for (size_t i = left; i < right; i++) {
			if (a[i] < pivot) {
				float t = a[p]; a[p] = a[i]; a[i] = t;
				p++;
			}
		}
		a[right] = a[p];
		a[p] = pivot;
		if (p < k) left = p + 1;
		else right = p;
	}
	return (n % 2 == 0) ? ((double)a[k - 1] + a[k]) / 2.0 : (double)a[k];
}

/* gsl_stats_float_median_from_sorted_data (GSL statistics/median_source.c,
 * BASE=float; GSL is not vendored, this is its published formula): the two
 * middle elements are added in float, then divided by 2.0 in double. */
double or_gsl_median_sorted_f(const float *s, size_t n) {
	if (n == 0) return 0.0;
	size_t lhs = (n - 1) / 2, rhs = n / 2;
	if (lhs == rhs) return s[lhs];
	return (s[lhs] + s[rhs]) / 2.0;
}

/* -------------------------------------------------------------- statistics */

/* Summation order of the reference's `#pragma omp simd reduction(+:...)`
 * loops (algos/statistics.h:93-101 for N >= 24, stacking/median_and_mean.c
 * :1085-1090 for kept >= STACK_SIMD_N_THRESHOLD = 16, stacking.h:14).
 * g_simd_lanes == 0: the sequential order (the scalar branch, which is also
 * what the sorted path's exact kernel restates).  L > 0: a model of GCC's
 * vectorised reduction for the default x86-64 (SSE2, no -march=native,
 * meson.build:170-175) build: the float loads are converted to double in
 * L lanes (L = 4: one 4-float load -> two 2-double accumulators), lane j sums
 * the elements i = j (mod L) of the vector body in order, the lanes are
 * combined by halving (upper half added to lower half: for L = 4
 * (l0 + l2) + (l1 + l3)), then the N mod L tail elements are added in order.
 * Test infrastructure for measuring how many results depend on the order
 * (DESIGN.md §2); the default stays sequential. */
static int g_simd_lanes = 0;
void or_set_simd_lanes(int lanes) { g_simd_lanes = (lanes == 2 || lanes == 4 || lanes == 8) ? lanes : 0; }

static double simd_sum_f(const float *x, int n, const float *sub, int sq) {
	/* sum of (double)x[i] (sq == 0) or of (double)(d*d), d = x[i] - *sub in float */
	double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	const int L = g_simd_lanes, body = n - n % L;
	int i, l;
	for (i = 0; i < body; i += L)
		for (l = 0; l < L; l++) {
			float d = sq ? x[i + l] - *sub : x[i + l];
			acc[l] += sq ? (double)(d * d) : (double)d;
		}
	for (l = L / 2; l >= 1; l /= 2)
		for (i = 0; i < l; i++) acc[i] += acc[i + l];
	for (i = body; i < n; i++) {
		float d = sq ? x[i] - *sub : x[i];
		acc[0] += sq ? (double)(d * d) : (double)d;
	}
	return acc[0];
}

/* the double sum of x in the order selected by or_set_simd_lanes (tests) */
double or_sum_f(const float *x, int n) {
	double s = 0.0;
	if (g_simd_lanes) return simd_sum_f(x, n, NULL, 0);
	for (int i = 0; i < n; i++) s += (double)x[i];
	return s;
}

/* siril_stats_float_sd, algos/statistics.h:80-106: the sequential branch,
 * and for N >= 24 the `omp simd` branch in the order g_simd_lanes models
 * (sequential when 0). */
float or_stats_float_sd(const float *x, int n, float *mean_out) {
	double sum = 0.0, vsum = 0.0;
	float mean;
	if (g_simd_lanes && n >= 24) {
		sum = simd_sum_f(x, n, NULL, 0);
		mean = (float)(sum / n);
		vsum = simd_sum_f(x, n, &mean, 1);
	} else {
		for (int i = 0; i < n; i++) sum += (double)x[i];
		mean = (float)(sum / n);
		for (int i = 0; i < n; i++) {
			float d = x[i] - mean;
			vsum += (double)(d * d);
		}
	}
	if (mean_out) *mean_out = mean;
	return sqrtf((float)(vsum / (n - 1)));
}

/* std::min / std::max as used by rt_algo.cc:58-61 */
static inline float fminf_ref(float a, float b) { return (b < a) ? b : a; }
static inline float fmaxf_ref(float a, float b) { return (a < b) ? b : a; }

/* rtengine::findMinMaxPercentile, rt/rt_algo.cc:38-172, single-thread path,
 * called with minPrct == maxPrct == 0.5 and minOut == maxOut. */
static float or_histogram_percentile_f(const float *x, size_t n, float prct) {
	float lo = x[0], hi = x[0];
	for (size_t i = 1; i < n; ++i) {
		lo = fminf_ref(lo, x[i]);
		hi = fmaxf_ref(hi, x[i]);
	}
	if (fabsf(hi - lo) == 0.f) return lo;
	const unsigned hs = (unsigned)(n < 65536 ? n : 65536);
	const float scale = (hs - 1) / (hi - lo);
	uint32_t *h = calloc(hs, sizeof *h);
	for (size_t i = 0; i < n; ++i) h[(uint16_t)(scale * (x[i] - lo))]++;
	size_t k = 0, count = 0;
	float out = 0.f;
	for (int pass = 0; pass < 2; pass++) {	/* min, then max: same percentile */
		const float thr = prct * n;
		while (count < thr) count += h[k++];
		if (k > 0) {
			const size_t before = count - h[k - 1];
			const float c0 = count - thr;
			const float c1 = thr - before;
			out = (c1 * k + c0 * (k - 1)) / (c0 + c1);
		} else {
			out = k;
		}
		out /= scale;
		out += lo;
		float m = fminf_ref(out, hi);		/* rtengine::LIM, rt_math.h:84-87 */
		out = fmaxf_ref(lo, m);
	}
	free(h);
	return out;
}

/* siril_stats_float_mad, algos/statistics_float.c:79-101 -> histogram_median_float,
 * sorting.c:644-649: the (approximate) histogram-interpolated median of
 * |x - (float)m|. */
double or_stats_float_mad(const float *x, size_t n, double m) {
	const float med = (float)m;
	float *t = malloc(n * sizeof *t);
	for (size_t i = 0; i < n; i++) t[i] = fabsf(x[i] - med);
	double mad = or_histogram_percentile_f(t, n, 0.5f);
	free(t);
	return mad;
}

/* siril_fit_linear, stacking/siril_fit_linear.c:24-50 (running-mean least
 * squares in float; x[i] = 1/(i+1), m_x and m_dx2 precomputed for the
 * ORIGINAL frame count, median_and_mean.c:1487-1500). */
void or_fit_linear(const float *x, const float *y, float m_x, float m_dx2,
		size_t n, float *c0, float *c1) {
	float m_y = y[0];
	for (size_t i = 1; i < n; i++) m_y += (y[i] - m_y) * x[i];
	float m_dxdy = 0.f, dx = -m_x;
	for (size_t i = 0; i < n; i++, dx += 1.f) {
		const float dy = y[i] - m_y;
		m_dxdy += (dx * dy - m_dxdy) * x[i];
	}
	const float b = m_dxdy * m_dx2;
	*c0 = m_y - m_x * b;
	*c1 = b;
}

/* LINEARFIT precomputation, median_and_mean.c:1487-1500 */
void or_linear_fit_setup(int nb_frames, float *xf, float *m_x, float *m_dx2) {
	float mx = (nb_frames - 1) * 0.5f, md = 0.f;
	for (int j = 0; j < nb_frames; ++j) {
		const float dx = j - mx;
		xf[j] = 1.f / (j + 1);
		md += (dx * dx - md) * xf[j];
	}
	*m_x = mx;
	*m_dx2 = 1.f / md;
}

/* ---------------------------------------------------------------- rejection */

typedef struct {
	int type;		/* rejection enum */
	float sig[2];		/* sig[0] low / sig[1] high (or GESD fraction, alpha) */
	const float *crit;	/* GESD critical values, indexed by iter + removed */
	const float *xf;	/* LINEARFIT 1/(j+1) table, nb_frames long */
	float m_x, m_dx2;	/* LINEARFIT constants */
} or_rej_params;

typedef struct {		/* per-thread scratch, struct _data_block (stacking.h:152-165) */
	float *stack, *o_stack, *w_stack, *yf;
	int *rejected;
	const float *dstack;	/* drizzle weights of the column (args->drizzle), or NULL */
	const float *mstack;	/* feather-mask weights of the column (masking), or NULL */
} or_scratch;

/* percentile_clipping, rejection_float.c:31-44 */
static int or_pclip(float x, const float sig[2], float med, int rej[2]) {
	if (med - x > med * sig[0]) { rej[0]++; return -1; }
	if (x - med > med * sig[1]) { rej[1]++; return 1; }
	return 0;
}

/* sigma_clipping_float, rejection_float.c:49-60 */
static int or_sclip(float x, float s, float slo, float shi, float med, int rej[2]) {
	if (med - x > s * slo) { rej[0]++; return -1; }
	if (x - med > s * shi) { rej[1]++; return 1; }
	return 0;
}

/* line_clipping, rejection_float.c:62-75 */
static int or_lclip(float x, const float sig[2], float s, int i, float a, float b, int rej[2]) {
	if (a * i + b - x > s * sig[0]) { rej[0]++; return -1; }
	if (x - a * i - b > s * sig[1]) { rej[1]++; return 1; }
	return 0;
}

/* order-preserving compaction of the kept samples (e.g. rejection_float.c:198-207) */
static int or_compact(float *s, const int *rej, int n) {
	int o = 0;
	for (int p = 0; p < n; p++)
		if (!rej[p]) s[o++] = s[p];
	return o;
}

/* grubbs_stat, rejection_float.c:82-98 (data sorted) */
static void or_grubbs(const float *s, int n, float *g, int *imax) {
	float avg;
	float sd = or_stats_float_sd(s, n, &avg);
	float dev = avg - s[0];
	float d2 = s[n - 1] - avg;
	if (d2 > dev) { dev = d2; *imax = n - 1; }
	else *imax = 0;
	*g = dev / sd;
}

typedef struct { float x; int i; int out; } or_esd;	/* struct ESD_outliers, stacking.h:171-175 */

/* confirm_outliers, median_and_mean.c:685-701 (NOTE: always confirms the
 * first two candidates, and high candidates carry their index in the
 * shrinking working copy -- reproduced as is). */
static void or_confirm(or_esd *o, int n, double med, int *rejected, int rej[2]) {
	int i = n - 1;
	while (i > 1 && !o[i].out) i--;
	for (int j = i; j >= 0; j--) {
		o[j].out = 1;
		if (o[j].x >= med) { rejected[o[j].i] = 1; rej[1]++; }
		else { rejected[o[j].i] = -1; rej[0]++; }
	}
}

/* apply_rejection_float, stacking/rejection_float.c:100-354 (no drizzle
 * weights).  Returns the number of kept samples, left compacted at the
 * front of sc->stack; crej[0]/[1] count low/high rejections. */
int or_apply_rejection_f(const or_rej_params *P, or_scratch *sc, int nb_frames, int crej[2]) {
	int N = nb_frames, r = 0, firstloop = 1, kept = 0, changed, n;
	double median = 0.0;
	float *stack = sc->stack, *w = sc->w_stack;
	int *rejected = sc->rejected;
	const float slo = P->sig[0], shi = P->sig[1];

	memcpy(sc->o_stack, stack, N * sizeof(float));			/* :114 */
	if (sc->dstack) {						/* :117-126 */
		for (int f = 0; f < N; f++)
			if (stack[f] != 0.f && sc->dstack[f] != 0.f) {
				if (f != kept) stack[kept] = stack[f];
				kept++;
			}
	} else {
		for (int f = 0; f < N; f++)				/* :128-135 */
			if (stack[f] != 0.f) {
				if (f != kept) stack[kept] = stack[f];
				kept++;
			}
	}
	if (kept <= 1) return kept;					/* :140-142 */
	const int removed = N - kept;
	N = kept;

	switch (P->type) {						/* :147-157 */
	case OR_PERCENTILE: case OR_SIGMA: case OR_MAD:
		median = or_quickmedian_f(stack, N);
		if (median == 0.0) return 0;
		break;
	default: break;
	}

	switch (P->type) {
	case OR_PERCENTILE:						/* :160-173 */
		for (int f = 0; f < N; f++)
			rejected[f] = or_pclip(stack[f], P->sig, (float)median, crej);
		N = or_compact(stack, rejected, N);
		break;
	case OR_SIGMA: case OR_MAD:					/* :174-209 */
		do {
			float var;
			if (P->type == OR_SIGMA) var = or_stats_float_sd(stack, N, NULL);
			else var = (float)or_stats_float_mad(stack, N, median);
			if (!firstloop) median = or_quickmedian_f(stack, N);
			else firstloop = 0;
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_sclip(stack[f], var, slo, shi, (float)median, crej);
					if (rejected[f]) r++;
				}
			}
			int out = or_compact(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_SIGMEDIAN:						/* :210-222 */
		do {
			const float sigma = or_stats_float_sd(stack, N, NULL);
			const float mf = (float)or_quickmedian_f(stack, N);
			n = 0;
			for (int f = 0; f < N; f++)
				if (or_sclip(stack[f], sigma, slo, shi, mf, crej)) {
					stack[f] = mf;
					n++;
				}
		} while (n > 0);
		break;
	case OR_WINSORIZED:						/* :223-259 */
		do {
			float sigma0, sigma = or_stats_float_sd(stack, N, NULL);
			const float mf = (float)or_quickmedian_f(stack, N);
			memcpy(w, stack, N * sizeof(float));
			do {
				const float m0 = mf - 1.5f * sigma, m1 = mf + 1.5f * sigma;
				for (int j = 0; j < N; j++) {
					float v = w[j] < m0 ? m0 : w[j];	/* max(m0, w) */
					w[j] = m1 < v ? m1 : v;			/* min(m1, .) */
				}
				sigma0 = sigma;
				sigma = 1.134f * or_stats_float_sd(w, N, NULL);
			} while (fabsf(sigma - sigma0) > sigma0 * 0.0005f);
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_sclip(stack[f], sigma, slo, shi, mf, crej);
					if (rejected[f] != 0) r++;
				}
			}
			int out = or_compact(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_LINEARFIT:						/* :260-300 */
		do {
			or_quicksort_f(stack, N);
			for (int f = 0; f < N; f++) sc->yf[f] = stack[f];
			float a, b;
			or_fit_linear(P->xf, sc->yf, P->m_x, P->m_dx2, N, &b, &a);
			float sigma = 0.f;
			for (int f = 0; f < N; f++) sigma += fabsf(stack[f] - (a * f + b));
			sigma /= (float)N;
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_lclip(stack[f], P->sig, sigma, f, a, b, crej);
					if (rejected[f] != 0) r++;
				}
			}
			int out = or_compact(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_GESDT: {						/* :301-348 */
		or_quicksort_f(stack, N);
		median = or_gsl_median_sorted_f(stack, N);
		int max_out = (int)nb_frames * P->sig[0];
		if (removed >= max_out) return kept;
		max_out -= removed;
		or_esd *o = malloc(max_out * sizeof *o);
		memcpy(w, stack, N * sizeof(float));
		memset(rejected, 0, N * sizeof(int));
		int cold = 0;
		for (int it = 0, size = N; it < max_out; it++, size--) {
			float g;
			int im = 0;
			or_grubbs(w, size, &g, &im);
			o[it].out = g > P->crit[it + removed];		/* check_G_values */
			o[it].x = w[im];
			o[it].i = (im == 0) ? cold++ : im;
			for (int q = im; q < size - 1; q++) w[q] = w[q + 1];	/* remove_element */
		}
		or_confirm(o, max_out, median, rejected, crej);
		free(o);
		N = or_compact(stack, rejected, N);
		break;
	}
	default:
		break;
	}
	return N;
}

/* mean_and_reject, float branch, median_and_mean.c:1038-1099.  `weights`
 * (nb_frames doubles, or NULL) selects the weighted branch :1043-1082. */
double or_mean_and_reject_f(const or_rej_params *P, or_scratch *sc, int n,
		const double *weights, int rej[2]) {
	int kept = or_apply_rejection_f(P, sc, n, rej);
	if (kept == 0) return or_quickmedian_f(sc->stack, n);		/* :1040-1041 */
	if (weights || sc->dstack || sc->mstack) {
		float pmin = FLT_MAX, pmax = -FLT_MAX;
		for (int f = 0; f < kept; ++f) {
			if (pmin > sc->stack[f]) pmin = sc->stack[f];
			if (pmax < sc->stack[f]) pmax = sc->stack[f];
		}
		double sum = 0.0, norm = 0.0;
		for (int f = 0; f < n; ++f) {
			float v = sc->o_stack[f];
			if (v >= pmin && v <= pmax && v != 0.f) {
				double w = 1.;					/* :1060-1066 */
				if (sc->dstack) w *= sc->dstack[f];
				if (sc->mstack) w *= sc->mstack[f];
				if (weights) w *= weights[f];
				sum += (double)v * w;
				norm += w;
			}
		}
		if (norm == 0. || sum == 0.) {
			sum = 0.;
			for (int f = 0; f < n; ++f) {
				float v = sc->o_stack[f];
				if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
			}
			return sum / (double)kept;
		}
		return sum / norm;
	}
	double sum = 0.0;						/* :1083-1097 */
	if (g_simd_lanes && kept >= 16) return simd_sum_f(sc->stack, kept, NULL, 0) / (double)kept;
	for (int f = 0; f < kept; ++f) sum += (double)sc->stack[f];
	return sum / (double)kept;
}

/* round_to_int, core/proto.h:208-213 */
static int or_round_to_int(double x) {
	x = (x > (double)INT32_MAX - 0.5) ? (double)INT32_MAX - 0.5 : x;
	x = (x < (double)INT32_MIN + 0.5) ? (double)INT32_MIN + 0.5 : x;
	return (int)(x + ((x >= 0.0) ? 0.5 : -0.5));
}

/* ------------------------------------------------------------ block driver */

/* Per-pixel loop of stack_mean_or_median, median_and_mean.c:1592-1737, over
 * a frame-major block frames[f*frame_stride + y*W + x] of `rows` rows.
 *   method 0 = mean with rejection (mean_and_reject), 1 = median (quickmedian_float)
 *   shift_dx: per-frame registration x shift (double, already minus offset[0]),
 *             converted by round_to_int(dx*scale) as :1618-1622; NULL = none
 *   norm: normalization enum; scale/offset/mul per frame (doubles)
 *   output_norm: 0 -> clamp to [0,1] (set_float_in_interval, :1725-1727)
 * Output row y of the block is out[y*W + x] (the caller does the FITS
 * bottom-up flip, :1597).  rej_lo/rej_hi may be NULL; counts[2] accumulate. */
int or_stack_rows_planes_f(const float *frames, const float *drizz, const float *mask, int nframes, long W,
		long rows, long frame_stride, int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads);

int or_stack_rows_f(const float *frames, int nframes, long W, long rows, long frame_stride,
		int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads) {
	return or_stack_rows_planes_f(frames, NULL, NULL, nframes, W, rows, frame_stride, method, P, norm, scale,
			offset, mul, shift_dx, shift_scale, weights, output_norm, out, rej_lo, rej_hi, counts, nthreads);
}

/* Same with the per-sample weight planes of the block (data->drizz with
 * args->drizzle, data->mask with feather masking; frame-major like frames,
 * NULL when unused), read at the shifted index as :1687-1692 do. */
int or_stack_rows_planes_f(const float *frames, const float *drizz, const float *mask, int nframes, long W,
		long rows, long frame_stride, int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads) {
	uint64_t c0 = 0, c1 = 0;
	int *shx = NULL;
	if (shift_dx) {
		shx = malloc(nframes * sizeof(int));
		for (int f = 0; f < nframes; f++) shx[f] = or_round_to_int(shift_dx[f] * shift_scale);
	}
#ifdef _OPENMP
	if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+:c0, c1)
#endif
	{
		or_scratch sc;
		float *buf = malloc(7 * (size_t)nframes * sizeof(float));
		sc.stack = buf;
		sc.o_stack = buf + nframes;
		sc.w_stack = buf + 2 * nframes;
		sc.yf = buf + 3 * nframes;
		sc.rejected = (int *)(buf + 4 * nframes);
		float *dst = buf + 5 * nframes, *mst = buf + 6 * nframes;
		sc.dstack = drizz ? dst : NULL;
		sc.mstack = mask ? mst : NULL;
		/* out-of-frame samples keep the previous pixel's weights, as the
		 * reference's `continue` does (:1626-1633); they are zero samples, so
		 * the weights never count */
		for (int f = 0; f < nframes; f++) dst[f] = mst[f] = 0.f;
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
		for (long y = 0; y < rows; y++) {
			for (long x = 0; x < W; x++) {
				for (int f = 0; f < nframes; f++) {
					long pix = y * W + x;
					if (shx) {
						int s = shx[f];
						if (s && (x - s >= W || x - s < 0)) {	/* :1624-1631 */
							sc.stack[f] = 0.0f;
							continue;
						}
						pix -= s;
					}
					float v = frames[(size_t)f * frame_stride + pix];
					if (drizz) dst[f] = drizz[(size_t)f * frame_stride + pix];	/* :1690-1692 */
					if (mask) mst[f] = mask[(size_t)f * frame_stride + pix];	/* :1687-1689 */
					double t;
					switch (norm) {					/* :1644-1686 */
					default:
					case OR_NO_NORM:
						sc.stack[f] = v;
						break;
					case OR_ADDITIVE: case OR_ADDITIVE_SCALING:
						if (v != 0.f) {
							t = v * scale[f];
							sc.stack[f] = (float)(t - offset[f]);
						} else sc.stack[f] = 0.f;
						break;
					case OR_MULTIPLICATIVE: case OR_MULTIPLICATIVE_SCALING:
						t = v * scale[f];
						sc.stack[f] = (float)(t * mul[f]);
						break;
					}
				}
				double res;
				int rj[2] = {0, 0};
				if (method == 0) {
					res = or_mean_and_reject_f(P, &sc, nframes, weights, rj);
					c0 += rj[0];
					c1 += rj[1];
					long o = y * W + x;
					if (rej_lo) rej_lo[o] = (uint16_t)(rj[0] < 0 ? 0 : (rj[0] > 65535 ? 65535 : rj[0]));
					if (rej_hi) rej_hi[o] = (uint16_t)(rj[1] < 0 ? 0 : (rj[1] > 65535 ? 65535 : rj[1]));
				} else {
					res = or_quickmedian_f(sc.stack, nframes);
				}
				float fr = (float)res;
				if (!output_norm) {					/* set_float_in_interval, proto.h:384-388 */
					fr = (fr < 0.f) ? 0.f : fr;
					fr = (fr > 1.f) ? 1.f : fr;
				}
				out[y * W + x] = fr;
			}
		}
		free(buf);
	}
	free(shx);
	if (counts) { counts[0] += c0; counts[1] += c1; }
	return 0;
}

/* One-pixel entry point for tests: runs mean_and_reject (method 0) or the
 * median (method 1) on a single column; returns the double result. */
double or_stack_column_f(const float *col, int n, int method, const or_rej_params *P,
		const double *weights, int rej[2], int *kept_out) {
	float *buf = malloc(5 * (size_t)n * sizeof(float) + 16);
	or_scratch sc = { buf, buf + n, buf + 2 * n, buf + 3 * n, (int *)(buf + 4 * n), NULL, NULL };
	memcpy(sc.stack, col, n * sizeof(float));
	double r;
	rej[0] = rej[1] = 0;
	if (method == 0) {
		r = or_mean_and_reject_f(P, &sc, n, weights, rej);
	} else {
		r = or_quickmedian_f(sc.stack, n);
	}
	if (kept_out) *kept_out = 0;
	free(buf);
	return r;
}

/* ================================================================ 16-bit ==
 * DATA_USHORT path: apply_rejection_ushort (median_and_mean.c:703-954),
 * mean_and_reject ushort branch (:961-1036), with the WORD helpers of
 * sorting.c and statistics.c.  WORD == uint16_t. */

typedef uint16_t WORD;

/* sortnet_median (WORD), sorting.c:366-410 -- same comparator lists as the
 * float network, plus case 9 (used by histogram_median) */
static const unsigned char net9[] = {1,8, 2,7, 3,6, 4,5, 1,4, 5,8, 0,2, 6,7, 2,6, 7,8, 0,3, 4,5,
				     0,1, 3,5, 6,7, 2,4, 1,3, 5,7, 4,6, 1,2, 3,4, 5,6, 7,8, 2,3, 4,5};
double or_sortnet_median_u16(WORD *a, size_t n) {
	size_t k = n / 2;
	if (n == 1) return a[0];
	if (n < 2 || n > 9) return 0.0;
	const unsigned char *p = (n == 9) ? net9 : nets[n];
	const int len = (n == 9) ? (int)(sizeof net9 / 2) : net_len[n];
	for (int c = 0; c < len; c++) {
		int i = p[2 * c], j = p[2 * c + 1];
		if (a[i] > a[j]) { WORD t = a[i]; a[i] = a[j]; a[j] = t; }
	}
	return (n % 2 == 0) ? (a[k - 1] + a[k]) / 2.0 : a[k];
}

/* quickmedian (WORD), sorting.c:195-230 */
double or_quickmedian_u16(WORD *a, size_t n) {
	if (n < 9) return or_sortnet_median_u16(a, n);
	size_t k = n / 2, left = 0, right = n - 1;
	while (left < right) {
		size_t p = (left + right) / 2;
		WORD pivot = a[p];
		a[p] = a[right];
		a[right] = pivot;
		p = left;
		for (size_t i = left; i < right; i++) {
			if (a[i] < pivot) {
				WORD t = a[p]; a[p] = a[i]; a[i] = t;
				p++;
			}
		}
		a[right] = a[p];
		a[p] = pivot;
		if (p < k) left = p + 1;
		else right = p;
	}
	return (n % 2 == 0) ? ((double)a[k - 1] + (double)a[k]) / 2.0 : (double)a[k];
}

/* quicksort_s, sorting.c:160-185 (result = sorted array) */
static void or_quicksort_u16(WORD *a, size_t n) {
	if (n <= 32) {
		for (long i = 1; i < (long)n; i++) {
			const WORD v = a[i];
			long j = i - 1;
			while (j >= 0 && a[j] > v) { a[j + 1] = a[j]; --j; }
			a[j + 1] = v;
		}
		return;
	}
	const WORD pivot = a[n / 2];
	WORD *lo = a, *hi = a + n - 1;
	while (lo <= hi) {
		if (*lo < pivot) { lo++; continue; }
		if (*hi > pivot) { hi--; continue; }
		WORD t = *lo;
		*lo++ = *hi;
		*hi-- = t;
	}
	or_quicksort_u16(a, hi - a + 1);
	or_quicksort_u16(lo, a + n - lo);
}

/* histogram_median (WORD), sorting.c:577-642, single thread (exported: the
 * sorting.c:59-72 pin, tests/test_oracle.py) */
double or_histogram_median_u16(WORD *a, size_t n) {
	if (n < 10) return or_sortnet_median_u16(a, n);
	unsigned int *h = calloc(65536, sizeof *h);
	for (size_t i = 0; i < n; i++) h[a[i]]++;
	unsigned int i = 0, j = 0, k = n / 2, sum = 0;
	if (n % 2 == 0) {
		for (; sum <= k - 1; j++) sum += h[j];
		i = j;
	}
	for (; sum <= k; i++) sum += h[i];
	free(h);
	return (n % 2 == 0) ? (double)(i + j - 2) / 2.0 : (double)(i - 1);
}

/* siril_stats_ushort_sd_32, statistics.c:115-127 */
float or_stats_ushort_sd(const WORD *d, int n) {
	uint32_t isum = 0;
	for (int i = 0; i < n; ++i) isum += d[i];
	float mean = (float)(((double)isum) / ((double)n));
	double acc = 0.0;
	for (int i = 0; i < n; ++i) {
		float px = (float)d[i];
		acc += (px - mean) * (px - mean);
	}
	return sqrtf((float)(acc / (n - 1)));
}

/* siril_stats_ushort_sd (static, median_and_mean.c:647-660) used by grubbs */
static float or_stats_ushort_sd_m(const WORD *d, int n, float *m) {
	double acc = 0.0;
	for (int i = 0; i < n; ++i) acc += d[i];
	float mean = (float)(acc / n);
	acc = 0.0;
	for (int i = 0; i < n; ++i) acc += (d[i] - mean) * (d[i] - mean);
	if (m) *m = mean;
	return sqrtf((float)(acc / (n - 1)));
}

/* siril_stats_ushort_mad, statistics.c:133-154 */
static float or_stats_ushort_mad(const WORD *d, size_t n, double m) {
	int med = or_round_to_int(m);
	WORD *t = malloc(n * sizeof *t);
	for (size_t i = 0; i < n; i++) t[i] = (WORD)abs(d[i] - med);
	float mad = (float)or_histogram_median_u16(t, n);
	free(t);
	return mad;
}

/* roundf_to_WORD, proto.h:341-346; round_to_WORD, :232-237 */
static WORD or_roundf_to_word(float f) {
	f = f + 0.5f;
	f = (f > 65535.f) ? 65535.f : f;
	f = (f < 0.0f) ? 0.0f : f;
	return (WORD)f;
}
static WORD or_round_to_word(double x) {
	x = x + 0.5;
	x = (x > 65535.0) ? 65535.0 : x;
	x = (x < 0.0) ? 0.0 : x;
	return (WORD)x;
}

typedef struct {
	WORD *stack, *o_stack, *w_stack;
	float *yf;
	int *rejected;
	const float *dstack, *mstack;	/* drizzle / feather-mask weights of the column, or NULL */
} or_scratch_u16;

/* percentile_clipping (WORD), median_and_mean.c:589-603 */
static int or_pclip_u16(WORD x, const float sig[2], float med, int rej[2]) {
	if ((med - (float)x) / med > sig[0]) { rej[0]++; return -1; }
	if (((float)x - med) / med > sig[1]) { rej[1]++; return 1; }
	return 0;
}
/* sigma_clipping (WORD), median_and_mean.c:608-621 */
static int or_sclip_u16(WORD x, const float sig[2], float s, float med, int rej[2]) {
	if (med - x > sig[0] * s) { rej[0]++; return -1; }
	if (x - med > sig[1] * s) { rej[1]++; return 1; }
	return 0;
}
/* line_clipping (WORD), median_and_mean.c:630-643 */
static int or_lclip_u16(WORD x, const float sig[2], float s, int i, float a, float b, int rej[2]) {
	if (a * i + b - x > s * sig[0]) { rej[0]++; return -1; }
	if (x - a * i - b > s * sig[1]) { rej[1]++; return 1; }
	return 0;
}
static int or_compact_u16(WORD *s, const int *rej, int n) {
	int o = 0;
	for (int p = 0; p < n; p++)
		if (!rej[p]) s[o++] = s[p];
	return o;
}

/* apply_rejection_ushort, median_and_mean.c:703-954 (no drizzle) */
int or_apply_rejection_u16(const or_rej_params *P, or_scratch_u16 *sc, int nb_frames, int rej[2]) {
	int N = nb_frames, r = 0, firstloop = 1, kept = 0, changed, n;
	float median = 0.f;
	WORD *stack = sc->stack, *w = sc->w_stack;
	int *rejected = sc->rejected;
	memcpy(sc->o_stack, stack, N * sizeof(WORD));
	for (int f = 0; f < N; f++)					/* median_and_mean.c:716-731 */
		if (stack[f] != 0.f && (!sc->dstack || sc->dstack[f] != 0.f)) {
			if (f != kept) stack[kept] = stack[f];
			kept++;
		}
	if (kept <= 1) return kept;
	const int removed = N - kept;
	N = kept;
	switch (P->type) {						/* :747-759 */
	case OR_PERCENTILE: case OR_SIGMA: case OR_MAD: case OR_SIGMEDIAN: case OR_WINSORIZED:
		median = or_quickmedian_u16(stack, N);
		if (median == 0.f) return 0;
		break;
	default: break;
	}
	switch (P->type) {
	case OR_PERCENTILE:
		for (int f = 0; f < N; f++) rejected[f] = or_pclip_u16(stack[f], P->sig, median, rej);
		N = or_compact_u16(stack, rejected, N);
		break;
	case OR_SIGMA: case OR_MAD:
		do {
			float var;
			if (P->type == OR_SIGMA) var = or_stats_ushort_sd(stack, N);
			else var = or_stats_ushort_mad(stack, N, median);
			if (!firstloop) median = or_quickmedian_u16(stack, N);
			else firstloop = 0;
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_sclip_u16(stack[f], P->sig, var, median, rej);
					if (rejected[f]) r++;
				}
			}
			int out = or_compact_u16(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_SIGMEDIAN:
		do {
			const float sigma = or_stats_ushort_sd(stack, N);
			if (!firstloop) median = or_quickmedian_u16(stack, N);
			else firstloop = 0;
			n = 0;
			for (int f = 0; f < N; f++)
				if (or_sclip_u16(stack[f], P->sig, sigma, median, rej)) {
					stack[f] = median;
					n++;
				}
		} while (n > 0);
		break;
	case OR_WINSORIZED:
		do {
			float sigma0, sigma = or_stats_ushort_sd(stack, N);
			if (!firstloop) median = or_quickmedian_u16(stack, N);
			else firstloop = 0;
			memcpy(w, stack, N * sizeof(WORD));
			do {
				const WORD m0 = or_roundf_to_word(median - 1.5f * sigma);
				const WORD m1 = or_roundf_to_word(median + 1.5f * sigma);
				for (int j = 0; j < N; ++j) {		/* Winsorize, :623-628 */
					w[j] = w[j] < m0 ? m0 : w[j];
					w[j] = w[j] > m1 ? m1 : w[j];
				}
				sigma0 = sigma;
				sigma = 1.134f * or_stats_ushort_sd(w, N);
			} while (fabs(sigma - sigma0) > sigma0 * 0.0005f);
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_sclip_u16(stack[f], P->sig, sigma, median, rej);
					if (rejected[f] != 0) r++;
				}
			}
			int out = or_compact_u16(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_LINEARFIT:
		do {
			or_quicksort_u16(stack, N);
			for (int f = 0; f < N; f++) sc->yf[f] = (float)stack[f];
			float a, b;
			or_fit_linear(P->xf, sc->yf, P->m_x, P->m_dx2, N, &b, &a);
			float sigma = 0.f;
			for (int f = 0; f < N; f++) sigma += fabsf(stack[f] - (a * f + b));
			sigma /= (float)N;
			for (int f = 0; f < N; f++) {
				if (N - r <= 4) rejected[f] = 0;
				else {
					rejected[f] = or_lclip_u16(stack[f], P->sig, sigma, f, a, b, rej);
					if (rejected[f] != 0) r++;
				}
			}
			int out = or_compact_u16(stack, rejected, N);
			changed = N != out;
			N = out;
		} while (changed && N > 3);
		break;
	case OR_GESDT: {
		or_quicksort_u16(stack, N);
		{	/* gsl_stats_ushort_median_from_sorted_data into a float */
			size_t lhs = (N - 1) / 2, rhs = N / 2;
			median = (lhs == rhs) ? stack[lhs] : (stack[lhs] + stack[rhs]) / 2.0;
		}
		int max_out = (int)nb_frames * P->sig[0];
		if (removed >= max_out) return kept;
		max_out -= removed;
		or_esd *o = malloc(max_out * sizeof *o);
		memcpy(w, stack, N * sizeof(WORD));
		memset(rejected, 0, N * sizeof(int));
		int cold = 0;
		for (int it = 0, size = N; it < max_out; it++, size--) {
			float avg;
			float sd = or_stats_ushort_sd_m(w, size, &avg);
			float dev = avg - w[0];
			float d2 = w[size - 1] - avg;
			int im;
			if (d2 > dev) { dev = d2; im = size - 1; } else im = 0;
			float g = dev / sd;
			o[it].out = g > P->crit[it + removed];
			o[it].x = w[im];
			o[it].i = (im == 0) ? cold++ : im;
			for (int q = im; q < size - 1; q++) w[q] = w[q + 1];
		}
		or_confirm(o, max_out, median, rejected, rej);
		free(o);
		N = or_compact_u16(stack, rejected, N);
		break;
	}
	default:
		break;
	}
	return N;
}

/* mean_and_reject, ushort branch, median_and_mean.c:961-1036 */
double or_mean_and_reject_u16(const or_rej_params *P, or_scratch_u16 *sc, int n,
		const double *weights, int rej[2]) {
	int kept = or_apply_rejection_u16(P, sc, n, rej);
	if (kept == 0) return or_quickmedian_u16(sc->stack, n);
	if (weights || sc->dstack || sc->mstack) {
		WORD pmin = 65535, pmax = 0;
		for (int f = 0; f < kept; ++f) {
			WORD px = sc->stack[f];
			if (pmin > px) pmin = px;
			if (pmax < px) pmax = px;
		}
		double sum = 0.0, norm = 0.0;
		for (int f = 0; f < n; ++f) {
			WORD v = sc->o_stack[f];
			if (v >= pmin && v <= pmax && v > 0) {
				double w = 1.;					/* :998-1004 */
				if (sc->dstack) w *= sc->dstack[f];
				if (sc->mstack) w *= sc->mstack[f];
				if (weights) w *= weights[f];
				sum += (double)v * w;
				norm += w;
			}
		}
		if (norm == 0. || sum == 0.) {
			sum = 0.;
			for (int f = 0; f < n; ++f) {
				WORD v = sc->o_stack[f];
				if (v >= pmin && v <= pmax && v > 0) sum += (double)v;
			}
			return sum / (double)kept;
		}
		return sum / norm;
	}
	int64_t sum = 0;
	for (int f = 0; f < kept; ++f) sum += sc->stack[f];
	return sum / (double)kept;
}

/* normalize_to16bit (median_and_mean.c:547-555), applied to the 16-bit
 * result when output_norm (:1729-1732): x 65535/255 for BYTE_IMG sources.
 * Set by the caller per call (or_set_out16_mul), 1 by default. */
static double g_out16_mul = 1.0;
void or_set_out16_mul(double m) { g_out16_mul = m; }

/* Block driver for DATA_USHORT frames (median_and_mean.c:1592-1737):
 * normalization with round_to_WORD, output either 32-bit
 * (double_ushort_to_float_range, clamped unless output_norm) into out_f, or
 * 16-bit round_to_WORD into out_u16. */
int or_stack_rows_u16_planes(const WORD *frames, const float *drizz, const float *mask, int nframes, long W,
		long rows, long frame_stride, int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out_f, WORD *out_u16, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads);

int or_stack_rows_u16(const WORD *frames, int nframes, long W, long rows, long frame_stride,
		int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out_f, WORD *out_u16, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads) {
	return or_stack_rows_u16_planes(frames, NULL, NULL, nframes, W, rows, frame_stride, method, P, norm, scale,
			offset, mul, shift_dx, shift_scale, weights, output_norm, out_f, out_u16, rej_lo, rej_hi, counts,
			nthreads);
}

/* Same with per-sample drizzle / feather-mask weight planes (see
 * or_stack_rows_planes_f). */
int or_stack_rows_u16_planes(const WORD *frames, const float *drizz, const float *mask, int nframes, long W,
		long rows, long frame_stride, int method, const or_rej_params *P, int norm, const double *scale,
		const double *offset, const double *mul, const double *shift_dx, double shift_scale,
		const double *weights, int output_norm, float *out_f, WORD *out_u16, uint16_t *rej_lo,
		uint16_t *rej_hi, uint64_t counts[2], int nthreads) {
	uint64_t c0 = 0, c1 = 0;
	int *shx = NULL;
	if (shift_dx) {
		shx = malloc(nframes * sizeof(int));
		for (int f = 0; f < nframes; f++) shx[f] = or_round_to_int(shift_dx[f] * shift_scale);
	}
#ifdef _OPENMP
	if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+:c0, c1)
#endif
	{
		or_scratch_u16 sc;
		WORD *wb = malloc(3 * (size_t)nframes * sizeof(WORD));
		sc.stack = wb;
		sc.o_stack = wb + nframes;
		sc.w_stack = wb + 2 * nframes;
		sc.yf = malloc((size_t)nframes * sizeof(float));
		sc.rejected = malloc((size_t)nframes * sizeof(int));
		float *dst = calloc(2 * (size_t)nframes, sizeof(float)), *mst = dst + nframes;
		sc.dstack = drizz ? dst : NULL;
		sc.mstack = mask ? mst : NULL;
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
		for (long y = 0; y < rows; y++) {
			for (long x = 0; x < W; x++) {
				for (int f = 0; f < nframes; f++) {
					long pix = y * W + x;
					if (shx) {
						int s = shx[f];
						if (s && (x - s >= W || x - s < 0)) { sc.stack[f] = 0; continue; }
						pix -= s;
					}
					WORD v = frames[(size_t)f * frame_stride + pix];
					if (drizz) dst[f] = drizz[(size_t)f * frame_stride + pix];
					if (mask) mst[f] = mask[(size_t)f * frame_stride + pix];
					double t;
					switch (norm) {
					default:
					case OR_NO_NORM: sc.stack[f] = v; break;
					case OR_ADDITIVE: case OR_ADDITIVE_SCALING:
						if (v > 0) {
							t = (double)v * scale[f];
							sc.stack[f] = or_round_to_word(t - offset[f]);
						} else sc.stack[f] = 0;
						break;
					case OR_MULTIPLICATIVE: case OR_MULTIPLICATIVE_SCALING:
						t = (double)v * scale[f];
						sc.stack[f] = or_round_to_word(t * mul[f]);
						break;
					}
				}
				double res;
				int rj[2] = {0, 0};
				if (method == 0) {
					res = or_mean_and_reject_u16(P, &sc, nframes, weights, rj);
					c0 += rj[0];
					c1 += rj[1];
					long o = y * W + x;
					if (rej_lo) rej_lo[o] = (uint16_t)(rj[0] > 65535 ? 65535 : rj[0]);
					if (rej_hi) rej_hi[o] = (uint16_t)(rj[1] > 65535 ? 65535 : rj[1]);
				} else {
					res = or_quickmedian_u16(sc.stack, nframes);
				}
				long o = y * W + x;
				if (out_f) {
					float fr = (float)res * .000015259022f;	/* double_ushort_to_float_range */
					if (!output_norm) {
						fr = (fr < 0.f) ? 0.f : fr;
						fr = (fr > 1.f) ? 1.f : fr;
					}
					out_f[o] = fr;
				}
				if (out_u16) out_u16[o] = or_round_to_word(output_norm ? res * g_out16_mul : res);
			}
		}
		free(wb);
		free(sc.yf);
		free(sc.rejected);
		free(dst);
	}
	free(shx);
	if (counts) { counts[0] += c0; counts[1] += c1; }
	return 0;
}

/* ---------------------------------------------------------------------------
 * Per-frame normalization estimators, DATA_FLOAT.
 * statistics_internal_float (algos/statistics_float.c:281-480) with
 * option STATS_NORM (IKSS) or STATS_LITENORM (median + MAD), normValue 1:
 *   data   = non-zero, non-NaN samples (reassign_to_non_null_data_float :231-252)
 *   median = histogram_median_float(data)            (:425, sorting.c:644-649)
 *   mad    = siril_stats_float_mad(data, median)     (:450, :79-101)
 *   IKSSlite(data, median, mad) -> location, scale   (:469, :199-229)
 *   bwmv   = siril_stats_float_bwmv                  (:103-127)
 * out[0..3] = median, mad, location, scale.  Returns 0, or 1 where the
 * reference returns NULL stats (no good pixel, IKSS kept == 0, MAD == 0).
 * The bwmv double sums are accumulated in index order (the reference's
 * OpenMP reduction order depends on its thread count).
 * ------------------------------------------------------------------------- */
static double or_bwmv_f(const float *x, size_t n, float mad, float median) {
	double up = 0.0, down = 0.0;
	if (!(mad > 0.f)) return 0.0;
	const float factor = 1.f / (9.f * mad);
	for (size_t i = 0; i < n; i++) {
		const float i_med = x[i] - median;
		const float yi = i_med * factor;
		const float yi2 = fabsf(yi) < 1.f ? yi * yi : 1.f;
		const float t = (1 - yi2) * (1 - yi2);
		const float u = i_med * t;
		up += u * u;
		down += (1 - yi2) * (1 - 5 * yi2);
	}
	return down ? n * (up / (down * down)) : 0.0;
}

/* IKSSlite (statistics_float.c:199-229) on float samples: *loc, *scale. */
static int or_ikss_lite(float *d, size_t n, float med, float madf, double *loc_out, double *scale_out) {
	/* xlow = median - 6.0 * mad in double, stored as float */
	const float xlow = med - 6.0 * madf, xhigh = med + 6.0 * madf;
	size_t kept = 0;
	for (size_t i = 0; i < n; i++)
		if (d[i] >= xlow && d[i] <= xhigh) d[kept++] = d[i];
	if (kept == 0) return 1;
	const float loc = or_histogram_percentile_f(d, kept, 0.5f);
	*loc_out = loc;
	const float mad2 = (float)or_stats_float_mad(d, kept, *loc_out);
	if (mad2 == 0.0f) return 1;
	*scale_out = sqrt(or_bwmv_f(d, kept, mad2, (float)*loc_out)) * .991;
	return 0;
}

int or_norm_stats_f(const float *frame, size_t total, int lite, double out[4], size_t *ngood_out) {
	out[0] = out[1] = out[2] = out[3] = 0.0;
	float *d = malloc((total ? total : 1) * sizeof *d);
	size_t n = 0;
	for (size_t i = 0; i < total; i++)
		if (frame[i] != 0.f && !isnan(frame[i])) d[n++] = frame[i];
	if (ngood_out) *ngood_out = n;
	if (n == 0) { free(d); return 1; }
	const float med = or_histogram_percentile_f(d, n, 0.5f);
	out[0] = med;
	const double mad = or_stats_float_mad(d, n, out[0]);
	out[1] = mad;
	int st = lite ? 0 : or_ikss_lite(d, n, med, (float)mad, &out[2], &out[3]);
	free(d);
	return st;
}

/* statistics_internal_ushort (algos/statistics.c:231-449) with STATS_NORM /
 * STATS_LITENORM: data = samples > 0 (reassign_to_non_null_data_ushort
 * :183-204); median = histogram_median (sorting.c:575-641, exact order
 * statistics); mad = siril_stats_ushort_mad (:133-154); IKSSlite on
 * (float)x * (float)(1/65535.0) with median and mad scaled the same way
 * (:402-438); location and scale multiplied back by 65535.0. */
int or_norm_stats_u16(const WORD *frame, size_t total, int lite, double out[4], size_t *ngood_out) {
	out[0] = out[1] = out[2] = out[3] = 0.0;
	WORD *d = malloc((total ? total : 1) * sizeof *d);
	size_t n = 0;
	for (size_t i = 0; i < total; i++)
		if (frame[i] > 0) d[n++] = frame[i];
	if (ngood_out) *ngood_out = n;
	if (n == 0) { free(d); return 1; }
	out[0] = or_histogram_median_u16(d, n);
	out[1] = or_stats_ushort_mad(d, n, out[0]);
	if (lite) { free(d); return 0; }
	const double normValue = 65535.0;		/* USHRT_MAX_DOUBLE */
	const float inv = (float)(1.0 / normValue);
	float *f = malloc(n * sizeof *f);
	for (size_t i = 0; i < n; i++) f[i] = (float)d[i] * inv;
	const float med = (float)(out[0]) * inv;
	const float mad = (float)(out[1]) * inv;
	int st = or_ikss_lite(f, n, med, mad, &out[2], &out[3]);
	out[2] *= normValue;
	out[3] *= normValue;
	free(f);
	free(d);
	return st;
}
