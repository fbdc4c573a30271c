// overlap_norm.hip -- overlap normalization (stacking/normalization.c:296-938,
// `stack ... -overlap_norm`): per-pair estimators on the overlap of every two
// registered frames, then the least-squares coefficients.
//
// Reference flow (compute_normalization_overlaps, :666-906):
//   * compute_overlap (:420-456): with the integer translation between frames
//     i and j (dx = round_to_int(dxj - dxi), dy = round_to_int(dyi - dyj) from
//     translation_from_H), the two equal-size rectangles the frames share;
//   * _compute_estimators_for_images (:458-598): the samples non-zero in BOTH
//     frames (16-bit data as (float)x * (float)(1/USHRT_MAX)); with more than
//     3 of them, on each side: median = histogram_median_float, mad =
//     siril_stats_float_mad (both cast to float), and unless lite
//     IKSSlite(location, scale) cast to float (location 0 / scale 1 where
//     IKSSlite returns early);
//   * solve_overlap_coeffs (:296-355): an (N-1) x (N-1) linear system per
//     layer (GSL LU with partial pivoting), scales from the scale estimators
//     (ADDITIVE_SCALING / MULTIPLICATIVE_SCALING), then offsets
//     (ADDITIVE[_SCALING], on the rescaled locations) or multipliers
//     (MULTIPLICATIVE).
//
// GPU mapping: the pairs' masked samples are packed side by side into a
// workspace (k_overlap_pack: one read of each overlap, one write; zeros mark
// "not in both", padding to the batch's largest overlap is zero too) and the
// packed planes run through the STATS_NORM estimator kernels of norm_stats.hip
// (which count non-zero samples only), all pairs of a batch in the same
// launches.  The estimators are order independent (histogram percentiles;
// the bwmv sums are compared to a relative 1e-12 as for per-frame stats), so
// packing order does not matter.  Differences: samples that are NaN are
// skipped by the estimator kernels while the reference keeps them in datai
// (NaN is non-zero); frames are the stacked list only (the reference's cache
// seq->ostats is not kept).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <limits>
#include <vector>

#include "sgpu_internal.h"

namespace sgpu {
namespace ov {

struct PairRect {
    int i, j;          // frame indices in the stacked list
    int xi, yi, xj, yj;
    int w, h;
};

// one pair per blockIdx.y; side 0 -> plane 2p, side 1 -> plane 2p + 1
template <typename T>
__global__ __launch_bounds__(256) void k_overlap_pack(const T *frames, long long fstride, long long W,
                                                      const PairRect *pairs, float *out, long long plane) {
    const PairRect pr = pairs[blockIdx.y];
    const long long n = (long long)pr.w * pr.h;
    float *oi = out + (size_t)(2 * blockIdx.y) * plane;
    float *oj = oi + plane;
    const T *fi = frames + (size_t)pr.i * fstride;
    const T *fj = frames + (size_t)pr.j * fstride;
    const float inv = (float)(1.0 / 65535.0);   // invnorm = 1. / USHRT_MAX (normalization.c:464)
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < plane;
         k += (long long)gridDim.x * blockDim.x) {
        float a = 0.f, b = 0.f;
        if (k < n) {
            const long long r = k / pr.w, cc = k - r * pr.w;
            const T ta = fi[(pr.yi + r) * W + pr.xi + cc];
            const T tb = fj[(pr.yj + r) * W + pr.xj + cc];
            if (ta != (T)0 && tb != (T)0) {      // :555 / :560
                if constexpr (sizeof(T) == 2) {
                    a = (float)ta * inv;
                    b = (float)tb * inv;
                } else {
                    a = (float)ta;
                    b = (float)tb;
                }
            }
        }
        oi[k] = a;
        oj[k] = b;
    }
}

}  // namespace ov
}  // namespace sgpu

namespace {

using sgpu::ov::PairRect;

int round_to_int(double x) {   // core/proto.h:208-213
    x = (x > (double)INT_MAX - 0.5) ? (double)INT_MAX - 0.5 : x;
    x = (x < (double)INT_MIN + 0.5) ? (double)INT_MIN + 0.5 : x;
    const double offset = (x >= 0.0) ? 0.5 : -0.5;
    return (int)(x + offset);
}

// compute_overlap (normalization.c:420-456) for frames of one size
long overlap_rect(int W, int H, double dxi, double dyi, double dxj, double dyj, int *ri, int *rj) {
    int dx = round_to_int(dxj - dxi);
    int dy = round_to_int(dyi - dyj);
    if (dx == INT_MIN) dx += 1;
    if (dy == INT_MIN) dy += 1;
    const int x_tli = std::max(0, dx), y_tli = std::max(0, dy);
    const int x_bri = std::min(W, dx + W), y_bri = std::min(H, dy + H);
    const int x_tlj = std::max(0, -dx), y_tlj = std::max(0, -dy);
    if (x_tli < x_bri && y_tli < y_bri) {
        ri[0] = x_tli; ri[1] = y_tli; ri[2] = x_bri - x_tli; ri[3] = y_bri - y_tli;
        rj[0] = x_tlj; rj[1] = y_tlj; rj[2] = x_bri - x_tli; rj[3] = y_bri - y_tli;
        return (long)(x_bri - x_tli) * (y_bri - y_tli);
    }
    return 0;
}

inline int pair_index(int N, int i, int j) { return i * (2 * N - i - 1) / 2 + j - i - 1; }   // :412-414

template <typename T>
int overlap_stats(sgpu_context *c, const T *d_frames, int nframes, long W, long H, long fstride,
                  const double *h02, const double *h12, int lite, long *nij, double *stats) {
    HIP_TRY(hipSetDevice(c->device));
    const int npairs = nframes * (nframes - 1) / 2;
    std::vector<PairRect> pr;
    std::vector<int> pidx;
    long maxn = 0;
    for (int i = 0; i < nframes; ++i)
        for (int j = i + 1; j < nframes; ++j) {
            const int p = pair_index(nframes, i, j);
            nij[p] = 0;
            for (int k = 0; k < 8; ++k) stats[8 * p + k] = 0.0;
            int ri[4], rj[4];
            // translation_from_H (registration.c:301-304): dx = h02, dy = -h12
            const long n = overlap_rect((int)W, (int)H, h02[i], -h12[i], h02[j], -h12[j], ri, rj);
            if (n <= 0) continue;
            pr.push_back(PairRect{i, j, ri[0], ri[1], rj[0], rj[1], ri[2], ri[3]});
            pidx.push_back(p);
            maxn = std::max(maxn, n);
        }
    (void)npairs;
    if (pr.empty()) return SGPU_OK;
    // batches of pairs whose packed planes fit a 4 GiB workspace
    const long long plane = (maxn + 63) & ~63LL;
    const size_t pair_bytes = 2 * sizeof(float) * (size_t)plane;
    const int batch = (int)std::max<size_t>(1, std::min<size_t>(pr.size(), ((size_t)4 << 30) / pair_bytes));
    int rc;
    if ((rc = c->ov_ws.ensure(pair_bytes * batch)) || (rc = c->ov_tab.ensure(sizeof(PairRect) * batch))) return rc;
    std::vector<double> st(4 * 2 * (size_t)batch);
    std::vector<long> ng(2 * (size_t)batch);
    std::vector<int> status(2 * (size_t)batch);
    for (size_t b0 = 0; b0 < pr.size(); b0 += batch) {
        const int nb = (int)std::min<size_t>(batch, pr.size() - b0);
        HIP_TRY(hipMemcpyAsync(c->ov_tab.p, pr.data() + b0, sizeof(PairRect) * nb, hipMemcpyHostToDevice,
                               c->stream));
        const unsigned gx = (unsigned)std::min<long long>(1024, (plane + 255) / 256);
        hipLaunchKernelGGL(sgpu::ov::k_overlap_pack<T>, dim3(gx, (unsigned)nb), dim3(256), 0, c->stream, d_frames,
                           (long long)fstride, (long long)W, (const PairRect *)c->ov_tab.p, (float *)c->ov_ws.p,
                           plane);
        HIP_TRY(hipGetLastError());
        if ((rc = sgpu_norm_stats_device(c, (const float *)c->ov_ws.p, 2 * nb, (long)plane, (long)plane, lite,
                                         st.data(), ng.data(), status.data())))
            return rc;
        for (int q = 0; q < nb; ++q) {
            const int p = pidx[b0 + q];
            const long n = ng[2 * q];            // same mask on both sides
            if (n <= 3) continue;                // :567 "at least 3 pixels"
            nij[p] = n;
            for (int side = 0; side < 2; ++side) {
                const double *s = &st[4 * (2 * q + side)];
                const int bad = status[2 * q + side];
                stats[8 * p + 0 + side] = (double)(float)s[0];                    // medij / medji
                stats[8 * p + 2 + side] = (double)(float)s[1];                    // madij / madji
                if (!lite) {
                    // IKSSlite: location set unless kept == 0 (then 0, its
                    // initial value), scale only on success (else 1)
                    stats[8 * p + 4 + side] = (double)(float)s[2];                // locij / locji
                    stats[8 * p + 6 + side] = bad ? 1.0 : (double)(float)s[3];    // scaij / scaji
                }
            }
        }
    }
    return SGPU_OK;
}

// gsl_linalg_LU_decomp (unblocked, partial pivoting on the first largest
// |a|) + gsl_linalg_LU_solve, row-major n x n
void lu_solve(int n, std::vector<double> &A, std::vector<double> &b, std::vector<double> &x) {
    std::vector<int> perm((size_t)n);
    for (int i = 0; i < n; ++i) perm[(size_t)i] = i;
    auto a = [&](int r, int cc) -> double & { return A[(size_t)r * n + cc]; };
    for (int j = 0; j < n - 1; ++j) {
        double mx = std::fabs(a(j, j));
        int ip = j;
        for (int i = j + 1; i < n; ++i) {
            const double v = std::fabs(a(i, j));
            if (v > mx) { mx = v; ip = i; }
        }
        if (ip != j) {
            for (int cc = 0; cc < n; ++cc) std::swap(a(j, cc), a(ip, cc));
            std::swap(perm[(size_t)j], perm[(size_t)ip]);
        }
        const double ajj = a(j, j);
        if (ajj != 0.0) {
            for (int i = j + 1; i < n; ++i) {
                const double aij = (a(i, j) /= ajj);
                for (int k = j + 1; k < n; ++k) a(i, k) -= aij * a(j, k);
            }
        }
    }
    x.assign((size_t)n, 0.0);
    for (int i = 0; i < n; ++i) x[(size_t)i] = b[(size_t)perm[(size_t)i]];
    for (int i = 0; i < n; ++i)            // L y = P b (unit lower)
        for (int k = 0; k < i; ++k) x[(size_t)i] -= a(i, k) * x[(size_t)k];
    for (int i = n - 1; i >= 0; --i) {     // U x = y
        for (int k = i + 1; k < n; ++k) x[(size_t)i] -= a(i, k) * x[(size_t)k];
        x[(size_t)i] /= a(i, i);
    }
}

// solve_overlap_coeffs (normalization.c:296-355); M[i*n + j] = Mij[i][j]
void solve_coeffs(int n, const std::vector<int> &index, int ref, const std::vector<double> &Nij,
                  const std::vector<double> &M, bool additive, std::vector<double> &coeffs) {
    const int N = n - 1;
    std::vector<double> A((size_t)N * N, 0.0), B((size_t)N, 0.0);
    auto nn = [&](int i, int j) { return Nij[(size_t)i * n + j]; };
    auto mm = [&](int i, int j) { return M[(size_t)i * n + j]; };
    int c = 0;
    for (int i = 0; i < N; ++i) {
        const int ii = index[(size_t)i];
        B[(size_t)i] = additive ? nn(ii, ref) * (mm(ref, ii) - mm(ii, ref)) : nn(ii, ref) * mm(ref, ii) * mm(ii, ref);
        for (int j = 0; j < N; ++j) {
            const int ij = index[(size_t)j];
            if (ii == ij) {
                for (int k = 0; k < n; ++k)
                    if (k != ii) A[(size_t)c] += additive ? nn(ii, k) : nn(ii, k) * mm(ii, k) * mm(ii, k);
            } else {
                A[(size_t)c] = additive ? -nn(ii, ij) : -nn(ii, ij) * mm(ii, ij) * mm(ij, ii);
                if (additive) B[(size_t)i] += nn(ii, ij) * (mm(ij, ii) - mm(ii, ij));
            }
            c++;
        }
    }
    lu_solve(N, A, B, coeffs);
}

}  // namespace

extern "C" int sgpu_overlap_rect(int width, int height, double dxi, double dyi, double dxj, double dyj,
                                 int *area_i, int *area_j, long *npix) {
    if (!area_i || !area_j || !npix || width <= 0 || height <= 0)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_overlap_rect: bad arguments");
    for (int k = 0; k < 4; ++k) area_i[k] = area_j[k] = 0;
    *npix = overlap_rect(width, height, dxi, dyi, dxj, dyj, area_i, area_j);
    return SGPU_OK;
}

#define OV_ARGS_OK(fr) (c && (fr) && nframes >= 2 && width > 0 && height > 0 && \
                        frame_stride >= width * height && h02 && h12 && nij && stats)

extern "C" int sgpu_overlap_stats_device(sgpu_context *c, const float *d_frames, int nframes, long width,
                                         long height, long frame_stride, const double *h02, const double *h12,
                                         int lite, long *nij, double *stats) {
    if (!OV_ARGS_OK(d_frames)) return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_overlap_stats_device: bad arguments");
    return overlap_stats<float>(c, d_frames, nframes, width, height, frame_stride, h02, h12, lite, nij, stats);
}

extern "C" int sgpu_overlap_stats_u16_device(sgpu_context *c, const uint16_t *d_frames, int nframes, long width,
                                             long height, long frame_stride, const double *h02,
                                             const double *h12, int lite, long *nij, double *stats) {
    if (!OV_ARGS_OK(d_frames))
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_overlap_stats_u16_device: bad arguments");
    return overlap_stats<unsigned short>(c, d_frames, nframes, width, height, frame_stride, h02, h12, lite, nij,
                                         stats);
}

extern "C" int sgpu_overlap_factors(int normalize, int lite, int nframes, int ref_index, const long *nij,
                                    const double *stats, double *offset, double *mul, double *scale) {
    if (nframes < 2 || ref_index < 0 || ref_index >= nframes || !nij || !stats || !offset || !mul || !scale)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_overlap_factors: bad arguments");
    for (int i = 0; i < nframes; ++i) {   // init_coeffs
        offset[i] = 0.0;
        mul[i] = 1.0;
        scale[i] = 1.0;
    }
    if (normalize == SGPU_NO_NORM) return SGPU_OK;
    if (normalize != SGPU_ADDITIVE && normalize != SGPU_MULTIPLICATIVE && normalize != SGPU_ADDITIVE_SCALING &&
        normalize != SGPU_MULTIPLICATIVE_SCALING)
        return sgpu_host::fail(SGPU_BAD_ARGUMENT, "sgpu_overlap_factors: unknown normalization");
    const int n = nframes;
    std::vector<double> Nm((size_t)n * n, 0.0), M((size_t)n * n, 0.0), S((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {       // :804-821
            const int p = pair_index(n, i, j);
            if (nij[p] == 0) continue;
            const double *s = stats + 8 * (size_t)p;
            M[(size_t)i * n + j] = lite ? s[0] : s[4];
            M[(size_t)j * n + i] = lite ? s[1] : s[5];
            S[(size_t)i * n + j] = lite ? s[2] : s[6];
            S[(size_t)j * n + i] = lite ? s[3] : s[7];
            Nm[(size_t)i * n + j] = Nm[(size_t)j * n + i] = (double)nij[p];
        }
    std::vector<int> index;
    for (int i = 0; i < n; ++i)
        if (i != ref_index) index.push_back(i);
    std::vector<double> coeffs;
    if (normalize == SGPU_MULTIPLICATIVE_SCALING || normalize == SGPU_ADDITIVE_SCALING) {   // :875-888
        solve_coeffs(n, index, ref_index, Nm, S, false, coeffs);
        for (int i = 0; i < n - 1; ++i) scale[index[(size_t)i]] = coeffs[(size_t)i];
        for (int ii = 0; ii < n; ++ii)
            for (int jj = 0; jj < n; ++jj) M[(size_t)ii * n + jj] *= scale[ii];
    }
    if (normalize == SGPU_ADDITIVE || normalize == SGPU_ADDITIVE_SCALING) {                 // :890-897
        solve_coeffs(n, index, ref_index, Nm, M, true, coeffs);
        for (int i = 0; i < n - 1; ++i) offset[index[(size_t)i]] = -coeffs[(size_t)i];
    }
    if (normalize == SGPU_MULTIPLICATIVE) {                                                   // :899-905
        solve_coeffs(n, index, ref_index, Nm, M, false, coeffs);
        for (int i = 0; i < n - 1; ++i) mul[index[(size_t)i]] = coeffs[(size_t)i];
    }
    return SGPU_OK;
}
