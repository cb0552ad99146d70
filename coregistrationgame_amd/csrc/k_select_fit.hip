// k_select_fit.hip -- FRMSD-optimal fraction selection (ficp.py:54-60, 73-86) and the
// 2D rigid least-squares fit (ficp.py:89-110) on the device.
//
// Fraction: the reference evaluates FRMSD(k) = (1.0 / (k/N)**lambda) * sqrt(S_k / k) for
// every prefix k of argsort(dist), each with a fresh O(k) sum -> O(N^2) (ficp.py:80-85).
// Here S_k is ONE prefix scan of r_(j) = sum_md (src - corr)^2 in the sorted order
// (tile sums -> scan of tile sums -> per-tile scan fused with the FRMSD evaluation and
// a first-minimum argmin), all deterministic (fixed reduction trees, no float atomics).
//
// Fit: two passes like the reference (centroids, then the 2x2 cross-covariance of the
// centred pairs), reduced per tile and combined in a fixed order; coordinates are
// shifted by a pivot (the CHM-layer centre) before summation so geo-referenced inputs
// (~6.5e6 m) keep full precision.  R comes from the closed form of the 2x2 Kabsch
// problem: rotation angle atan2(H01 - H10, H00 + H11) -- identical to the SVD path
// R = Vt^T U^T with the det fix of ficp.py:101-103; with
// allow_reflection the SVD path returns a reflection iff det(H) < 0, given here by the
// angle atan2(H01 + H10, H00 - H11).
#include "ficp_internal.h"

#include <math.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int FB = 256;
constexpr int FI = 16;
constexpr int FTILE = FB * FI;

__device__ __forceinline__ double block_sum_d(double v, double *s /*[256]*/) {
    // fixed-order tree: deterministic
    s[threadIdx.x] = v;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
        __syncthreads();
    }
    const double r = s[0];
    __syncthreads();
    return r;
}

// exclusive scan of one double per thread (Hillis-Steele in LDS, deterministic)
__device__ __forceinline__ double block_excl_scan_d(double v, double *s /*[2][256]*/) {
    double *a = s, *b = s + 256;
    a[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const double x =
            ((int)threadIdx.x >= o) ? a[threadIdx.x - o] + a[threadIdx.x] : a[threadIdx.x];
        b[threadIdx.x] = x;
        __syncthreads();
        double *t = a;
        a = b;
        b = t;
    }
    const double ex = threadIdx.x ? a[threadIdx.x - 1] : 0.0;
    __syncthreads();
    return ex;
}

__device__ __forceinline__ double frmsd_of(long long k, long long N, double S, double lam) {
    const double frac = (double)k / (double)N;
    return (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
}

__device__ __forceinline__ bool better(double f, long long k, double bf, long long bk) {
    return f < bf || (f == bf && k < bk);
}

__global__ __launch_bounds__(256) void k_residuals(const double *sx, const double *sy,
                                                   const double *sz, const double *cx,
                                                   const double *cy, const double *cz,
                                                   int64_t n, int md, double *r) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double dx = sx[i] - cx[i];
    const double dy = sy[i] - cy[i];
    double s = dx * dx;
    s = s + dy * dy;
    if (md == 3) {
        const double dz = sz[i] - cz[i];
        s = s + dz * dz;
    }
    r[i] = s;
}

// per tile: sum of r in sorted order
__global__ __launch_bounds__(FB) void k_frac_tilesum(const uint32_t *order, const double *r,
                                                     int64_t n, double *tsum, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[256];
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + (int64_t)threadIdx.x * FI;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < FI; ++q)
        if (j0 + q < n) acc = acc + r[order[j0 + q]];
    const double t = block_sum_d(acc, s);
    if (threadIdx.x == 0) tsum[blockIdx.x] = t;
}

// single block: exclusive scan of the tile sums (sequential per thread segment)
__global__ __launch_bounds__(256) void k_frac_tilescan(double *tsum, int nb, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[512];
    const int per = (nb + 255) / 256;
    const int b0 = threadIdx.x * per;
    double acc = 0.0;
    for (int b = b0; b < min(nb, b0 + per); ++b) acc = acc + tsum[b];
    double pre = block_excl_scan_d(acc, s);
    for (int b = b0; b < min(nb, b0 + per); ++b) {
        const double c = tsum[b];
        tsum[b] = pre;
        pre = pre + c;
    }
    if (threadIdx.x == 255) tsum[nb] = pre;  // grand total (last segment's running sum)
}

struct BestRec {
    double f;
    long long k;
};

__global__ __launch_bounds__(FB) void k_frac_eval(const uint32_t *order, const double *r,
                                                  int64_t n, int64_t N, double lam,
                                                  const double *tpre, BestRec *tbest,
                                                  const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[512];
    __shared__ double s_f[256];
    __shared__ long long s_k[256];
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + (int64_t)threadIdx.x * FI;
    double v[FI];
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < FI; ++q) {
        v[q] = (j0 + q < n) ? r[order[j0 + q]] : 0.0;
        acc = acc + v[q];
    }
    double S = tpre[blockIdx.x] + block_excl_scan_d(acc, s);
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
#pragma unroll
    for (int q = 0; q < FI; ++q) {
        const int64_t j = j0 + q;
        if (j < n && j < N) {
            S = S + v[q];
            const long long k = j + 1;
            const double f = frmsd_of(k, N, S, lam);
            if (f < bf) {  // ascending k: strict < keeps the first minimum
                bf = f;
                bk = k;
            }
        }
    }
    s_f[threadIdx.x] = bf;
    s_k[threadIdx.x] = bk;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            if (better(s_f[threadIdx.x + w], s_k[threadIdx.x + w], s_f[threadIdx.x], s_k[threadIdx.x])) {
                s_f[threadIdx.x] = s_f[threadIdx.x + w];
                s_k[threadIdx.x] = s_k[threadIdx.x + w];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tbest[blockIdx.x].f = s_f[0];
        tbest[blockIdx.x].k = s_k[0];
    }
}

__global__ __launch_bounds__(256) void k_frac_final(const BestRec *tbest, int nb, const double *tpre,
                                                    int64_t n, int64_t N, double lam,
                                                    IterState *st, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s_f[256];
    __shared__ long long s_k[256];
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    for (int b = threadIdx.x; b < nb; b += 256)
        if (better(tbest[b].f, tbest[b].k, bf, bk)) {
            bf = tbest[b].f;
            bk = tbest[b].k;
        }
    s_f[threadIdx.x] = bf;
    s_k[threadIdx.x] = bk;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            if (better(s_f[threadIdx.x + w], s_k[threadIdx.x + w], s_f[threadIdx.x], s_k[threadIdx.x])) {
                s_f[threadIdx.x] = s_f[threadIdx.x + w];
                s_k[threadIdx.x] = s_k[threadIdx.x + w];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        bf = s_f[0];
        bk = s_k[0];
        if (N > n) {
            // k in (n, N]: the selection saturates at n rows, S stays S_n and FRMSD falls
            // with k, so only k = N can win there (ficp.py:80-85 with len(order) < N)
            const double f = frmsd_of(N, N, tpre[nb], lam);
            if (f < bf) {
                bf = f;
                bk = N;
            }
        }
        if (bk == 0x7fffffffffffffffLL) {  // every FRMSD was NaN/inf: reference keeps (0.0, 0)
            st->k = 0;
            st->frac = 0.0;
            st->frmsd = INFINITY;
        } else {
            st->k = bk;
            st->frac = (double)bk / (double)N;
            st->frmsd = bf;
        }
        st->n_src = N;
    }
}

// ------------------------------------------------------------------------- fit
struct FitIn {
    const uint32_t *order;  // selection order (null: rows 0..k-1)
    const double *sx, *sy;
    const int32_t *idx;     // partner index (null: same row)
    const double *tx, *ty;
    int64_t kfixed;         // k when order == null
    double px, py;          // pivot
    const IterState *st;
};

__device__ __forceinline__ int64_t fit_k(const FitIn &a) { return a.order ? (int64_t)a.st->k : a.kfixed; }

__device__ __forceinline__ void fit_pair(const FitIn &a, int64_t j, double &xs, double &ys,
                                         double &xt, double &yt) {
    const int64_t i = a.order ? (int64_t)a.order[j] : j;
    const int64_t m = a.idx ? (int64_t)a.idx[i] : i;
    xs = a.sx[i] - a.px;
    ys = a.sy[i] - a.py;
    xt = a.tx[m] - a.px;
    yt = a.ty[m] - a.py;
}

__global__ __launch_bounds__(FB) void k_fit_pass1(FitIn a, double *part, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[256];
    const int64_t k = fit_k(a);
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + (int64_t)threadIdx.x * FI;
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int q = 0; q < FI; ++q) {
        const int64_t j = j0 + q;
        if (j < k) {
            double xs, ys, xt, yt;
            fit_pair(a, j, xs, ys, xt, yt);
            c0 = c0 + xs;
            c1 = c1 + ys;
            c2 = c2 + xt;
            c3 = c3 + yt;
        }
    }
    c0 = block_sum_d(c0, s);
    c1 = block_sum_d(c1, s);
    c2 = block_sum_d(c2, s);
    c3 = block_sum_d(c3, s);
    if (threadIdx.x == 0) {
        part[4 * blockIdx.x + 0] = c0;
        part[4 * blockIdx.x + 1] = c1;
        part[4 * blockIdx.x + 2] = c2;
        part[4 * blockIdx.x + 3] = c3;
    }
}

// identical fixed-order reduction of the pass-1 partials in every block that needs it
__device__ __forceinline__ void fit_centroids(const double *part, int nb, int64_t k, double *s,
                                              double c[4]) {
    for (int e = 0; e < 4; ++e) {
        double acc = 0.0;
        for (int b = threadIdx.x; b < nb; b += 256) acc = acc + part[4 * b + e];
        c[e] = block_sum_d(acc, s) / (double)k;
    }
}

__global__ __launch_bounds__(FB) void k_fit_pass2(FitIn a, const double *part1, int nb,
                                                  double *part2, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[256];
    const int64_t k = fit_k(a);
    const int64_t j0b = (int64_t)blockIdx.x * FTILE;
    if (j0b >= k) {
        if (threadIdx.x < 4) part2[4 * blockIdx.x + threadIdx.x] = 0.0;
        return;
    }
    double c[4];
    fit_centroids(part1, nb, k, s, c);
    const int64_t j0 = j0b + (int64_t)threadIdx.x * FI;
    double h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (int q = 0; q < FI; ++q) {
        const int64_t j = j0 + q;
        if (j < k) {
            double xs, ys, xt, yt;
            fit_pair(a, j, xs, ys, xt, yt);
            xs = xs - c[0];
            ys = ys - c[1];
            xt = xt - c[2];
            yt = yt - c[3];
            h0 = h0 + xs * xt;
            h1 = h1 + xs * yt;
            h2 = h2 + ys * xt;
            h3 = h3 + ys * yt;
        }
    }
    h0 = block_sum_d(h0, s);
    h1 = block_sum_d(h1, s);
    h2 = block_sum_d(h2, s);
    h3 = block_sum_d(h3, s);
    if (threadIdx.x == 0) {
        part2[4 * blockIdx.x + 0] = h0;
        part2[4 * blockIdx.x + 1] = h1;
        part2[4 * blockIdx.x + 2] = h2;
        part2[4 * blockIdx.x + 3] = h3;
    }
}

__global__ __launch_bounds__(256) void k_fit_final(FitIn a, const double *part1,
                                                   const double *part2, int nb, int allow_refl,
                                                   IterState *st, const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[256];
    const int64_t k = fit_k(a);
    double c[4];
    fit_centroids(part1, nb, k, s, c);
    double H[4];
    for (int e = 0; e < 4; ++e) {
        double acc = 0.0;
        for (int b = threadIdx.x; b < nb; b += 256) acc = acc + part2[4 * b + e];
        H[e] = block_sum_d(acc, s);
    }
    if (threadIdx.x != 0) return;
    double R00, R01, R10, R11;
    const double det = H[0] * H[3] - H[1] * H[2];
    if (allow_refl && det < 0.0) {
        // SVD path without the det fix: R = V U^T is the reflection Rot(a1) diag(1,-1)
        const double F = H[0] - H[3], G = H[2] + H[1];
        const double nrm = hypot(F, G);
        const double cc = F / nrm, ss = G / nrm;
        R00 = cc;
        R01 = ss;
        R10 = ss;
        R11 = -cc;
    } else {
        const double A = H[0] + H[3], B = H[1] - H[2];
        const double nrm = hypot(A, B);
        double cc = 1.0, ss = 0.0;  // H = 0 (k = 1): the SVD path gives R = I
        if (nrm > 0.0) {
            cc = A / nrm;
            ss = B / nrm;
        }
        R00 = cc;
        R01 = -ss;
        R10 = ss;
        R11 = cc;
    }
    // centroids in world coordinates, t = ct - cs @ R^T (ficp.py:105)
    const double csx = c[0] + a.px, csy = c[1] + a.py;
    const double ctx = c[2] + a.px, cty = c[3] + a.py;
    const double tx = ctx - (csx * R00 + csy * R01);
    const double ty = cty - (csx * R10 + csy * R11);
    st->T[0] = R00;
    st->T[1] = R01;
    st->T[2] = tx;
    st->T[3] = R10;
    st->T[4] = R11;
    st->T[5] = ty;
    st->T[6] = 0.0;
    st->T[7] = 0.0;
    st->T[8] = 1.0;
    st->csx = c[0];
    st->csy = c[1];
    st->ctx = c[2];
    st->cty = c[3];
    for (int e = 0; e < 4; ++e) st->H[e] = H[e];
}

// --------------------------------------------------------------- frmsd (public API)
__global__ __launch_bounds__(256) void k_ssd_partial(const double *sx, const double *sy,
                                                     const double *sz, const double *cx,
                                                     const double *cy, const double *cz,
                                                     int64_t k, int md, double *part) {
    __shared__ double s[256];
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + (int64_t)threadIdx.x * FI;
    double acc = 0.0;
    for (int q = 0; q < FI; ++q) {
        const int64_t i = j0 + q;
        if (i < k) {
            const double dx = sx[i] - cx[i], dy = sy[i] - cy[i];
            double r = dx * dx;
            r = r + dy * dy;
            if (md == 3) {
                const double dz = sz[i] - cz[i];
                r = r + dz * dz;
            }
            acc = acc + r;
        }
    }
    acc = block_sum_d(acc, s);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_ssd_final(const double *part, int nb, double *out) {
    __shared__ double s[256];
    double acc = 0.0;
    for (int b = threadIdx.x; b < nb; b += 256) acc = acc + part[b];
    acc = block_sum_d(acc, s);
    if (threadIdx.x == 0) *out = acc;
}

__global__ __launch_bounds__(256) void k_gather_xy(const int32_t *idx, const double *tx,
                                                   const double *ty, int64_t n, double *ox,
                                                   double *oy) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int j = idx[i];
    ox[i] = tx[j];
    oy[i] = ty[j];
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }
inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

}  // namespace

int64_t frac_tmp_bytes(int64_t n) {
    const int64_t nb = (n + FTILE - 1) / FTILE + 1;
    return align_up((nb + 1) * 8, 256) + align_up(nb * (int64_t)sizeof(BestRec), 256);
}

hipError_t launch_residuals(const double *sx, const double *sy, const double *sz,
                            const double *cx, const double *cy, const double *cz, int64_t n,
                            int md, double *r, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_residuals, dim3(nblk(n)), dim3(256), 0, s, sx, sy, sz, cx, cy, cz, n, md,
                       r);
    return hipGetLastError();
}

hipError_t launch_fraction(const uint32_t *order, const double *r, int64_t n, int64_t n_src,
                           double lam, void *tmp, IterState *st, const int *skip, hipStream_t s) {
    const int nb = (int)((n + FTILE - 1) / FTILE);
    char *p = (char *)tmp;
    double *tsum = (double *)p;
    p += align_up((int64_t)(nb + 2) * 8, 256);
    BestRec *tbest = (BestRec *)p;
    if (nb > 0) {
        hipLaunchKernelGGL(k_frac_tilesum, dim3(nb), dim3(FB), 0, s, order, r, n, tsum, skip);
        hipLaunchKernelGGL(k_frac_tilescan, dim3(1), dim3(256), 0, s, tsum, nb, skip);
        hipLaunchKernelGGL(k_frac_eval, dim3(nb), dim3(FB), 0, s, order, r, n, n_src, lam, tsum,
                           tbest, skip);
    }
    hipLaunchKernelGGL(k_frac_final, dim3(1), dim3(256), 0, s, tbest, nb, tsum, n, n_src, lam, st,
                       skip);
    return hipGetLastError();
}

int64_t fit_tmp_bytes(int64_t n) {
    const int64_t nb = (n + FTILE - 1) / FTILE + 1;
    return 2 * align_up(nb * 4 * 8, 256);
}

hipError_t launch_fit(const uint32_t *order, const double *sx, const double *sy,
                      const int32_t *idx, const double *tx, const double *ty, int64_t n,
                      double px, double py, int allow_reflection, void *tmp, IterState *st,
                      const int *skip, hipStream_t s) {
    // n = number of rows available (grid size); the kernels read k from st when order != null
    const int nb = (int)std::max<int64_t>(1, (n + FTILE - 1) / FTILE);
    char *p = (char *)tmp;
    double *part1 = (double *)p;
    p += align_up((int64_t)nb * 4 * 8, 256);
    double *part2 = (double *)p;
    FitIn a{order, sx, sy, idx, tx, ty, n, px, py, st};
    hipLaunchKernelGGL(k_fit_pass1, dim3(nb), dim3(FB), 0, s, a, part1, skip);
    hipLaunchKernelGGL(k_fit_pass2, dim3(nb), dim3(FB), 0, s, a, part1, nb, part2, skip);
    hipLaunchKernelGGL(k_fit_final, dim3(1), dim3(256), 0, s, a, part1, part2, nb,
                       allow_reflection, st, skip);
    return hipGetLastError();
}

hipError_t launch_sum_sq_diff(const double *sx, const double *sy, const double *sz,
                              const double *cx, const double *cy, const double *cz, int64_t k,
                              int md, void *tmp, double *out, hipStream_t s) {
    const int nb = (int)std::max<int64_t>(1, (k + FTILE - 1) / FTILE);
    double *part = (double *)tmp;
    hipLaunchKernelGGL(k_ssd_partial, dim3(nb), dim3(256), 0, s, sx, sy, sz, cx, cy, cz, k, md,
                       part);
    hipLaunchKernelGGL(k_ssd_final, dim3(1), dim3(256), 0, s, part, nb, out);
    return hipGetLastError();
}

hipError_t launch_gather_xy(const int32_t *idx, const double *tx, const double *ty, int64_t n,
                            double *ox, double *oy, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_xy, dim3(nblk(n)), dim3(256), 0, s, idx, tx, ty, n, ox, oy);
    return hipGetLastError();
}

}  // namespace ficp
