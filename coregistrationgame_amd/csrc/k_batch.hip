// k_batch.hip -- many plots per launch (BASELINE config C4: 1024 plots x 10k trees vs 10k
// CHM stems).  Every plot runs the reference's two-stage _iterate (ficp.py:122-154); the
// plots advance together, one batch iteration = {fit of looping plots -> NN with the fit
// applied -> segmented sort -> per-plot FRMSD scan -> per-plot state machine}, and a plot
// leaves the batch when its own convergence test fires (per-plot masks, no host work).
//
//  * k_batch_bbox / k_fill_plot_ids / k_batch_grid_count: per-plot CHM grids in one set of
//    arrays (cell ids offset by each plot's cell_base).
//  * k_batch_fraction: one workgroup per plot scans r in the plot's (distance, index)
//    order -> first-minimum FRMSD argmin (same formula and tie rule as k_frac_eval).
//  * k_batch_fit: one workgroup per looping plot streams the plot's trees, selects
//    (key, index) <= (key_t, t), reduces the 8 pivot-shifted sums and solves the 2x2
//    Kabsch problem in closed form (same as k_fit_final).
//  * k_batch_update: one thread per plot advances HEAD -> LOOP -> (stage 2) -> DONE.
#include "ficp_internal.h"

#include <math.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int BB = 256;  // threads per per-plot workgroup
constexpr int BI = 4;    // items per thread per chunk

__device__ __forceinline__ double bsum(double v, double *s) {
    s[threadIdx.x] = v;
    __syncthreads();
    for (int w = BB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
        __syncthreads();
    }
    const double r = s[0];
    __syncthreads();
    return r;
}

// exclusive scan over the workgroup + total (Hillis-Steele, deterministic)
__device__ __forceinline__ double bscan(double v, double *s /*[2*BB]*/, double &total) {
    double *a = s, *b = s + BB;
    a[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < BB; o <<= 1) {
        const double x =
            ((int)threadIdx.x >= o) ? a[threadIdx.x - o] + a[threadIdx.x] : a[threadIdx.x];
        b[threadIdx.x] = x;
        __syncthreads();
        double *t = a;
        a = b;
        b = t;
    }
    const double ex = threadIdx.x ? a[threadIdx.x - 1] : 0.0;
    total = a[BB - 1];
    __syncthreads();
    return ex;
}

__device__ __forceinline__ bool better(double f, long long k, double bf, long long bk) {
    return f < bf || (f == bf && k < bk);
}

__global__ __launch_bounds__(BB) void k_batch_bbox(const double *tx, const double *ty,
                                                   const int64_t *to, double *bb) {
    __shared__ double s[4][BB];
    const int p = blockIdx.x;
    double a0 = INFINITY, a1 = -INFINITY, b0 = INFINITY, b1 = -INFINITY;
    for (int64_t j = to[p] + threadIdx.x; j < to[p + 1]; j += BB) {
        a0 = fmin(a0, tx[j]);
        a1 = fmax(a1, tx[j]);
        b0 = fmin(b0, ty[j]);
        b1 = fmax(b1, ty[j]);
    }
    s[0][threadIdx.x] = a0;
    s[1][threadIdx.x] = a1;
    s[2][threadIdx.x] = b0;
    s[3][threadIdx.x] = b1;
    __syncthreads();
    for (int w = BB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + w]);
            s[1][threadIdx.x] = fmax(s[1][threadIdx.x], s[1][threadIdx.x + w]);
            s[2][threadIdx.x] = fmin(s[2][threadIdx.x], s[2][threadIdx.x + w]);
            s[3][threadIdx.x] = fmax(s[3][threadIdx.x], s[3][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) bb[4 * p + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(BB) void k_fill_plot_ids(const int64_t *off, int32_t *plot_of) {
    const int p = blockIdx.x;
    for (int64_t j = off[p] + threadIdx.x; j < off[p + 1]; j += BB) plot_of[j] = p;
}

__device__ __forceinline__ int cell_coord_b(double v, double v0, double inv_h, int g) {
    double f = (v - v0) * inv_h;
    if (!(f >= 0.0)) return 0;
    if (f >= (double)(g - 1)) return g - 1;
    return (int)f;
}

__global__ __launch_bounds__(256) void k_batch_grid_count(const double *tx, const double *ty,
                                                          int64_t m, const int32_t *tplot,
                                                          const PlotGrid *grids,
                                                          int32_t *cell_of, int32_t *counts) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const PlotGrid g = grids[tplot[j]];
    const int cx = cell_coord_b(tx[j], g.x0, g.inv_h, g.gx);
    const int cy = cell_coord_b(ty[j], g.y0, g.inv_h, g.gy);
    const int c = (int)g.cell_base + cy * g.gx + cx;
    cell_of[j] = c;
    atomicAdd(&counts[c], 1);
}

__global__ void k_batch_init(const int64_t *so, const int64_t *to, int nplots, int nstages,
                             PlotState *st) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nplots) return;
    PlotState z{};
    for (int e = 0; e < 9; ++e) {
        z.T[e] = (e % 4 == 0) ? 1.0 : 0.0;
        z.Ttot[e] = z.T[e];
    }
    z.cur = INFINITY;
    z.frmsd = INFINITY;
    // empty layers: find_correspondences returns nothing, k = 0, nothing moves
    // (ficp.py:66-68, 75-77, 125-126)
    const bool empty = (so[p + 1] == so[p]) || (to[p + 1] == to[p]);
    z.phase = (empty || nstages <= 0) ? PH_DONE : PH_HEAD;
    st[p] = z;
}

// one workgroup per plot: FRMSD argmin over the plot's r in (distance, index) order
__global__ __launch_bounds__(BB) void k_batch_fraction(const double *rs, const int64_t *so,
                                                       const double *lams, PlotState *st) {
    __shared__ double s[2 * BB];
    __shared__ double s_f[BB];
    __shared__ long long s_k[BB];
    const int p = blockIdx.x;
    if (st[p].phase == PH_DONE) return;  // uniform per workgroup
    const double lam = lams[st[p].stage];
    const int64_t b = so[p], e = so[p + 1];
    const long long N = e - b;
    double run = 0.0, bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    for (int64_t c = b; c < e; c += BB * BI) {
        const int64_t j0 = c + (int64_t)threadIdx.x * BI;
        double v[BI];
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < BI; ++q) {
            v[q] = (j0 + q < e) ? rs[j0 + q] : 0.0;
            acc = acc + v[q];
        }
        double tot;
        double S = run + bscan(acc, s, tot);
#pragma unroll
        for (int q = 0; q < BI; ++q) {
            if (j0 + q < e) {
                S = S + v[q];
                const long long k = j0 + q - b + 1;
                const double frac = (double)k / (double)N;
                const double f = (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
                if (f < bf) {  // ascending k: strict < keeps the first minimum (ficp.py:84)
                    bf = f;
                    bk = k;
                }
            }
        }
        run = run + tot;
    }
    s_f[threadIdx.x] = bf;
    s_k[threadIdx.x] = bk;
    __syncthreads();
    for (int w = BB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w &&
            better(s_f[threadIdx.x + w], s_k[threadIdx.x + w], s_f[threadIdx.x], s_k[threadIdx.x])) {
            s_f[threadIdx.x] = s_f[threadIdx.x + w];
            s_k[threadIdx.x] = s_k[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (s_k[0] == 0x7fffffffffffffffLL) {  // every FRMSD NaN: the reference keeps (0.0, 0)
            st[p].k = 0;
            st[p].frac = 0.0;
            st[p].frmsd = INFINITY;
        } else {
            st[p].k = s_k[0];
            st[p].frac = (double)s_k[0] / (double)N;
            st[p].frmsd = s_f[0];
        }
    }
}

// one workgroup per looping plot: rigid fit on the plot's first k trees of the order
__global__ __launch_bounds__(BB) void k_batch_fit(const double *sx, const double *sy,
                                                  const double *cx, const double *cy,
                                                  const unsigned long long *key,
                                                  const uint32_t *order, const int64_t *so,
                                                  const PlotGrid *grids, int allow_refl,
                                                  PlotState *st) {
    __shared__ double s[BB];
    const int p = blockIdx.x;
    if (st[p].phase != PH_LOOP) {
        if (threadIdx.x == 0) st[p].apply = 0;
        return;
    }
    const int64_t b = so[p], e = so[p + 1];
    const long long k = st[p].k;
    const int64_t t = (int64_t)order[b + k - 1];  // k >= 1 in the loop phase
    const unsigned long long tk = key[t];
    const double px = grids[p].px, py = grids[p].py;
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = b + threadIdx.x; i < e; i += BB) {
        const unsigned long long ki = key[i];
        if (ki < tk || (ki == tk && i <= t)) {
            const double xs = sx[i] - px, ys = sy[i] - py;
            const double xt = cx[i] - px, yt = cy[i] - py;
            c[0] = c[0] + xs;
            c[1] = c[1] + ys;
            c[2] = c[2] + xt;
            c[3] = c[3] + yt;
            c[4] = c[4] + xs * xt;
            c[5] = c[5] + xs * yt;
            c[6] = c[6] + ys * xt;
            c[7] = c[7] + ys * yt;
        }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = bsum(c[q], s);
    if (threadIdx.x != 0) return;
    const double kk = (double)k;
    const double csx = c[0] / kk, csy = c[1] / kk, ctx = c[2] / kk, cty = c[3] / kk;
    const double H0 = c[4] - c[0] * ctx, H1 = c[5] - c[0] * cty;
    const double H2 = c[6] - c[1] * ctx, H3 = c[7] - c[1] * cty;
    double R00, R01, R10, R11;
    if (allow_refl && H0 * H3 - H1 * H2 < 0.0) {
        const double F = H0 - H3, G = H2 + H1, nrm = hypot(F, G);
        R00 = F / nrm;
        R01 = G / nrm;
        R10 = G / nrm;
        R11 = -F / nrm;
    } else {
        const double A = H0 + H3, B = H1 - H2, nrm = hypot(A, B);
        double cc = 1.0, ss = 0.0;
        if (nrm > 0.0) {
            cc = A / nrm;
            ss = B / nrm;
        }
        R00 = cc;
        R01 = -ss;
        R10 = ss;
        R11 = cc;
    }
    const double wsx = csx + px, wsy = csy + py, wtx = ctx + px, wty = cty + py;
    double *T = st[p].T;
    T[0] = R00;
    T[1] = R01;
    T[2] = wtx - (wsx * R00 + wsy * R01);
    T[3] = R10;
    T[4] = R11;
    T[5] = wty - (wsx * R10 + wsy * R11);
    T[6] = 0.0;
    T[7] = 0.0;
    T[8] = 1.0;
    st[p].apply = 1;
}

__device__ __forceinline__ void end_stage(PlotState &s, int nstages) {
    if (s.stage == 0) s.iters0 = s.it;
    else if (s.stage == 1) s.iters1 = s.it;
    if (s.stage + 1 < nstages) {
        s.stage += 1;  // ficp.py:152: lambda switches, stage 2 starts with a head NN call
        s.phase = PH_HEAD;
        s.it = 0;
    } else {
        s.phase = PH_DONE;
    }
}

// one thread per plot: the convergence logic of ficp.py:125-145 per plot
__global__ void k_batch_update(int nplots, int nstages, double threshold, int max_iter,
                               PlotState *st, unsigned int *active) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nplots) return;
    PlotState s = st[p];
    if (s.phase != PH_DONE) {
        s.n_nn += 1;
        if (s.phase == PH_HEAD) {
            if (s.k == 0) {
                end_stage(s, nstages);
            } else {
                s.cur = s.frmsd;
                s.phase = PH_LOOP;
                s.it = 0;
                if (max_iter <= 0) end_stage(s, nstages);
            }
        } else {  // a loop body just ran: fit -> apply -> NN -> fraction
            s.n_fit += 1;
            double R[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    R[3 * i + j] = s.T[3 * i] * s.Ttot[j] + s.T[3 * i + 1] * s.Ttot[3 + j] +
                                   s.T[3 * i + 2] * s.Ttot[6 + j];
            for (int e = 0; e < 9; ++e) s.Ttot[e] = R[e];
            const double nw = s.frmsd;
            if (s.cur - nw <= threshold) {  // ficp.py:142
                end_stage(s, nstages);
            } else {
                s.cur = nw;
                s.it += 1;
                if (s.it >= max_iter) end_stage(s, nstages);
            }
        }
        s.apply = 0;
        st[p] = s;
    }
    if (s.phase != PH_DONE) atomicAdd(active, 1u);
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t launch_batch_bbox(const double *tx, const double *ty, const int64_t *to, int nplots,
                             double *bb, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_bbox, dim3(nplots), dim3(BB), 0, s, tx, ty, to, bb);
    return hipGetLastError();
}

hipError_t launch_fill_plot_ids(const int64_t *off, int nplots, int32_t *plot_of, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_plot_ids, dim3(nplots), dim3(BB), 0, s, off, plot_of);
    return hipGetLastError();
}

hipError_t launch_batch_grid_count(const double *tx, const double *ty, int64_t m,
                                   const int32_t *tplot, const PlotGrid *grids, int32_t *cell_of,
                                   int32_t *counts, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_grid_count, dim3(nblk(m)), dim3(256), 0, s, tx, ty, m, tplot,
                       grids, cell_of, counts);
    return hipGetLastError();
}

hipError_t launch_batch_init(const int64_t *so, const int64_t *to, int nplots, int nstages,
                             PlotState *st, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_init, dim3(nblk(nplots)), dim3(256), 0, s, so, to, nplots, nstages,
                       st);
    return hipGetLastError();
}

hipError_t launch_batch_fit(const double *sx, const double *sy, const double *cx,
                            const double *cy, const unsigned long long *key,
                            const uint32_t *order, const int64_t *so, const PlotGrid *grids,
                            int nplots, int allow_refl, PlotState *st, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_fit, dim3(nplots), dim3(BB), 0, s, sx, sy, cx, cy, key, order, so,
                       grids, allow_refl, st);
    return hipGetLastError();
}

hipError_t launch_batch_fraction(const double *rs, const int64_t *so, int nplots,
                                 const double *lambdas, PlotState *st, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_fraction, dim3(nplots), dim3(BB), 0, s, rs, so, lambdas, st);
    return hipGetLastError();
}

hipError_t launch_batch_update(int nplots, int nstages, double threshold, int max_iter,
                               PlotState *st, unsigned int *active, hipStream_t s) {
    hipError_t e = launch_atomic_zero32(active, 1, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_batch_update, dim3(nblk(std::max(nplots, 1))), dim3(256), 0, s, nplots,
                       nstages, threshold, max_iter, st, active);
    return hipGetLastError();
}

}  // namespace ficp
