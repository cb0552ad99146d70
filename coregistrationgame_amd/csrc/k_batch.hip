// k_batch.hip -- many plots per launch (BASELINE config C4: 1024 plots x 10k trees vs 10k
// CHM stems).  Every plot runs the reference's two-stage _iterate (ficp.py:122-154); the
// plots advance together, one batch iteration = {fit of looping plots -> NN with the fit
// applied -> per-plot FRMSD selection -> per-plot state machine}, and a plot leaves the
// batch when its own convergence test fires (per-plot masks, no host work).
//
//  * k_batch_bbox / k_fill_plot_ids / k_batch_grid_count: per-plot CHM grids in one set of
//    arrays (cell ids offset by each plot's cell_base).
//  * k_batch_select: one workgroup per live plot: bucketed FRMSD bounds, exact order of
//    the candidate window only -> first-minimum FRMSD argmin and the selection threshold.
//  * k_batch_fit: one workgroup per looping plot streams the plot's trees, selects
//    (key, index) <= (key_t, t), reduces the 8 pivot-shifted sums and solves the 2x2
//    Kabsch problem in closed form (same as k_fit_final).
//  * k_batch_update: one thread per plot advances HEAD -> LOOP -> (stage 2) -> DONE.
#include "ficp_internal.h"
#include "frmsd_bounds.h"

#include <math.h>
#include <stdlib.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int BB = 256;  // threads per per-plot workgroup (bbox, fit)

__device__ __forceinline__ bool better(double f, long long k, double bf, long long bk) {
    return f < bf || (f == bf && k < bk);
}

__global__ __launch_bounds__(BB) void k_batch_bbox(const double *tx, const double *ty,
                                                   const int64_t *to, double *bb) {
    __shared__ double s[4][BB];
    const int p = blockIdx.x;
    double a0 = INFINITY, a1 = -INFINITY, b0 = INFINITY, b1 = -INFINITY;
    // 8 rows per thread in flight (one row per trip was one load latency per row)
    const int64_t je = to[p + 1];
    for (int64_t j0 = to[p] + threadIdx.x; j0 < je; j0 += 8 * BB) {
        double vx[8], vy[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t j = j0 + (int64_t)u * BB;
            vx[u] = j < je ? tx[j] : NAN;  // fmin / fmax ignore NaN
            vy[u] = j < je ? ty[j] : NAN;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = fmin(a0, vx[u]);
            a1 = fmax(a1, vx[u]);
            b0 = fmin(b0, vy[u]);
            b1 = fmax(b1, vy[u]);
        }
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

// The run's offsets and lambdas come straight from the host's coherent pinned staging
// (so_h, to_h, lam_h): this kernel stores the device copies the later kernels read, zeroes
// the fused step's arrival counters and initialises every plot's state.  Three staged
// copies and a memset were four runtime blit launches (~20 us at the head of a run).
__global__ void k_batch_init(BatchInitArgs a) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p <= a.nplots) {
        a.so[p] = a.so_h[p];
        a.to[p] = a.to_h[p];
    }
    if (p < a.nl) a.lams[p] = a.lam_h[p];
    if (p < a.narrive) a.arrive[p] = 0ULL;
    if (p >= a.nplots) return;
    PlotState z{};
    for (int e = 0; e < 9; ++e) {
        z.T[e] = (e % 4 == 0) ? 1.0 : 0.0;
        z.Ttot[e] = z.T[e];
    }
    z.cur = INFINITY;
    z.frmsd = INFINITY;
    z.wfloor = 0;  // (win_start_log of the plot's rows)
    // empty layers: find_correspondences returns nothing, k = 0, nothing moves
    // (ficp.py:66-68, 75-77, 125-126)
    const bool empty = (a.so_h[p + 1] == a.so_h[p]) || (a.to_h[p + 1] == a.to_h[p]);
    z.phase = (empty || a.nstages <= 0) ? PH_DONE : PH_HEAD;
    a.st[p] = z;
}

// ---------------------------------------------------------------- per-plot selection
// ficp.py:73-86 for one plot per workgroup, without sorting the plot: the FRMSD-optimal
// k needs the exact order only where the FRMSD curve can hold its minimum.
//  1. key range of the plot's finite rows (r = inf / NaN rows sort last and never win:
//     every FRMSD from them on is inf or NaN, never < the running minimum);
//  2. LDS histogram of the keys into SB buckets (count + fp64 sum of r);
//  3. prefix counts/sums over the buckets; U = the smallest upper bound of h (the log2
//     form of FRMSD, frmsd_bounds.h) at a bucket end; the candidate window = the buckets
//     from the first to the last whose lower bound is <= U (the minimum lies inside);
//  4. S_base = the sum of r below the window (each thread's rows in a fixed order, then a
//     fixed reduction tree: deterministic), window rows appended to a scratch region;
//  5. exact (key, row) order of the window: rank of each row inside its bucket;
//  6. prefix sums over the window in that order, FRMSD of every window position, first
//     minimum (strict <, ascending k).
// The bucket sums only feed the bounds (kMarg covers their rounding); every FRMSD value
// compared comes from the deterministic S_base + window prefix sums.
#ifndef FICP_BSEL_ST
#define FICP_BSEL_ST 512
#endif
#ifndef FICP_BSEL_RCACHE
#define FICP_BSEL_RCACHE 1  // r kept in registers too (0: re-read from L2 in its two passes)
#endif
#ifndef FICP_BSEL_RPT
#define FICP_BSEL_RPT 32
#endif
constexpr int ST = FICP_BSEL_ST; // threads
constexpr int SB = 2048;         // buckets
constexpr int SB_LOG = 11;
constexpr int RPT = FICP_BSEL_RPT;  // rows per thread kept in registers (plots <= ST * RPT rows)
constexpr int SRP = 4;           // window rows per thread per scan chunk
constexpr int WCAP = 1024;          // candidate windows up to this many rows stay in LDS

typedef unsigned long long u64;

template <int NW>
struct SelRed {
    double d[NW];
    u64 a[NW], b[NW];
    unsigned c[NW];
    long long l[NW];
};

// block sum of a double in a fixed order (deterministic, same value on every thread)
template <int NW>
__device__ __forceinline__ double blk_sum_d(double x, SelRed<NW> &r) {
    x = wave_sum63(x);  // DPP (ficp_internal.h), lane 63
    if ((threadIdx.x & 63) == 63) r.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = r.d[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) t = t + r.d[w];
    __syncthreads();
    return t;
}

template <int NW>
__device__ __forceinline__ double blk_min_d(double x, SelRed<NW> &r) {
    x = wave_min63(x);
    if ((threadIdx.x & 63) == 63) r.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = r.d[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) t = fmin(t, r.d[w]);
    __syncthreads();
    return t;
}

// {max a, max b, sum c} over the block
template <int NW>
__device__ __forceinline__ void blk_max2_sum(u64 &a, u64 &b, unsigned &c, SelRed<NW> &r) {
    // DPP steps; a lane a step does not write reads 0 (neutral for max of u64 and for +)
#define MAX2SUM_STEP(CTRL, ROWM)                                                      \
    {                                                                                 \
        const u64 xa = (u64)dpp::mov_ll<CTRL, ROWM>(0, (long long)a);                 \
        const u64 xb = (u64)dpp::mov_ll<CTRL, ROWM>(0, (long long)b);                 \
        const unsigned xc = (unsigned)__builtin_amdgcn_update_dpp(0, (int)c, CTRL, ROWM, 0xf, false); \
        a = xa > a ? xa : a;                                                          \
        b = xb > b ? xb : b;                                                          \
        c += xc;                                                                      \
    }
    MAX2SUM_STEP(dpp::QP_XOR1, 0xf)
    MAX2SUM_STEP(dpp::QP_XOR2, 0xf)
    MAX2SUM_STEP(dpp::ROW_HALF_MIRROR, 0xf)
    MAX2SUM_STEP(dpp::ROW_MIRROR, 0xf)
    MAX2SUM_STEP(dpp::ROW_BCAST15, 0xA)
    MAX2SUM_STEP(dpp::ROW_BCAST31, 0xC)
#undef MAX2SUM_STEP
    if ((threadIdx.x & 63) == 63) {
        r.a[threadIdx.x >> 6] = a;
        r.b[threadIdx.x >> 6] = b;
        r.c[threadIdx.x >> 6] = c;
    }
    __syncthreads();
    a = r.a[0];
    b = r.b[0];
    c = r.c[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        a = r.a[w] > a ? r.a[w] : a;
        b = r.b[w] > b ? r.b[w] : b;
        c += r.c[w];
    }
    __syncthreads();
}

// exclusive scan over the block (thread order) of a count and a sum; fixed schedule
template <int NW>
__device__ __forceinline__ void blk_excl_scan2(unsigned &c, double &x, SelRed<NW> &r) {
    // DPP wave scans (ficp_internal.h)
    const unsigned ci = (unsigned)wave_incl_scan_ll((long long)c);
    const double xi = wave_incl_scan_d(x);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned ce = (unsigned)wave_shr1_ll((long long)ci);
    const double xe = wave_shr1_d(xi);
    if (lane == 63) {
        r.c[w] = ci;
        r.d[w] = xi;
    }
    __syncthreads();
    unsigned cp = 0;
    double xp = 0.0;
    for (int v = 0; v < w; ++v) {
        cp += r.c[v];
        xp = xp + r.d[v];
    }
    __syncthreads();
    c = cp + ce;
    x = xp + xe;
}

// exclusive scan of a double over the block + the block total; fixed schedule
template <int NW>
__device__ __forceinline__ double blk_excl_scan_d(double x, double &total, SelRed<NW> &r) {
    const double xi = wave_incl_scan_d(x);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double xe = wave_shr1_d(xi);
    if (lane == 63) r.d[w] = xi;
    __syncthreads();
    double xp = 0.0, tot = 0.0;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
        if (v < w) xp = xp + r.d[v];
        tot = tot + r.d[v];
    }
    __syncthreads();
    total = tot;
    return xp + xe;
}

template <int NW>
__device__ __forceinline__ void blk_argmin(double &f, long long &k, SelRed<NW> &r) {
#define ARGMIN_STEP(CTRL, ROWM)                                                      \
    {                                                                                \
        const double of = dpp::mov_d<CTRL, ROWM>(INFINITY, f);                       \
        const long long ok = dpp::mov_ll<CTRL, ROWM>(0x7fffffffffffffffLL, k);       \
        if (better(of, ok, f, k)) {                                                  \
            f = of;                                                                  \
            k = ok;                                                                  \
        }                                                                            \
    }
    ARGMIN_STEP(dpp::QP_XOR1, 0xf)
    ARGMIN_STEP(dpp::QP_XOR2, 0xf)
    ARGMIN_STEP(dpp::ROW_HALF_MIRROR, 0xf)
    ARGMIN_STEP(dpp::ROW_MIRROR, 0xf)
    ARGMIN_STEP(dpp::ROW_BCAST15, 0xA)
    ARGMIN_STEP(dpp::ROW_BCAST31, 0xC)
#undef ARGMIN_STEP
    if ((threadIdx.x & 63) == 63) {
        r.d[threadIdx.x >> 6] = f;
        r.l[threadIdx.x >> 6] = k;
    }
    __syncthreads();
    f = r.d[0];
    k = r.l[0];
#pragma unroll
    for (int w = 1; w < NW; ++w)
        if (better(r.d[w], r.l[w], f, k)) {
            f = r.d[w];
            k = r.l[w];
        }
    __syncthreads();
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

// one workgroup, one thread per plot (strided): the convergence logic of ficp.py:125-145
// per plot; the number of plots still running is stored (system scope, release) into
// *flag in coherent pinned host memory, which the host polls while the next batch
// iteration already runs
constexpr int UT = 1024;
// trace (nullable): this plot's row of the per-call k trace (ficp_set_batch_trace)
__device__ __forceinline__ void step_plot(PlotState &s, int nstages, double threshold,
                                          int max_iter, long long *trace = nullptr,
                                          int max_trace = 0) {
    if (s.phase != PH_DONE) {
        if (trace && s.n_nn < max_trace) trace[s.n_nn] = s.k;
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
    }
}

__device__ __forceinline__ bool update_plot(PlotState *st, int p, int nstages, double threshold,
                                            int max_iter, long long *trace, int max_trace) {
    PlotState s = st[p];
    if (s.phase != PH_DONE) {
        step_plot(s, nstages, threshold, max_iter, trace ? trace + (int64_t)p * max_trace : nullptr,
                  max_trace);
        st[p] = s;
    }
    return s.phase != PH_DONE;
}


// The batch iteration's tail in the plot's selection workgroup (BatchStep::fuse): thread
// 0 takes the loop step of ficp.py:125-145 (k_batch_update's update_plot) with this call's
// k and FRMSD, and when a loop body follows, the workgroup fits it on this call's selection
// (ficp.py:133-134: k_batch_fit's 8 pivot-shifted sums of the rows (key, row) <= (tkey,
// trow), here per thread in row order, then a wave butterfly and the waves in order), so
// the next NN call applies T with no fit launch in between.
struct BatchStep {
    const double *sx, *sy, *cx, *cy;
    const PlotGrid *grids;
    int fuse, allow_refl, nstages, max_iter;
    double threshold;
    unsigned long long *arrive;  // (arrivals << 32) + live plots of this launch (nullable)
    int *flag;                   // the last arrival stores the live count (pinned host word)
    int nplots;
    long long *trace;            // per-call k trace, max_trace per plot of this launch (nullable)
    int max_trace;
    const uint32_t *worig;       // caller row of each work row (nullable: caller order)
    const double *r;             // the NN call's r (the keys are derived from it when the
                                 // NN stored none: key == nullptr)
};

// thread 0 of plot p's workgroup, its state final for this call: one agent-scope atomic
// adds (1 << 32) + live; the workgroup that completes the count stores the number of live
// plots into the host's flag and resets the counter for the next launch (stream-ordered)
// (in two halves: the fused step issues the add before its fit and tests the returned
// count after it, so the atomic's round trip is off the workgroup's chain)
__device__ __forceinline__ u64 batch_arrive_add(const BatchStep &bs, int live) {
    if (!bs.arrive) return 0ULL;
    const u64 add = (1ULL << 32) | (u64)(unsigned)live;
    return __hip_atomic_fetch_add(bs.arrive, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void batch_arrive_last(const BatchStep &bs, u64 old, int live) {
    if (!bs.arrive) return;
    if ((int)(old >> 32) + 1 == bs.nplots) {
        const int tot = (int)(old & 0xffffffffULL) + live;
        __hip_atomic_exchange(bs.arrive, 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(bs.flag, tot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__device__ __forceinline__ void batch_arrive(const BatchStep &bs, int live) {
    batch_arrive_last(bs, batch_arrive_add(bs, live), live);
}

// KR > 1: the caller's registers hold the keys of rows b + t + q NT (q < KR; ~0 past the
// plot), so the fit loads only the pairs, FU rows at a time
template <int NW, int KR>
__device__ __forceinline__ void plot_step_fit(PlotState *st, const PlotState *ps, int p, long long k,
                                              double frac, double frmsd, u64 tkey, long long trow,
                                              int64_t b, int64_t e, const u64 *key, const u64 (&kc)[KR],
                                              const BatchStep &bs, double *s8, int *s_flag,
                                              int wrows = -1, long long *pt = nullptr) {
    const int t = threadIdx.x;
    constexpr int NT = NW * 64;
    u64 arr = 0ULL;  // (thread 0) the arrival add's returned word
    int live = 0;
    if (t == 0) {
        PlotState s = *ps;  // (the workgroup's LDS copy, loaded with its rows)
        // the threshold's move since the previous loop-body call (the window's half-width)
        const bool prev = s.phase == PH_LOOP && s.k > 0 && k > 0;
        const u64 mv = prev ? (tkey > s.tkey ? tkey - s.tkey : s.tkey - tkey) : 0ULL;
        s.k = k;
        s.frac = frac;
        s.frmsd = frmsd;
        if (k > 0) {
            s.tkey = tkey;
            s.trow = trow;
        }
        s.tmove = mv;
        // the window path's floor from its row count (wrows >= 0: this call took it)
        const long long nrow = e - b;
        const int f = win_floor(s.wfloor, nrow);
        if (wrows > 256) s.wfloor = max(kWinHMinLog, f - 1);
        else if (wrows >= 0 && wrows < 16) s.wfloor = min(win_hmax_log(nrow) - 1, f + 1);
        step_plot(s, bs.nstages, bs.threshold, bs.max_iter,
                  bs.trace ? bs.trace + (int64_t)p * bs.max_trace : nullptr, bs.max_trace);
        s_flag[0] = s.phase == PH_LOOP && s.k > 0;  // a loop body (fit -> apply -> NN) follows
        st[p] = s;
        live = s.phase != PH_DONE ? 1 : 0;
        arr = batch_arrive_add(bs, live);
    }
    __syncthreads();
    if (pt && t == 0) pt[13] = wall_clock64();  // (FICP_BSEL_PROF)
    if (!s_flag[0]) {
        if (t == 0) batch_arrive_last(bs, arr, live);
        return;
    }
    const PlotGrid g = bs.grids[p];
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifndef FICP_BFIT_FU
#define FICP_BFIT_FU 8
#endif
    // (the tie at the threshold key: the caller's row, loaded only then)
    auto sel = [&](u64 kk, int64_t i) {
        return kk < tkey || (kk == tkey && (bs.worig ? (long long)bs.worig[i] : i) <= trow);
    };
    if constexpr (KR > 1) {
        // cached keys: 10 rows' pairs in flight per thread (C4's 10k-row plots: two round
        // trips, the key-loading loop below took three), the rows in the same order
        constexpr int FK = 10;
#pragma unroll
        for (int q0 = 0; q0 < KR; q0 += FK) {
            if (b + t + (int64_t)q0 * NT >= e) break;
            double xs[FK], ys[FK], xt[FK], yt[FK];
#pragma unroll
            for (int u = 0; u < FK; ++u) {
                const int64_t i = b + t + (int64_t)(q0 + u) * NT;
                const bool in = q0 + u < KR && i < e;
                xs[u] = in ? bs.sx[i] : 0.0;
                ys[u] = in ? bs.sy[i] : 0.0;
                xt[u] = in ? bs.cx[i] : 0.0;
                yt[u] = in ? bs.cy[i] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < FK; ++u) {
                const int64_t i = b + t + (int64_t)(q0 + u) * NT;
                if (q0 + u < KR && i < e && sel(kc[q0 + u < KR ? q0 + u : 0], i))
                    fit_add(c, xs[u], ys[u], xt[u], yt[u], g.px, g.py);
            }
        }
    } else {
    constexpr int FU = FICP_BFIT_FU;  // rows in flight per thread (every load before its predicate)
    for (int64_t i0 = b + t; i0 < e; i0 += (int64_t)FU * NT) {
        u64 kv[FU];
        double xs[FU], ys[FU], xt[FU], yt[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int64_t i = i0 + (int64_t)u * NT;
            const bool in = i < e;
            kv[u] = in ? (key ? key[i] : key_of_r(bs.r[i])) : ~0ULL;
            xs[u] = in ? bs.sx[i] : 0.0;
            ys[u] = in ? bs.sy[i] : 0.0;
            xt[u] = in ? bs.cx[i] : 0.0;
            yt[u] = in ? bs.cy[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int64_t i = i0 + (int64_t)u * NT;
            if (i < e && sel(kv[u], i)) fit_add(c, xs[u], ys[u], xt[u], yt[u], g.px, g.py);
        }
    }
    }
    if (pt && t == 0) pt[14] = wall_clock64();
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = wave_sum63(c[q]);
    if ((t & 63) == 63)
#pragma unroll
        for (int q = 0; q < 8; ++q) s8[8 * (t >> 6) + q] = c[q];
    __syncthreads();
    if (t != 0) return;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        double v = s8[q];
        for (int w = 1; w < NW; ++w) v = v + s8[8 * w + q];
        c[q] = v;
    }
    fit_solve_T(c, (double)k, g.px, g.py, bs.allow_refl, st[p].T);
    st[p].apply = 1;
    batch_arrive_last(bs, arr, live);
    if (pt) {
        pt[15] = wall_clock64();
        printf("BSELF p=%d pre %lld sel %lld step %lld fit %lld solve %lld (10 ns)\n", p, pt[0] - pt[12],
               pt[7] - pt[0], pt[13] - pt[7], pt[14] - pt[13], pt[15] - pt[14]);
    }
}

// every row of the plot with its key and r: CACHED keeps them in registers (RPT per
// thread, rows past the plot hold r = inf), otherwise they are re-read per pass
#define SEL_ROWS(BODY)                                                              \
    if (CACHED) {                                                                   \
        _Pragma("unroll") for (int q = 0; q < RPT; ++q) {                           \
            const int64_t i = b + t + (int64_t)q * ST;                              \
            const u64 kk = kc[q];                                                   \
            const double rv = BSEL_RCACHE ? rc[q] : (i < e ? r[i] : INFINITY);       \
            (void)i;                                                                \
            BODY                                                                    \
        }                                                                           \
    } else {                                                                        \
        for (int64_t i = b + t; i < e; i += ST) {                                   \
            const double rv = r[i];                                                 \
            const u64 kk = key ? key[i] : key_of_r(rv);                             \
            constexpr int q = 0;                                                    \
            (void)i;                                                                \
            (void)q;                                                                \
            BODY                                                                    \
        }                                                                           \
    }

#ifdef FICP_BSEL_PROF
#define BSEL_T(i) bt_[i] = wall_clock64()
#else
#define BSEL_T(i)
#endif
#if defined(FICP_BSEL_WPE) && FICP_BSEL_WPE > 0
#define BSEL_WPE __attribute__((amdgpu_waves_per_eu(FICP_BSEL_WPE, FICP_BSEL_WPE)))
#else
#define BSEL_WPE
#endif
// KST threads (512; 1024 when the plots are fewer than the CUs: half the rows per thread
// on the same per-plot latency chain), KRPT rows per thread kept in registers
template <bool CACHED, int KST, int KRPT, bool KRC = (bool)FICP_BSEL_RCACHE>
__global__ __launch_bounds__(KST) BSEL_WPE void k_batch_select(const u64 *__restrict__ key,
                                                     const double *__restrict__ r,
                                                     const int64_t *__restrict__ so,
                                                     const double *__restrict__ lams,
                                                     PlotState *__restrict__ st,
                                                     BatchSelScratch ws, BatchStep bs) {
    constexpr int ST = KST;                // (these hide the namespace-scope defaults)
    constexpr int RPT = KRPT;
    constexpr bool BSEL_RCACHE = KRC;
    constexpr int SPER = SB / ST;          // buckets per thread in the scans
    constexpr int BMAXACT = ST / SPER;     // active bound chunks evaluated one bucket per lane
    __shared__ unsigned s_cnt[SB];  // exclusive bucket starts
    __shared__ double s_sum[SB];    // (count, sum) words, then per-bucket fill counters (as unsigned)
    __shared__ SelRed<ST / 64> red;
    __shared__ double s_fit8[8 * (ST / 64)];
    __shared__ int s_fitflag[1];
    __shared__ long long s_k[2];
    __shared__ u64 l_wk[WCAP], l_sk[WCAP];       // a small window's rows (phases 4-6)
    __shared__ double l_wr[WCAP], l_sr[WCAP];
    __shared__ uint32_t l_wrow[WCAP], l_srow[WCAP];
    __shared__ int s_act[BMAXACT];               // active chunks (thread ids)
    __shared__ int s_nact;
    __shared__ long long s_eC[BMAXACT * SPER];   // rows before each of their buckets
    __shared__ double s_eP[BMAXACT * SPER];      // sum of r before it
    const int p = blockIdx.x;
    const int t = threadIdx.x;
#ifdef FICP_BSEL_PROF
    const long long t_entry = wall_clock64();
#endif
    // the phase, the stage and the plot's row range load together (one latency, not two)
    const int ph = st[p].phase, stg = st[p].stage, s_it = st[p].it, s_wfl = st[p].wfloor;
    const long long s_kprev = st[p].k;
    const u64 s_tkey = st[p].tkey, s_tmove = st[p].tmove;
    const int64_t b = so[p], e = so[p + 1];
    if (ph == PH_DONE) {  // uniform per workgroup
        if (t == 0) batch_arrive(bs, 0);
        return;
    }
    // the plot's state for the step (thread 0, plot_step_fit), loaded with the rows: a load
    // there was one more round trip on the workgroup's chain
    __shared__ PlotState s_ps;
    constexpr int PSW = (int)(sizeof(PlotState) / 4);
    static_assert(PSW <= KST, "one state word per thread");
    if (t < PSW) reinterpret_cast<uint32_t *>(&s_ps)[t] = reinterpret_cast<const uint32_t *>(st + p)[t];
#ifdef FICP_BSEL_PROF
    long long bt_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    __shared__ long long s_bt[16];
#endif
    const double lam = lams[stg];
    const double pe = 2.0 * lam + 1.0;
    const long long N = e - b;
    u64 kc[CACHED ? RPT : 1];
    double rc[CACHED && BSEL_RCACHE ? RPT : 1];
    // the rows' caller rows too when the registers allow (the 20-row form): the window
    // rows' tie-break words were a dependent load inside the S_base pass (~1.5 us)
    constexpr bool OCACHE = CACHED && RPT <= 20;
    uint32_t oc[OCACHE ? RPT : 1];
    if (CACHED) {
        // (key == nullptr: the NN stored no keys, each is derived from its row's r --
        // key_of_r, the NN's own operations -- once the loads have issued)
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t i = b + t + (int64_t)q * ST;
            kc[q] = (key && i < e) ? key[i] : ~0ULL;
            if (BSEL_RCACHE) rc[q] = i < e ? r[i] : INFINITY;
            if (OCACHE) oc[q] = (i < e && ws.worig) ? ws.worig[i] : (uint32_t)i;
        }
        if (!key) {
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t i = b + t + (int64_t)q * ST;
                if (i < e) kc[q] = key_of_r(BSEL_RCACHE ? rc[q] : r[i]);
            }
        }
    }
    BSEL_T(0);
    // (A per-plot window path as k_sel_win measured slower here: 128 plots 793-797k vs
    // 866-867k plot-it/s, 1024 plots equal -- 255 VGPRs with spills, and a 10k-row plot's
    // window holds few rows; removed in round 5.)
    (void)s_it;
    (void)s_kprev;
    (void)s_tkey;
    (void)s_tmove;
    (void)s_wfl;
    // 1. key range of the finite rows
    u64 amin = 0, kmax = 0;
    unsigned nfin = 0;
    SEL_ROWS(if (rv < INFINITY) {
        amin = max(amin, ~kk);
        kmax = max(kmax, kk);
        ++nfin;
    })
    blk_max2_sum(amin, kmax, nfin, red);
    if (nfin == 0) {  // every distance inf / NaN: the reference keeps (0.0, 0)
        if (bs.fuse) {
            plot_step_fit<ST / 64>(st, &s_ps, p, 0, 0.0, INFINITY, 0, 0, b, e, key, kc, bs, s_fit8, s_fitflag);
        } else if (t == 0) {
            st[p].k = 0;
            st[p].frac = 0.0;
            st[p].frmsd = INFINITY;
        }
        return;
    }
    const u64 kmin = ~amin;
    const int nb = fb::bits_of(kmax - kmin);
    const int sh = nb > SB_LOG ? nb - SB_LOG : 0;
    // bucket sums of r as integers on the grid 2^Lq (floor per row): the same bits in any
    // atomic order (a double LDS atomic sum was not; its last bits moved the window and so
    // the split between S_base and the window's scan).  r < 2^e1 for every finite row
    // (d <= dmax, d = sqrt(r) rounded), so nfin rows fit in 62 bits; a bucket's true sum
    // lies in [lo, lo + count) units.
    // Each bucket is one u64 LDS word: its count in the top HB_CB bits, its sum in the low
    // HB_SB (one atomic per row instead of two): nfin < 2^15 rows below 2^HB_SB units.
    const double dmax = __longlong_as_double((long long)(kmax & 0x7fffffffffffffffULL));
    const int e1 = dmax > 0.0 ? 2 * (ilogb(dmax) + 1) : 0;
    constexpr int HB_SB = 49;
    constexpr u64 HB_SM = (1ULL << HB_SB) - 1ULL;
    static_assert(KST * KRPT < (1 << (64 - HB_SB)), "bucket counts in the top bits");
    const int Lq = e1 - (HB_SB - fb::bits_of((u64)nfin));
    u64 *s_fx = reinterpret_cast<u64 *>(s_sum);
    BSEL_T(1);
    // 2. histogram
#pragma unroll
    for (int j = 0; j < SPER; ++j) s_fx[t * SPER + j] = 0ULL;
    if (t == 0) s_nact = 0;
    __syncthreads();
    SEL_ROWS(if (rv < INFINITY) {
        const int bk = (int)((kk - kmin) >> sh);
        atomicAdd(&s_fx[bk], (1ULL << HB_SB) | fx_floor(rv, Lq));
    })
    __syncthreads();
    BSEL_T(2);
    // 3. bounds over the buckets (thread t owns buckets t*SPER .. t*SPER + SPER - 1): the
    // lower sums P (prefix of the lo values); the upper sum before a bucket is P + C units
    unsigned c[SPER];
    double sm[SPER];
    unsigned tc = 0;
    double ts = 0.0;
#pragma unroll
    for (int j = 0; j < SPER; ++j) {
        const u64 hv = s_fx[t * SPER + j];
        c[j] = (unsigned)(hv >> HB_SB);
        sm[j] = ldexp((double)(hv & HB_SM), Lq);
        tc += c[j];
        ts = ts + sm[j];
    }
    unsigned Cex = tc;
    double Pex = ts;
    blk_excl_scan2(Cex, Pex, red);
    const double unit = ldexp(1.0, Lq);
    BSEL_T(8);
    // coarse to fine (as k_select.hip k_sel_bounds): U1 = the bound at each thread's chunk
    // end; a chunk whose lower bound (its rows are all >= its first bucket's lo_r) exceeds
    // U1 holds neither the minimising bucket end nor a candidate bucket, so only the few
    // chunks near the minimum evaluate their buckets (every thread evaluating its 4
    // buckets twice was ~40 % of the workgroup's time: 24 fp64 log2 per thread)
    double U1 = tc ? fb::h_of((long long)Cex + tc, (Pex + ts) + (double)(Cex + tc) * unit, pe) + fb::kMarg
                   : INFINITY;
    U1 = blk_min_d(U1, red);
    BSEL_T(9);
    // (the extra 1e-9 covers the different rounding of the chunk's and its buckets' sums)
    const bool active = tc && (!(fb::block_lb(Cex, tc, Pex, fb::lo_r(kmin + ((u64)(t * SPER) << sh)), pe) -
                                     1e-9 > U1) ||
                               !(pe >= 1.0));
    // the active chunks' buckets, one per lane: a chunk walked by its own thread chained
    // ~24 dependent fp64 log2 (8 us per plot at C4); per-lane they take two rounds
    if (active) {
        const int a = atomicAdd(&s_nact, 1);
        if (a < BMAXACT) {
            s_act[a] = t;
            long long C = Cex;
            double P = Pex;
#pragma unroll
            for (int j = 0; j < SPER; ++j) {
                s_eC[a * SPER + j] = C;  // rows and sum before bucket j of the chunk
                s_eP[a * SPER + j] = P;
                C += c[j];
                P = P + sm[j];
            }
        }
    }
    __syncthreads();
    const int nact = s_nact;
    double U = INFINITY;
    long long bmin = SB, bmax = -1;
    if (nact <= BMAXACT) {
        static_assert(BMAXACT * SPER <= ST, "one work item per lane");
        const int q = t;
        const bool has = q < nact * SPER;
        const int bk = has ? s_act[q / SPER] * SPER + (q % SPER) : 0;
        const u64 hq = has ? s_fx[bk] : 0ULL;
        const unsigned cq = (unsigned)(hq >> HB_SB);
        const long long C0 = has ? s_eC[q] : 0;
        const double P0 = has ? s_eP[q] : 0.0;
        // the same additions in the same order as the chunk walk: same bits; the bucket's
        // end value and its lower bound in one round of independent log2
        double lb = INFINITY;
        if (cq) {
            U = fb::h_of(C0 + cq, (P0 + ldexp((double)(hq & HB_SM), Lq)) + (double)(C0 + cq) * unit, pe) +
                fb::kMarg;
            lb = fb::block_lb(C0, cq, P0, fb::lo_r(kmin + ((u64)bk << sh)), pe);
        }
        BSEL_T(10);
        U = fmin(blk_min_d(U, red), U1);
        if (cq && (!(lb > U) || !(pe >= 1.0))) {
            bmin = bk;
            bmax = bk;
        }
    } else {  // many active chunks (pe < 1: every non-empty one): each walks its buckets
        if (active) {
            long long C = Cex;
            double P = Pex;
#pragma unroll
            for (int j = 0; j < SPER; ++j) {
                if (c[j]) {
                    C += c[j];
                    P = P + sm[j];
                    U = fmin(U, fb::h_of(C, P + (double)C * unit, pe) + fb::kMarg);
                }
            }
        }
        U = fmin(blk_min_d(U, red), U1);
        if (active) {
            long long C = Cex;
            double P = Pex;
#pragma unroll
            for (int j = 0; j < SPER; ++j) {
                const int bk = t * SPER + j;
                if (c[j]) {
                    const double lb = fb::block_lb(C, c[j], P, fb::lo_r(kmin + ((u64)bk << sh)), pe);
                    if (!(lb > U) || !(pe >= 1.0)) {
                        bmin = min(bmin, (long long)bk);
                        bmax = max(bmax, (long long)bk);
                    }
                }
                C += c[j];
                P = P + sm[j];
            }
        }
    }
    {  // {min bmin, max bmax} as two maxima of non-negative words (DPP, blk_max2_sum)
        u64 ma = (u64)(SB - bmin), mb = (u64)(bmax + 1);
        unsigned mc = 0;
        blk_max2_sum(ma, mb, mc, red);
        bmin = SB - (long long)ma;
        bmax = (long long)mb - 1;
    }
    BSEL_T(11);
    // bucket starts (rows before each bucket) replace the counts; fill counters zeroed
    unsigned *fill = reinterpret_cast<unsigned *>(s_sum);
    {
        unsigned C = Cex;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const int bk = t * SPER + j;
            s_cnt[bk] = C;
            fill[bk] = 0u;
            if (bk == bmin) s_k[0] = C;
            if (bk == bmax) s_k[1] = C + c[j];
            C += c[j];
        }
    }
    __syncthreads();
    const long long K0 = s_k[0];
    const long long W = s_k[1] - K0;
    BSEL_T(3);
    // 4. sum of r below the window (deterministic), window rows to scratch: LDS when the
    // window is small (the normal case: tens of rows), the global scratch otherwise
    const bool inl = W <= WCAP;
    u64 *wk = inl ? l_wk : ws.wkey + b;
    uint32_t *wrw = inl ? l_wrow : ws.wrow + b;
    double *wr = inl ? l_wr : ws.wr + b;
    u64 *sk = inl ? l_sk : ws.skey + b;
    uint32_t *srw = inl ? l_srow : ws.srow + b;
    double *sr = inl ? l_sr : ws.sr + b;
    double sb = 0.0;
    SEL_ROWS(if (rv < INFINITY) {
        const int bk = (int)((kk - kmin) >> sh);
        if (bk < bmin) {
            sb = sb + rv;
        } else if (bk <= bmax) {
            const int64_t slot = (int64_t)s_cnt[bk] - K0 + atomicAdd(&fill[bk], 1u);
            wk[slot] = kk;
            // (ties: the caller's row)
            wrw[slot] = OCACHE ? oc[q < RPT ? q : 0] : (ws.worig ? ws.worig[i] : (uint32_t)i);
            wr[slot] = rv;
        }
    })
    const double S_base = blk_sum_d(sb, red);  // its barriers also publish the scratch
    BSEL_T(4);
    // 5. exact (key, row) order of the window: rank inside the row's bucket
    for (long long q = t; q < W; q += ST) {
        const u64 kq = wk[q];
        const uint32_t rq = wrw[q];
        const int bk = (int)((kq - kmin) >> sh);
        const long long s0 = (long long)s_cnt[bk] - K0;
        const long long s1 = (long long)(bk + 1 < SB ? s_cnt[bk + 1] : nfin) - K0;
        long long rank = 0;
        for (long long j = s0; j < s1; ++j) {
            const u64 kj = wk[j];
            rank += (kj < kq) || (kj == kq && wrw[j] < rq);
        }
        const int64_t pos = s0 + rank;
        sk[pos] = kq;
        srw[pos] = rq;
        sr[pos] = wr[q];
    }
    __syncthreads();
    BSEL_T(5);
    // 6. prefix sums in window order, FRMSD of every window position, first minimum
    double run = S_base, bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    for (long long c0 = 0; c0 < W; c0 += (long long)ST * SRP) {
        const long long j0 = c0 + (long long)t * SRP;
        double v[SRP];
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < SRP; ++q) {
            v[q] = (j0 + q < W) ? sr[j0 + q] : 0.0;
            acc = acc + v[q];
        }
        double tot;
        double S = run + blk_excl_scan_d(acc, tot, red);
#pragma unroll
        for (int q = 0; q < SRP; ++q) {
            if (j0 + q < W) {
                S = S + v[q];
                const long long k = K0 + j0 + q + 1;
                const double f = (1.0 / pow((double)k / (double)N, lam)) * sqrt(S / (double)k);
                if (f < bf) {  // ascending k: strict < keeps the first minimum (ficp.py:84)
                    bf = f;
                    bk = k;
                }
            }
        }
        run = run + tot;
    }
    BSEL_T(6);
    blk_argmin(bf, bk, red);
    BSEL_T(7);
#ifdef FICP_BSEL_PROF
    if (t == 0 && (p % 97) == 5)
        printf("BSEL p=%d N=%lld W=%lld sh=%d t: %lld %lld %lld %lld %lld %lld %lld | %lld %lld %lld %lld %lld\n", p, N, W, sh,
               bt_[1] - bt_[0], bt_[2] - bt_[1], bt_[3] - bt_[2], bt_[4] - bt_[3], bt_[5] - bt_[4],
               bt_[6] - bt_[5], bt_[7] - bt_[6], bt_[8] - bt_[2], bt_[9] - bt_[8], bt_[10] - bt_[9],
               bt_[11] - bt_[10], bt_[3] - bt_[11]);
#endif
    long long *pt = nullptr;
#ifdef FICP_BSEL_PROF
    if (t == 0) {
        for (int q = 0; q < 12; ++q) s_bt[q] = bt_[q];
        s_bt[12] = t_entry;
    }
    if ((p % 97) == 5) pt = s_bt;
#endif
    if (bs.fuse) {
        const bool none = bk == 0x7fffffffffffffffLL;  // every FRMSD NaN: (0.0, 0)
        plot_step_fit<ST / 64>(st, &s_ps, p, none ? 0 : bk, none ? 0.0 : (double)bk / (double)N,
                               none ? INFINITY : bf, none ? 0ULL : sk[bk - K0 - 1],
                               none ? 0LL : (long long)srw[bk - K0 - 1], b, e, key, kc, bs, s_fit8,
                               s_fitflag, -1, pt);
        return;
    }
    if (t == 0) {
        if (bk == 0x7fffffffffffffffLL) {  // every FRMSD NaN: the reference keeps (0.0, 0)
            st[p].k = 0;
            st[p].frac = 0.0;
            st[p].frmsd = INFINITY;
        } else {
            st[p].k = bk;
            st[p].frac = (double)bk / (double)N;
            st[p].frmsd = bf;
            st[p].tkey = sk[bk - K0 - 1];
            st[p].trow = (long long)srw[bk - K0 - 1];
        }
    }
}
#undef SEL_ROWS

// Rigid fit of every looping plot on its first k trees of the order: the plot's rows in
// chunks of FCH (one workgroup each, 8 rows per thread in flight), each chunk's 8 sums
// handed to the plot's last arriving chunk (sc1 stores, one agent-scope atomic add per
// workgroup on the plot's counter, sc1 loads: the k_fit_sums pattern), which adds them in
// chunk order and solves.  The chunking depends on the plot alone, so a plot's result does
// not depend on the rest of the batch.  (One workgroup per plot streamed 410 MB at 6.8
// TB/s with 1024 plots, but with 128 plots per GPU -- the N = 8 share -- a single round
// of 128 workgroups took 13 us per launch.)
constexpr int FCH = BB * 8;
__global__ __launch_bounds__(BB) void k_batch_fit(const double *sx, const double *sy,
                                                  const double *cx, const double *cy,
                                                  const unsigned long long *key, const double *r,
                                                  const int64_t *so, const PlotGrid *grids,
                                                  int allow_refl, PlotState *st, double *part,
                                                  unsigned *ctr, int gmax, const uint32_t *worig) {
    __shared__ double s[8 * (BB / 64)];
    __shared__ int s_last;
    const int p = blockIdx.x / gmax, g = blockIdx.x % gmax;
    // the phase and the plot's row range load together (one latency, not two)
    const int ph = st[p].phase;
    const int64_t b = so[p], e = so[p + 1];
    if (ph != PH_LOOP) {
        if (g == 0 && threadIdx.x == 0) st[p].apply = 0;
        return;
    }
    const long long k = st[p].k;  // k >= 1 in the loop phase
    const int64_t t = st[p].trow;  // the k-th row of the (key, row) order (k_batch_select)
    const unsigned long long tk = st[p].tkey;
    const double px = grids[p].px, py = grids[p].py;
    const int gp = (int)((e - b + FCH - 1) / FCH);  // chunks of this plot (<= gmax)
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // every load issued before the predicate (a row loop with a key load and then the
    // dependent row loads took two round trips per row)
    constexpr int FU = 8;
    {
        const int64_t i0 = b + (int64_t)g * FCH + threadIdx.x;
        unsigned long long kv[FU];
        double xs[FU], ys[FU], xt[FU], yt[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int64_t i = i0 + (int64_t)u * BB;
            const bool in = i < e;
            kv[u] = in ? (key ? key[i] : key_of_r(r[i])) : ~0ULL;
            xs[u] = in ? sx[i] : 0.0;
            ys[u] = in ? sy[i] : 0.0;
            xt[u] = in ? cx[i] : 0.0;
            yt[u] = in ? cy[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int64_t i = i0 + (int64_t)u * BB;
            if (i < e && (kv[u] < tk || (kv[u] == tk && (worig ? (int64_t)worig[i] : i) <= t))) {
                const double a0 = xs[u] - px, a1 = ys[u] - py;
                const double b0 = xt[u] - px, b1 = yt[u] - py;
                c[0] = c[0] + a0;
                c[1] = c[1] + a1;
                c[2] = c[2] + b0;
                c[3] = c[3] + b1;
                c[4] = c[4] + a0 * b0;
                c[5] = c[5] + a0 * b1;
                c[6] = c[6] + a1 * b0;
                c[7] = c[7] + a1 * b1;
            }
        }
    }
    // the chunk's sums: DPP wave sums, then the waves in order (fixed tree)
    constexpr int FW = BB / 64;
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = wave_sum63(c[q]);
    if ((threadIdx.x & 63) == 63)
#pragma unroll
        for (int q = 0; q < 8; ++q) s[8 * (threadIdx.x >> 6) + q] = c[q];
    __syncthreads();
    if (g >= gp) return;  // (uniform) no rows in this chunk
    if (threadIdx.x < 8) {
        double v = s[threadIdx.x];
#pragma unroll
        for (int w = 1; w < FW; ++w) v = v + s[8 * w + threadIdx.x];
        __hip_atomic_store(&part[8 * ((int64_t)p * gmax + g) + threadIdx.x], v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const bool last = __hip_atomic_fetch_add(&ctr[p], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) == (unsigned)gp - 1u;
        if (last) __hip_atomic_exchange(&ctr[p], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
    }
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = 0.0;
    for (int h = 0; h < gp; ++h)  // the chunks in order
#pragma unroll
        for (int q = 0; q < 8; ++q)
            c[q] = c[q] + __hip_atomic_load(&part[8 * ((int64_t)p * gmax + h) + q], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
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

__global__ __launch_bounds__(UT) void k_batch_update(int nplots, int nstages, double threshold,
                                                     int max_iter, PlotState *st, int *flag,
                                                     long long *trace, int max_trace) {
    __shared__ int s_live[UT / 64];
    int live = 0;
    for (int p = threadIdx.x; p < nplots; p += UT)
        live += update_plot(st, p, nstages, threshold, max_iter, trace, max_trace) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o, 64);
    if ((threadIdx.x & 63) == 0) s_live[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < UT / 64; ++w) tot += s_live[w];
        __threadfence_system();
        __hip_atomic_store(flag, tot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// the number of plots still running (the selection took the loop step: BatchStep::fuse)
__global__ __launch_bounds__(UT) void k_batch_live(int nplots, const PlotState *st, int *flag) {
    __shared__ int s_live[UT / 64];
    int live = 0;
    for (int p = threadIdx.x; p < nplots; p += UT) live += st[p].phase != PH_DONE ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o, 64);
    if ((threadIdx.x & 63) == 0) s_live[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < UT / 64; ++w) tot += s_live[w];
        __threadfence_system();
        __hip_atomic_store(flag, tot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------- per-plot sorts
// The batch grid (stems by the cell of their plot's grid, row-major) and the batch work
// order (trees by 8x8-cell supertile, then cell) as one LDS counting sort per plot: one
// workgroup holds a plot's points in registers (PS_R per thread), counts their keys in LDS,
// scans the counts, drops each point into its key's bin and ranks it there by its row
// (bins hold ~1 point), then writes it at its final position -- scattered stores inside the
// plot's own ~80-320 KB region, which its CU's L2 merges into whole lines.  The order is the
// two-level bucket sort's (key, row), so the outputs are bit-identical to it; that sort moved
// every point's 32-B record through global memory twice (~0.45 ms per 10M points).
constexpr int PS_T = 1024;
constexpr int PS_R = 12;
constexpr int PS_MAXN = PS_T * PS_R;  // points of one plot (16-bit indices)
constexpr int PS_MAXK = PS_T * PS_R;  // keys of one plot
constexpr int PS_KPT = PS_MAXK / PS_T;

__device__ __forceinline__ uint32_t ps_st_key(int cx, int cy, int gx) {  // (k_bsort.hip st_key)
    const uint32_t nstx = (uint32_t)(gx + 7) >> 3;
    const uint32_t stl = ((uint32_t)cy >> 3) * nstx + ((uint32_t)cx >> 3);
    return (stl << 6) | ((uint32_t)(cy & 7) << 3) | (uint32_t)(cx & 7);
}

// an LDS-only barrier: __syncthreads() also waits for every outstanding global access
// (vmcnt(0)), stores included, so each stage hand-off below waited for the previous
// column's global stores to complete
#define PS_LDS_SYNC() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
__global__ __launch_bounds__(PS_T) void k_plot_sort(PlotSortJob A, PlotSortJob B, const PlotGrid *grids,
                                                    int nplots) {
    const bool jb = (int)blockIdx.x >= nplots;
    const PlotSortJob J = jb ? B : A;
    const int p = (int)blockIdx.x - (jb ? nplots : 0);
    const PlotGrid g = grids[p];
    const int64_t b = J.off[p], e = J.off[p + 1];
    const int N = (int)(e - b);
    const int nk = J.mode == 0 ? g.gx * g.gy : ((g.gx + 7) >> 3) * ((g.gy + 7) >> 3) * 64;
    if (N > PS_MAXN || nk >= PS_MAXK) return;  // (the host checks every plot: never)
    // the sort's arrays, and afterwards (aliased) one output column staged in final order
    __shared__ __align__(16) unsigned char s_mem[PS_MAXN * 8];
    static_assert(PS_MAXK / 2 * 4 + PS_MAXK * 4 + PS_MAXN * 2 <= PS_MAXN * 8, "sort arrays in the stage");
    uint32_t *s_cnt2 = (uint32_t *)s_mem;                            // two 16-bit counts per word
    uint32_t *s_start = s_cnt2 + PS_MAXK / 2;                        // bin starts, then fill
    uint16_t *s_idx = (uint16_t *)(s_start + PS_MAXK);               // bin slot -> point
    __shared__ uint32_t s_w[PS_T / 64];
    const int t = threadIdx.x;
    for (int k = t; k < PS_MAXK / 2; k += PS_T) s_cnt2[k] = 0u;
    // the points' keys (their coordinates are reloaded, coalesced and L2-hot, when the
    // outputs are written: holding x, y, z of PS_R points per thread spilled 98 VGPRs)
    int key[PS_R];
    {
        double px[PS_R], py[PS_R];
#pragma unroll
        for (int u = 0; u < PS_R; ++u) {
            const int i = t + u * PS_T;
            const bool in = i < N;
            px[u] = in ? J.x[b + i] : 0.0;
            py[u] = in ? J.y[b + i] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PS_R; ++u) {
            key[u] = -1;
            if (t + u * PS_T < N) {
                const int cx = cell_coord_b(px[u], g.x0, g.inv_h, g.gx);
                const int cy = cell_coord_b(py[u], g.y0, g.inv_h, g.gy);
                key[u] = J.mode == 0 ? cy * g.gx + cx : (int)ps_st_key(cx, cy, g.gx);
                atomicAdd(&s_cnt2[key[u] >> 1], (key[u] & 1) ? 0x10000u : 1u);
            }
        }
    }
    __syncthreads();
    auto cnt_of = [&](int k) -> uint32_t { return (s_cnt2[k >> 1] >> (16 * (k & 1))) & 0xffffu; };
    {  // exclusive scan of the counts, PS_KPT keys per thread (a contiguous run)
        uint32_t c[PS_KPT], tot = 0;
#pragma unroll
        for (int j = 0; j < PS_KPT; ++j) {
            const int k = t * PS_KPT + j;
            c[j] = k < nk ? cnt_of(k) : 0u;
            tot += c[j];
        }
        const uint32_t xi = (uint32_t)wave_incl_scan_ll((long long)tot);
        const int lane = t & 63, w = t >> 6;
        if (lane == 63) s_w[w] = xi;
        __syncthreads();
        uint32_t run = xi - tot;
        for (int q = 0; q < w; ++q) run += s_w[q];
#pragma unroll
        for (int j = 0; j < PS_KPT; ++j) {
            const int k = t * PS_KPT + j;
            s_start[k] = run;
            run += c[j];
        }
    }
    __syncthreads();
    // the grid's cell starts (global rows; the cell after the plot's last one is the next
    // plot's first: the same value from both plots), coalesced from LDS before the bins
    // fill: stored from the scan's registers, each lane's 12 consecutive keys put every
    // lane of a store 48 B from its neighbour (~5 us per plot of uncoalesced stores)
    if (J.mode == 0) {  // (uniform per workgroup)
        for (int k = t; k <= nk; k += PS_T) J.cell_start[g.cell_base + k] = (int32_t)(b + s_start[k]);
        PS_LDS_SYNC();
    }
    // a point alone in its bin (most of them) has its final position already: the slot
    // its atomic returned (re-reading the bin's bounds for every point took ~4 us per plot)
    int slot[PS_R];
#pragma unroll
    for (int u = 0; u < PS_R; ++u) {
        slot[u] = -1;
        if (key[u] >= 0) {
            const uint32_t c = cnt_of(key[u]);
            const uint32_t sl = atomicAdd(&s_start[key[u]], 1u);
            s_idx[sl] = (uint16_t)(t + u * PS_T);
            slot[u] = c == 1u ? (int)sl : -2;
        }
    }
    __syncthreads();
    // final position of each point (its rank inside its bin by row), in key[]'s registers
#pragma unroll
    for (int u = 0; u < PS_R; ++u) {
        if (key[u] < 0) continue;
        if (slot[u] >= 0) {
            key[u] = slot[u];
            continue;
        }
        const int i = t + u * PS_T;
        const uint32_t be = s_start[key[u]], bs = be - cnt_of(key[u]);
        uint32_t rank = 0;
        for (uint32_t q = bs; q < be; ++q) rank += s_idx[q] < (uint16_t)i ? 1u : 0u;
        key[u] = (int)(bs + rank);
    }
    const int *pos = key;
    // the outputs field by field through the stage: each point's value reloaded (coalesced,
    // L2-hot) and stored into the stage at its final position, then coalesced global stores
    // (scattered 8-B global stores: every lane of a store on its own cache line).  Grid
    // records (32 B: x, y, z, row) in two halves of positions, 16 B per record per pass: the
    // columns of a field pair are loaded once for both halves (reloaded per half, every
    // grid workgroup waited for four load round trips more).
    double *sd = (double *)s_mem;
    uint32_t *su = (uint32_t *)s_mem;
    const int half = PS_MAXN / 2;
    if (J.mode == 0) {
        for (int f = 0; f < 2; ++f) {  // 0: (x, y); 1: (z, row)
            const double *c0 = f == 0 ? J.x : J.z;  // (z nullable: 2-D layers store 0)
            double v0[PS_R], v1[PS_R];
#pragma unroll
            for (int u = 0; u < PS_R; ++u) {
                const int i = t + u * PS_T;
                v0[u] = (pos[u] >= 0 && c0) ? c0[b + i] : 0.0;
                v1[u] = (pos[u] >= 0 && f == 0) ? J.y[b + i] : 0.0;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // (unrolled: the halves' waits know v0 / v1 landed)
                const int r0 = h * half, r1 = min(N, r0 + half);
                PS_LDS_SYNC();  // (the sort's arrays / the previous half are consumed)
#pragma unroll
                for (int u = 0; u < PS_R; ++u) {
                    if (pos[u] < r0 || pos[u] >= r1) continue;
                    const uint32_t row = (uint32_t)(b + t + u * PS_T);
                    sd[2 * (pos[u] - r0)] = v0[u];
                    sd[2 * (pos[u] - r0) + 1] = f == 0 ? v1[u] : __longlong_as_double((long long)row);
                }
                PS_LDS_SYNC();
                for (int r = r0 + t; r < r1; r += PS_T)
                    *reinterpret_cast<double2 *>(reinterpret_cast<double *>(J.pts + b + r) + 2 * f) =
                        make_double2(sd[2 * (r - r0)], sd[2 * (r - r0) + 1]);
            }
        }
        return;
    }
    // mode 1: x and y loaded together (one round trip for both columns), then z, then the
    // rows, each staged in full and stored coalesced
    for (int f = 0; f < 2; ++f) {  // 0: x, y; 1: z (3-D), row
        const double *c0 = f == 0 ? J.x : J.z;
        double v0[PS_R], v1[PS_R];
#pragma unroll
        for (int u = 0; u < PS_R; ++u) {
            const int i = t + u * PS_T;
            v0[u] = (pos[u] >= 0 && c0) ? c0[b + i] : 0.0;
            v1[u] = (pos[u] >= 0 && f == 0) ? J.y[b + i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // x, y, z, row (unrolled, as mode 0's halves)
            const int ps = 2 * f + q;
            if (ps == 2 && !J.wz) continue;  // (uniform: 2-D plots have no z)
            PS_LDS_SYNC();  // (the sort's arrays / the previous column are consumed)
#pragma unroll
            for (int u = 0; u < PS_R; ++u) {
                if (pos[u] < 0) continue;
                if (ps == 3) su[pos[u]] = (uint32_t)(b + t + u * PS_T);
                else sd[pos[u]] = ps == 1 ? v1[u] : v0[u];
            }
            PS_LDS_SYNC();
            double *dst = ps == 0 ? J.wx : (ps == 1 ? J.wy : J.wz);
            for (int r = t; r < N; r += PS_T) {
                if (ps == 3) J.worig[b + r] = su[r];
                else dst[b + r] = sd[r];
            }
        }
    }
}

// The batch's moved XY back into the caller's rows, one workgroup per plot: the plot's work
// rows (caller row worig, wx, wy) read coalesced, each value placed at its caller position in
// an LDS stage, then written coalesced (k_scatter_xy's scattered 8-B stores: 166 us at C4).
__global__ __launch_bounds__(PS_T) void k_plot_scatter_xy(const uint32_t *worig, const double *wx,
                                                          const double *wy, const int64_t *off,
                                                          double *sx, double *sy) {
    const int p = blockIdx.x;
    const int64_t b = off[p], e = off[p + 1];
    const int N = (int)(e - b);
    if (N > PS_MAXN) return;  // (the host checks every plot: never)
    __shared__ double s_v[PS_MAXN];
    const int t = threadIdx.x;
    int dst[PS_R];
    double vx[PS_R], vy[PS_R];
#pragma unroll
    for (int u = 0; u < PS_R; ++u) {
        const int i = t + u * PS_T;
        const bool in = i < N;
        dst[u] = in ? (int)(worig[b + i] - (uint32_t)b) : -1;
        vx[u] = in ? wx[b + i] : 0.0;
        vy[u] = in ? wy[b + i] : 0.0;
    }
    for (int c = 0; c < 2; ++c) {
        if (c) __syncthreads();  // (the x column is written out)
#pragma unroll
        for (int u = 0; u < PS_R; ++u)
            if (dst[u] >= 0) s_v[dst[u]] = c ? vy[u] : vx[u];
        __syncthreads();
        double *out = c ? sy : sx;
        for (int r = t; r < N; r += PS_T) out[b + r] = s_v[r];
    }
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

hipError_t launch_batch_init(const BatchInitArgs &a, hipStream_t s) {
    const int nt = std::max(a.nplots + 1, std::max(a.nl, a.narrive));
    hipLaunchKernelGGL(k_batch_init, dim3(nblk(nt)), dim3(256), 0, s, a);
    return hipGetLastError();
}

int batch_fit_chunks(int64_t max_rows) {
    return (int)std::max<int64_t>(1, (max_rows + FCH - 1) / FCH);
}

hipError_t launch_batch_fit(const double *sx, const double *sy, const double *cx,
                            const double *cy, const unsigned long long *key, const double *r,
                            const int64_t *so, const PlotGrid *grids, int nplots, int64_t max_rows,
                            int allow_refl, PlotState *st, double *part, unsigned *ctr, hipStream_t s,
                            const uint32_t *worig) {
    if (nplots <= 0) return hipSuccess;
    const int gmax = batch_fit_chunks(max_rows);
    hipLaunchKernelGGL(k_batch_fit, dim3((unsigned)nplots * (unsigned)gmax), dim3(BB), 0, s, sx, sy,
                       cx, cy, key, r, so, grids, allow_refl, st, part, ctr, gmax, worig);
    return hipGetLastError();
}

__global__ void k_zero_u32_atomic(unsigned *p, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        __hip_atomic_exchange(&p[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_batch_fit_ctr_zero(unsigned *ctr, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_zero_u32_atomic, dim3((unsigned)std::min(1024, (n + 255) / 256)), dim3(256), 0,
                       s, ctr, n);
    return hipGetLastError();
}

bool plot_sort_fits(int64_t max_points, int64_t max_keys) {
    return max_points <= PS_MAXN && max_keys < PS_MAXK;  // (key nk: the plot's end)
}

hipError_t launch_plot_sort(const PlotSortJob &a, const PlotSortJob *b, const PlotGrid *grids,
                            int nplots, hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    const PlotSortJob bb = b ? *b : a;
    hipLaunchKernelGGL(k_plot_sort, dim3((unsigned)nplots * (b ? 2u : 1u)), dim3(PS_T), 0, s, a, bb,
                       grids, nplots);
    return hipGetLastError();
}

hipError_t launch_plot_scatter_xy(const uint32_t *worig, const double *wx, const double *wy,
                                  const int64_t *off, int nplots, double *sx, double *sy,
                                  hipStream_t s) {
    if (nplots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_plot_scatter_xy, dim3((unsigned)nplots), dim3(PS_T), 0, s, worig, wx, wy, off, sx, sy);
    return hipGetLastError();
}

hipError_t launch_batch_live(int nplots, const PlotState *st, int *flag, hipStream_t s) {
    hipLaunchKernelGGL(k_batch_live, dim3(1), dim3(UT), 0, s, nplots, st, flag);
    return hipGetLastError();
}

hipError_t launch_batch_select(const unsigned long long *key, const double *r, const int64_t *so,
                               int nplots, int64_t max_rows, const double *lambdas,
                               PlotState *st, BatchSelScratch ws, hipStream_t s,
                               const BatchStepArgs *step) {
    if (nplots <= 0) return hipSuccess;
    BatchStep bs{};
    if (step) {
        bs.sx = step->sx;
        bs.sy = step->sy;
        bs.cx = step->cx;
        bs.cy = step->cy;
        bs.grids = step->grids;
        bs.fuse = 1;
        bs.allow_refl = step->allow_refl;
        bs.nstages = step->nstages;
        bs.max_iter = step->max_iter;
        bs.threshold = step->threshold;
        bs.arrive = step->arrive;
        bs.flag = step->flag;
        bs.nplots = nplots;
        bs.trace = step->trace;
        bs.max_trace = step->max_trace;
        bs.worig = step->worig;
        bs.r = r;
    }
    // (1024-thread workgroups for plots fewer than the CUs measured slower: 128 plots 0.53 vs
    // 0.38 ms of selection per batch run -- 128 VGPRs with spills, 16-wave barriers; round 5
    // with 16 cached rows per thread: 131 VGPRs spilled, with 10: 200 B of scratch per lane
    // at the 128-VGPR cap, since the uncached form alone holds 141; not run)
    // cached rows per thread by plot size: 20 (plots up to 10,240 rows: C4's 10k) or RPT (the
    // unrolled row loops skip no padding slot, so a 10k-row plot ran 32 iterations per pass)
    constexpr int RPT_S = 20;
    if (max_rows <= (int64_t)ST * RPT_S)
        hipLaunchKernelGGL((k_batch_select<true, ST, RPT_S>), dim3(nplots), dim3(ST), 0, s, key, r, so,
                           lambdas, st, ws, bs);
    else if (max_rows <= (int64_t)ST * RPT)
        hipLaunchKernelGGL((k_batch_select<true, ST, RPT>), dim3(nplots), dim3(ST), 0, s, key, r, so,
                           lambdas, st, ws, bs);
    else
        hipLaunchKernelGGL((k_batch_select<false, ST, RPT>), dim3(nplots), dim3(ST), 0, s, key, r, so,
                           lambdas, st, ws, bs);
    return hipGetLastError();
}

hipError_t launch_batch_update(int nplots, int nstages, double threshold, int max_iter,
                               PlotState *st, int *flag, hipStream_t s, long long *trace,
                               int max_trace) {
    hipLaunchKernelGGL(k_batch_update, dim3(1), dim3(UT), 0, s, nplots, nstages, threshold,
                       max_iter, st, flag, trace, max_trace);
    return hipGetLastError();
}

}  // namespace ficp
