// k_small.hip -- the whole two-stage ICP of one small plot in ONE workgroup.
//
// The production caller joins one field plot at a time: 5-44 trees against the ~260 CHM
// stems within 70 m (app.py:630-661, Data/*/Stand_10_trees.csv).  At that size the
// multi-kernel loop (capi.hip run_core: six launches per NN call, a bbox read-back, a
// grid build) is all launch and hand-off latency: ~0.5 ms per Join on the box, slower
// than the one-thread C oracle (bench.py app_scale_join).  Here the CHM layer is staged
// in LDS once, every tree lives in one thread's registers, and each NN call of
// ficp.py:122-154 is a few block-wide steps with no global round trip:
//   apply T (ficp.py:112-119, the NN kernels' exact fma form)
//   exact 1-NN by brute force over the LDS stems (ficp.py:65-71: d2 = ((0 + dx^2) + dy^2)
//     + dz^2, no contraction, ascending index with strict <: the lowest index wins a tie)
//   the stable (d, row) order by rank counting, prefix sums of r in that order, FRMSD of
//     every k, first minimum (ficp.py:73-86; strict <, frmsd_of's operation order)
//   the rigid fit of the first k rows (ficp.py:89-110: k_fit_sums' 8 pivot-shifted sums,
//     in thread order, fit_solve's closed form)
//   the loop step (k_loop.hip loop_step: stage head, `cur - new <= threshold`,
//     max_iterations, the lambda switch of ficp.py:152)
// One launch per run(); the host reads the IterState and XY once at the end.
#include "ficp_internal.h"

#include <math.h>

namespace ficp {

namespace {

typedef unsigned long long u64;

template <int BT>
struct SmallRed {
    double d[BT / 64][8];
    u64 u[BT / 64];
    long long l[BT / 64];
};

// block sum of 8 doubles, fixed tree (wave butterfly, then the waves in order): every
// thread gets the same bits
template <int BT>
__device__ __forceinline__ void small_sum8(double (&c)[8], SmallRed<BT> &r) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c[e] = c[e] + __shfl_xor(c[e], o, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) r.d[w][e] = c[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        double t = 0.0;
#pragma unroll
        for (int v = 0; v < BT / 64; ++v) t = t + r.d[v][e];
        c[e] = t;
    }
    __syncthreads();
}

// exclusive scan of x in thread order + the block total (fixed schedule)
template <int BT>
__device__ __forceinline__ double small_excl_scan(double x, double &total, SmallRed<BT> &r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double xi = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(xi, o, 64);
        if (lane >= o) xi = y + xi;
    }
    double xe = __shfl_up(xi, 1, 64);
    if (lane == 0) xe = 0.0;
    if (lane == 63) r.d[w][0] = xi;
    __syncthreads();
    double off = 0.0, tot = 0.0;
#pragma unroll
    for (int v = 0; v < BT / 64; ++v) {
        if (v < w) off = off + r.d[v][0];
        tot = tot + r.d[v][0];
    }
    __syncthreads();
    total = tot;
    return w ? off + xe : xe;
}

// first minimum of (f, k) over the block (better(): smaller f, then smaller k)
template <int BT>
__device__ __forceinline__ void small_argmin(double &f, long long &k, SmallRed<BT> &r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double of = __shfl_xor(f, o, 64);
        const long long ok = __shfl_xor(k, o, 64);
        if (of < f || (of == f && ok < k)) {
            f = of;
            k = ok;
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        r.d[w][0] = f;
        r.l[w] = k;
    }
    __syncthreads();
    f = r.d[0][0];
    k = r.l[0];
#pragma unroll
    for (int v = 1; v < BT / 64; ++v)
        if (r.d[v][0] < f || (r.d[v][0] == f && r.l[v] < k)) {
            f = r.d[v][0];
            k = r.l[v];
        }
    __syncthreads();
}

// {min x, max x, min y, max y} of the stems (bbox -> the fit's pivot, as ensure_bbox)
template <int BT>
__device__ __forceinline__ void small_bbox(double (&b)[4], SmallRed<BT> &r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        b[0] = fmin(b[0], __shfl_xor(b[0], o, 64));
        b[1] = fmax(b[1], __shfl_xor(b[1], o, 64));
        b[2] = fmin(b[2], __shfl_xor(b[2], o, 64));
        b[3] = fmax(b[3], __shfl_xor(b[3], o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e) r.d[w][e] = b[e];
    __syncthreads();
#pragma unroll
    for (int v = 0; v < BT / 64; ++v) {
        b[0] = fmin(b[0], r.d[v][0]);
        b[1] = fmax(b[1], r.d[v][1]);
        b[2] = fmin(b[2], r.d[v][2]);
        b[3] = fmax(b[3], r.d[v][3]);
    }
    __syncthreads();
}

__device__ __forceinline__ void small_apply(const double *T, double &x, double &y) {
    // numpy's ([x, y, 1] @ T.T)[:, :2] through OpenBLAS dgemm (ficp.py:117), the NN
    // kernels' apply_T: fma(y, T01, x*T00) + T02 -- pinned by tests/golden/apply.npz
    const double nx = __fma_rn(y, T[1], x * T[0]) + T[2];
    const double ny = __fma_rn(y, T[4], x * T[3]) + T[5];
    x = nx;
    y = ny;
}

template <int BT, int MD>
__global__ __launch_bounds__(BT) void k_small_run(SmallArgs a, LoopCtl lc) {
    __shared__ double s_tx[kSmallMaxM], s_ty[kSmallMaxM], s_tz[MD == 3 ? kSmallMaxM : 1];
    __shared__ u64 s_key[BT];
    __shared__ double s_r[BT];
    __shared__ IterState s_st;
    __shared__ SmallRed<BT> red;
    const int t = threadIdx.x;
    const int n = a.n, m = a.m;
    const bool mine = t < n;
    if (a.host_t && t == 0)
        __hip_atomic_store(&a.host_t[0], (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // the CHM layer into LDS (it never moves, ficp.py:123,137), its bbox for the pivot
    double bb[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    for (int j = t; j < m; j += BT) {
        const double x = a.tx[j], y = a.ty[j];
        s_tx[j] = x;
        s_ty[j] = y;
        if (MD == 3) s_tz[j] = a.tz[j];
        bb[0] = fmin(bb[0], x);
        bb[1] = fmax(bb[1], x);
        bb[2] = fmin(bb[2], y);
        bb[3] = fmax(bb[3], y);
    }
    small_bbox<BT>(bb, red);
    const double px = bb[0] + 0.5 * (bb[1] - bb[0]), py = bb[2] + 0.5 * (bb[3] - bb[2]);
    // this thread's tree (the caller's rows straight from the upload, or SoA columns)
    double x = 0.0, y = 0.0, z = 0.0;
    if (mine) {
        if (a.rows) {
            const double *row = a.rows + (int64_t)t * a.ld;
            x = row[0];
            y = row[1];
            if (MD == 3) z = row[2];
        } else {
            x = a.sx[t];
            y = a.sy[t];
            if (MD == 3) z = a.sz[t];
        }
    }
    double r = INFINITY, cx = 0.0, cy = 0.0;
    u64 key = ~0ULL;
    int bi = 0x7fffffff;  // matched stem of the last NN call (a reused call keeps it)
    bool sel = false;  // in the selection of the last fraction call (the fit's input)
    if (t == 0) {
        IterState &s = s_st;
        for (int e = 0; e < 9; ++e) s.Ttot[e] = (e % 4 == 0) ? 1.0 : 0.0;
        s.cur = INFINITY;
        s.frmsd_last[0] = s.frmsd_last[1] = INFINITY;
        s.k = 0;
        s.k_last = 0;
        s.stage = 0;
        s.it = 0;
        s.n_nn = s.n_fit = 0;
        s.n_reuse = 0;
        s.iters[0] = s.iters[1] = 0;
        s.tkey = 0;
        s.torig = 0;
        s.tmove = 0;
        s.phase = lc.nstages > 0 ? PH_HEAD : PH_DONE;
        s.lam_cur = lc.nstages > 0 ? lam_of(lc, 0) : 0.0;
        loop_set_flags(s);
    }
    __syncthreads();
    for (;;) {
        const int done = s_st.done, no_fit = s_st.no_fit, apply = s_st.apply;
        const int reuse = s_st.nn_reuse;
        const double lam = s_st.lam_cur;
        const long long kprev = s_st.k;
        if (done) break;
        // ---- fit on the previous call's selection (ficp.py:133-134)
        if (!no_fit) {
            double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (sel) fit_add(c, x, y, cx, cy, px, py);
            small_sum8<BT>(c, red);
            if (t == 0 && kprev > 0) fit_solve(c, (double)kprev, px, py, a.allow_refl, &s_st);
            __syncthreads();
        }
        // ---- apply (ficp.py:135) and the NN call (ficp.py:137)
        if (apply && mine) small_apply(s_st.T, x, y);
        if (!reuse) {
            double best = INFINITY;
            bi = 0x7fffffff;
            if (mine) {
                for (int j = 0; j < m; ++j) {  // ascending j: strict < keeps the lowest index
                    const double s = sq_dist<MD>(x, y, z, s_tx[j], s_ty[j], MD == 3 ? s_tz[j] : 0.0);
                    if (s < best) {
                        best = s;
                        bi = j;
                    }
                }
                const int bj = bi < m ? bi : 0;  // no stem matched (NaN query): no gather out of the layer
                cx = s_tx[bj];
                cy = s_ty[bj];
                r = best;
                key = ordkey(sqrt(best));
            }
        }
        if (a.tidx && mine && s_st.n_nn < lc.max_trace_idx) a.tidx[(int64_t)s_st.n_nn * n + t] = bi;
        // ---- the stable order of (d, row), prefix sums, FRMSD of every k, first minimum
        s_key[t] = key;
        __syncthreads();
        int rank = 0;
        if (mine)
            for (int j = 0; j < n; ++j) {
                const u64 kj = s_key[j];
                rank += (kj < key) || (kj == key && j < t);
            }
        s_r[mine ? rank : t] = mine ? r : 0.0;
        __syncthreads();
        const double rp = s_r[t];
        double tot;
        const double S = small_excl_scan<BT>(rp, tot, red) + rp;  // sum of positions 0..t
        double bf = INFINITY;
        long long bk = 0x7fffffffffffffffLL;
        if (t < n) {
            const long long k = t + 1;
            const double f = frmsd_of(k, n, S, lam);
            if (f < bf) {
                bf = f;
                bk = k;
            }
        }
        small_argmin<BT>(bf, bk, red);
        const bool none = bk == 0x7fffffffffffffffLL;  // every FRMSD NaN: (0.0, 0)
        sel = mine && !none && rank < bk;
        if (t == 0) {
            IterState &s = s_st;
            s.k = none ? 0 : bk;
            s.frac = none ? 0.0 : (double)bk / (double)n;
            s.frmsd = none ? INFINITY : bf;
            s.n_src = n;
            loop_step(&s, lc);
        }
        __syncthreads();
    }
    if (mine && a.sx) {
        a.sx[t] = x;
        a.sy[t] = y;
    }
    if (a.host_flag) {
        // pinned host report: XY, the state and the end stamp, then the flag (system
        // scope release: every thread's stores are drained and made visible first)
        if (mine) {
            a.host_xy[2 * t] = x;
            a.host_xy[2 * t + 1] = y;
        }
        if (t == 0) {
            *a.host_st = s_st;
            __hip_atomic_store(&a.host_t[1], (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __threadfence_system();
        __syncthreads();
        if (t == 0) __hip_atomic_store(a.host_flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t == 0) {
        *a.st = s_st;
    }
}

}  // namespace

bool small_run_fits(int64_t n, int64_t m) {
    return n >= 1 && m >= 1 && n <= kSmallMaxN && m <= kSmallMaxM && n * m <= kSmallMaxPairs;
}

hipError_t launch_small_run(const SmallArgs &a, int md, const LoopCtl &lc, hipStream_t s) {
    if (a.n <= 256) {
        if (md == 3) hipLaunchKernelGGL((k_small_run<256, 3>), dim3(1), dim3(256), 0, s, a, lc);
        else hipLaunchKernelGGL((k_small_run<256, 2>), dim3(1), dim3(256), 0, s, a, lc);
    } else {
        if (md == 3) hipLaunchKernelGGL((k_small_run<1024, 3>), dim3(1), dim3(1024), 0, s, a, lc);
        else hipLaunchKernelGGL((k_small_run<1024, 2>), dim3(1), dim3(1024), 0, s, a, lc);
    }
    return hipGetLastError();
}

}  // namespace ficp
