// k_select_fit.hip -- FRMSD-optimal fraction selection (ficp.py:54-60, 73-86) and the
// 2D rigid least-squares fit (ficp.py:89-110) on the device.
//
// Fraction: the reference evaluates FRMSD(k) = (1.0 / (k/N)**lambda) * sqrt(S_k / k) for
// every prefix k of argsort(dist), each with a fresh O(k) sum -> O(N^2) (ficp.py:80-85).
// Here S_k is ONE prefix scan of r_(j) = sum_md (src - corr)^2 in selection order (the
// sort already wrote r in that order, so every read is coalesced): tile sums -> scan of
// the tile sums -> per-tile scan fused with the FRMSD evaluation and a first-minimum
// argmin.  Deterministic: fixed reduction trees, no float atomics.
//
// Fit: the selected set is {i : (key_i, i) <= (key_t, t)} with t = order[k-1] (the k-th
// entry of the stable order), so the fit streams every source point in index order
// (coalesced x, y, corr x, corr y, key) instead of gathering through the permutation.
// One pass accumulates the 8 sums of the pivot-shifted pairs (pivot = CHM-layer centre,
// so geo-referenced ~6.5e6 m coordinates keep their precision); H = sum s't'^T -
// k cs' ct'^T.  R from the closed form of the 2x2 Kabsch problem: rotation angle
// atan2(H01 - H10, H00 + H11), identical to the SVD path R = Vt^T U^T with the det fix
// of ficp.py:101-103; with allow_reflection the SVD path returns a
// reflection iff det(H) < 0, given by the angle atan2(H01 + H10, H00 - H11).
#include "ficp_internal.h"

#include <math.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int FB = 256;
constexpr int FI = 4;
constexpr int FTILE = FB * FI;
// k_fit_sums: FIT_I rows per thread.  Each workgroup arrives once at one of 8 group
// counters (blockIdx % 8: one per XCD under round-robin dispatch) and the last of each
// group at the top counter: one word takes only ~88 atomics/us, so ~245 arrivals on one
// word serialised ~2.8 us
#ifndef FICP_FIT_I
#define FICP_FIT_I 8
#endif
#ifndef FICP_FIT_B
#define FICP_FIT_B 512
#endif
constexpr int FIT_I = FICP_FIT_I;
constexpr int FIT_B = FICP_FIT_B;  // threads of k_fit_sums
constexpr int FIT_CTR = 64;        // counter stride (u32 words: 256 B apart)
constexpr int FIT_PART = 4096;     // byte offset of the partial sums in the scratch
constexpr int FIT_W = FIT_B / 64;
constexpr int FIT_TILE = FIT_B * FIT_I;

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

// per tile: sum of r in selection order
__global__ __launch_bounds__(FB) void k_frac_tilesum(const double *rs, int64_t n, double *tsum,
                                                     const int *skip) {
    if (skip && *skip) return;
    __shared__ double s[256];
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + threadIdx.x;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < FI; ++q)  // strided within the tile: coalesced; order fixed
        if (j0 + q * FB < n) acc = acc + rs[j0 + q * FB];
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

__global__ __launch_bounds__(FB) void k_frac_eval(const double *rs, int64_t n, int64_t N,
                                                  double lam, const double *lam_dev,
                                                  const double *tpre, BestRec *tbest,
                                                  const int *skip) {
    if (skip && *skip) return;
    if (lam_dev) lam = *lam_dev;
    __shared__ double s[512];
    __shared__ double s_f[256];
    __shared__ long long s_k[256];
    const int64_t j0 = (int64_t)blockIdx.x * FTILE + (int64_t)threadIdx.x * FI;
    double v[FI];
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < FI; ++q) {
        v[q] = (j0 + q < n) ? rs[j0 + q] : 0.0;
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
            if (f < bf) {  // ascending k: strict < keeps the first minimum (ficp.py:84)
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
                                                    const double *lam_dev, IterState *st,
                                                    const int *skip) {
    if (skip && *skip) return;
    if (lam_dev) lam = *lam_dev;
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
        if (bk == 0x7fffffffffffffffLL) {  // every FRMSD was NaN: reference keeps (0.0, 0)
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
// threshold pair (key, orig) of the k-th entry of the stable order
__device__ __forceinline__ bool fit_threshold(const FitIn &a, unsigned long long &tk,
                                              int64_t &to) {
    if (!a.key) return true;  // every row selected
    // k and the threshold pair load together (the pair's loads used to wait for k's)
    const long long k = a.st->k;
    const unsigned long long tk0 = a.st->tkey;
    const int64_t to0 = a.st->torig;
    if (k <= 0) {
        tk = 0;
        to = -1;
        return false;
    }
    if (!a.order) {  // threshold pair from the bucketed selection
        tk = tk0;
        to = to0;
        return false;
    }
    const int64_t tp = (int64_t)a.order[k - 1];
    tk = a.key[tp];
    to = a.orig ? (int64_t)a.orig[tp] : tp;
    return false;
}

// The finishing step (k_fit_final's work) runs in the block that arrives last at the
// counter: partials are handed off with sc1 stores/loads and one agent-scope atomic add
// per block (MI355X_MICROARCH.md hand-off table, first row); the last block resets the
// counter (atomic exchange) for the next launch.
__device__ void fit_finish(const FitIn &a, const double *part, int nb, int allow_refl,
                           IterState *st, double *s, double *out8);

// out8 (distributed runs): the last block stores the 8 sums there instead of solving
__global__ __launch_bounds__(FIT_B) void k_fit_sums(FitIn a, double *part, unsigned *ctr,
                                                 int allow_refl, IterState *st,
                                                 const int *skip, double *out8) {
    // the skip flag and the threshold state load together; the rows after the skip test
    // (a no-op launch, 3 per C3 run, would otherwise read every row)
    const int sk = skip ? *skip : 0;
    __shared__ double s[256];
    __shared__ int s_last;
    unsigned long long tk = 0;
    int64_t ti = 0;
    const bool all = fit_threshold(a, tk, ti);
    if (sk) return;
    const int64_t i0 = (int64_t)blockIdx.x * FIT_TILE + threadIdx.x;
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // FIT_I rows per thread in chunks of 4, every load of a chunk in flight at once.  The
    // rows' coordinates are loaded whether selected or not: selection is scattered over
    // the work order, so a skipped row saves no cache line.
#pragma unroll
    for (int q0 = 0; q0 < FIT_I; q0 += 4) {
        unsigned long long kv[4];
        double xs[4], ys[4], xt[4], yt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + (int64_t)(q0 + u) * FIT_B;
            const bool in = i < a.n;
            kv[u] = (in && !all) ? a.key[i] : 0ULL;
            xs[u] = in ? a.sx[i] : 0.0;
            ys[u] = in ? a.sy[i] : 0.0;
            xt[u] = in ? a.cx[i] : 0.0;
            yt[u] = in ? a.cy[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + (int64_t)(q0 + u) * FIT_B;
            if (i < a.n) {
                bool sel = all;
                if (!all) {
                    const unsigned long long ki = kv[u];
                    sel = ki < tk || (ki == tk && (a.orig ? (int64_t)a.orig[i] : i) <= ti);
                }
                if (sel) {
                    const double dxs = xs[u] - a.px, dys = ys[u] - a.py;
                    const double dxt = xt[u] - a.px, dyt = yt[u] - a.py;
                    c[0] = c[0] + dxs;
                    c[1] = c[1] + dys;
                    c[2] = c[2] + dxt;
                    c[3] = c[3] + dyt;
                    c[4] = c[4] + dxs * dxt;
                    c[5] = c[5] + dxs * dyt;
                    c[6] = c[6] + dys * dxt;
                    c[7] = c[7] + dys * dyt;
                }
            }
        }
    }
    // fixed-order reduction: wave butterfly (every lane ends with the same bits), then the
    // four waves in order
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c[e] = c[e] + __shfl_xor(c[e], o, 64);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[8 * (threadIdx.x >> 6) + e] = c[e];
    __syncthreads();
    if (threadIdx.x < 8) {
        const int e = threadIdx.x;
        double t = s[e];
        for (int w = 1; w < FIT_W; ++w) t = t + s[8 * w + e];
        __hip_atomic_store(&part[8 * blockIdx.x + e], t, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned grp = blockIdx.x & 7u, ng = min(gridDim.x, 8u);
        const unsigned gsz = (gridDim.x - grp + 7u) / 8u;  // workgroups of this group
        unsigned *gc = ctr + FIT_CTR * (1 + grp);
        bool last = false;
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
            __hip_atomic_exchange(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
            if (last) __hip_atomic_exchange(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    fit_finish(a, part, (int)gridDim.x, allow_refl, st, s, out8);
}

__device__ void fit_finish(const FitIn &a, const double *part, int nb, int allow_refl,
                           IterState *st, double *s, double *out8) {
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < nb; b += FIT_B) {  // fixed order per thread
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
            v[e] = __hip_atomic_load(&part[8 * b + e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int e = 0; e < 8; ++e) c[e] = c[e] + v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c[e] = c[e] + __shfl_xor(c[e], o, 64);
    __syncthreads();  // s[] was used by the caller
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[8 * (threadIdx.x >> 6) + e] = c[e];
    __syncthreads();
    if (threadIdx.x != 0) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        double t = s[e];
        for (int w = 1; w < FIT_W; ++w) t = t + s[8 * w + e];
        c[e] = t;
    }
    if (out8) {
        for (int e = 0; e < 8; ++e) out8[e] = c[e];
        return;
    }
    const double k = a.key ? (double)a.st->k : (double)a.n;
    fit_solve(c, k, a.px, a.py, allow_refl, st);
}

// --------------------------------------------------------------- frmsd (public API)
__global__ __launch_bounds__(256) void k_ssd_partial(const double *sx, const double *sy,
                                                     const double *sz, const double *cx,
                                                     const double *cy, const double *cz,
                                                     int64_t k, int md, double *part) {
    __shared__ double s[256];
    const int64_t i0 = (int64_t)blockIdx.x * FTILE + threadIdx.x;
    double acc = 0.0;
    for (int q = 0; q < FI; ++q) {
        const int64_t i = i0 + q * FB;
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

hipError_t launch_fraction(const double *rs, int64_t n, int64_t n_src, double lam,
                           const double *lam_dev, void *tmp, IterState *st, const int *skip,
                           hipStream_t s) {
    const int nb = (int)((n + FTILE - 1) / FTILE);
    char *p = (char *)tmp;
    double *tsum = (double *)p;
    p += align_up((int64_t)(nb + 2) * 8, 256);
    BestRec *tbest = (BestRec *)p;
    if (nb > 0) {
        hipLaunchKernelGGL(k_frac_tilesum, dim3(nb), dim3(FB), 0, s, rs, n, tsum, skip);
        hipLaunchKernelGGL(k_frac_tilescan, dim3(1), dim3(256), 0, s, tsum, nb, skip);
        hipLaunchKernelGGL(k_frac_eval, dim3(nb), dim3(FB), 0, s, rs, n, n_src, lam, lam_dev, tsum,
                           tbest, skip);
    }
    hipLaunchKernelGGL(k_frac_final, dim3(1), dim3(256), 0, s, tbest, nb, tsum, n, n_src, lam,
                       lam_dev, st, skip);
    return hipGetLastError();
}

// fit scratch: [0, 256) the arrival counter (atomics only; zeroed once per allocation by
// launch_fit_init), then 8 partial sums per block
int64_t fit_tmp_bytes(int64_t n) {
    const int64_t nb = (n + FTILE - 1) / FTILE + 1;
    return FIT_PART + align_up(nb * 8 * 8, 256);
}

int64_t fit_scratch_offset() { return FIT_PART; }

hipError_t launch_fit_init(void *tmp, hipStream_t s) {
    return launch_atomic_zero32((uint32_t *)tmp, FIT_PART / 4, s);
}

hipError_t launch_fit(const FitIn &a, int allow_reflection, void *tmp, IterState *st,
                      const int *skip, hipStream_t s) {
    const int nb = (int)std::max<int64_t>(1, (a.n + FIT_TILE - 1) / FIT_TILE);
    unsigned *ctr = (unsigned *)tmp;
    double *part = (double *)((char *)tmp + FIT_PART);
    hipLaunchKernelGGL(k_fit_sums, dim3(nb), dim3(FIT_B), 0, s, a, part, ctr, allow_reflection, st,
                       skip, (double *)nullptr);
    return hipGetLastError();
}

// distributed runs: this rank's 8 fit sums (k_fit_sums without the solve), then, once the
// caller has gathered every rank's sums, the solve on their sum in rank order
hipError_t launch_fit_sums(const FitIn &a, void *tmp, const int *skip, double *out8,
                           hipStream_t s) {
    const int nb = (int)std::max<int64_t>(1, (a.n + FIT_TILE - 1) / FIT_TILE);
    unsigned *ctr = (unsigned *)tmp;
    double *part = (double *)((char *)tmp + FIT_PART);
    hipLaunchKernelGGL(k_fit_sums, dim3(nb), dim3(FIT_B), 0, s, a, part, ctr, 0,
                       const_cast<IterState *>(a.st), skip, out8);
    return hipGetLastError();
}

__global__ void k_fit_solve_ranks(const double *sums, int world, double px, double py,
                                  int allow_refl, IterState *st, const int *skip) {
    if ((skip && *skip) || threadIdx.x != 0) return;
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = 0; q < world; ++q)
        for (int e = 0; e < 8; ++e) c[e] = c[e] + sums[8 * q + e];
    fit_solve(c, (double)st->k, px, py, allow_refl, st);
}

hipError_t launch_fit_solve_ranks(const double *sums, int world, double px, double py,
                                  int allow_refl, IterState *st, const int *skip, hipStream_t s) {
    hipLaunchKernelGGL(k_fit_solve_ranks, dim3(1), dim3(64), 0, s, sums, world, px, py, allow_refl,
                       st, skip);
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

}  // namespace ficp
