// k_bsort.hip -- points sorted by a grid key in two levels, without global atomics:
// the CHM grid build (stems by cell) and the spatial work order of the tree layer (trees
// by 8x8-cell supertile, then cell).  Both orders are deterministic: (key, index).
//
//  1. k_bs_count   : B1 workgroups, each a contiguous slice of the points; LDS histogram
//                    of the coarse digit (key >> fs, <= 4096 buckets), stored per
//                    workgroup with plain stores.
//  2. k_bs_colscan : per bucket, the exclusive prefix over workgroups and the total.
//  3. k_bs_scatter : every workgroup scans the bucket totals itself (bases), then appends
//                    its points' 32-B records (x, y, z, index) to their buckets (LDS
//                    fill counters: the order inside a bucket is not yet fixed).
//  4. k_bs_bucket  : one workgroup per bucket: orders its points by (fine digit, index)
//                    -- a counting sort on the fine digit, then each point's rank among
//                    the equal-digit points of smaller index -- and writes the outputs
//                    in that order (grid: TPt records + cell_start; work order: SoA
//                    coordinates + caller index).  A bucket larger than the LDS tile is
//                    ordered the same way through global scratch.
// The previous grid build (global atomic counting sort + per-cell insertion sort) took
// ~150 us at 1M stems and the work order (64-bit radix sort + gather) ~170 us: scattered
// global atomics execute at the memory side, one 64-B request per lane.
#include "ficp_internal.h"

#include <math.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int BT = 1024;        // threads of k_bs_count / k_bs_scatter
constexpr int BMAXB = 16384;    // coarse buckets (max)
constexpr int BMAXB_LOG = 14;
constexpr int B4T = 256;        // threads of k_bs_bucket
constexpr int BMAXF_LOG = 12;   // fine digits per bucket (max 4096)

__device__ __forceinline__ int bs_coord(double v, double v0, double inv_h, int g) {
    double f = (v - v0) * inv_h;
    if (!(f >= 0.0)) return 0;  // also NaN
    if (f >= (double)(g - 1)) return g - 1;
    return (int)f;
}

// key of a point: mode 0 = cell id cy * gx + cx (the grid layout); mode 1 = 8x8-supertile
// order (supertile row-major, then the cell inside it row-major); mode 2 = the global cell
// id of the batch grids (the point's plot's cell_base + its cell in that plot's grid, as
// k_batch_grid_count); mode 3 = the batch work order (the point's plot's wbase + its mode-1
// key in that plot's grid: plot-major, so every plot keeps its contiguous row range)
__device__ __forceinline__ uint32_t st_key(int cx, int cy, int gx) {
    const uint32_t nstx = (uint32_t)(gx + 7) >> 3;
    const uint32_t st = ((uint32_t)cy >> 3) * nstx + ((uint32_t)cx >> 3);
    return (st << 6) | ((uint32_t)(cy & 7) << 3) | (uint32_t)(cx & 7);
}
__device__ __forceinline__ uint32_t bs_key(double x, double y, const BSortGeom &g, int64_t i) {
    if (g.mode >= 2) {
        const PlotGrid &pg = g.grids[g.plot[i]];
        const int cx = bs_coord(x, pg.x0, pg.inv_h, pg.gx);
        const int cy = bs_coord(y, pg.y0, pg.inv_h, pg.gy);
        if (g.mode == 2) return (uint32_t)(pg.cell_base + (long long)cy * pg.gx + cx);
        return (uint32_t)(pg.wbase + (long long)st_key(cx, cy, pg.gx));
    }
    const int cx = bs_coord(x, g.x0, g.inv_h, g.gx);
    const int cy = bs_coord(y, g.y0, g.inv_h, g.gy);
    if (g.mode == 0) return (uint32_t)cy * (uint32_t)g.gx + (uint32_t)cx;
    return st_key(cx, cy, g.gx);
}

// Every kernel runs one or two sort jobs side by side (the grid build and the work
// order): workgroups [0, split) take job a, the rest job b.  J is the workgroup's job,
// bid its workgroup index inside that job.
#define BS_PICK(SPLIT)                                         \
    const bool bs_b = (int)blockIdx.x >= (SPLIT);              \
    const BSJob &J = bs_b ? P.b : P.a;                         \
    const int bid = (int)blockIdx.x - (bs_b ? (SPLIT) : 0);    \
    const BSortGeom g = J.g;                                   \
    const BSortPlan p = J.p;

// The slices of k_bs_count / k_bs_scatter are dealt XCD-aware (slice = xcd_block of the
// workgroup within its job; each job's workgroups start at a multiple of 8): an XCD's
// slices are one contiguous range of points, so when the keys follow the point order (the
// batch: plot-major) its scattered records fill whole lines of its own L2.
__global__ __launch_bounds__(BT) void k_bs_count(BSPair P) {
    BS_PICK(P.split[0])
    if (bid >= p.nb1) return;  // (the padding of job a's workgroups to a multiple of 8)
    const int sl = (int)xcd_block(bid, p.nb1);
    const double *x = J.x, *y = J.y;
    const int64_t n = J.n;
    uint32_t *counts = J.counts;
    __shared__ uint32_t h[BMAXB];
    for (int b = threadIdx.x; b < p.nbk; b += BT) h[b] = 0u;
    __syncthreads();
    const int64_t i0 = (int64_t)sl * p.per, i1 = min(n, i0 + p.per);
    constexpr int U = 8;  // points in flight per thread
    for (int64_t i = i0 + threadIdx.x; i < i1; i += (int64_t)U * BT) {
        double xv[U], yv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = i + (int64_t)u * BT;
            xv[u] = q < i1 ? x[q] : 0.0;
            yv[u] = q < i1 ? y[q] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + (int64_t)u * BT < i1)
                atomicAdd(&h[bs_key(xv[u], yv[u], g, i + (int64_t)u * BT) >> p.fs], 1u);
    }
    __syncthreads();
    uint32_t *c = counts + (int64_t)sl * p.nbk;
    for (int b = threadIdx.x; b < p.nbk; b += BT) c[b] = h[b];
}

// counts[blk][b] -> exclusive prefix over blk (in place); totals[b].  One workgroup per
// 64 buckets: thread (c, l) holds slices 16c..16c+15 of bucket l, so every load and store
// is a coalesced 256-B row segment (a wave per bucket with lanes over slices read 4 B per
// 16 KB stride: 17 us at 1M points), and the 16 chunk sums are scanned through LDS.
__global__ __launch_bounds__(1024) void k_bs_colscan(BSPair P) {
    BS_PICK(P.split[1])
    (void)g;
    uint32_t *counts = J.counts, *totals = J.totals;
    __shared__ uint32_t s_c[16][64];
    const int l = threadIdx.x & 63, c = threadIdx.x >> 6;
    const int b = bid * 64 + l;
    const bool ok = b < p.nbk;
    constexpr int R = 16;  // slices per thread (nb1 <= 256)
    uint32_t v[R], tot = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int k = c * R + j;
        v[j] = (ok && k < p.nb1) ? counts[(int64_t)k * p.nbk + b] : 0u;
        tot += v[j];
    }
    s_c[c][l] = tot;
    __syncthreads();
    uint32_t run = 0;
    for (int q = 0; q < c; ++q) run += s_c[q][l];
    if (c == 15 && ok) totals[b] = run + tot;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int k = c * R + j;
        if (ok && k < p.nb1) counts[(int64_t)k * p.nbk + b] = run;
        run += v[j];
    }
}

__global__ __launch_bounds__(BT) void k_bs_scatter(BSPair P) {
    BS_PICK(P.split[2])
    if (bid >= p.nb1) return;  // (padding, as k_bs_count)
    const int sl = (int)xcd_block(bid, p.nb1);
    const double *x = J.x, *y = J.y, *z = J.z;
    const int64_t n = J.n;
    const uint32_t *colpref = J.counts, *totals = J.totals;
    uint32_t *base_out = J.base;
    TPt *rec = J.rec;
    __shared__ uint32_t fill[BMAXB];
    __shared__ uint32_t s_w[BT / 64];
    // bases: exclusive scan of the bucket totals (each workgroup redoes it: 16 KB)
    constexpr int PB = BMAXB / BT;
    uint32_t v[PB], tot = 0;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        const int b = threadIdx.x * PB + j;
        v[j] = b < p.nbk ? totals[b] : 0u;
        tot += v[j];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t xs = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(xs, o, 64);
        if (lane >= o) xs += t;
    }
    if (lane == 63) s_w[wave] = xs;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; ++w) off += s_w[w];
    uint32_t run = off + xs - tot;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        const int b = threadIdx.x * PB + j;
        if (b < p.nbk) {
            fill[b] = run + colpref[(int64_t)sl * p.nbk + b];
            if (sl == 0) base_out[b] = run;
        }
        run += v[j];
    }
    if (sl == 0 && threadIdx.x == 0) base_out[p.nbk] = (uint32_t)n;
    __syncthreads();
    const int64_t i0 = (int64_t)sl * p.per, i1 = min(n, i0 + p.per);
#ifndef FICP_BS_SU
#define FICP_BS_SU 8
#endif
    constexpr int U = FICP_BS_SU;  // points in flight per thread (the loop was load-latency bound)
    for (int64_t i = i0 + threadIdx.x; i < i1; i += (int64_t)U * BT) {
        double xv[U], yv[U], zv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = i + (int64_t)u * BT;
            const bool in = q < i1;
            xv[u] = in ? x[q] : 0.0;
            yv[u] = in ? y[q] : 0.0;
            zv[u] = (in && z) ? z[q] : 0.0;
        }
        uint32_t slot[U], kv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = i + (int64_t)u * BT < i1;
            kv[u] = in ? bs_key(xv[u], yv[u], g, i + (int64_t)u * BT) : 0u;
            slot[u] = in ? atomicAdd(&fill[kv[u] >> p.fs], 1u) : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = i + (int64_t)u * BT;
            if (q < i1) {
                // the record carries its key above the index: k_bs_bucket reads it instead of
                // recomputing it (mode 2 recomputed it twice per point with two dependent
                // loads each, the plot and its grid; C4 batch run 7.61 -> 7.44 ms)
                double4 r;
                r.x = xv[u];
                r.y = yv[u];
                r.z = zv[u];
                r.w = __longlong_as_double((long long)(((unsigned long long)kv[u] << 32) |
                                                       (unsigned long long)q));
                *reinterpret_cast<double4 *>(rec + slot[u]) = r;
            }
        }
    }
}

// rank of item e among the items of its fine bin [b0, b0 + nb) with a smaller index
__device__ __forceinline__ uint32_t bin_rank(const uint64_t *comp, uint32_t b0, uint32_t nb,
                                             uint64_t me) {
    uint32_t r = 0;
    for (uint32_t j = b0; j < b0 + nb; ++j) r += comp[j] < me ? 1u : 0u;
    return r;
}

// the key a record carries above its index (k_bs_scatter)
__device__ __forceinline__ uint32_t rec_key(const TPt &t) {
    return (uint32_t)((unsigned long long)t.idx >> 32);
}

__device__ __forceinline__ void bs_emit(const BSortOut &o, int64_t q, const TPt &t) {
    if (o.pts) {
        TPt u = t;
        u.idx = (long long)(uint32_t)t.idx;  // the index alone
        o.pts[q] = u;
    } else {
        o.wx[q] = t.x;
        o.wy[q] = t.y;
        if (o.wz) o.wz[q] = t.z;
        o.worig[q] = (uint32_t)t.idx;
    }
}

__global__ __launch_bounds__(B4T) void k_bs_bucket(BSPair P) {
    BS_PICK(P.split[3])
    (void)g;  // the keys travel in the records
    const TPt *rec = J.rec;
    const uint32_t *base = J.base;
    const BSortOut o = J.o;
    uint64_t *gcomp = J.gcomp;
    uint32_t *gpos = J.gpos;
    // dynamic LDS sized by the plan (bs_bucket_lds): ~23 KB at 1M points, so several
    // workgroups share a CU
    extern __shared__ __align__(32) unsigned char dyn[];
    const int nf = 1 << p.fs;
    TPt *lrec = (TPt *)dyn;                                     // [bcap]
    uint64_t *lcomp = (uint64_t *)(dyn + p.bcap * sizeof(TPt));  // [bcap] (fine << 32 | index)
    uint32_t *fc = (uint32_t *)(lcomp + p.bcap);                // [nf] counts, then bin starts
    uint32_t *ff = fc + nf;                                   // [nf] fill counters
    uint16_t *lsrc = (uint16_t *)(ff + nf);                     // [bcap] bin slot -> record
    __shared__ uint32_t s_w[B4T / 64];
    const int b = bid;
    const uint32_t lo = base[b], hi = base[b + 1], cnt = hi - lo;
    const uint32_t mask = (uint32_t)nf - 1u;
    for (int f = threadIdx.x; f < nf; f += B4T) {
        fc[f] = 0u;
        ff[f] = 0u;
    }
    __syncthreads();
    const bool small = cnt <= (uint32_t)p.bcap;
    for (uint32_t e = threadIdx.x; e < cnt; e += B4T) {
        const TPt t = rec[lo + e];
        if (small) lrec[e] = t;
        atomicAdd(&fc[rec_key(t) & mask], 1u);
    }
    __syncthreads();
    // exclusive scan of the fine counts (nf <= BMAXF; PF per thread)
    {
        const int PF = (nf + B4T - 1) / B4T;
        const int f0 = threadIdx.x * PF;
        uint32_t tot = 0;
        for (int j = 0; j < PF; ++j)
            if (f0 + j < nf) tot += fc[f0 + j];
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t xs = tot;
#pragma unroll
        for (int q = 1; q < 64; q <<= 1) {
            const uint32_t t = __shfl_up(xs, q, 64);
            if (lane >= q) xs += t;
        }
        if (lane == 63) s_w[wave] = xs;
        __syncthreads();
        uint32_t run = xs - tot;
        for (int w = 0; w < wave; ++w) run += s_w[w];
        for (int j = 0; j < PF; ++j)
            if (f0 + j < nf) {
                const uint32_t c = fc[f0 + j];
                fc[f0 + j] = run;
                run += c;
            }
    }
    __syncthreads();
    // cell_start of this bucket's keys (grid layout)
    if (o.cell_start) {
        const uint32_t k0 = (uint32_t)b << p.fs;
        for (int f = threadIdx.x; f < nf; f += B4T)
            if ((uint64_t)k0 + (uint64_t)f < (uint64_t)p.nkeys) o.cell_start[k0 + f] = lo + fc[f];
        if (b == p.nbk - 1 && threadIdx.x == 0) o.cell_start[p.nkeys] = hi;
    }
    if (small) {
        for (uint32_t e = threadIdx.x; e < cnt; e += B4T) {
            const TPt t = lrec[e];
            const uint32_t f = rec_key(t) & mask;
            const uint32_t s = fc[f] + atomicAdd(&ff[f], 1u);
            lcomp[s] = ((uint64_t)f << 32) | (uint64_t)(uint32_t)t.idx;
            lsrc[s] = (uint16_t)e;
        }
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < cnt; s += B4T) {
            const uint64_t me = lcomp[s];
            const uint32_t f = (uint32_t)(me >> 32);
            const uint32_t b0 = fc[f];
            const uint32_t r = b0 + bin_rank(lcomp, b0, ff[f], me);
            bs_emit(o, (int64_t)lo + r, lrec[lsrc[s]]);
        }
    } else {  // a bucket larger than the LDS tile: the same ordering through global scratch
        for (uint32_t e = threadIdx.x; e < cnt; e += B4T) {
            const TPt t = rec[lo + e];
            const uint32_t f = rec_key(t) & mask;
            const uint32_t s = fc[f] + atomicAdd(&ff[f], 1u);
            gcomp[lo + s] = ((uint64_t)f << 32) | (uint64_t)(uint32_t)t.idx;
            gpos[lo + s] = e;
        }
        __threadfence_block();
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < cnt; s += B4T) {
            const uint64_t me = gcomp[lo + s];
            const uint32_t f = (uint32_t)(me >> 32);
            const uint32_t b0 = fc[f];
            const uint32_t r = b0 + bin_rank(gcomp + lo, b0, ff[f], me);
            bs_emit(o, (int64_t)lo + r, rec[lo + gpos[lo + s]]);
        }
    }
}

}  // namespace

// coarse buckets of ~256 points on average (at most 2^14), slices of >= 4K points (at
// most 256, one per CU): the per-slice bucket counts are ~4 MB at 1M points
BSortPlan bsort_plan(int64_t n, int64_t nkeys) {
    BSortPlan p{};
    p.nkeys = nkeys;
    int kb = 0;
    while (kb < 40 && (((int64_t)1) << kb) < nkeys) ++kb;
    // -DFICP_BS_BPTS / -DFICP_BS_SLICE (and -DFICP_BS_SU, k_bs_scatter's points in flight
    // per thread): compile-time sizes for A/B builds (tools/build_variant.sh)
    // ~256 points per coarse bucket, slices of 4096 points (512-1024 and 8K-16K within 1 %)
#ifndef FICP_BS_BPTS
#define FICP_BS_BPTS 256
#endif
    constexpr int64_t bpts = FICP_BS_BPTS;
#ifndef FICP_BS_SLICE
#define FICP_BS_SLICE 4096
#endif
    constexpr int64_t slice = FICP_BS_SLICE;
    int want = 0;
    while (want < BMAXB_LOG && (bpts << want) < n) ++want;
    p.fs = std::max(0, kb - want);
    p.nbk = (int)std::max<int64_t>(1, (nkeys + (((int64_t)1) << p.fs) - 1) >> p.fs);
    p.nb1 = (int)std::min<int64_t>(256, std::max<int64_t>(1, (n + slice - 1) / slice));
    // LDS tile: twice the mean bucket (at 10M points the 16384 buckets hold ~610 points:
    // a 512 tile sent most of them through the global-scratch path, 467 us per C4 grid
    // build), within 64 KB of LDS so two workgroups still share a CU
    {
        const int64_t mean = (n + p.nbk - 1) / p.nbk;
        int64_t cap = std::max<int64_t>(2 * bpts, ((2 * mean + 255) / 256) * 256);
        const int64_t fit = (65536 - (int64_t)2 * 4 * (((int64_t)1) << p.fs)) / (int64_t)(sizeof(TPt) + 8 + 2);
        cap = std::min<int64_t>(cap, std::max<int64_t>(2 * bpts, (fit / 256) * 256));
        p.bcap = (int)std::min<int64_t>(4096, cap);
    }
    p.per = (n + p.nb1 - 1) / p.nb1;
    return p;
}

bool bsort_supported(int64_t n, int64_t nkeys) {
    const BSortPlan p = bsort_plan(n, nkeys);
    return p.fs <= BMAXF_LOG && p.nbk <= BMAXB && nkeys < (((int64_t)1) << 32) && n < (1LL << 31);
}

int64_t bsort_tmp_bytes(int64_t n, int64_t nkeys) {
    const BSortPlan p = bsort_plan(n, nkeys);
    const int64_t nn = std::max<int64_t>(n, 1);
    return 256 + (int64_t)p.nb1 * p.nbk * 4 + 2 * (int64_t)(p.nbk + 1) * 4 + 3 * 256 +
           nn * (int64_t)sizeof(TPt) + nn * 8 + nn * 4 + 256;
}

// a job's scratch carved from tmp (bsort_tmp_bytes(n, nkeys) bytes)
BSJob bsort_job(const double *x, const double *y, const double *z, int64_t n, const BSortGeom &g,
                int64_t nkeys, const BSortOut &o, void *tmp) {
    BSJob j{};
    j.x = x;
    j.y = y;
    j.z = z;
    j.n = n;
    j.g = g;
    j.p = bsort_plan(n, nkeys);
    j.o = o;
    auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
    char *q = (char *)tmp;
    q += 256;
    j.counts = (uint32_t *)q;
    q += al((int64_t)j.p.nb1 * j.p.nbk * 4);
    j.totals = (uint32_t *)q;
    q += al((int64_t)(j.p.nbk + 1) * 4);
    j.base = (uint32_t *)q;
    q += al((int64_t)(j.p.nbk + 1) * 4);
    j.rec = (TPt *)q;
    q += al(n * (int64_t)sizeof(TPt));
    j.gcomp = (uint64_t *)q;
    q += al(n * 8);
    j.gpos = (uint32_t *)q;
    return j;
}

// one or two jobs (b.n == 0: a alone), four launches for both
hipError_t launch_bsort2(const BSJob &a, const BSJob &b, hipStream_t s) {
    BSPair P{a, b, {0, 0, 0, 0}};
    const bool two = b.n > 0;
    auto blocks = [](const BSJob &j, int k) -> int {
        if (j.n <= 0) return 0;
        if (k == 0 || k == 2) return j.p.nb1;
        if (k == 1) return (j.p.nbk + 63) / 64;
        return j.p.nbk;
    };
    int tot[4];
    for (int k = 0; k < 4; ++k) {
        P.split[k] = blocks(a, k);
        // the slice kernels: job b's workgroups start at a multiple of 8 (XCD-aware slices)
        if (two && (k == 0 || k == 2)) P.split[k] = (P.split[k] + 7) & ~7;
        tot[k] = P.split[k] + (two ? blocks(b, k) : 0);
    }
    auto lds_of = [](const BSJob &j) {
        return (size_t)j.p.bcap * (sizeof(TPt) + 8 + 2) + (size_t)2 * 4 * (1 << j.p.fs);
    };
    const size_t lds = std::max(lds_of(a), two ? lds_of(b) : (size_t)0);
    hipLaunchKernelGGL(k_bs_count, dim3(tot[0]), dim3(BT), 0, s, P);
    hipLaunchKernelGGL(k_bs_colscan, dim3(tot[1]), dim3(1024), 0, s, P);
    hipLaunchKernelGGL(k_bs_scatter, dim3(tot[2]), dim3(BT), 0, s, P);
    hipLaunchKernelGGL(k_bs_bucket, dim3(tot[3]), dim3(B4T), lds, s, P);
    return hipGetLastError();
}

hipError_t launch_bsort(const double *x, const double *y, const double *z, int64_t n,
                        const BSortGeom &g, int64_t nkeys, const BSortOut &o, void *tmp,
                        hipStream_t s) {
    if (n <= 0) {
        if (o.cell_start && nkeys >= 0)
            return hipMemsetAsync(o.cell_start, 0, (size_t)(nkeys + 1) * 4, s);
        return hipSuccess;
    }
    if (!bsort_supported(n, nkeys)) return hipErrorInvalidValue;
    return launch_bsort2(bsort_job(x, y, z, n, g, nkeys, o, tmp), BSJob{}, s);
}

}  // namespace ficp
