// k_grid_nn.hip -- exact 1-NN correspondence search of the tree layer against the
// static CHM layer (replaces cKDTree(target).query(source, k=1), ficp.py:65-71).
//
// Parity rule (probe-verified against cKDTree): squared distance
// d2 = ((0 + dx*dx) + dy*dy) + dz*dz in fp64 with NO FMA contraction (this TU is built
// with -ffp-contract=off; `0 + x` is the identity for x >= 0), argmin over d2, exact ties
// to the lowest target index, dist = sqrt(d2).
//
// Two exact searches:
//  * k_nn_grid  -- the CHM layer is binned once into a uniform XY grid (cell-sorted AoS,
//    32 B per stem); a query scans square rings of cells around its own cell until a
//    conservative lower bound on the distance to everything outside the scanned block
//    exceeds the best d2.  Queries run in a spatial work order (8x8-cell supertiles) so
//    the 64 lanes of a wave scan overlapping cells: their candidate loads coalesce and
//    hit L1/L2 instead of 64 scattered cache lines.
//  * k_nn_brute -- LDS-tiled all-pairs scan (target tiles of 256 stems staged in LDS and
//    read as broadcasts, QPT queries per lane held in registers), fp64-VALU bound; used
//    for small layers and as an independent cross-check of the grid kernel.
// Both fuse the pending rigid transform of the previous fit (ficp.py:135) into the
// source load, and write idx, dist, d2, the sort key, and the matched stem's XY.
#include "ficp_internal.h"

#include <hip/hip_ext.h>

#include <math.h>
#include <stdlib.h>

#include <algorithm>

namespace ficp {

namespace {

__device__ __forceinline__ int cell_coord(double v, double v0, double inv_h, int g) {
    double f = (v - v0) * inv_h;
    if (!(f >= 0.0)) return 0;           // also catches NaN
    if (f >= (double)(g - 1)) return g - 1;
    return (int)f;
}


// The cell-sorted stems are read through a buffer descriptor: 32-bit per-lane byte
// offsets, no 64-bit address arithmetic per candidate (cdna_hip_programming.md T8).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

// z and index of a record: 12 B (dwordx3).  A dwordx4 load of them left its unused 4th
// dword free for the register allocator, which placed the next candidate's address there
// and so made every candidate wait for the previous one's loads (s_waitcnt vmcnt(0)).
__device__ __forceinline__ u32x3 load_zid(__amdgpu_buffer_rsrc_t r, int p) {
    return __builtin_amdgcn_raw_buffer_load_b96(r, p * 32 + 16, 0, 0);
}
__device__ __forceinline__ double zid_z(const u32x3 &v) {
    return __longlong_as_double((long long)(((unsigned long long)v.y << 32) | v.x));
}

#ifndef FICP_NN_UNROLL
#define FICP_NN_UNROLL 2  // candidate loads in flight per lane (2: best of 1, 2, 4, 8 at C3)
#endif

struct Stems {
    __amdgpu_buffer_rsrc_t r;
};

// FICP_NN_STATS (diagnostic builds only): per-launch counts of candidate evaluations,
// certified / scanned queries, printed by a one-thread kernel after each NN launch
#ifdef FICP_NN_STATS
__device__ unsigned long long g_nnst[8];
#define NNST(i)                                                                      \
    do {                                                                             \
        const unsigned long long m_ = __ballot(1);                                   \
        if ((threadIdx.x & 63) == (unsigned)__builtin_ctzll(m_))                    \
            atomicAdd(&g_nnst[i], (unsigned long long)__popcll(m_));                 \
    } while (0)
#else
#define NNST(i) \
    do {        \
    } while (0)
#endif

__device__ __forceinline__ Stems stems_of(const TPt *pts, int64_t m) {
    Stems st;
    st.r = __builtin_amdgcn_make_buffer_rsrc((void *)pts, 0, (int)(m * (int64_t)sizeof(TPt)),
                                             0x00020000);
    return st;
}

// best candidate so far: d2, stem index (tie-break), grid slot.  The kernel is VALU-bound
// (~70 % busy at C3), so the loop carries only what the comparison needs; the matched
// record is reloaded once at the end.
struct Best {
    double d2;
    int id, slot;
};

template <int MD>
__device__ __forceinline__ void eval_slot(const Stems &S, int p, double qx, double qy, double qz,
                                          Best &b) {
    NNST(1);
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(S.r, p * 32, 0, 0);
    const u32x3 hi = load_zid(S.r, p);
    const double2 xy = __builtin_bit_cast(double2, lo);
    const double pz = zid_z(hi);
    const int id = (int)hi.z;
    // sq_dist's operations in its order, with dz^2 kept
    const double dx = qx - xy.x, dy = qy - xy.y;
    double s = dx * dx;
    s = s + dy * dy;
    double dzz = 0.0;
    if (MD == 3) {
        const double dz = qz - pz;
        dzz = dz * dz;
        s = s + dzz;
    }
    // strict < keeps the best; an equal distance goes to the lower stem index
    const bool take = (s < b.d2) | ((s == b.d2) & (id < b.id));
    b.d2 = take ? s : b.d2;
    b.id = take ? id : b.id;
    b.slot = take ? p : b.slot;
}

// stems [p0, p1) of the cell-sorted layer, several loads in flight per step (a step past
// the end re-reads the last stem: evaluating a candidate twice changes nothing)
template <int MD>
__device__ __forceinline__ void scan_pts(const Stems &S, int p0, int p1, double qx, double qy,
                                         double qz, Best &b) {
    for (int p = p0; p < p1; p += FICP_NN_UNROLL) {
#pragma unroll
        for (int u = 0; u < FICP_NN_UNROLL; ++u)
            eval_slot<MD>(S, min(p + u, p1 - 1), qx, qy, qz, b);
    }
}

// gap between q and the band [v0 + c0 h, v0 + c1 h) along one axis, less the margin
__device__ __forceinline__ double band_gap(double q, double v0, double h, int c0, int c1,
                                           double mq) {
    const double lo = v0 + (double)c0 * h, hi = v0 + (double)c1 * h;
    return fmax(fmax(lo - q, q - hi), 0.0) - mq;
}

__device__ __forceinline__ bool beyond(double gap, double d2) { return gap > 0.0 && gap * gap > d2; }

__device__ __forceinline__ double query_margin(const GridView &g, double qx, double qy) {
    return g.margin + 1e-15 * (fabs(qx) + fabs(qy));
}

// Disk-clipped row scan: every stem within sqrt(best) of q (in XY, a lower bound of the
// md-dimensional distance) lies in a row band whose y-gap is <= sqrt(best) and, inside
// that row, within +-sqrt(best - gap^2) of qx.  Rows are visited outward from q's own
// row and each row scans only the cells under that chord, so the work follows the
// shrinking disk of the best match.  Requires a finite best on entry.
template <int MD>
__device__ __forceinline__ void disk_scan(const GridView &g, const Stems &S, double qx, double qy,
                                          double qz, int cy, double mq, Best &b) {
    for (int k = 0;; ++k) {
        bool any = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (k == 0 && side == 1) continue;
            const int yy = side ? cy + k : cy - k;
            if (yy < 0 || yy >= g.gy) continue;
            const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
            if (beyond(gy, b.d2)) continue;
            any = true;
            const double gy0 = fmax(gy, 0.0);
            const double w = sqrt(fmax(b.d2 - gy0 * gy0, 0.0)) + mq;
            const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
            const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
            const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
            scan_pts<MD>(S, row[xl], row[xh + 1], qx, qy, qz, b);
        }
        if (!any) break;  // both rows at this offset are beyond the disk: so are all farther
    }
}

// The same disk scan with its first three rows (cy - 1, cy, cy + 1) batched: their
// chords come from the entry bound (a superset of what the shrinking disk needs, so the
// scan stays exact), all six cell_start loads issue together and then all their stems,
// FICP_NN_UNROLL loads in flight.  The row-by-row walk made every row's loads wait for
// the previous row's stems (about 8 dependent memory latencies per query at C3; batched:
// 4).  Rows at offset >= 2 follow row by row, as before.
// sa <= sb: the columns [sa, sb] of these three rows were evaluated already (the cold
// start's 3x3 block): each row's chord is split around them, so no stem is evaluated twice
template <int MD>
__device__ __forceinline__ void disk_scan_batched(const GridView &g, const Stems &S, double qx,
                                                  double qy, double qz, int cy, double mq,
                                                  Best &b, int sa = 1, int sb = 0) {
    int p0[6], len[6];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        p0[2 * r] = p0[2 * r + 1] = 0;
        len[2 * r] = len[2 * r + 1] = 0;
        const int yy = cy + r - 1;
        if (yy < 0 || yy >= g.gy) continue;
        const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
        if (beyond(gy, b.d2)) continue;
        const double gy0 = fmax(gy, 0.0);
        const double w = sqrt(fmax(b.d2 - gy0 * gy0, 0.0)) + mq;
        const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
        const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
        const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
        // [xl, xh] minus [sa, sb]: [xl, min(xh, sa - 1)] and [max(xl, sb + 1), xh]
        const int a1 = sa <= sb ? min(xh, sa - 1) : xh;
        const int a2 = sa <= sb ? max(xl, sb + 1) : xh + 1;
        if (a1 >= xl) {
            p0[2 * r] = row[xl];
            len[2 * r] = row[a1 + 1] - p0[2 * r];
        }
        if (a2 <= xh) {
            p0[2 * r + 1] = row[a2];
            len[2 * r + 1] = row[xh + 1] - p0[2 * r + 1];
        }
    }
    int tot = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) tot += len[r];
    for (int t = 0; t < tot; t += FICP_NN_UNROLL) {
#pragma unroll
        for (int u = 0; u < FICP_NN_UNROLL; ++u) {
            int q = min(t + u, tot - 1), slot = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r) {  // the segment holding position q
                if (q >= 0 && q < len[r]) slot = p0[r] + q;
                q -= len[r];
            }
            eval_slot<MD>(S, slot, qx, qy, qz, b);
        }
    }
    for (int k = 2;; ++k) {
        bool any = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const int yy = side ? cy + k : cy - k;
            if (yy < 0 || yy >= g.gy) continue;
            const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
            if (beyond(gy, b.d2)) continue;
            any = true;
            const double gy0 = fmax(gy, 0.0);
            const double w = sqrt(fmax(b.d2 - gy0 * gy0, 0.0)) + mq;
            const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
            const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
            const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
            scan_pts<MD>(S, row[xl], row[xh + 1], qx, qy, qz, b);
        }
        if (!any) break;
    }
}

#ifndef FICP_NN_BATCHED
#define FICP_NN_BATCHED 1
#endif

// Exact 1-NN: a finite first bound from q's own cell (or the warm-start stem, or the
// first non-empty ring), then the disk-clipped rows.
template <int MD>
__device__ __forceinline__ void grid_nn(const GridView &g, const Stems &S, double qx, double qy,
                                        double qz, Best &b) {
    const int cx = cell_coord(qx, g.x0, g.inv_h, g.gx);
    const int cy = cell_coord(qy, g.y0, g.inv_h, g.gy);
    const double mq = query_margin(g, qx, qy);
    int sa = 1, sb = 0;  // columns of rows cy-1..cy+1 evaluated by the cold start
    if (!(b.d2 < INFINITY)) {
        // cold start (no previous match): the 3x3 cells around q as one batch -- a bound
        // near the true distance (the own cell's stem alone was often 5-13 m away in 3-D,
        // which widened every chord of the disk scan)
        int p0[3], len[3];
        const int xa = max(cx - 1, 0), xb = min(cx + 1, g.gx - 1);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            p0[r] = 0;
            len[r] = 0;
            const int yy = cy + r - 1;
            if (yy < 0 || yy >= g.gy) continue;
            const int32_t *rw = g.cell_start + (int64_t)yy * g.gx;
            p0[r] = rw[xa];
            len[r] = rw[xb + 1] - p0[r];
        }
        const int l01 = len[0] + len[1], tot = l01 + len[2];
        for (int t = 0; t < tot; t += FICP_NN_UNROLL) {
#pragma unroll
            for (int u = 0; u < FICP_NN_UNROLL; ++u) {
                const int q = min(t + u, tot - 1);
                const int slot = q < len[0] ? p0[0] + q : (q < l01 ? p0[1] + (q - len[0]) : p0[2] + (q - l01));
                eval_slot<MD>(S, slot, qx, qy, qz, b);
            }
        }
        sa = xa;
        sb = xb;
        for (int r = 2; !(b.d2 < INFINITY); ++r) {  // empty 3x3 block: grow square rings
            const int xa = cx - r, xb = cx + r, ya = cy - r, yb = cy + r;
            if (xa < 0 && ya < 0 && xb >= g.gx && yb >= g.gy) break;  // empty layer
            const int xlo = max(xa, 0), xhi = min(xb, g.gx - 1);
            for (int yy = max(ya, 0); yy <= min(yb, g.gy - 1); ++yy) {
                const int32_t *rw = g.cell_start + (int64_t)yy * g.gx;
                if (yy == ya || yy == yb) {
                    scan_pts<MD>(S, rw[xlo], rw[xhi + 1], qx, qy, qz, b);
                } else {
                    if (xa >= 0) scan_pts<MD>(S, rw[xa], rw[xa + 1], qx, qy, qz, b);
                    if (xb < g.gx) scan_pts<MD>(S, rw[xb], rw[xb + 1], qx, qy, qz, b);
                }
            }
        }
        if (!(b.d2 < INFINITY)) return;
    }
    if (FICP_NN_BATCHED) disk_scan_batched<MD>(g, S, qx, qy, qz, cy, mq, b, sa, sb);
    else disk_scan<MD>(g, S, qx, qy, qz, cy, mq, b);
}

// ---------------------------------------------------------------- k nearest (remove_matches)
// CHMPlot.remove_matches (chm_plot.py:223-285) matches with scipy's cdist + argmin: the
// ORDER is by the rounded distance d = sqrt(d2) and then by stem index (np.argmin keeps
// the first of equal distances).  The K best (d, index) of a query, skipping stems
// flagged in `removed` (indexed by stem index; nullable).
constexpr int KNN = KNN_K;

template <int MD>
__device__ __forceinline__ void knn_eval(const Stems &S, int p, double qx, double qy, double qz,
                                         const uint8_t *removed, double (&kd)[KNN],
                                         int (&kid)[KNN]) {
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(S.r, p * 32, 0, 0);
    const u32x3 hi = load_zid(S.r, p);
    const int id = (int)hi.z;
    if (removed && removed[id]) return;
    const double2 xy = __builtin_bit_cast(double2, lo);
    const double dd = sqrt(sq_dist<MD>(qx, qy, qz, xy.x, xy.y, zid_z(hi)));
    if (!(dd < kd[KNN - 1] || (dd == kd[KNN - 1] && id < kid[KNN - 1]))) return;
    kd[KNN - 1] = dd;
    kid[KNN - 1] = id;
#pragma unroll
    for (int u = KNN - 1; u > 0; --u) {  // bubble the new entry to its place (stable)
        const bool sw = kd[u] < kd[u - 1] || (kd[u] == kd[u - 1] && kid[u] < kid[u - 1]);
        const double td = sw ? kd[u - 1] : kd[u];
        const int ti = sw ? kid[u - 1] : kid[u];
        kd[u - 1] = sw ? kd[u] : kd[u - 1];
        kid[u - 1] = sw ? kid[u] : kid[u - 1];
        kd[u] = td;
        kid[u] = ti;
    }
}

template <int MD>
__device__ __forceinline__ void knn_range(const Stems &S, int p0, int p1, double qx, double qy,
                                          double qz, const uint8_t *removed, double (&kd)[KNN],
                                          int (&kid)[KNN]) {
    for (int p = p0; p < p1; ++p) knn_eval<MD>(S, p, qx, qy, qz, removed, kd, kid);
}

template <int MD>
__global__ __launch_bounds__(256) void k_knn_grid(const double *sx, const double *sy,
                                                  const double *sz, int64_t q0, int64_t n,
                                                  GridView g, const uint8_t *removed,
                                                  int32_t *out_id, double *out_d) {
    const int64_t i = q0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Stems S = stems_of(g.pts, g.m);
    const double qx = sx[i], qy = sy[i], qz = (MD == 3) ? sz[i] : 0.0;
    double kd[KNN];
    int kid[KNN];
#pragma unroll
    for (int u = 0; u < KNN; ++u) {
        kd[u] = INFINITY;
        kid[u] = 0x7fffffff;
    }
    const int cx = cell_coord(qx, g.x0, g.inv_h, g.gx);
    const int cy = cell_coord(qy, g.y0, g.inv_h, g.gy);
    const double mq = query_margin(g, qx, qy);
    // square rings until K stems are held (or the grid is exhausted): a finite radius
    for (int r = 0; kid[KNN - 1] == 0x7fffffff; ++r) {
        const int xa = cx - r, xb = cx + r, ya = cy - r, yb = cy + r;
        if (r > 0 && xa < 0 && ya < 0 && xb >= g.gx && yb >= g.gy) break;
        const int xlo = max(xa, 0), xhi = min(xb, g.gx - 1);
        for (int yy = max(ya, 0); yy <= min(yb, g.gy - 1); ++yy) {
            const int32_t *rw = g.cell_start + (int64_t)yy * g.gx;
            if (yy == ya || yy == yb) {
                knn_range<MD>(S, rw[xlo], rw[xhi + 1], qx, qy, qz, removed, kd, kid);
            } else {
                if (xa >= 0) knn_range<MD>(S, rw[xa], rw[xa + 1], qx, qy, qz, removed, kd, kid);
                if (xb < g.gx) knn_range<MD>(S, rw[xb], rw[xb + 1], qx, qy, qz, removed, kd, kid);
            }
        }
    }
    if (kid[KNN - 1] != 0x7fffffff) {
        // disk-clipped rows within the K-th distance (inflated: a d2 a few ulps below
        // kd^2 can still round to the same d and win on its index)
        for (int k = 0;; ++k) {
            bool any = false;
            for (int side = 0; side < 2; ++side) {
                if (k == 0 && side == 1) continue;
                const int yy = side ? cy + k : cy - k;
                if (yy < 0 || yy >= g.gy) continue;
                const double b2 = kd[KNN - 1] * kd[KNN - 1] * (1.0 + 1e-12);
                const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
                if (beyond(gy, b2)) continue;
                any = true;
                const double gy0 = fmax(gy, 0.0);
                const double w = sqrt(fmax(b2 - gy0 * gy0, 0.0)) + mq;
                const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
                const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
                const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
                knn_range<MD>(S, row[xl], row[xh + 1], qx, qy, qz, removed, kd, kid);
            }
            if (!any) break;
        }
    }
#pragma unroll
    for (int u = 0; u < KNN; ++u) {
        out_id[i * KNN + u] = kid[u];
        out_d[i * KNN + u] = kd[u];
    }
}

__device__ __forceinline__ void apply_T(const double *__restrict__ T, double &x, double &y) {
    // numpy's ([x, y, 1] @ T.T)[:, :2] through OpenBLAS dgemm (ficp.py:117):
    // fma(y, T01, x*T00) + T02 -- pinned bit-exactly by tests/golden/apply.npz
    const double nx = __fma_rn(y, T[1], x * T[0]) + T[2];
    const double ny = __fma_rn(y, T[4], x * T[3]) + T[5];
    x = nx;
    y = ny;
}

// per-point outputs; returns the sort key
__device__ __forceinline__ unsigned long long write_out(const NNArgs &a, int64_t i, double best,
                                                        int bi) {
    if (a.idx) a.idx[i] = bi;
    const double d = sqrt(best);
    const unsigned long long k = ordkey(d);
    if (a.dist) a.dist[i] = d;
    if (a.r) a.r[i] = best;
    if (a.key) a.key[i] = k;
    if (a.val) a.val[i] = (uint32_t)i;
    return k;
}

// Per-query finish: matched slot, correspondence XY, idx/dist/r/key; folds the key into
// this thread's range accumulator.
// A warm scan that ends on the stem it matched before leaves (cx, cy, dz2, bp) as they are
// -- they describe that stem already -- and writes only r / key / idx: 28 B per query less
// written and no record reload, for one more load (the previous slot) before the scan.  The
// batch kernels take it (C4 1024 plots: +2 %, 1.222M vs 1.200M plot-it/s); the single-plot
// ones do not (C3 cover scans: -1.2 %, 8,470 vs 8,575 it/s).  FICP_NN_SKIP_SAME=0: never.
#ifndef FICP_NN_SKIP_SAME
#define FICP_NN_SKIP_SAME 1
#endif
#ifndef FICP_NN_SKIP_SINGLE  // (the single-plot kernels: A/B, tools/build_variant.sh)
#define FICP_NN_SKIP_SINGLE 0
#endif
__device__ __forceinline__ void finish_same(const NNArgs &a, int64_t i, const Best &b,
                                            unsigned long long &kmin_c, unsigned long long &kmax);

__device__ __forceinline__ void finish(const NNArgs &a, const Stems &S, int64_t i, double qz,
                                       const Best &b,
                                       unsigned long long &kmin_c, unsigned long long &kmax) {
    if (a.out_bp) a.out_bp[i] = b.slot;
    if (a.cx || a.dz2) {  // the matched record (L1-hot); slot 0 for an unmatched query
        const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(S.r, b.slot * 32, 0, 0);
        const double2 c = __builtin_bit_cast(double2, lo);
        if (a.cx) {
            a.cx[i] = c.x;
            a.cy[i] = c.y;
        }
        if (a.dz2) {  // the next call's warm start: z never moves, d2 = dx^2 + dy^2 + dz2
            const double dz = qz - zid_z(load_zid(S.r, b.slot));
            a.dz2[i] = dz * dz;
        }
    }
    const unsigned long long k = write_out(a, i, b.d2, b.id);
    kmin_c = max(kmin_c, ~k);
    kmax = max(kmax, k);
}

__device__ __forceinline__ void finish_same(const NNArgs &a, int64_t i, const Best &b,
                                            unsigned long long &kmin_c, unsigned long long &kmax) {
    const unsigned long long k = write_out(a, i, b.d2, b.id);
    kmin_c = max(kmin_c, ~k);
    kmax = max(kmax, k);
}

// ------------------------------------------------------- certified reuse of the match
// Between ICP iterations a query moves by a small rigid step and its nearest stem rarely
// changes.  A full scan here covers every stem within sqrt(cover2) of q, cover2 =
// (d_match + pad)^2, and records G = a lower bound on the distance from q to every stem
// other than the match: min(runner-up distance among the scanned stems, sqrt(cover2)
// less the margins).  At the next call the query has moved by delta (XY only; z never
// moves), so every other stem is at >= G - delta (triangle inequality) while the match
// is at the recomputed d_new (the exact eval_slot operations on its stored XY and dz^2).
// d_new + eps < G - delta - eps proves the match is still the unique nearest stem: the
// result is the scan's, bit for bit, with no candidate read.  G then carries over as
// G - delta - eps until a step fails the test and the query scans again.
struct Best2 {
    double d2;
    int id, slot;  // slot -1: the bound is not (yet) a scanned stem
    double s2;     // smallest d2 among scanned stems other than the best
};

template <int MD>
__device__ __forceinline__ void eval2(const Stems &S, int p, double qx, double qy, double qz,
                                      Best2 &b) {
    NNST(0);
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(S.r, p * 32, 0, 0);
    const u32x3 hi = load_zid(S.r, p);
    const double2 xy = __builtin_bit_cast(double2, lo);
    const int id = (int)hi.z;
    const double dx = qx - xy.x, dy = qy - xy.y;
    double s = dx * dx;
    s = s + dy * dy;
    if (MD == 3) {
        const double dz = qz - zid_z(hi);
        s = s + dz * dz;
    }
    const bool take = (s < b.d2) | ((s == b.d2) & (id < b.id));
    // the runner-up: a displaced best that was a scanned stem, or this stem unless it is
    // the best itself (evaluated twice)
    const double other = take ? (b.slot >= 0 ? b.d2 : INFINITY) : (p == b.slot ? INFINITY : s);
    b.s2 = fmin(b.s2, other);
    b.d2 = take ? s : b.d2;
    b.id = take ? id : b.id;
    b.slot = take ? p : b.slot;
}

template <int MD>
__device__ __forceinline__ void scan2(const Stems &S, int p0, int p1, double qx, double qy,
                                      double qz, Best2 &b) {
    for (int p = p0; p < p1; p += FICP_NN_UNROLL) {
#pragma unroll
        for (int u = 0; u < FICP_NN_UNROLL; ++u) eval2<MD>(S, min(p + u, p1 - 1), qx, qy, qz, b);
    }
}

// every stem within sqrt(cover2) of q (XY) evaluated: rows cy-1..cy+1 batched, then the
// rows beyond while their band is within sqrt(cover2); chords from cover2
template <int MD>
__device__ __forceinline__ void cover_scan(const GridView &g, const Stems &S, double qx, double qy,
                                           double qz, int cy, double mq, double cover2, Best2 &b) {
    int p0[3], len[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        p0[r] = 0;
        len[r] = 0;
        const int yy = cy + r - 1;
        if (yy < 0 || yy >= g.gy) continue;
        const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
        if (beyond(gy, cover2)) continue;
        const double gy0 = fmax(gy, 0.0);
        const double w = sqrt(fmax(cover2 - gy0 * gy0, 0.0)) + mq;
        const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
        const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
        const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
        p0[r] = row[xl];
        len[r] = row[xh + 1] - p0[r];
    }
    const int l01 = len[0] + len[1], tot = l01 + len[2];
    for (int t = 0; t < tot; t += FICP_NN_UNROLL) {
#pragma unroll
        for (int u = 0; u < FICP_NN_UNROLL; ++u) {
            const int q = min(t + u, tot - 1);
            const int slot = q < len[0] ? p0[0] + q : (q < l01 ? p0[1] + (q - len[0]) : p0[2] + (q - l01));
            eval2<MD>(S, slot, qx, qy, qz, b);
        }
    }
    for (int k = 2;; ++k) {
        bool any = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const int yy = side ? cy + k : cy - k;
            if (yy < 0 || yy >= g.gy) continue;
            const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
            if (beyond(gy, cover2)) continue;
            any = true;
            const double gy0 = fmax(gy, 0.0);
            const double w = sqrt(fmax(cover2 - gy0 * gy0, 0.0)) + mq;
            const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
            const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
            const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
            scan2<MD>(S, row[xl], row[xh + 1], qx, qy, qz, b);
        }
        if (!any) break;
    }
}

#ifndef FICP_CERT_PAD
#define FICP_CERT_PAD 0.25  // scans cover d_match + 0.25 cell sizes (0.1-0.4 within 1 % at C3)
#endif

// rounding allowance of the certificate's distances (coordinates up to ~1e7 m: ulp ~2e-9 m)
// G stored rounded down: a lower bound stays a lower bound (a few 1e-7 m at G ~ 5 m)
__device__ __forceinline__ gap_t gap_rd(double g) { return __double2float_rd(g); }

__device__ __forceinline__ double cert_eps(const GridView &g, double qx, double qy) {
    return 2.0 * g.margin + 1e-12 * (fabs(qx) + fabs(qy)) + 1e-9;
}

#ifndef FICP_CERT_DMUL
#define FICP_CERT_DMUL 4.0
#endif
#ifndef FICP_CERT_PADMIN
#define FICP_CERT_PADMIN 0.02
#endif
// how far beyond the match a full scan reaches: pad h, or DMUL times this call's move
// when that is smaller (but at least PADMIN h).  The next certificate needs the cover to
// exceed about twice the next move, and ICP moves shrink call by call: a cover sized
// from the move is enough and cheaper in the later calls (C3: +1 % for DMUL 2-8)
__device__ __forceinline__ double cert_pad(const GridView &g, double mv) {
    const double p = FICP_CERT_PAD * g.h;
    if (!(FICP_CERT_DMUL > 0.0)) return p;
    return fmin(p, fmax(FICP_CERT_DMUL * mv, FICP_CERT_PADMIN * g.h));
}

// the stored match's exact d2 at the (moved) query: eval_slot's operations on (cx, cy, dz2)
template <int MD>
__device__ __forceinline__ double warm_d2(const NNArgs &a, int64_t i, double qx, double qy) {
    const double dx = qx - a.cx[i], dy = qy - a.cy[i];
    double d2 = dx * dx;
    d2 = d2 + dy * dy;
    if (MD == 3) d2 = d2 + a.dz2[i];
    return d2;
}

// Step 1 (warm calls): apply T, then try the certificate.  Returns true when the stored
// match stands (outputs written, no scan); false leaves the moved query for cert_scan.
template <int MD>
__device__ __forceinline__ bool cert_try(const NNArgs &a, const GridView &g, const Stems &S,
                                         int64_t i, const double *T, unsigned long long &kmin_c,
                                         unsigned long long &kmax, double &mv, double &qx,
                                         double &qy) {
    const double ox = a.sx[i], oy = a.sy[i];
    qx = ox;
    qy = oy;
    if (T) {
        apply_T(T, qx, qy);
        a.sx[i] = qx;
        a.sy[i] = qy;
    }
    const double eps = cert_eps(g, qx, qy);
    const double d2w = warm_d2<MD>(a, i, qx, qy);
    const double mx = qx - ox, my = qy - oy;
    mv = sqrt(mx * mx + my * my);
    const double G = (a.gap_cold ? 0.0 : (double)a.gap[i]) - mv - eps;
    if (!(d2w < INFINITY && sqrt(d2w) + eps < G)) return false;
    NNST(2);
    a.gap[i] = gap_rd(G);
    if (a.idx) a.idx[i] = (int)load_zid(S.r, a.out_bp[i]).z;
    const double d = sqrt(d2w);
    const unsigned long long k = ordkey(d);
    if (a.dist) a.dist[i] = d;
    if (a.r) a.r[i] = d2w;
    if (a.key) a.key[i] = k;
    if (a.val) a.val[i] = (uint32_t)i;
    kmin_c = max(kmin_c, ~k);
    kmax = max(kmax, k);
    return true;
}

// cold start of a scan: the 3x3 cells around q, then rings until a stem is found
template <int MD>
__device__ __forceinline__ void cold_start(const GridView &g, const Stems &S, double qx, double qy,
                                           double qz, int cx, int cy, Best2 &b) {
    for (int yy = max(cy - 1, 0); yy <= min(cy + 1, g.gy - 1); ++yy) {
        const int32_t *rw = g.cell_start + (int64_t)yy * g.gx;
        scan2<MD>(S, rw[max(cx - 1, 0)], rw[min(cx + 1, g.gx - 1) + 1], qx, qy, qz, b);
    }
    for (int r = 2; !(b.d2 < INFINITY); ++r) {
        const int xa = cx - r, xb = cx + r, ya = cy - r, yb = cy + r;
        if (xa < 0 && ya < 0 && xb >= g.gx && yb >= g.gy) break;  // empty layer
        const int xlo = max(xa, 0), xhi = min(xb, g.gx - 1);
        for (int yy = max(ya, 0); yy <= min(yb, g.gy - 1); ++yy) {
            const int32_t *rw = g.cell_start + (int64_t)yy * g.gx;
            if (yy == ya || yy == yb) {
                scan2<MD>(S, rw[xlo], rw[xhi + 1], qx, qy, qz, b);
            } else {
                if (xa >= 0) scan2<MD>(S, rw[xa], rw[xa + 1], qx, qy, qz, b);
                if (xb < g.gx) scan2<MD>(S, rw[xb], rw[xb + 1], qx, qy, qz, b);
            }
        }
    }
}

// Step 2: the full scan of an uncertified query at its (already moved) position: warm
// bound from the stored match (or the cold 3x3 start), every stem within d + pad
// evaluated, the new bound G and the match slot stored, outputs written.
// (qx, qy: the query's moved position, as cert_try stored it; a scan in the workgroup's
// compacted phase takes it from LDS, not from the store another lane made)
template <int MD, bool SKIP = false>
__device__ __forceinline__ void cert_scan(const NNArgs &a, const GridView &g, const Stems &S,
                                          int64_t i, double qx, double qy, bool warm, double pad,
                                          unsigned long long &kmin_c, unsigned long long &kmax) {
    const double qz = (MD == 3) ? a.sz[i] : 0.0;
    const double eps = cert_eps(g, qx, qy);
    Best2 b{INFINITY, 0x7fffffff, -1, INFINITY};
    NNST(3);
    const int pslot = (SKIP && warm) ? a.out_bp[i] : -2;  // the previous match
    if (warm) {
        const double d2w = warm_d2<MD>(a, i, qx, qy);
        if (d2w < INFINITY) b.d2 = d2w;  // a stem's exact d2, its slot unknown (-1)
    }
    const int cx = cell_coord(qx, g.x0, g.inv_h, g.gx);
    const int cy = cell_coord(qy, g.y0, g.inv_h, g.gy);
    const double mq = query_margin(g, qx, qy);
    if (!(b.d2 < INFINITY)) cold_start<MD>(g, S, qx, qy, qz, cx, cy, b);
    double gnew = 0.0;
    if (b.d2 < INFINITY) {
        double rc = sqrt(b.d2) + pad;
        cover_scan<MD>(g, S, qx, qy, qz, cy, mq, rc * rc, b);
        if (b.slot < 0) {
            // A warm bound whose stem the cover did not re-evaluate.  The cover contains
            // the stored match (it lies at exactly sqrt(d2w) < rc), so this is not
            // expected; should it happen, search again from scratch rather than write
            // slot -1: the result is then the cold search's, still exact.
            b = Best2{INFINITY, 0x7fffffff, -1, INFINITY};
            cold_start<MD>(g, S, qx, qy, qz, cx, cy, b);
            rc = sqrt(b.d2) + pad;
            if (b.d2 < INFINITY) cover_scan<MD>(g, S, qx, qy, qz, cy, mq, rc * rc, b);
        }
        gnew = fmin(sqrt(b.s2), rc - mq) - eps;
    }
    a.gap[i] = gap_rd(b.slot >= 0 ? gnew : 0.0);
    if (b.slot >= 0 && b.slot == pslot) {
        finish_same(a, i, Best{b.d2, b.id, b.slot}, kmin_c, kmax);
        return;
    }
    a.out_bp[i] = b.slot;
    finish(a, S, i, qz, Best{b.d2, b.id, max(b.slot, 0)}, kmin_c, kmax);
}

// cert_scan with the candidate stems of one query split over a group of GS lanes
// (stride GS over each row segment), then a butterfly merge of the partial Best2s:
// lowest (d2, id) among real stems wins; the runner-up takes every lane's s2 and each
// losing lane's real best.  Lane lg == 0 writes the outputs.  Every lane of a group runs
// the same row bounds (same query, same cover), so the group stays convergent.
template <int MD, int GS>
__device__ __forceinline__ void group_eval(const Stems &S, int p0, int p1, int lg, double qx,
                                           double qy, double qz, Best2 &b) {
    for (int p = p0 + lg; p < p1; p += GS) eval2<MD>(S, p, qx, qy, qz, b);
}

template <int MD, int GS, bool SKIP = false>
__device__ __forceinline__ void cert_scan_group(const NNArgs &a, const GridView &g, const Stems &S,
                                                int64_t i, double qx, double qy, int lg, double pad,
                                                unsigned long long &kmin_c, unsigned long long &kmax) {
    const double qz = (MD == 3) ? a.sz[i] : 0.0;
    const double eps = cert_eps(g, qx, qy);
    const double d2w = warm_d2<MD>(a, i, qx, qy);
    if (!(d2w < INFINITY)) {  // no finite previous match: the serial cold search
        if (lg == 0) cert_scan<MD>(a, g, S, i, qx, qy, false, pad, kmin_c, kmax);
        return;
    }
    Best2 b{d2w, 0x7fffffff, -1, INFINITY};
    const int pslot = SKIP ? a.out_bp[i] : -2;  // the previous match
    const int cy = cell_coord(qy, g.y0, g.inv_h, g.gy);
    const double mq = query_margin(g, qx, qy);
    const double rc = sqrt(d2w) + pad;
    if (lg == 0) NNST(4);
    const double cover2 = rc * rc;
    for (int k = -1;; ++k) {  // rows cy-1, cy, cy+1, then cy -+ 2, 3, ... while in cover
        bool any = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const int yy = k <= 1 ? (side ? -1 : cy + k) : (side ? cy + k : cy - k);
            if (yy < 0 || yy >= g.gy) continue;
            const double gy = band_gap(qy, g.y0, g.h, yy, yy + 1, mq);
            if (beyond(gy, cover2)) continue;
            any = true;
            const double gy0 = fmax(gy, 0.0);
            const double w = sqrt(fmax(cover2 - gy0 * gy0, 0.0)) + mq;
            const int xl = cell_coord(qx - w, g.x0, g.inv_h, g.gx);
            const int xh = cell_coord(qx + w, g.x0, g.inv_h, g.gx);
            const int32_t *row = g.cell_start + (int64_t)yy * g.gx;
            group_eval<MD, GS>(S, row[xl], row[xh + 1], lg, qx, qy, qz, b);
        }
        if (!any && k >= 2) break;
    }
#pragma unroll
    for (int off = GS / 2; off > 0; off >>= 1) {
        const double od2 = __shfl_xor(b.d2, off, GS);
        const int oid = __shfl_xor(b.id, off, GS);
        const int oslot = __shfl_xor(b.slot, off, GS);
        const double os2 = __shfl_xor(b.s2, off, GS);
        const bool mine_real = b.slot >= 0, other_real = oslot >= 0;
        const bool take = other_real &&
                          (!mine_real || od2 < b.d2 || (od2 == b.d2 && oid < b.id));
        const double lose = take ? (mine_real ? b.d2 : INFINITY) : (other_real ? od2 : INFINITY);
        b.s2 = fmin(fmin(b.s2, os2), lose);
        b.d2 = take ? od2 : b.d2;
        b.id = take ? oid : b.id;
        b.slot = take ? oslot : b.slot;
    }
    if (lg != 0) return;
    if (b.slot < 0) {  // the stored match was not re-evaluated (not expected): cold search
        cert_scan<MD>(a, g, S, i, qx, qy, false, pad, kmin_c, kmax);
        return;
    }
    const double gnew = fmin(sqrt(b.s2), rc - mq) - eps;
    a.gap[i] = gap_rd(gnew);
    if (b.slot == pslot) {
        finish_same(a, i, Best{b.d2, b.id, b.slot}, kmin_c, kmax);
        return;
    }
    finish(a, S, i, qz, Best{b.d2, b.id, max(b.slot, 0)}, kmin_c, kmax);
}

// one query of the certified path, both steps inline; returns true when certified
template <int MD>
__device__ __forceinline__ bool nn_query_cert(const NNArgs &a, const GridView &g, const Stems &S,
                                              int64_t i, const double *T,
                                              unsigned long long &kmin_c, unsigned long long &kmax) {
    double mv = 0.0, qx = 0.0, qy = 0.0;
    if (a.warm_c && cert_try<MD>(a, g, S, i, T, kmin_c, kmax, mv, qx, qy)) return true;
    if (!a.warm_c) {
        qx = a.sx[i];
        qy = a.sy[i];
        if (T) {
            apply_T(T, qx, qy);
            a.sx[i] = qx;
            a.sy[i] = qy;
        }
    }
    cert_scan<MD>(a, g, S, i, qx, qy, a.warm_c != 0, cert_pad(g, a.warm_c ? mv : INFINITY), kmin_c, kmax);
    return false;
}

// Exact 1-NN of one query (lane): warm start from the stem it matched in the previous
// call, then the disk-clipped row scan of grid_nn.
template <int MD>
__device__ __forceinline__ void nn_query(const NNArgs &a, const GridView &g, const Stems &S,
                                         int64_t i, const double *T, unsigned long long &kmin_c,
                                         unsigned long long &kmax) {
    NNST(5);
    double qx = a.sx[i], qy = a.sy[i];
    if (T) {
        apply_T(T, qx, qy);
        a.sx[i] = qx;
        a.sy[i] = qy;
    }
    const double qz = (MD == 3) ? a.sz[i] : 0.0;
    Best b{INFINITY, 0x7fffffff, 0};
    if (a.warm_c) {
        // the previous match as a finite bound: its exact d2 to the moved query (the
        // operations of eval_slot), index unknown -- the scan meets it again and an
        // equal d2 at a lower index still wins the tie
        const double px = a.cx[i], py = a.cy[i];
        const double dzz = (MD == 3) ? a.dz2[i] : 0.0;
        const double dx = qx - px, dy = qy - py;
        double s = dx * dx;
        s = s + dy * dy;
        if (MD == 3) s = s + dzz;
        if (s < INFINITY) b.d2 = s;
    } else if (a.prev_bp) {
        const int pb = a.prev_bp[i];
        if (pb >= 0) eval_slot<MD>(S, pb, qx, qy, qz, b);
    }
    grid_nn<MD>(g, S, qx, qy, qz, b);
    finish(a, S, i, qz, b, kmin_c, kmax);
}

// Waves per SIMD.  k_nn_grid (one query per thread): 7 kept 71 VGPRs and 94 SGPRs (40
// spilled to VGPR lanes): NN 43.4 -> 42.3 us per C3 call; 8 spilled VGPRs to scratch.
// k_nn_grid_q (QPT = 4 queries per thread; the certified step holds 4 queries' inputs):
// 7 spills 49 VGPRs to scratch, 6 spills 4, 5 none (87 VGPRs).
#ifndef FICP_NN_WPE
#define FICP_NN_WPE 7
#endif
#if FICP_NN_WPE > 0
#define NN_WPE __attribute__((amdgpu_waves_per_eu(FICP_NN_WPE, FICP_NN_WPE)))
#else
#define NN_WPE
#endif
#ifndef FICP_NNQ_WPE
#define FICP_NNQ_WPE 5
#endif
#define NNQ_WPE __attribute__((amdgpu_waves_per_eu(FICP_NNQ_WPE, FICP_NNQ_WPE)))
// Queries per thread of k_nn_grid: a workgroup takes 256 * QPT consecutive queries (in
// the work order), thread t queries t, t + 256, ...  The certified calls (most of a run)
// are a short load-test-store per query whose time was latency: 1 query per thread left
// ~22 us per 1M-query call with >99.5 % certified; QPT queries' loads issue together.
#ifndef FICP_NN_QPT
#define FICP_NN_QPT 4
#endif
constexpr int QPT = FICP_NN_QPT;
// the first calls of a run scan most queries (cold start, then every query's first cover
// scan): those run one query per thread at 7 waves per SIMD (k_nn_grid); the later calls,
// mostly certified, take QPT queries per thread at 5 waves (k_nn_grid_q) -- per call at
// C3 the QPT form was 2-7 us faster from the 5th call on and 3-23 us slower before it
#ifndef FICP_NN_QPT_FROM
#define FICP_NN_QPT_FROM 4
#endif

// Step 1 of the certified path for the QPT queries of this thread: every input loaded
// first (no store between them, so the loads issue back to back), then apply T, try the
// certificate, store.  pend bit q: query q needs the scan (its moved XY stored), mv[q] its
// move.
template <int MD, int Q>
__device__ __forceinline__ unsigned cert_try_qpt(const NNArgs &a, const GridView &g, const Stems &S,
                                                 int64_t i0, const double *T,
                                                 unsigned long long &kmin_c,
                                                 unsigned long long &kmax, double (&mv)[Q],
                                                 double (&mqx)[Q], double (&mqy)[Q]) {
    double ox[Q], oy[Q], wx[Q], wy[Q], wz[Q];
    float gp[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t i = i0 + (int64_t)q * 256;
        const bool v = i < a.n;
        ox[q] = v ? a.sx[i] : 0.0;
        oy[q] = v ? a.sy[i] : 0.0;
        wx[q] = v ? a.cx[i] : 0.0;
        wy[q] = v ? a.cy[i] : 0.0;
        wz[q] = (v && MD == 3) ? a.dz2[i] : 0.0;
        gp[q] = (v && !a.gap_cold) ? a.gap[i] : 0.0f;
    }
    unsigned pend = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t i = i0 + (int64_t)q * 256;
        mv[q] = 0.0;
        mqx[q] = mqy[q] = 0.0;
        if (i >= a.n) continue;
        double qx = ox[q], qy = oy[q];
        if (T) {
            apply_T(T, qx, qy);
            a.sx[i] = qx;
            a.sy[i] = qy;
        }
        mqx[q] = qx;
        mqy[q] = qy;
        const double eps = cert_eps(g, qx, qy);
        // the stored match's exact d2 at the moved query (eval_slot's operations)
        const double dx = qx - wx[q], dy = qy - wy[q];
        double d2w = dx * dx;
        d2w = d2w + dy * dy;
        if (MD == 3) d2w = d2w + wz[q];
        const double mx = qx - ox[q], my = qy - oy[q];
        mv[q] = sqrt(mx * mx + my * my);
        const double G = (double)gp[q] - mv[q] - eps;
        if (!(d2w < INFINITY && sqrt(d2w) + eps < G)) {
            pend |= 1u << q;
            continue;
        }
        NNST(2);
        a.gap[i] = gap_rd(G);
        if (a.idx) a.idx[i] = (int)load_zid(S.r, a.out_bp[i]).z;
        const double d = sqrt(d2w);
        const unsigned long long k = ordkey(d);
        if (a.dist) a.dist[i] = d;
        if (a.r) a.r[i] = d2w;
        if (a.key) a.key[i] = k;
        if (a.val) a.val[i] = (uint32_t)i;
        kmin_c = max(kmin_c, ~k);
        kmax = max(kmax, k);
    }
    return pend;
}


// The compacted phase's hand-off is an LDS-only barrier: the scanning lanes take each
// query's moved position from LDS (s_qx, s_qy) instead of loading the store another lane
// made, so the barrier need not wait for the certified lanes' stores (__syncthreads()
// waits for every outstanding global access, vmcnt(0)).
#define NN_LDS_SYNC() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
// LQ: the single-plot kernels (the batch kernels keep the global hand-off: the two LDS
// arrays cost their 5 waves per SIMD, 1,024 plots -1.4 %)
template <int MD, bool APPLY, int Q, bool SKIP = false, bool LQ = false>
__device__ __forceinline__ void nn_grid_body(const NNArgs &a, const GridView &g, int64_t i0) {
    // the three flags load together (the apply flag's load used to wait for the other two)
    const int sk = a.skip ? *a.skip : 0, ru = a.reuse ? *a.reuse : 0;
    const int ap = (APPLY && a.apply_flag) ? *a.apply_flag : 1;
    if (sk && a.fin_orig) fin_scatter(a, (int64_t)blockIdx.x * (256 * Q), 256 * Q);
    if (sk || ru) return;
    const int t = threadIdx.x;
    unsigned long long kmin_c = 0, kmax = 0;
    const double *T = (APPLY && ap) ? a.T : nullptr;
    if (a.cert_block && a.gap && a.warm_c) {
        // block-compacted: certificates first, then the workgroup's uncertified queries
        // packed densely onto its lanes (GS lanes per query when there are few of them)
        __shared__ int s_list[256 * Q];
        __shared__ double s_mv[256 * Q];
        __shared__ double s_qx[LQ ? 256 * Q : 1], s_qy[LQ ? 256 * Q : 1];
        __shared__ int s_n;
        if (t == 0) s_n = 0;
        __syncthreads();
        const Stems S = stems_of(g.pts, g.m);
        double mv[Q], mqx[Q], mqy[Q];
        const unsigned pend = cert_try_qpt<MD, Q>(a, g, S, i0 + t, T, kmin_c, kmax, mv, mqx, mqy);
        const int lane = t & 63;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const bool pq = (pend >> q) & 1u;
            const unsigned long long m = __ballot(pq);
            int base = 0;
            if (lane == 0 && m) base = atomicAdd(&s_n, __popcll(m));
            base = __shfl(base, 0);
            if (pq) {
                const int e = base + __popcll(m & ((1ULL << lane) - 1));
                s_list[e] = q * 256 + t;
                s_mv[e] = mv[q];
                if constexpr (LQ) {
                    s_qx[e] = mqx[q];
                    s_qy[e] = mqy[q];
                }
            }
        }
        if constexpr (LQ) NN_LDS_SYNC();
        else __syncthreads();  // (the certified lanes' moved positions land first)
        const int tot = s_n;
#define NN_QXY(e) (LQ ? s_qx[(LQ ? (e) : 0)] : a.sx[i0 + s_list[e]]), (LQ ? s_qy[(LQ ? (e) : 0)] : a.sy[i0 + s_list[e]])
        if (a.cert_block >= 16 && tot <= 16) {
            if (t < tot * 16) cert_scan_group<MD, 16, SKIP>(a, g, S, i0 + s_list[t >> 4], NN_QXY(t >> 4), t & 15, cert_pad(g, s_mv[t >> 4]), kmin_c, kmax);
        } else if (a.cert_block >= 8 && tot <= 32) {
            if (t < tot * 8) cert_scan_group<MD, 8, SKIP>(a, g, S, i0 + s_list[t >> 3], NN_QXY(t >> 3), t & 7, cert_pad(g, s_mv[t >> 3]), kmin_c, kmax);
        } else if (a.cert_block >= 4 && tot <= 64) {
            if (t < tot * 4) cert_scan_group<MD, 4, SKIP>(a, g, S, i0 + s_list[t >> 2], NN_QXY(t >> 2), t & 3, cert_pad(g, s_mv[t >> 2]), kmin_c, kmax);
        } else if (a.cert_block >= 2 && tot <= 128) {
            if (t < tot * 2) cert_scan_group<MD, 2, SKIP>(a, g, S, i0 + s_list[t >> 1], NN_QXY(t >> 1), t & 1, cert_pad(g, s_mv[t >> 1]), kmin_c, kmax);
        } else if constexpr (Q == 1) {
            if (t < tot) cert_scan<MD, SKIP>(a, g, S, i0 + s_list[t], NN_QXY(t), true, cert_pad(g, s_mv[t]), kmin_c, kmax);
        } else {
            for (int e = t; e < tot; e += 256)
                cert_scan<MD, SKIP>(a, g, S, i0 + s_list[e], NN_QXY(e), true, cert_pad(g, s_mv[e]), kmin_c, kmax);
        }
    } else {
        const Stems S = stems_of(g.pts, g.m);
        for (int q = 0; q < Q; ++q) {
            const int64_t i = i0 + (int64_t)q * 256 + t;
            if (i >= a.n) break;
            if (a.gap && !a.warm_c) {
                // the cold call: the plain scan (no cover) and no certificate for the next
                // call, which scans every query with its cover.  A cold scan with the cover
                // cost more than that first warm call saved (C3: +1.8 % without it)
                nn_query<MD>(a, g, S, i, T, kmin_c, kmax);
                if (!a.gap_cold) a.gap[i] = 0;
            } else if (a.gap) {
                nn_query_cert<MD>(a, g, S, i, T, kmin_c, kmax);
            } else {
                nn_query<MD>(a, g, S, i, T, kmin_c, kmax);
            }
        }
    }
    if (a.range) {
        if constexpr (Q == 1) {
            block_range_store(a.range, true, kmin_c, kmax);
        } else {
            // the parts keep the one-query-per-thread layout (nblk(n) of them, whichever
            // kernel ran): this workgroup's range in part Q b, neutral (0, 0) in the next
            // Q - 1, so the selection reads no stale part
            __shared__ unsigned long long s_ra[4], s_rb[4];
            unsigned long long ra = kmin_c, rb = kmax;
            wave_range_reduce(ra, rb);  // (lane 63)
            if ((t & 63) == 63) {
                s_ra[t >> 6] = ra;
                s_rb[t >> 6] = rb;
            }
            __syncthreads();
            const int64_t np = (a.n + 255) / 256, p0 = (int64_t)blockIdx.x * Q;
            if (t < Q && p0 + t < np) {
                unsigned long long x = 0, y = 0;
                if (t == 0)
                    for (int w = 0; w < 4; ++w) {
                        x = s_ra[w] > x ? s_ra[w] : x;
                        y = s_rb[w] > y ? s_rb[w] : y;
                    }
                a.range[2 + 2 * (p0 + t)] = x;
                a.range[3 + 2 * (p0 + t)] = y;
            }
        }
    }
}

template <int MD, bool APPLY>
__global__ __launch_bounds__(256) NN_WPE void k_nn_grid(NNArgs a, GridView g) {
    constexpr bool SK1 = FICP_NN_SKIP_SINGLE != 0;
    // the three flags load together (the apply flag's load used to wait for the other two)
    const int sk = a.skip ? *a.skip : 0, ru = a.reuse ? *a.reuse : 0;
    const int ap = (APPLY && a.apply_flag) ? *a.apply_flag : 1;
    if (sk && a.fin_orig) fin_scatter(a, (int64_t)blockIdx.x * blockDim.x, (int)blockDim.x);
    if (sk || ru) return;
    const int64_t i = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    unsigned long long kmin_c = 0, kmax = 0;
    const double *T = (APPLY && ap) ? a.T : nullptr;
    if (a.cert_block && a.gap && a.warm_c) {
        // block-compacted: certificates first, then the workgroup's uncertified queries
        // packed densely onto its lanes (GS lanes per query when there are few of them)
        __shared__ int s_list[256];
        __shared__ double s_mv[256], s_qx[256], s_qy[256];
        __shared__ int s_n;
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        const Stems S = stems_of(g.pts, g.m);
        double mv = 0.0, mqx = 0.0, mqy = 0.0;
        const bool pend = i < a.n && !cert_try<MD>(a, g, S, i, T, kmin_c, kmax, mv, mqx, mqy);
        const unsigned long long m = __ballot(pend);
        const int lane = threadIdx.x & 63;
        int base = 0;
        if (lane == 0 && m) base = atomicAdd(&s_n, __popcll(m));
        base = __shfl(base, 0);
        if (pend) {
            const int q = base + __popcll(m & ((1ULL << lane) - 1));
            s_list[q] = (int)(i & 255);
            s_mv[q] = mv;
            s_qx[q] = mqx;
            s_qy[q] = mqy;
        }
        NN_LDS_SYNC();  // (as nn_grid_body: the moved positions travel in LDS)
        const int tot = s_n;
        const int64_t i0 = i - threadIdx.x;
        const int t = threadIdx.x;
        constexpr bool LQ = true;
        if (a.cert_block >= 16 && tot <= 16) {
            if (t < tot * 16) cert_scan_group<MD, 16, SK1>(a, g, S, i0 + s_list[t >> 4], NN_QXY(t >> 4), t & 15, cert_pad(g, s_mv[t >> 4]), kmin_c, kmax);
        } else if (a.cert_block >= 8 && tot <= 32) {
            if (t < tot * 8) cert_scan_group<MD, 8, SK1>(a, g, S, i0 + s_list[t >> 3], NN_QXY(t >> 3), t & 7, cert_pad(g, s_mv[t >> 3]), kmin_c, kmax);
        } else if (a.cert_block >= 4 && tot <= 64) {
            if (t < tot * 4) cert_scan_group<MD, 4, SK1>(a, g, S, i0 + s_list[t >> 2], NN_QXY(t >> 2), t & 3, cert_pad(g, s_mv[t >> 2]), kmin_c, kmax);
        } else if (a.cert_block >= 2 && tot <= 128) {
            if (t < tot * 2) cert_scan_group<MD, 2, SK1>(a, g, S, i0 + s_list[t >> 1], NN_QXY(t >> 1), t & 1, cert_pad(g, s_mv[t >> 1]), kmin_c, kmax);
        } else if (t < tot) {
            cert_scan<MD, SK1>(a, g, S, i0 + s_list[t], NN_QXY(t), true, cert_pad(g, s_mv[t]), kmin_c, kmax);
        }
    } else if (i < a.n) {
        if (a.gap && !a.warm_c) {
            // the cold call: the plain scan (no cover) and no certificate for the next
            // call, which scans every query with its cover.  A cold scan with the cover
            // cost more than that first warm call saved (C3: +1.8 % without it)
            nn_query<MD>(a, g, stems_of(g.pts, g.m), i, T, kmin_c, kmax);
            if (!a.gap_cold) a.gap[i] = 0;
        } else if (a.gap) {
            nn_query_cert<MD>(a, g, stems_of(g.pts, g.m), i, T, kmin_c, kmax);
        } else {
            nn_query<MD>(a, g, stems_of(g.pts, g.m), i, T, kmin_c, kmax);
        }
    }
    if (a.range) block_range_store(a.range, true, kmin_c, kmax);
}

template <int MD, bool APPLY>
__global__ __launch_bounds__(256) NNQ_WPE void k_nn_grid_q(NNArgs a, GridView g) {
    nn_grid_body<MD, APPLY, QPT, FICP_NN_SKIP_SINGLE != 0, true>(a, g, xcd_block(blockIdx.x, gridDim.x) * (256 * QPT));
}

// Batch of plots (C4): tree i belongs to plot p = plot_of[i] and is matched against
// plot p's own CHM grid (cells cell_base_p.., stems indexed in the concatenated layer).
__device__ __forceinline__ GridView plot_view(const PlotGrid &pg, const TPt *pts,
                                              const int32_t *cell_start, int64_t m) {
    GridView g;
    g.pts = pts;
    g.cell_start = cell_start + pg.cell_base;
    g.x0 = pg.x0;
    g.y0 = pg.y0;
    g.h = pg.h;
    g.inv_h = pg.inv_h;
    g.margin = pg.margin;
    g.gx = pg.gx;
    g.gy = pg.gy;
    g.m = m;
    return g;
}

// The single-plot kernel's certified reuse per plot: warm calls (a.warm_c) try every
// live query's certificate (cert_try) against its own plot's grid; the workgroup's
// uncertified queries are then packed onto its first lanes, GS lanes per query when
// few remain, each scanning with its own plot's grid (a workgroup may straddle plots).
// The cold call runs the plain scan and stores G = 0.  Converged plots are skipped.
#ifndef FICP_NNB_WPE
#define FICP_NNB_WPE 6  // 84 -> 80 VGPRs, 5 -> 6 waves per SIMD: batch NN 375 -> 367 us per launch
#endif
#if FICP_NNB_WPE > 0
#define NNB_WPE __attribute__((amdgpu_waves_per_eu(FICP_NNB_WPE, FICP_NNB_WPE)))
#else
#define NNB_WPE
#endif
template <int MD>
__device__ __forceinline__ void nn_batch_rows(const NNArgs &a, const int32_t *__restrict__ plot_of,
                                              const PlotGrid *__restrict__ grids,
                                              const TPt *__restrict__ pts, int64_t m,
                                              const int32_t *__restrict__ cell_start,
                                              const PlotState *__restrict__ st, int64_t i) {
    unsigned long long kmin_c = 0, kmax = 0;  // (no key range: the batch selection is per plot)
    const Stems S = stems_of(pts, m);
    int p = 0;
    bool live = false;
    if (i < a.n) {
        p = plot_of[i];
        live = st[p].phase != PH_DONE;
    }
    const double *T = (live && st[p].apply) ? st[p].T : nullptr;
    if (a.gap && a.warm_c) {
        __shared__ int s_list[256];
        __shared__ double s_mv[256];
        __shared__ int s_n;
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        double mv = 0.0, mqx = 0.0, mqy = 0.0;
        bool pend = false;
        if (live) {
            const GridView g = plot_view(grids[p], pts, cell_start, m);
            pend = !cert_try<MD>(a, g, S, i, T, kmin_c, kmax, mv, mqx, mqy);
        }
        const unsigned long long msk = __ballot(pend);
        const int lane = threadIdx.x & 63;
        int base = 0;
        if (lane == 0 && msk) base = atomicAdd(&s_n, __popcll(msk));
        base = __shfl(base, 0);
        if (pend) {
            const int q = base + __popcll(msk & ((1ULL << lane) - 1));
            s_list[q] = (int)(i & 255);
            s_mv[q] = mv;
        }
        __syncthreads();  // (the certified lanes' moved positions land first)
        const int tot = s_n;
        const int64_t i0 = i - threadIdx.x;
        const int t = threadIdx.x;
        int gs = 1;
        if (a.cert_block >= 8 && tot <= 32) gs = 8;
        else if (a.cert_block >= 4 && tot <= 64) gs = 4;
        else if (a.cert_block >= 2 && tot <= 128) gs = 2;
        if (t < tot * gs) {
            const int q = t / gs;
            const int64_t iq = i0 + s_list[q];
            const GridView gq = plot_view(grids[plot_of[iq]], pts, cell_start, m);
            const double pad = cert_pad(gq, s_mv[q]);
            constexpr bool SK = FICP_NN_SKIP_SAME != 0;
            const double qx = a.sx[iq], qy = a.sy[iq];
            if (gs == 8) cert_scan_group<MD, 8, SK>(a, gq, S, iq, qx, qy, t & 7, pad, kmin_c, kmax);
            else if (gs == 4) cert_scan_group<MD, 4, SK>(a, gq, S, iq, qx, qy, t & 3, pad, kmin_c, kmax);
            else if (gs == 2) cert_scan_group<MD, 2, SK>(a, gq, S, iq, qx, qy, t & 1, pad, kmin_c, kmax);
            else cert_scan<MD, SK>(a, gq, S, iq, qx, qy, true, pad, kmin_c, kmax);
        }
    } else if (live) {
        const GridView g = plot_view(grids[p], pts, cell_start, m);
        nn_query<MD>(a, g, S, i, T, kmin_c, kmax);
        if (a.gap && !a.gap_cold) a.gap[i] = 0;  // the cold call stores no certificate (k_nn_grid)
    }
}

template <int MD>
__global__ __launch_bounds__(256) NNB_WPE void k_nn_grid_batch(NNArgs a, const int32_t *__restrict__ plot_of,
                                                       const PlotGrid *__restrict__ grids,
                                                       const TPt *__restrict__ pts, int64_t m,
                                                       const int32_t *__restrict__ cell_start,
                                                       const PlotState *__restrict__ st) {
    nn_batch_rows<MD>(a, plot_of, grids, pts, m, cell_start, st,
                      xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x);
}

// The cold batch call, one query per thread: a workgroup whose 256 trees belong to one plot
// (10k-tree plots: ~39 in 40) reads that plot's state and grid once, as scalars, and runs
// the single-plot kernel's body against it (k_nn_grid's cold form: the plain scan, G = 0);
// a workgroup that straddles plots takes k_nn_grid_batch's per-row form.  The per-row
// form kept every lane's grid view in VGPRs behind two dependent per-lane loads (plot id,
// then grid): the cold launch ran ~2x the single-plot cold call's time per query.
#ifndef FICP_NNBU_WPE
#define FICP_NNBU_WPE 6  // 72 VGPRs with 73 spilled at 7; 6: 128 plots +1.5-2.8 %, 1024 +0.4 % (5: -3 %)
#endif
template <int MD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FICP_NNBU_WPE, FICP_NNBU_WPE)))
void k_nn_grid_batch_u(NNArgs a, const int32_t *__restrict__ plot_of, const PlotGrid *__restrict__ grids,
                       const TPt *__restrict__ pts, int64_t m, const int32_t *__restrict__ cell_start,
                       PlotState *__restrict__ st) {
    const int64_t i0 = xcd_block(blockIdx.x, gridDim.x) * 256;
    const int64_t ilast = min(i0 + 256, a.n) - 1;
    const int p0 = plot_of[i0], p1 = plot_of[ilast];
    if (p0 == p1) {  // (uniform)
        if (st[p0].phase == PH_DONE) return;
        NNArgs b = a;
        b.T = st[p0].T;
        b.apply_flag = &st[p0].apply;
        b.skip = nullptr;
        b.reuse = nullptr;
        nn_grid_body<MD, true, 1, FICP_NN_SKIP_SAME != 0>(b, plot_view(grids[p0], pts, cell_start, m), i0);
        return;
    }
    nn_batch_rows<MD>(a, plot_of, grids, pts, m, cell_start, st, i0 + threadIdx.x);
}

// Warm batch calls, QPT queries per thread (the single-plot k_nn_grid_q's form): a
// workgroup takes 256 * QPT consecutive trees.  When they all belong to one plot (10k-tree
// plots: ~9 in 10 workgroups) the plot's state, transform and grid are uniform and the
// rows run nn_grid_body against that plot's grid; a workgroup that straddles plots runs
// k_nn_grid_batch's per-row form on each of its QPT row blocks in turn.
template <int MD>
__global__ __launch_bounds__(256) NNQ_WPE void k_nn_grid_batch_q(NNArgs a, const int32_t *__restrict__ plot_of,
                                                         const PlotGrid *__restrict__ grids,
                                                         const TPt *__restrict__ pts, int64_t m,
                                                         const int32_t *__restrict__ cell_start,
                                                         PlotState *__restrict__ st) {
    const int64_t i0 = xcd_block(blockIdx.x, gridDim.x) * (256 * QPT);
    const int64_t ilast = min(i0 + 256 * QPT, a.n) - 1;
    const int p0 = plot_of[i0], p1 = plot_of[ilast];
    if (p0 == p1) {  // (uniform)
        if (st[p0].phase == PH_DONE) return;
        NNArgs b = a;
        b.T = st[p0].T;
        b.apply_flag = &st[p0].apply;
        b.skip = nullptr;
        b.reuse = nullptr;
        nn_grid_body<MD, true, QPT, FICP_NN_SKIP_SAME != 0>(b, plot_view(grids[p0], pts, cell_start, m), i0);
        return;
    }
    for (int q = 0; q < QPT; ++q) {
        const int64_t r0 = i0 + (int64_t)q * 256;
        if (r0 >= a.n) break;  // (uniform)
        nn_batch_rows<MD>(a, plot_of, grids, pts, m, cell_start, st, r0 + threadIdx.x);
        __syncthreads();  // (the per-row form's LDS list is reused by the next block)
    }
}

constexpr int kTile = 256;

// blockIdx.y = target chunk; one chunk -> final outputs, several -> partials then merge
template <int MD, int QPT>
__global__ __launch_bounds__(256) void k_nn_brute(NNArgs a, const double *__restrict__ tx,
                                                  const double *__restrict__ ty,
                                                  const double *__restrict__ tz, int64_t m,
                                                  int64_t chunk, double *part_d2,
                                                  int32_t *part_idx) {
    if (a.skip && *a.skip) return;
    __shared__ double s_x[kTile], s_y[kTile], s_z[kTile];
    const int64_t base = (int64_t)blockIdx.x * (256 * QPT) + threadIdx.x;
    double qx[QPT], qy[QPT], qz[QPT], best[QPT];
    int bi[QPT];
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
        const int64_t i = base + q * 256;
        const bool ok = i < a.n;
        qx[q] = ok ? a.sx[i] : 0.0;
        qy[q] = ok ? a.sy[i] : 0.0;
        qz[q] = (ok && MD == 3) ? a.sz[i] : 0.0;
        best[q] = INFINITY;
        bi[q] = 0x7fffffff;
    }
    const int64_t j0 = (int64_t)blockIdx.y * chunk;
    const int64_t j1 = min(m, j0 + chunk);
    for (int64_t t0 = j0; t0 < j1; t0 += kTile) {
        const int cnt = (int)min((int64_t)kTile, j1 - t0);
        __syncthreads();
        if (threadIdx.x < cnt) {
            s_x[threadIdx.x] = tx[t0 + threadIdx.x];
            s_y[threadIdx.x] = ty[t0 + threadIdx.x];
            if (MD == 3) s_z[threadIdx.x] = tz[t0 + threadIdx.x];
        }
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const double px = s_x[j], py = s_y[j];
            const double pz = (MD == 3) ? s_z[j] : 0.0;
            const int id = (int)(t0 + j);
#pragma unroll
            for (int q = 0; q < QPT; ++q) {
                const double s = sq_dist<MD>(qx[q], qy[q], qz[q], px, py, pz);
                const bool b = s < best[q];  // ascending j: strict < keeps the lowest index
                best[q] = b ? s : best[q];
                bi[q] = b ? id : bi[q];
            }
        }
    }
    unsigned long long kmin_c = 0, kmax = 0;
    bool any = false;
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
        const int64_t i = base + q * 256;
        if (i >= a.n) continue;
        if (gridDim.y == 1) {
            const unsigned long long k = write_out(a, i, best[q], bi[q]);
            if (a.cx) {  // no stem matched (NaN query): no gather out of the layer
                const int bj = bi[q] < (int)m ? bi[q] : 0;
                a.cx[i] = a.tx[bj];
                a.cy[i] = a.ty[bj];
            }
            kmin_c = max(kmin_c, ~k);
            kmax = max(kmax, k);
            any = true;
        } else {
            part_d2[(int64_t)blockIdx.y * a.n + i] = best[q];
            part_idx[(int64_t)blockIdx.y * a.n + i] = bi[q];
        }
    }
    if (gridDim.y == 1 && a.range) block_range_store(a.range, any, kmin_c, kmax);
}

__global__ __launch_bounds__(256) void k_nn_merge(NNArgs a, int nchunks, const double *part_d2,
                                                  const int32_t *part_idx) {
    if (a.skip && *a.skip) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < a.n;
    unsigned long long key = 0;
    if (valid) {
        double best = INFINITY;
        int bi = 0x7fffffff;
        for (int c = 0; c < nchunks; ++c) {  // chunks ascend in index: strict < keeps the lowest
            const double s = part_d2[(int64_t)c * a.n + i];
            const int id = part_idx[(int64_t)c * a.n + i];
            if (s < best || (s == best && id < bi)) {
                best = s;
                bi = id;
            }
        }
        key = write_out(a, i, best, bi);
        if (a.cx) {  // bi stays INT32_MAX only for a NaN query: never gather past the layer
            const int bj = bi != 0x7fffffff ? bi : 0;
            a.cx[i] = a.tx[bj];
            a.cy[i] = a.ty[bj];
        }
    }
    if (a.range) block_range_store(a.range, valid, ~key, key);
}

__global__ __launch_bounds__(256) void k_apply_inplace(double *x, double *y, int64_t n,
                                                       const double *T, const int *skip,
                                                       const int *apply_flag) {
    if ((skip && *skip) || (apply_flag && !*apply_flag)) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double qx = x[i], qy = y[i];
    apply_T(T, qx, qy);
    x[i] = qx;
    y[i] = qy;
}

// ---------------------------------------------------------------- grid build
// ox non-null: also copies x, y (and z when both non-null) to ox, oy, oz on the way
__global__ __launch_bounds__(256) void k_minmax2_partial(const double *x, const double *y,
                                                         int64_t m, double *partials,
                                                         const double *z, double *ox, double *oy,
                                                         double *oz) {
    __shared__ double s[4][256];
    double a0 = INFINITY, a1 = -INFINITY, b0 = INFINITY, b1 = -INFINITY;
    const int64_t stride = (int64_t)gridDim.x * 256;
    // 4 grid-stride rows in flight per thread (one at a time serialised 4 latencies)
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < m; i0 += 4 * stride) {
        double xs[4], ys[4], zs[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * stride;
            xs[u] = i < m ? x[i] : NAN;
            ys[u] = i < m ? y[i] : NAN;
            zs[u] = (i < m && ox && z && oz) ? z[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= m) continue;
            const double vx = xs[u], vy = ys[u];
            if (ox) {
                ox[i] = vx;
                oy[i] = vy;
                if (z && oz) oz[i] = zs[u];
            }
            a0 = fmin(a0, vx);
            a1 = fmax(a1, vx);
            b0 = fmin(b0, vy);
            b1 = fmax(b1, vy);
        }
    }
    s[0][threadIdx.x] = a0;
    s[1][threadIdx.x] = a1;
    s[2][threadIdx.x] = b0;
    s[3][threadIdx.x] = b1;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + w]);
            s[1][threadIdx.x] = fmax(s[1][threadIdx.x], s[1][threadIdx.x + w]);
            s[2][threadIdx.x] = fmin(s[2][threadIdx.x], s[2][threadIdx.x + w]);
            s[3][threadIdx.x] = fmax(s[3][threadIdx.x], s[3][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) partials[blockIdx.x * 4 + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_minmax2_final(const double *partials, int nb, double *out4) {
    __shared__ double s[4][256];
    double a0 = INFINITY, a1 = -INFINITY, b0 = INFINITY, b1 = -INFINITY;
    for (int b = threadIdx.x; b < nb; b += 256) {
        a0 = fmin(a0, partials[4 * b]);
        a1 = fmax(a1, partials[4 * b + 1]);
        b0 = fmin(b0, partials[4 * b + 2]);
        b1 = fmax(b1, partials[4 * b + 3]);
    }
    s[0][threadIdx.x] = a0;
    s[1][threadIdx.x] = a1;
    s[2][threadIdx.x] = b0;
    s[3][threadIdx.x] = b1;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + w]);
            s[1][threadIdx.x] = fmax(s[1][threadIdx.x], s[1][threadIdx.x + w]);
            s[2][threadIdx.x] = fmin(s[2][threadIdx.x], s[2][threadIdx.x + w]);
            s[3][threadIdx.x] = fmax(s[3][threadIdx.x], s[3][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) out4[threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_grid_count(const double *x, const double *y, int64_t m,
                                                    double x0, double y0, double inv_h, int gx,
                                                    int gy, int32_t *cell_of, int32_t *counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int cx = cell_coord(x[i], x0, inv_h, gx);
    const int cy = cell_coord(y[i], y0, inv_h, gy);
    const int c = cy * gx + cx;
    cell_of[i] = c;
    atomicAdd(&counts[c], 1);
}

__global__ __launch_bounds__(256) void k_grid_scatter(const double *x, const double *y,
                                                      const double *z, int64_t m,
                                                      const int32_t *cell_of,
                                                      const int32_t *cell_start, int32_t *fill,
                                                      TPt *pts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int c = cell_of[i];
    const int pos = cell_start[c] + atomicAdd(&fill[c], 1);
    double4 v;
    v.x = x[i];
    v.y = y[i];
    v.z = z ? z[i] : 0.0;
    v.w = __longlong_as_double((long long)i);
    *reinterpret_cast<double4 *>(pts + pos) = v;
}

// Order each cell's stems by index so the grid layout is deterministic (results are
// deterministic regardless: ties are resolved by index explicitly).
__global__ __launch_bounds__(256) void k_grid_sort_cells(TPt *pts, const int32_t *cell_start,
                                                         int64_t ncells) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    const int p0 = cell_start[c], p1 = cell_start[c + 1];
    if (p1 - p0 > 64) return;  // only small cells; large ones keep arrival order
    for (int a = p0 + 1; a < p1; ++a) {
        const TPt v = pts[a];
        int b = a - 1;
        while (b >= p0 && pts[b].idx > v.idx) {
            pts[b + 1] = pts[b];
            --b;
        }
        pts[b + 1] = v;
    }
}

// ---------------------------------------------------------------- work order
__global__ __launch_bounds__(256) void k_src_cellkey(const double *sx, const double *sy,
                                                     int64_t n, GridView g,
                                                     unsigned long long *key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int cx = cell_coord(sx[i], g.x0, g.inv_h, g.gx);
    const int cy = cell_coord(sy[i], g.y0, g.inv_h, g.gy);
    const unsigned nstx = (unsigned)(g.gx + 7) >> 3;
    const unsigned st = ((unsigned)cy >> 3) * nstx + ((unsigned)cx >> 3);
    const unsigned long long ck = ((unsigned long long)st << 6) | ((cy & 7) << 3) | (cx & 7);
    key[i] = (ck << 32) | (unsigned long long)i;
}

__global__ __launch_bounds__(256) void k_gather_work(const uint32_t *perm, const double *sx,
                                                     const double *sy, const double *sz,
                                                     int64_t n, double *wx, double *wy,
                                                     double *wz, uint32_t *worig) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = perm[p];
    wx[p] = sx[i];
    wy[p] = sy[i];
    if (sz) wz[p] = sz[i];
    worig[p] = i;
}

__global__ __launch_bounds__(256) void k_scatter_xy(const uint32_t *worig, const double *wx,
                                                    const double *wy, int64_t n, double *sx,
                                                    double *sy) {
    // XCD-aware: each XCD takes one contiguous eighth of the work rows, so the caller rows
    // one region of work rows scatters to (a batch plot's) fill whole lines in one L2
    // instead of partial lines from every XCD (C4, 10M rows: 250 us with the plain order)
    const int64_t p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = worig[p];
    sx[i] = wx[p];
    sy[i] = wy[p];
}

__global__ __launch_bounds__(256) void k_scatter_i32(const uint32_t *worig, const int32_t *w,
                                                     int64_t n, int32_t *out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    out[worig[p]] = w[p];
}

__global__ __launch_bounds__(256) void k_deinterleave(const double *rows, int64_t n, int64_t ld,
                                                      int ncols, double *c0, double *c1,
                                                      double *c2) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *r = rows + i * ld;
    c0[i] = r[0];
    if (ncols > 1) c1[i] = r[1];
    if (ncols > 2 && c2) c2[i] = r[2];
}

__global__ __launch_bounds__(256) void k_interleave_xy(const double *x, const double *y, int64_t n,
                                                       double *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[2 * i] = x[i];
    out[2 * i + 1] = y[i];
}

// the moved XY into columns 0, 1 of the uploaded (n x ld) rows (ficp_run_into's result)
__global__ __launch_bounds__(256) void k_put_xy_rows(const double *x, const double *y, int64_t n,
                                                     int64_t ld, double *rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    rows[i * ld] = x[i];
    rows[i * ld + 1] = y[i];
}

// device-to-device copy of n 16-B words (ficp_memcpy_d2d on aligned buffers): four
// independent loads per thread in flight, a grid that covers the array once
__global__ __launch_bounds__(256) void k_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// empty shard: +inf distance, an index no real stem has (never chosen by the merge)
__global__ __launch_bounds__(256) void k_fill_inf(double *d2, int32_t *idx, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        d2[i] = INFINITY;
        idx[i] = 0x7fffffff;
    }
}

// partitioned target (C5): shard-local idx -> global idx
__global__ __launch_bounds__(256) void k_add_offset(int32_t *idx, int64_t n, int64_t off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) idx[i] = (int32_t)(idx[i] + off);
}

// merged (d2, global idx) of every query -> the sort/fit inputs of one NN call: key of
// dist = sqrt(d2) (exactly as write_out), r = d2, the matched stem's XY; key-range parts
__global__ __launch_bounds__(256) void k_corr_from_merge(const double *d2, const int32_t *idx,
                                                         const double *tx, const double *ty,
                                                         int64_t n, unsigned long long *key,
                                                         double *r, double *cx, double *cy,
                                                         unsigned long long *range) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long k = 0;
    const bool valid = i < n;
    if (valid) {
        const double v = d2[i];
        k = ordkey(sqrt(v));
        key[i] = k;
        r[i] = v;
        const int32_t j = idx[i] != 0x7fffffff ? idx[i] : 0;  // unmatched (NaN) query
        cx[i] = tx[j];
        cy[i] = ty[j];
    }
    block_range_store(range, valid, ~k, k);
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t launch_minmax2(const double *x, const double *y, int64_t m, double *partials,
                          double *out4, hipStream_t s, const double *z, double *ox, double *oy,
                          double *oz) {
    int nb = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (m + 255) / 256));
    hipLaunchKernelGGL(k_minmax2_partial, dim3(nb), dim3(256), 0, s, x, y, m, partials, z, ox, oy,
                       oz);
    hipLaunchKernelGGL(k_minmax2_final, dim3(1), dim3(256), 0, s, partials, nb, out4);
    return hipGetLastError();
}

hipError_t launch_grid_count(const double *x, const double *y, int64_t m, double x0, double y0,
                             double inv_h, int gx, int gy, int32_t *cell_of, int32_t *counts,
                             hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_grid_count, dim3(nblk(m)), dim3(256), 0, s, x, y, m, x0, y0, inv_h, gx,
                       gy, cell_of, counts);
    return hipGetLastError();
}

hipError_t launch_grid_scatter(const double *x, const double *y, const double *z, int64_t m,
                               const int32_t *cell_of, const int32_t *cell_start, int32_t *fill,
                               TPt *pts, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_grid_scatter, dim3(nblk(m)), dim3(256), 0, s, x, y, z, m, cell_of,
                       cell_start, fill, pts);
    return hipGetLastError();
}

hipError_t launch_grid_sort_cells(TPt *pts, const int32_t *cell_start, int64_t ncells,
                                  hipStream_t s) {
    hipLaunchKernelGGL(k_grid_sort_cells, dim3(nblk(ncells)), dim3(256), 0, s, pts, cell_start,
                       ncells);
    return hipGetLastError();
}

#ifdef FICP_NN_STATS
__global__ void k_nn_stats_print(const int *skip, const int *reuse) {
    if (threadIdx.x != 0) return;
    if ((skip && *skip) || (reuse && *reuse)) return;
    printf("NNSTATS eval2 %llu evalslot %llu cert %llu scan %llu group %llu plain %llu\n", g_nnst[0],
           g_nnst[1], g_nnst[2], g_nnst[3], g_nnst[4], g_nnst[5]);
    for (int q = 0; q < 8; ++q) g_nnst[q] = 0;
}
#endif

hipError_t launch_nn_grid(const NNArgs &a, const GridView &g, int md, hipStream_t s,
                          bool reduce_range, hipEvent_t e0, hipEvent_t e1) {
    if (a.n == 0) return hipSuccess;
#ifdef FICP_NN_STATS
    struct Pr {
        hipStream_t s;
        const NNArgs &a;
        ~Pr() { hipLaunchKernelGGL(k_nn_stats_print, dim3(1), dim3(64), 0, s, a.skip, a.reuse); }
    } pr_{s, a};
#endif
    const bool q = a.multi && a.cert_block && a.gap && a.warm_c;
    dim3 grid(q ? nblk(a.n, 256 * QPT) : nblk(a.n)), blk(256);
    void (*kf)(NNArgs, GridView);
    if (md == 3) kf = q ? (a.T ? k_nn_grid_q<3, true> : k_nn_grid_q<3, false>)
                        : (a.T ? k_nn_grid<3, true> : k_nn_grid<3, false>);
    else kf = q ? (a.T ? k_nn_grid_q<2, true> : k_nn_grid_q<2, false>)
                : (a.T ? k_nn_grid<2, true> : k_nn_grid<2, false>);
    if (!e0) hipLaunchKernelGGL(kf, grid, blk, 0, s, a, g);  // plain dispatch without events
    else hipExtLaunchKernelGGL(kf, grid, blk, 0, s, e0, e1, 0, a, g);
    if (a.range && reduce_range) return launch_range_reduce(a.range, grid.x, s);
    return hipGetLastError();
}

hipError_t launch_nn_brute(const NNArgs &a0, const double *tx, const double *ty,
                           const double *tz, int64_t m, int md, double *part_d2,
                           int32_t *part_idx, hipStream_t s, bool reduce_range) {
    if (a0.n == 0 || m == 0) return hipSuccess;
    NNArgs a = a0;
    if (a.T) {  // apply first: with several target chunks every chunk reads the moved source
        hipLaunchKernelGGL(k_apply_inplace, dim3(nblk(a.n)), dim3(256), 0, s, a.sx, a.sy, a.n,
                           a.T, a.skip, a.apply_flag);
        a.T = nullptr;
    }
    constexpr int QPT = 2;
    const int64_t qblocks = (a.n + 256 * QPT - 1) / (256 * QPT);
    const int64_t nchunks = brute_chunk_count(a.n, m);
    const int64_t chunk = ((m + nchunks - 1) / nchunks + kTile - 1) / kTile * kTile;
    const int64_t nch = (m + chunk - 1) / chunk;
    dim3 grid((unsigned)qblocks, (unsigned)nch), blk(256);
    if (md == 3)
        hipLaunchKernelGGL((k_nn_brute<3, QPT>), grid, blk, 0, s, a, tx, ty, tz, m, chunk,
                           part_d2, part_idx);
    else
        hipLaunchKernelGGL((k_nn_brute<2, QPT>), grid, blk, 0, s, a, tx, ty, tz, m, chunk,
                           part_d2, part_idx);
    if (nch > 1)
        hipLaunchKernelGGL(k_nn_merge, dim3(nblk(a.n)), dim3(256), 0, s, a, (int)nch, part_d2,
                           part_idx);
    if (a.range && reduce_range)
        return launch_range_reduce(a.range, nn_range_parts(a.n, m, false), s);
    return hipGetLastError();
}

// workgroups that store key-range parts in one NN launch (grid: one per 256 queries;
// brute: one per 512 queries, or the merge kernel's one per 256 with several chunks)
int64_t nn_range_parts(int64_t n, int64_t m, bool grid) {
    if (grid || brute_chunk_count(n, m) > 1) return (int64_t)nblk(n);
    return (n + 511) / 512;
}

int nn_qpt_from() { return FICP_NN_QPT_FROM; }

// target chunks for the brute kernel: enough workgroups to fill 256 CUs
int64_t brute_chunk_count(int64_t n, int64_t m) {
    const int64_t qblocks = (n + 511) / 512;
    int64_t c = (2048 + qblocks - 1) / qblocks;
    const int64_t maxc = (m + kTile - 1) / kTile;
    if (c > maxc) c = maxc;
    if (c > 64) c = 64;
    if (c < 1) c = 1;
    return c;
}

hipError_t launch_deinterleave(const double *rows, int64_t n, int64_t ld, int ncols, double *c0,
                               double *c1, double *c2, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_deinterleave, dim3(nblk(n)), dim3(256), 0, s, rows, n, ld, ncols, c0, c1,
                       c2);
    return hipGetLastError();
}

hipError_t launch_interleave_xy(const double *x, const double *y, int64_t n, double *out_xy,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_interleave_xy, dim3(nblk(n)), dim3(256), 0, s, x, y, n, out_xy);
    return hipGetLastError();
}

hipError_t launch_put_xy_rows(const double *x, const double *y, int64_t n, int64_t ld, double *rows,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_put_xy_rows, dim3(nblk(n)), dim3(256), 0, s, x, y, n, ld, rows);
    return hipGetLastError();
}

hipError_t launch_copy16(const void *src, void *dst, int64_t n16, hipStream_t s) {
    if (n16 <= 0) return hipSuccess;
    // one pass of 4 words per thread: 1M x 16 B (C3's x, y columns) = 1,024 workgroups
    const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n16 + 1023) / 1024, 1), 8192);
    hipLaunchKernelGGL(k_copy16, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4 *)src, (uint4 *)dst,
                       n16);
    return hipGetLastError();
}

hipError_t launch_apply_xy_flags(double *x, double *y, int64_t n, const double *T, const int *skip,
                                const int *apply_flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_inplace, dim3(nblk(n)), dim3(256), 0, s, x, y, n, T, skip,
                       apply_flag);
    return hipGetLastError();
}

hipError_t launch_apply_xy(double *x, double *y, int64_t n, const double *T, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_inplace, dim3(nblk(n)), dim3(256), 0, s, x, y, n, T,
                       (const int *)nullptr, (const int *)nullptr);
    return hipGetLastError();
}

hipError_t launch_src_cellkey(const double *sx, const double *sy, int64_t n, const GridView &g,
                              unsigned long long *key, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_src_cellkey, dim3(nblk(n)), dim3(256), 0, s, sx, sy, n, g, key);
    return hipGetLastError();
}

hipError_t launch_gather_work(const uint32_t *perm, const double *sx, const double *sy,
                              const double *sz, int64_t n, double *wx, double *wy, double *wz,
                              uint32_t *worig, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_work, dim3(nblk(n)), dim3(256), 0, s, perm, sx, sy, sz, n, wx, wy,
                       wz, worig);
    return hipGetLastError();
}

hipError_t launch_scatter_xy(const uint32_t *worig, const double *wx, const double *wy, int64_t n,
                             double *sx, double *sy, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_xy, dim3(nblk(n)), dim3(256), 0, s, worig, wx, wy, n, sx, sy);
    return hipGetLastError();
}

hipError_t launch_nn_grid_batch(const NNArgs &a, const int32_t *plot_of, const PlotGrid *grids,
                                const TPt *pts, int64_t m, const int32_t *cell_start,
                                const PlotState *st, int md, hipStream_t s, int64_t call) {
    if (a.n == 0) return hipSuccess;
    // warm calls: QPT queries per thread from FICP_BATCH_QPT_MIN trees per launch on (default
    // 2M: ~2,000 workgroups of 1024 trees, enough to hide their latency chains; at 128 plots
    // of 10k, 640k trees per sub-batch, the 1-query form measured 39 vs 55 us per launch,
    // at 1024 plots the QPT form 264 vs 316 us), and from the batch iteration
    // FICP_BATCH_QPT_FROM on: the first warm calls scan most queries with their cover, which
    // wants one query per thread (the single-plot loop's FICP_NN_QPT_FROM); FICP_BATCH_QPT=0:
    // never.  The other calls run k_nn_grid_batch_u (one query per thread, the plot's grid
    // read once per workgroup); FICP_BATCH_COLD_U=0: the per-row k_nn_grid_batch instead.
    const char *qe = getenv("FICP_BATCH_QPT");
    const char *qm = getenv("FICP_BATCH_QPT_MIN");
    const char *qf = getenv("FICP_BATCH_QPT_FROM");
    const char *ue = getenv("FICP_BATCH_COLD_U");
    const int64_t qpt_min = qm ? atoll(qm) : (int64_t)2000000;
    const int64_t qpt_from = qf ? atoll(qf) : (int64_t)4;  // C4 1,024 plots: 1.373M vs 1.351M (1)
    const bool use_u = !(ue && atoi(ue) == 0);
    PlotState *stw = const_cast<PlotState *>(st);
    if (!(qe && atoi(qe) == 0) && a.n >= qpt_min && call >= qpt_from && a.warm_c && a.gap &&
        a.cert_block) {
        const dim3 gq(nblk(a.n, 256 * QPT));
        if (md == 3)
            hipLaunchKernelGGL(k_nn_grid_batch_q<3>, gq, dim3(256), 0, s, a, plot_of, grids, pts, m,
                               cell_start, stw);
        else
            hipLaunchKernelGGL(k_nn_grid_batch_q<2>, gq, dim3(256), 0, s, a, plot_of, grids, pts, m,
                               cell_start, stw);
    } else if (use_u) {
        if (md == 3)
            hipLaunchKernelGGL(k_nn_grid_batch_u<3>, dim3(nblk(a.n)), dim3(256), 0, s, a, plot_of, grids,
                               pts, m, cell_start, stw);
        else
            hipLaunchKernelGGL(k_nn_grid_batch_u<2>, dim3(nblk(a.n)), dim3(256), 0, s, a, plot_of, grids,
                               pts, m, cell_start, stw);
    } else if (md == 3)
        hipLaunchKernelGGL(k_nn_grid_batch<3>, dim3(nblk(a.n)), dim3(256), 0, s, a, plot_of, grids,
                           pts, m, cell_start, st);
    else
        hipLaunchKernelGGL(k_nn_grid_batch<2>, dim3(nblk(a.n)), dim3(256), 0, s, a, plot_of, grids,
                           pts, m, cell_start, st);
    if (a.range) return launch_range_reduce(a.range, nblk(a.n), s);
    return hipGetLastError();
}

hipError_t launch_knn_grid(const double *sx, const double *sy, const double *sz, int64_t q0,
                           int64_t n, const GridView &g, int md, const uint8_t *removed,
                           int32_t *out_id, double *out_d, hipStream_t s) {
    if (n <= q0) return hipSuccess;
    const unsigned nb = nblk(n - q0);
    if (md == 3)
        hipLaunchKernelGGL(k_knn_grid<3>, dim3(nb), dim3(256), 0, s, sx, sy, sz, q0, n, g, removed,
                           out_id, out_d);
    else
        hipLaunchKernelGGL(k_knn_grid<2>, dim3(nb), dim3(256), 0, s, sx, sy, sz, q0, n, g, removed,
                           out_id, out_d);
    return hipGetLastError();
}

hipError_t launch_fill_inf(double *d2, int32_t *idx, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_inf, dim3(nblk(n)), dim3(256), 0, s, d2, idx, n);
    return hipGetLastError();
}

hipError_t launch_add_offset(int32_t *idx, int64_t n, int64_t off, hipStream_t s) {
    if (n == 0 || off == 0) return hipSuccess;
    hipLaunchKernelGGL(k_add_offset, dim3(nblk(n)), dim3(256), 0, s, idx, n, off);
    return hipGetLastError();
}

hipError_t launch_corr_from_merge(const double *d2, const int32_t *idx, const double *tx,
                                  const double *ty, int64_t n, unsigned long long *key, double *r,
                                  double *cx, double *cy, unsigned long long *range,
                                  hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_corr_from_merge, dim3(nblk(n)), dim3(256), 0, s, d2, idx, tx, ty, n, key,
                       r, cx, cy, range);
    return launch_range_reduce(range, nblk(n), s);
}

hipError_t launch_scatter_i32(const uint32_t *worig, const int32_t *w, int64_t n, int32_t *out,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_i32, dim3(nblk(n)), dim3(256), 0, s, worig, w, n, out);
    return hipGetLastError();
}

}  // namespace ficp
