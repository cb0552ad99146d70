// frmsd_bounds.h -- bound arithmetic of the bucketed FRMSD-optimal-fraction selection,
// shared by the single-plot selection (k_select.hip) and the per-plot batch selection
// (k_batch.hip).  ficp.py:73-86 picks the first k minimising
//   FRMSD(k) = (1 / (k/N)^lambda) * sqrt(S_k / k),  S_k = sum of the k smallest r,
// which is monotone in h(k, S) = log2 S - p log2 k with p = 2 lambda + 1.  Inside a run
// of sorted positions whose rows are all >= lo, S_{C0+j} >= S_C0 + j lo makes h
// quasi-concave in j (p >= 1): the run's lower bound is the smaller of its end values.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ficp_internal.h"

namespace ficp {
namespace fb {

__device__ __forceinline__ int bits_of(unsigned long long v) {
    return v ? 64 - __clzll((long long)v) : 0;
}

// smallest r = d^2 of any row whose key (ordkey(d)) is >= klo (d = sqrt(d2) correctly
// rounded, so d >= d_lo implies d2 >= d_lo^2 up to the rounding the factor covers)
__device__ __forceinline__ double lo_r(unsigned long long klo) {
    if (!(klo >> 63)) return 0.0;
    const double d = __longlong_as_double((long long)(klo & 0x7fffffffffffffffULL));
    return d * d * (1.0 - 1e-15);
}

// lg2 is fast_log2 below (round 5; before it ocml's fp64 log2, ~1 ulp): absolute error
// ~1e-13 at |e| ~ 1000, measured over every exponent including subnormals by
// `tools/selcheck log2` (tests/test_gpu_parity.py::test_fast_log2_error_bound, which fails
// above kMarg / 100).  kMarg (log2 units) covers that error, the rounding of p log2 k and
// that of the fp64 prefix sums of the bucket sums the bounds are built from (relative
// ~1e-12 at 2^13 buckets or 16k rows): 1e-9 leaves a factor ~100.
// (The float log of round 1 forced 1e-5, which kept every position within ~3.5e-6 of the
// minimum FRMSD a candidate: 700-2200 rows at C3 whatever the bucket width.)
constexpr double kMarg = 1e-9;

// log2 for the bounds (round 5): x = 2^e m, m in [sqrt(1/2), sqrt(2)), log2 m = 2 atanh(s) /
// ln 2 with s = (m - 1) / (m + 1), |s| < 0.1716, the odd series to s^19 (the next term is
// ~4e-18), s from one reciprocal + a Newton step.  Absolute error ~1e-15 + the rounding of
// e + log2 m (~1e-13 at |e| ~ 1000), far inside kMarg.  ~25 dependent fp64 operations
// against ~60 in ocml's double-double log2, whose chains were the longest part of every
// bounds phase (the one-workgroup bounds of k_sel_bounds, the window tail, k_batch_select).
__device__ __forceinline__ double fast_log2(double x) {
    int e;
    double m = frexp(x, &e);  // m in [0.5, 1)
    if (m < 0.70710678118654752) {
        m = m + m;
        e -= 1;
    }
    const double a = m - 1.0, b = m + 1.0;  // (m - 1 exact)
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    const double s = a * r, z = s * s;
    double P = 1.0 / 19.0;
    P = fma(P, z, 1.0 / 17.0);
    P = fma(P, z, 1.0 / 15.0);
    P = fma(P, z, 1.0 / 13.0);
    P = fma(P, z, 1.0 / 11.0);
    P = fma(P, z, 1.0 / 9.0);
    P = fma(P, z, 1.0 / 7.0);
    P = fma(P, z, 1.0 / 5.0);
    P = fma(P, z, 1.0 / 3.0);
    P = fma(P, z, 1.0);
    constexpr double k2_ln2 = 2.8853900817779268;  // 2 / ln 2
    return (double)e + (s * P) * k2_ln2;
}

__device__ __forceinline__ double lg2(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -INFINITY : NAN;
    if (!(x < INFINITY)) return INFINITY;
    return fast_log2(x);
}

__device__ __forceinline__ double h_of(long long k, double S, double p) {
    return lg2(S) - p * lg2((double)k);
}

// lower bound of h over k in (C0, C0 + c] when the c rows there are all >= lo: the
// smaller end value, minus the margin
__device__ __forceinline__ double block_lb(long long C0, long long c, double P0, double lo,
                                           double p) {
    const double a = h_of(C0 + 1, P0 + lo, p);
    const double b = h_of(C0 + c, P0 + (double)c * lo, p);
    return fmin(a, b) - kMarg;
}

// ---- the window paths (k_select.hip k_sel_win, k_batch.hip k_batch_select): a key
// window [wlo, whi) around the previous threshold key and kWinNCS coarse buckets on each
// side whose widths grow with their distance from it (win_lh: ficp_internal.h)
constexpr int kWinNCS = 128;
typedef unsigned long long u64;

struct WMap {
    u64 kmin, kmax;  // the call's key range (the last workgroup: from the records)
    u64 wlo, whi;
    int su;   // coarse unit 2^su keys (H / 4)
    int fxb;  // fixed point: a row of bucket b adds floor(r * 2^(fxb - e_b)), r < 2^e_b
    int ok;
};

// the window [c - H, c + H) (saturated at the key range's ends), H = 2^win_lh; no key
// range needed: the coarse buckets are measured from the window's edges, and each has its
// own fixed-point exponent from its highest key
__device__ __forceinline__ WMap win_map(u64 c, u64 tmove, int wfloor, int64_t n) {
    WMap m{};
    m.kmin = 0;
    m.kmax = ~0ULL;
    const int lh = win_lh(tmove, win_floor(wfloor, n));
    const u64 H = 1ULL << lh;
    m.su = lh - 2;
    m.wlo = c > H ? c - H : 0ULL;
    m.whi = c < ~0ULL - H ? c + H : ~0ULL;
    m.ok = lh <= win_hmax_log(n);
    m.fxb = 62 - bits_of((u64)max<int64_t>(n, 1));
    return m;
}

// coarse bucket of a distance of q units from the window edge (0..3: one unit each, then 4
// per octave) and the smallest q of bucket j
__device__ __forceinline__ int win_cq(u64 q) {
    if (q < 4) return (int)q;
    const int e = 63 - __clzll((long long)q);
    return min(4 * (e - 1) + (int)((q >> (e - 2)) & 3ULL), kWinNCS - 1);
}
__device__ __forceinline__ u64 win_cq_lo(int j) {
    if (j < 4) return (u64)j;
    return (u64)(4 + (j & 3)) << (j / 4 - 1);
}

// lowest key any row of coarse bucket b (key order: b < kWinNCS below the window, kWinNCS - 1 the
// nearest; b >= kWinNCS above it, kWinNCS the nearest) can have
__device__ __forceinline__ u64 win_bucket_lo(const WMap &m, int b) {
    if (b < kWinNCS) {
        const int j = kWinNCS - 1 - b;  // rows with (wlo - 1 - key) >> su in [lo(j), lo(j + 1))
        if (j + 1 >= kWinNCS) return m.kmin;
        const u64 q = win_cq_lo(j + 1);
        if (q >= (1ULL << (64 - m.su))) return m.kmin;
        const u64 d = q << m.su;  // lowest key = wlo - d
        return d >= m.wlo - m.kmin ? m.kmin : m.wlo - d;
    }
    const u64 q = win_cq_lo(b - kWinNCS);
    if (q >= (1ULL << (64 - m.su))) return m.kmax;
    const u64 d = q << m.su;
    return d > m.kmax - m.whi ? m.kmax : m.whi + d;
}

// highest key any row of coarse bucket b can have (0: the bucket cannot hold a row)
__device__ __forceinline__ u64 win_bucket_hi(const WMap &m, int b) {
    if (b < kWinNCS) {
        const int j = kWinNCS - 1 - b;  // highest key = wlo - 1 - (lo(j) << su)
        const u64 q = win_cq_lo(j);
        if (q >= (1ULL << (64 - m.su))) return 0ULL;
        const u64 d = q << m.su;
        return (m.wlo == 0ULL || d > m.wlo - 1ULL) ? 0ULL : m.wlo - 1ULL - d;
    }
    const int j = b - kWinNCS;
    if (j + 1 >= kWinNCS) return ~0ULL;
    const u64 q = win_cq_lo(j + 1);
    if (q >= (1ULL << (64 - m.su))) return ~0ULL;
    const u64 d = q << m.su;
    return d - 1ULL > ~0ULL - m.whi ? ~0ULL : m.whi + (d - 1ULL);
}

// e with r < 2^e for every row of coarse bucket b (bucket_exp's rule; 1024: the bucket may
// hold inf / NaN, those rows fail the window path anyway)
__device__ __forceinline__ int win_bucket_exp(const WMap &m, int b) {
    const u64 khi = win_bucket_hi(m, b);
    if (!(khi >> 63)) return 0;
    const int ex = (int)((khi >> 52) & 0x7ffULL);
    return min(2 * ex - 2044, 1024);
}

}  // namespace fb
}  // namespace ficp
