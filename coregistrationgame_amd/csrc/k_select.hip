// k_select.hip -- the FRMSD-optimal fraction (ficp.py:54-60, 73-86) by bucketed
// selection instead of a full residual sort.
//
// The reference sorts every distance (argsort, ficp.py:63,78) and evaluates
// FRMSD(k) = (1 / (k/N)**lambda) * sqrt(S_k / k) for every prefix k.  Only three things
// of that sort are used by the rest of the iteration: the winning k, its FRMSD, and
// WHICH k rows are selected.  The selected set is {i : (key_i, orig_i) <= (key_t,
// orig_t)} for the k-th pair t of the stable order, so the fit needs t alone
// (k_fit_sums tests that predicate while it streams every row).
//
// FRMSD is a monotone function of g(k) = S_k / k^(2 lambda + 1).  Inside a block of
// consecutive sorted positions (C0, C0 + c] whose values r are all >= lo,
// S_{C0+j} >= S_C0 + j lo, and (S_C0 + j lo) / (C0 + j)^p is quasi-concave in j (its
// derivative changes sign at most once, + to -), so the block's lower bound is the
// smaller of its two end values.  Hence:
//  1. k_sel_hist    : 8192 buckets of (key - kmin) >> s over the NN call's key range;
//                     count + fixed-point sum of r per bucket (grid 2^(e_b - 37) with
//                     r < 2^e_b in the bucket: relative truncation < 2^-35), in LDS,
//                     then one integer atomic per non-empty bucket and workgroup.
//  2. k_sel_bounds  : one workgroup; prefix counts/sums over the buckets; U = the
//                     smallest FRMSD upper bound at any bucket end; candidate buckets
//                     [b0, b1] = those whose lower bound is <= U.  The true first
//                     minimum lies inside them.  Reads and resets the histogram.
//  3. k_sel_gather  : one pass: S_base = sum of r below b0 (fixed reduction tree, so
//                     bitwise deterministic), candidates (key, orig, r) appended.
//  4. k_sel_final   : one workgroup; (a) <= 4096 candidates: LDS bucket sort by
//                     (key, orig), exact prefix sums S_base + ..., FRMSD of every
//                     candidate k, first minimum (strict <, ficp.py:84); (b) more:
//                     refinement levels with 4096 sub-bins (exact integer sums of the
//                     rows that drop below, so still deterministic); (c) if that stalls
//                     (clustered or equal keys), an in-workgroup LSD radix sort.
// Level-0 bucket sums are bracketed exactly (truncated fixed point: [fx, fx + c) units);
// the bounds are compared in the log2 domain with a 1e-5 margin (see h_of).  The decided
// k and threshold pair depend only on the exact, deterministic prefix sums.
// At C3 (1M x 1M) the candidate set holds 15-5000 rows, so step (a) is the normal case.
#include "ficp_internal.h"

#include <math.h>

#include <algorithm>

namespace ficp {

namespace {

typedef unsigned long long u64;
typedef unsigned __int128 u128;

constexpr int NB = 8192;     // level-0 buckets
constexpr int NB_LOG = 13;
constexpr int HT = 1024;     // threads of the histogram / bounds / final kernels
constexpr int NWAVE = HT / 64;
constexpr int CAP = 4096;    // candidates sorted in LDS
constexpr int NSB = 2048;    // bins of the LDS bucket sort
constexpr int NSB_LOG = 11;
constexpr int NS = 4096;     // sub-bins of one refinement level
constexpr int NS_LOG = 12;
constexpr int MAXLEV = 4;
constexpr int GT = 256;      // gather: threads per block
constexpr int GI = 8;        // gather: rows per thread

// error bits of SelCtl::err (sticky; the host checks them after a run)
constexpr unsigned ERR_EMPTY = 1u;  // candidate set empty (cannot happen with finite r)

struct SelCtl {
    u64 kmin;
    int s, b0, b1, pad0;
    long long kbase;       // rows in buckets < b0
    double U;              // upper bound of h (log2 domain) at the minimum
    unsigned ccount;       // candidates appended (agent-scope atomics only)
    unsigned err;          // sticky error bits (agent-scope atomics only)
    unsigned levels;       // statistics: refinement levels run (plain, final kernel only)
    unsigned radix;        // statistics: radix fallbacks (plain, final kernel only)
};

struct SelWS {
    unsigned *hcnt;  // [NB] agent-scope atomics only
    u64 *hfix;       // [NB] fixed-point sums, agent-scope atomics only
    SelCtl *ctl;
    double *parts;   // [gather blocks]
    u64 *ka, *kb;    // candidate ping-pong buffers (n each)
    uint32_t *oa, *ob;
    double *ra, *rb;
};

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
inline int gather_blocks(int64_t n) { return (int)std::max<int64_t>(1, (n + GT * GI - 1) / (GT * GI)); }
inline int hist_blocks(int64_t n) { return (int)std::min<int64_t>(128, std::max<int64_t>(1, (n + 16383) / 16384)); }

SelWS carve(void *tmp, int64_t n) {
    char *p = (char *)tmp;
    SelWS w;
    w.hcnt = (unsigned *)p;
    p += align_up(NB * 4, 256);
    w.hfix = (u64 *)p;
    p += align_up(NB * 8, 256);
    w.ctl = (SelCtl *)p;
    p += 256;
    w.parts = (double *)p;
    p += align_up((int64_t)gather_blocks(n) * 8, 256);
    const int64_t nn = std::max<int64_t>(n, 1);
    w.ka = (u64 *)p;
    p += align_up(nn * 8, 256);
    w.kb = (u64 *)p;
    p += align_up(nn * 8, 256);
    w.ra = (double *)p;
    p += align_up(nn * 8, 256);
    w.rb = (double *)p;
    p += align_up(nn * 8, 256);
    w.oa = (uint32_t *)p;
    p += align_up(nn * 4, 256);
    w.ob = (uint32_t *)p;
    return w;
}

__device__ __forceinline__ int bits_of(u64 v) { return v ? 64 - __clzll((long long)v) : 0; }

__device__ __forceinline__ int sel_shift(u64 kmin, u64 kmax) {
    const int b = bits_of(kmax > kmin ? kmax - kmin : 0ULL);
    return b > NB_LOG ? b - NB_LOG : 0;
}

// smallest r = d^2 of any row whose key is >= klo (d = sqrt(d2) correctly rounded)
__device__ __forceinline__ double lo_r(u64 klo) {
    if (!(klo >> 63)) return 0.0;
    const double d = __longlong_as_double((long long)(klo & 0x7fffffffffffffffULL));
    return d * d * (1.0 - 1e-15);
}

// exponent e_b with r < 2^e_b for every row of bucket b (1024: the bucket holds inf/NaN)
__device__ __forceinline__ int bucket_exp(u64 kmin, u64 kmax, int s, int b) {
    const u64 wdt = ((u64)(b + 1) << s) - 1ULL;  // wraps to ~0 for the top bucket at s = 51
    const u64 khi = wdt > kmax - kmin ? kmax : kmin + wdt;
    if (!(khi >> 63)) return 0;
    const double d = __longlong_as_double((long long)(khi & 0x7fffffffffffffffULL));
    const double rhi = d * d * (1.0 + 1e-15);
    if (!(rhi < INFINITY)) return 1024;
    if (rhi == 0.0) return 0;
    return ilogb(rhi) + 1;
}
constexpr int FIXB = 37;  // bits of one row's fixed-point value

// Bounds work on h(k, S) = log2(S) - p log2(k), p = 2 lambda + 1, a monotone function of
// FRMSD(k) = N^lambda k^-lambda sqrt(S / k) (no pow per bucket).  lg2 is exact in the
// exponent and ~1e-7 in the mantissa (v_log_f32); kMarg (log2 units) covers that, the
// double rounding of the prefix sums and the refinement levels' LDS float sums.
constexpr double kMarg = 1e-5;

__device__ __forceinline__ double lg2(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -INFINITY : NAN;
    if (!(x < INFINITY)) return INFINITY;
    int e;
    const double m = frexp(x, &e);  // [0.5, 1)
    return (double)e + (double)__builtin_amdgcn_logf((float)m);
}

__device__ __forceinline__ double h_of(long long k, double S, double p) {
    return lg2(S) - p * lg2((double)k);
}

// lower bound of h over k in (C0, C0 + c] when the c rows there are all >= lo: the
// smaller end value (quasi-concave in k for p >= 1, see the header), minus the margin
__device__ __forceinline__ double block_lb(long long C0, long long c, double P0, double lo,
                                           double p) {
    const double a = h_of(C0 + 1, P0 + lo, p);
    const double b = h_of(C0 + c, P0 + (double)c * lo, p);
    return fmin(a, b) - kMarg;
}

__device__ __forceinline__ bool better(double f, long long k, double bf, long long bk) {
    return f < bf || (f == bf && k < bk);
}

// ------------------------------------------------- block primitives (HT threads)
struct Scr {
    double d[NWAVE];
    long long l[NWAVE];
    u64 u[NWAVE];
    u64 v[NWAVE];
};

// deterministic: butterfly inside the wave (every lane ends with the same bits), wave
// partials in wave order
__device__ __forceinline__ double blk_sum(double x, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = x + __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) t = t + s.d[w];
    __syncthreads();
    return t;
}

__device__ __forceinline__ double blk_min_d(double x, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, 64));
    if ((threadIdx.x & 63) == 0) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = s.d[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) t = fmin(t, s.d[w]);
    __syncthreads();
    return t;
}

__device__ __forceinline__ double blk_max_d(double x, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    if ((threadIdx.x & 63) == 0) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = s.d[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) t = fmax(t, s.d[w]);
    __syncthreads();
    return t;
}

// {min, max} of two u64 quantities at once: returns min(a), max(b)
__device__ __forceinline__ void blk_minmax_u64(u64 &a, u64 &b, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u64 xa = __shfl_xor(a, o, 64), xb = __shfl_xor(b, o, 64);
        a = xa < a ? xa : a;
        b = xb > b ? xb : b;
    }
    if ((threadIdx.x & 63) == 0) {
        s.u[threadIdx.x >> 6] = a;
        s.v[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    a = s.u[0];
    b = s.v[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) {
        a = s.u[w] < a ? s.u[w] : a;
        b = s.v[w] > b ? s.v[w] : b;
    }
    __syncthreads();
}

__device__ __forceinline__ long long blk_max_ll(long long x, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
    if ((threadIdx.x & 63) == 0) s.l[threadIdx.x >> 6] = x;
    __syncthreads();
    long long t = s.l[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) t = max(t, s.l[w]);
    __syncthreads();
    return t;
}

__device__ __forceinline__ long long blk_min_ll(long long x, Scr &s) {
    return -blk_max_ll(-x, s);
}

// exclusive scans (deterministic: Hillis-Steele in the wave, wave offsets in order)
__device__ __forceinline__ double blk_excl_scan_d(double v, Scr &s, double &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(x, o, 64);
        if (lane >= o) x = y + x;
    }
    if (lane == 63) s.d[wave] = x;
    double ex = __shfl_up(x, 1, 64);
    if (lane == 0) ex = 0.0;
    __syncthreads();
    double off = 0.0, tot = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
        if (w < wave) off = off + s.d[w];
        tot = tot + s.d[w];
    }
    __syncthreads();
    total = tot;
    return wave ? off + ex : ex;
}

__device__ __forceinline__ long long blk_excl_scan_ll(long long v, Scr &s, long long &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s.l[wave] = x;
    __syncthreads();
    long long off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
        if (w < wave) off += s.l[w];
        tot += s.l[w];
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

// block argmin of (f, k) with the first-minimum rule; result broadcast
__device__ __forceinline__ void blk_argmin(double &f, long long &k, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double xf = __shfl_xor(f, o, 64);
        const long long xk = __shfl_xor(k, o, 64);
        if (better(xf, xk, f, k)) {
            f = xf;
            k = xk;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        s.d[threadIdx.x >> 6] = f;
        s.l[threadIdx.x >> 6] = k;
    }
    __syncthreads();
    f = s.d[0];
    k = s.l[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w)
        if (better(s.d[w], s.l[w], f, k)) {
            f = s.d[w];
            k = s.l[w];
        }
    __syncthreads();
}

// ------------------------------------------------------------------ kernels
// range: with nparts > 0, every block reduces the producer's range parts itself (see
// block_range_store) and block 0 stores range[0..1] for the kernels that follow.
__global__ __launch_bounds__(HT) void k_sel_hist(const u64 *key, const double *r, int64_t n,
                                                 u64 *range, int64_t nparts, SelWS w,
                                                 const int *skip) {
    if (skip && *skip) return;
    __shared__ unsigned sc[NB];
    __shared__ u64 sf[NB];
    __shared__ short se[NB];
    __shared__ Scr scr;
    u64 kmin, kmax;
    if (nparts > 0) {
        u64 a = 0, b = 0;
        for (int64_t q = threadIdx.x; q < nparts; q += HT) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(range + 2 + 2 * q);
            a = max(a, v.x);
            b = max(b, v.y);
        }
        a = ~a;
        blk_minmax_u64(a, b, scr);
        kmin = a;
        kmax = b;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            range[0] = ~kmin;
            range[1] = kmax;
        }
    } else {
        kmin = ~range[0];
        kmax = range[1];
    }
    const int s = sel_shift(kmin, kmax);
    for (int b = threadIdx.x; b < NB; b += HT) {
        sc[b] = 0u;
        sf[b] = 0ULL;
        se[b] = (short)bucket_exp(kmin, kmax, s, b);
    }
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * per, i1 = min(n, i0 + per);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += HT) {
        const int b = (int)((key[i] - kmin) >> s);
        const int e = se[b];
        const double rv = r[i];
        const u64 m = (e < 1024 && rv < INFINITY) ? (u64)ldexp(rv, FIXB - e) : 0ULL;
        atomicAdd(&sc[b], 1u);
        atomicAdd(&sf[b], m);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += HT) {
        if (sc[b]) {
            __hip_atomic_fetch_add(&w.hcnt[b], sc[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&w.hfix[b], sf[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ __launch_bounds__(HT) void k_sel_bounds(SelWS w, int64_t N, double lam,
                                                   const double *lam_dev, const u64 *range,
                                                   const int *skip) {
    if (skip && *skip) return;
    if (lam_dev) lam = *lam_dev;
    __shared__ Scr scr;
    __shared__ unsigned lc[NB];
    __shared__ u64 lf[NB];
    constexpr int PER = NB / HT;
    const int t = threadIdx.x;
    const u64 kmin = ~range[0], kmax = range[1];
    const int s = sel_shift(kmin, kmax);
    // per bucket: count, and the sum of its rows bracketed by the truncated fixed-point
    // sum (each row loses < 1 unit): fx * 2^(e - FIXB) <= sum < (fx + c) * 2^(e - FIXB)
    auto sums = [&](int b, unsigned c, u64 fx, double &lo, double &hi) {
        const int e = bucket_exp(kmin, kmax, s, b);
        if (e >= 1024) {
            lo = hi = c ? INFINITY : 0.0;
        } else {
            lo = ldexp((double)fx, e - FIXB);
            hi = ldexp((double)(fx + c), e - FIXB);
        }
    };
    long long ct = 0;
    double tlo = 0.0, thi = 0.0;
    unsigned cc[PER];
    u64 ff[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // all 2 * PER exchanges in flight at once
        const int b = t * PER + j;
        cc[j] = __hip_atomic_exchange(&w.hcnt[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ff[j] = __hip_atomic_exchange(&w.hfix[b], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int b = t * PER + j;
        const unsigned c = cc[j];
        const u64 fx = ff[j];
        lc[b] = c;
        lf[b] = fx;
        double lo, hi;
        sums(b, c, fx, lo, hi);
        ct += c;
        tlo = tlo + lo;
        thi = thi + hi;
    }
    long long ctot;
    double stot;
    const long long Cex = blk_excl_scan_ll(ct, scr, ctot);
    const double Plo = blk_excl_scan_d(tlo, scr, stot);
    const double Phi = blk_excl_scan_d(thi, scr, stot);
    // U: the smallest upper bound of h at any bucket end
    const double p = 2.0 * lam + 1.0;
    double U = INFINITY;
    {
        long long C = Cex;
        double P = Phi;
        for (int j = 0; j < PER; ++j) {
            const int b = t * PER + j;
            const unsigned c = lc[b];
            if (c) {
                double lo, hi;
                sums(b, c, lf[b], lo, hi);
                C += c;
                P = P + hi;
                U = fmin(U, h_of(C, P, p) + kMarg);
            }
        }
    }
    U = blk_min_d(U, scr);
    // candidate buckets: lower bound <= U (NaN bounds count as candidates)
    long long bmin = 0x7fffffffLL, bmax = -1, kb = 0;
    {
        long long C = Cex;
        double P = Plo;
        for (int j = 0; j < PER; ++j) {
            const int b = t * PER + j;
            const unsigned c = lc[b];
            if (c) {
                double lo, hi;
                sums(b, c, lf[b], lo, hi);
                const double lb = block_lb(C, c, P, lo_r(kmin + ((u64)b << s)), p);
                if (!(lb > U) || !(p >= 1.0)) {
                    if (bmax < 0) kb = C;  // rows before this thread's first candidate
                    bmin = min(bmin, (long long)b);
                    bmax = max(bmax, (long long)b);
                }
                C += c;
                P = P + lo;
            }
        }
    }
    const long long my_bmin = bmin;
    bmin = blk_min_ll(bmin, scr);
    bmax = blk_max_ll(bmax, scr);
    if (bmax < 0) {  // no bucket qualifies (non-finite r): every row is a candidate
        bmin = 0;
        bmax = NB - 1;
        if (t == 0) w.ctl->kbase = 0;
    } else if (my_bmin == bmin) {
        w.ctl->kbase = kb;  // rows in buckets < b0
    }
    if (t == 0) {
        w.ctl->kmin = kmin;
        w.ctl->s = s;
        w.ctl->b0 = (int)bmin;
        w.ctl->b1 = (int)bmax;
        w.ctl->U = U;
        __hip_atomic_exchange(&w.ctl->ccount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(GT) void k_sel_gather(const u64 *key, const uint32_t *orig,
                                                   const double *r, int64_t n, SelWS w,
                                                   const int *skip) {
    if (skip && *skip) return;
    __shared__ double s_w[GT / 64];
    const u64 kmin = w.ctl->kmin;
    const int s = w.ctl->s, b0 = w.ctl->b0, b1 = w.ctl->b1;
    const int lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blockIdx.x * (GT * GI) + threadIdx.x;
    // all loads first (no load waits behind the append's atomic)
    u64 kk[GI];
    double rr[GI];
#pragma unroll
    for (int q = 0; q < GI; ++q) {
        const int64_t i = base + (int64_t)q * GT;
        kk[q] = i < n ? key[i] : 0ULL;
        rr[q] = i < n ? r[i] : 0.0;
    }
    double acc = 0.0;
    unsigned inm = 0;   // bit q: row q is a candidate
    unsigned wtot = 0;  // candidates of the wave
    u64 masks[GI];
#pragma unroll
    for (int q = 0; q < GI; ++q) {
        const int64_t i = base + (int64_t)q * GT;
        bool in = false;
        if (i < n) {
            const int b = (int)((kk[q] - kmin) >> s);
            if (b < b0) acc = acc + rr[q];
            else if (b <= b1) in = true;
        }
        masks[q] = __ballot(in);
        inm |= (in ? 1u : 0u) << q;
        wtot += (unsigned)__popcll(masks[q]);
    }
    if (wtot) {  // one append reservation per wave
        unsigned pos = 0;
        if (lane == 0)
            pos = __hip_atomic_fetch_add(&w.ctl->ccount, wtot, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        pos = __shfl(pos, 0, 64);
        const u64 lt = (1ULL << lane) - 1ULL;
#pragma unroll
        for (int q = 0; q < GI; ++q) {
            if ((inm >> q) & 1u) {
                const int64_t i = base + (int64_t)q * GT;
                const unsigned p = pos + (unsigned)__popcll(masks[q] & lt);
                w.ka[p] = kk[q];
                w.oa[p] = orig ? orig[i] : (uint32_t)i;
                w.ra[p] = rr[q];
            }
            pos += (unsigned)__popcll(masks[q]);
        }
    }
    // fixed tree: wave butterfly, then the waves in order
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc = acc + __shfl_xor(acc, o, 64);
    if (lane == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < GT / 64; ++q) t = t + s_w[q];
        w.parts[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------- the final workgroup
struct Cand {
    u64 *k;
    uint32_t *o;
    double *r;
};

struct FinalIn {
    long long N;
    double lam;
    double S0;      // exact (deterministic) sum of every row sorted before the candidates
    long long K0;   // number of those rows
    double U;
};

// composite order key of one candidate: ((key - kmin) << ob) | (orig - omin) when that fits
// in 63 bits (then strictly monotone in (key, orig)), else key - kmin (monotone in key)
struct Comp {
    u64 kmin;
    uint32_t omin;
    int ob;  // -1: key only
    __device__ __forceinline__ u64 operator()(u64 k, uint32_t o) const {
        return ob < 0 ? k - kmin : ((k - kmin) << ob) | (u64)(o - omin);
    }
    __device__ __forceinline__ u64 key_lo(u64 v) const { return kmin + (ob < 0 ? v : v >> ob); }
};

__device__ __forceinline__ Comp make_comp(u64 kmin, u64 kmax, uint32_t omin, uint32_t omax) {
    Comp c;
    c.kmin = kmin;
    c.omin = omin;
    const int kb = bits_of(kmax - kmin), ob = bits_of((u64)(omax - omin));
    c.ob = (kb + ob <= 63) ? ob : -1;
    return c;
}

__device__ __forceinline__ bool less_ko(u64 ka, uint32_t oa, u64 kb, uint32_t ob) {
    return ka < kb || (ka == kb && oa < ob);
}

// write the decision to the iteration state (thread 0)
__device__ __forceinline__ void publish(IterState *st, const FinalIn &in, double bf, long long bk,
                                        u64 tkey, uint32_t torig) {
    if (bk == 0x7fffffffffffffffLL) {  // every FRMSD was NaN: the reference keeps (0.0, 0)
        st->k = 0;
        st->frac = 0.0;
        st->frmsd = INFINITY;
    } else {
        st->k = bk;
        st->frac = (double)bk / (double)in.N;
        st->frmsd = bf;
    }
    st->n_src = in.N;
    st->tkey = tkey;
    st->torig = (long long)torig;
}

// LDS layout of the final kernel (bytes)
constexpr int L_K = 0;                          // u64[CAP]
constexpr int L_R = L_K + CAP * 8;              // f64[CAP]
constexpr int L_O = L_R + CAP * 8;              // u32[CAP]
constexpr int L_POS = L_O + CAP * 4;            // u16[CAP]
constexpr int L_MEM = L_POS + CAP * 2;          // u16[CAP]
constexpr int L_BC = L_MEM + CAP * 2;           // u32[NSB] counts / fill
constexpr int L_BO = L_BC + NSB * 4;            // u32[NSB] offsets
constexpr int L_END = L_BO + NSB * 4;
// refinement: u32[NS] counts + f64[NS] sums + u32 counter (aliases the above)
constexpr int R_C = 0;
constexpr int R_S = NS * 4;
constexpr int R_N = R_S + NS * 8;
constexpr int R_END = R_N + 16;
// radix: u32[12][256] histograms + u32[16][256] wave counts + u32[256] bases + u32[256] tile
constexpr int X_H = 0;
constexpr int X_W = 12 * 256 * 4;
constexpr int X_B = X_W + NWAVE * 256 * 4;
constexpr int X_T = X_B + 256 * 4;
constexpr int X_END = X_T + 256 * 4;
constexpr int SMEM = L_END > R_END ? (L_END > X_END ? L_END : X_END) : (R_END > X_END ? R_END : X_END);
static_assert(SMEM <= 150 * 1024, "final kernel LDS");

// (a) c <= CAP candidates: bucket sort in LDS, exact prefix sums, first minimum
__device__ void final_lds(const Cand &src, unsigned c, const FinalIn &in, unsigned char *sm,
                          Scr &scr, IterState *st) {
    u64 *lk = (u64 *)(sm + L_K);
    double *lr = (double *)(sm + L_R);
    uint32_t *lo = (uint32_t *)(sm + L_O);
    uint16_t *pos = (uint16_t *)(sm + L_POS);
    uint16_t *mem = (uint16_t *)(sm + L_MEM);
    unsigned *bc = (unsigned *)(sm + L_BC);
    unsigned *bo = (unsigned *)(sm + L_BO);
    const int t = threadIdx.x;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = src.k[i];
        const uint32_t o = src.o[i];
        lk[i] = k;
        lo[i] = o;
        lr[i] = src.r[i];
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
    }
    for (int b = t; b < NSB; b += HT) bc[b] = 0u;
    blk_minmax_u64(kmn, kmx, scr);
    blk_minmax_u64(omn, omx, scr);
    const Comp cmp = make_comp(kmn, kmx, (uint32_t)omn, (uint32_t)omx);
    const u64 vspan = cmp(kmx, (uint32_t)omx);
    const int vb = bits_of(vspan);
    const int sh = vb > NSB_LOG ? vb - NSB_LOG : 0;
    for (unsigned i = t; i < c; i += HT) atomicAdd(&bc[(int)(cmp(lk[i], lo[i]) >> sh)], 1u);
    __syncthreads();
    {
        constexpr int PB = NSB / HT;  // 2 bins per thread
        unsigned v[PB];
        long long tot = 0;
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            v[j] = bc[t * PB + j];
            tot += v[j];
        }
        long long all;
        long long ex = blk_excl_scan_ll(tot, scr, all);
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            bo[t * PB + j] = (unsigned)ex;
            ex += v[j];
            bc[t * PB + j] = 0u;  // becomes the fill counter
        }
    }
    __syncthreads();
    for (unsigned i = t; i < c; i += HT) {
        const int b = (int)(cmp(lk[i], lo[i]) >> sh);
        mem[bo[b] + atomicAdd(&bc[b], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    // rank inside the bin (bins hold few rows unless keys cluster)
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = lk[i];
        const uint32_t o = lo[i];
        const int b = (int)(cmp(k, o) >> sh);
        const unsigned b0 = bo[b], nb = bc[b];
        unsigned rank = b0;
        for (unsigned j = b0; j < b0 + nb; ++j) {
            const unsigned e = mem[j];
            rank += less_ko(lk[e], lo[e], k, o) ? 1u : 0u;
        }
        pos[rank] = (uint16_t)i;
    }
    __syncthreads();
    // exact prefix sums in sorted order, FRMSD of every candidate k
    constexpr int PP = CAP / HT;  // 4 positions per thread
    double v[PP];
    double tsum = 0.0;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        const unsigned p = (unsigned)(t * PP + q);
        v[q] = p < c ? lr[pos[p]] : 0.0;
        tsum = tsum + v[q];
    }
    double all;
    double run = blk_excl_scan_d(tsum, scr, all);
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        const unsigned p = (unsigned)(t * PP + q);
        if (p < c) {
            run = run + v[q];
            const long long k = in.K0 + (long long)p + 1;
            const double f = frmsd_of(k, in.N, in.S0 + run, in.lam);
            if (f < bf) {
                bf = f;
                bk = k;
            }
        }
    }
    blk_argmin(bf, bk, scr);
    if (t == 0) {
        u64 tk = 0;
        uint32_t to = 0;
        if (bk != 0x7fffffffffffffffLL) {
            const unsigned e = pos[(unsigned)(bk - in.K0 - 1)];
            tk = lk[e];
            to = lo[e];
        }
        publish(st, in, bf, bk, tk, to);
    }
}

// (b) one refinement level over c > CAP candidates in global memory: returns false when
// it cannot shrink the set (the caller then sorts it)
__device__ bool refine(Cand &src, Cand &dst, unsigned &c, FinalIn &in, unsigned char *sm,
                       Scr &scr) {
    unsigned *rc = (unsigned *)(sm + R_C);
    double *rs = (double *)(sm + R_S);
    unsigned *rn = (unsigned *)(sm + R_N);
    const int t = threadIdx.x;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    double rmax = 0.0;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = src.k[i];
        const uint32_t o = src.o[i];
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
        rmax = fmax(rmax, src.r[i]);
    }
    for (int b = t; b < NS; b += HT) {
        rc[b] = 0u;
        rs[b] = 0.0;
    }
    if (t == 0) *rn = 0u;
    blk_minmax_u64(kmn, kmx, scr);
    blk_minmax_u64(omn, omx, scr);
    rmax = blk_max_d(rmax, scr);
    if (!(rmax < INFINITY)) return false;
    const Comp cmp = make_comp(kmn, kmx, (uint32_t)omn, (uint32_t)omx);
    const int vb = bits_of(cmp(kmx, (uint32_t)omx));
    if (vb == 0) return false;
    const int sh = vb > NS_LOG ? vb - NS_LOG : 0;
    for (unsigned i = t; i < c; i += HT) {
        const int b = (int)(cmp(src.k[i], src.o[i]) >> sh);
        atomicAdd(&rc[b], 1u);
        atomicAdd(&rs[b], src.r[i]);
    }
    __syncthreads();
    constexpr int PB = NS / HT;  // 4 sub-bins per thread
    unsigned cn[PB];
    double sv[PB];
    long long ct = 0;
    double stt = 0.0;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        cn[j] = rc[t * PB + j];
        sv[j] = rs[t * PB + j];
        ct += cn[j];
        stt = stt + sv[j];
    }
    long long ctot;
    double stot;
    const long long Cex = blk_excl_scan_ll(ct, scr, ctot);
    const double Pex = blk_excl_scan_d(stt, scr, stot);
    const double p = 2.0 * in.lam + 1.0;
    double U = in.U;
    {
        long long C = in.K0 + Cex;
        double P = in.S0 + Pex;
#pragma unroll
        for (int j = 0; j < PB; ++j)
            if (cn[j]) {
                C += cn[j];
                P = P + sv[j];
                U = fmin(U, h_of(C, P, p) + kMarg);
            }
    }
    U = blk_min_d(U, scr);
    long long bmin = 0x7fffffffLL, bmax = -1, nfirst = 0x7fffffffLL, nlast = -1;
    {
        long long C = in.K0 + Cex;
        double P = in.S0 + Pex;
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int b = t * PB + j;
            if (cn[j]) {
                nfirst = min(nfirst, (long long)b);
                nlast = max(nlast, (long long)b);
                const double lb = block_lb(C, cn[j], P, lo_r(cmp.key_lo((u64)b << sh)), p);
                if (!(lb > U) || !(p >= 1.0)) {
                    bmin = min(bmin, (long long)b);
                    bmax = max(bmax, (long long)b);
                }
                C += cn[j];
                P = P + sv[j];
            }
        }
    }
    bmin = blk_min_ll(bmin, scr);
    bmax = blk_max_ll(bmax, scr);
    nfirst = blk_min_ll(nfirst, scr);
    nlast = blk_max_ll(nlast, scr);
    if (bmax < 0 || (bmin == nfirst && bmax == nlast)) return false;
    // rows that drop below the new range: exact integer sum on the grid 2^(e - 96)
    const int e = rmax > 0.0 ? ilogb(rmax) : 0;
    const int L = e - 96;
    u128 acc = 0;
    long long below = 0;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = src.k[i];
        const uint32_t o = src.o[i];
        const double rv = src.r[i];
        const int b = (int)(cmp(k, o) >> sh);
        if (b < bmin) {
            below += 1;
            const u64 bitsr = (u64)__double_as_longlong(rv);
            const int ex = (int)((bitsr >> 52) & 0x7ff);
            u64 m = bitsr & 0xfffffffffffffULL;
            int p2;
            if (ex == 0) {
                p2 = -1074;
            } else {
                m |= 1ULL << 52;
                p2 = ex - 1075;
            }
            const int sft = p2 - L;
            if (sft >= 0) acc += (u128)m << sft;
            else if (sft > -64) acc += (u128)(m >> (-sft));
        } else if (b <= bmax) {
            const unsigned slot = atomicAdd(rn, 1u);
            dst.k[slot] = k;
            dst.o[slot] = o;
            dst.r[slot] = rv;
        }
    }
    // integer sums are order-free: reduce hi/lo with carries through LDS
    u64 *hi = (u64 *)(sm + R_S);  // sub-bin sums are no longer needed
    u64 *lo64 = hi + HT;
    long long *cnt = (long long *)(lo64 + HT);
    __syncthreads();
    hi[t] = (u64)(acc >> 64);
    lo64[t] = (u64)acc;
    cnt[t] = below;
    __syncthreads();
    for (int wdt = HT / 2; wdt > 0; wdt >>= 1) {
        if (t < wdt) {
            const u128 a = ((u128)hi[t] << 64) | lo64[t];
            const u128 b = ((u128)hi[t + wdt] << 64) | lo64[t + wdt];
            const u128 s = a + b;
            hi[t] = (u64)(s >> 64);
            lo64[t] = (u64)s;
            cnt[t] += cnt[t + wdt];
        }
        __syncthreads();
    }
    const double add = ldexp((double)hi[0], L + 64) + ldexp((double)lo64[0], L);
    const long long nbelow = cnt[0];
    const unsigned nc = *rn;
    __syncthreads();
    in.S0 = in.S0 + add;
    in.K0 += nbelow;
    in.U = U;
    c = nc;
    Cand tmp = src;
    src = dst;
    dst = tmp;
    return true;
}

// (c) in-workgroup stable LSD radix sort of the candidates by (key, orig), then the scan
__device__ void final_radix(Cand &src, Cand &dst, unsigned c, const FinalIn &in,
                            unsigned char *sm, Scr &scr, IterState *st) {
    unsigned *hist = (unsigned *)(sm + X_H);
    unsigned *wc = (unsigned *)(sm + X_W);
    unsigned *gb = (unsigned *)(sm + X_B);
    unsigned *tt = (unsigned *)(sm + X_T);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = src.k[i];
        const uint32_t o = src.o[i];
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
    }
    blk_minmax_u64(kmn, kmx, scr);
    blk_minmax_u64(omn, omx, scr);
    const int po = (bits_of(omx - omn) + 7) / 8, pk = (bits_of(kmx - kmn) + 7) / 8;
    const int np = po + pk;  // <= 4 + 8
    for (int j = t; j < 12 * 256; j += HT) hist[j] = 0u;
    __syncthreads();
    auto digit = [&](u64 k, uint32_t o, int p) -> unsigned {
        return p < po ? (unsigned)(((o - (uint32_t)omn) >> (8 * p)) & 0xffu)
                      : (unsigned)(((k - kmn) >> (8 * (p - po))) & 0xffu);
    };
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = src.k[i];
        const uint32_t o = src.o[i];
        for (int p = 0; p < np; ++p) atomicAdd(&hist[p * 256 + digit(k, o, p)], 1u);
    }
    __syncthreads();
    for (int p = 0; p < np; ++p) {
        {
            const long long v = t < 256 ? (long long)hist[p * 256 + t] : 0;
            long long all;
            const long long ex = blk_excl_scan_ll(v, scr, all);
            if (t < 256) gb[t] = (unsigned)ex;
        }
        __syncthreads();
        for (unsigned t0 = 0; t0 < c; t0 += HT) {
            const unsigned i = t0 + t;
            const bool valid = i < c;
            u64 k = 0;
            uint32_t o = 0;
            double rv = 0.0;
            unsigned d = 0;
            if (valid) {
                k = src.k[i];
                o = src.o[i];
                rv = src.r[i];
                d = digit(k, o, p);
            }
            u64 m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const u64 bb = __ballot(valid && ((d >> b) & 1u));
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const unsigned lr = (unsigned)__popcll(m & ((1ULL << lane) - 1ULL));
            for (int j = t; j < NWAVE * 256; j += HT) wc[j] = 0u;
            __syncthreads();
            if (valid && lr == 0) wc[wave * 256 + d] = (unsigned)__popcll(m);
            __syncthreads();
            if (t < 256) {
                unsigned run = 0;
                for (int w2 = 0; w2 < NWAVE; ++w2) {
                    const unsigned x = wc[w2 * 256 + t];
                    wc[w2 * 256 + t] = run;
                    run += x;
                }
                tt[t] = run;
            }
            __syncthreads();
            if (valid) {
                const unsigned q = gb[d] + wc[wave * 256 + d] + lr;
                dst.k[q] = k;
                dst.o[q] = o;
                dst.r[q] = rv;
            }
            __syncthreads();
            if (t < 256) gb[t] += tt[t];
            __syncthreads();
        }
        Cand tmp = src;
        src = dst;
        dst = tmp;
        __threadfence_block();
        __syncthreads();
    }
    // scan of the sorted candidates in chunks of HT rows
    double carry = 0.0;
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    for (unsigned t0 = 0; t0 < c; t0 += HT) {
        const unsigned i = t0 + t;
        const double v = i < c ? src.r[i] : 0.0;
        double all;
        const double ex = blk_excl_scan_d(v, scr, all);
        if (i < c) {
            const double run = (carry + ex) + v;
            const long long k = in.K0 + (long long)i + 1;
            const double f = frmsd_of(k, in.N, in.S0 + run, in.lam);
            if (f < bf) {
                bf = f;
                bk = k;
            }
        }
        carry = carry + all;
    }
    blk_argmin(bf, bk, scr);
    if (t == 0) {
        u64 tk = 0;
        uint32_t to = 0;
        if (bk != 0x7fffffffffffffffLL) {
            const unsigned e = (unsigned)(bk - in.K0 - 1);
            tk = src.k[e];
            to = src.o[e];
        }
        publish(st, in, bf, bk, tk, to);
    }
}

// With fuse_loop, thread 0 also runs the loop step of k_loop_update (ficp.py:122-154)
// and, with host_flag, stores the state's done flag to that (coherent pinned) host word.
__global__ __launch_bounds__(HT) void k_sel_final(SelWS w, int nparts, int64_t N, double lam,
                                                  const double *lam_dev, IterState *st,
                                                  const int *skip, LoopCtl lc, int fuse_loop,
                                                  int *host_flag) {
    if (skip && *skip) {
        if (host_flag && threadIdx.x == 0)
            __hip_atomic_store(host_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (lam_dev) lam = *lam_dev;
    __shared__ __align__(16) unsigned char sm[SMEM];
    __shared__ Scr scr;
    __shared__ IterState s_st;  // thread 0's working copy of the state (one load, one store)
    const int t = threadIdx.x;
    if (t == 0) s_st = *st;
    double a = 0.0;
    for (int p = t; p < nparts; p += HT) a = a + w.parts[p];  // fixed order per thread
    FinalIn in;
    in.N = N;
    in.lam = lam;
    in.S0 = blk_sum(a, scr);
    in.K0 = w.ctl->kbase;
    in.U = w.ctl->U;
    unsigned c = __hip_atomic_fetch_add(&w.ctl->ccount, 0u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    if (c == 0) {
        if (t == 0) {
            __hip_atomic_fetch_or(&w.ctl->err, ERR_EMPTY, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
            publish(&s_st, in, INFINITY, 0x7fffffffffffffffLL, 0, 0);
        }
    } else {
        Cand src{w.ka, w.oa, w.ra}, dst{w.kb, w.ob, w.rb};
        int lev = 0;
        bool stalled = false;
        while (c > (unsigned)CAP && lev < MAXLEV && !stalled) {
            stalled = !refine(src, dst, c, in, sm, scr);
            if (!stalled) ++lev;
            __threadfence_block();
            __syncthreads();
        }
        if (t == 0) w.ctl->levels += lev;
        if (c <= (unsigned)CAP) {
            final_lds(src, c, in, sm, scr, &s_st);
        } else {
            if (t == 0) w.ctl->radix += 1;
            final_radix(src, dst, c, in, sm, scr, &s_st);
        }
    }
    if (t == 0) {
        if (fuse_loop) loop_step(&s_st, lc);
        *st = s_st;
        if (host_flag)
            __hip_atomic_store(host_flag, s_st.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_sel_init(SelWS w) {
    for (int b = threadIdx.x; b < NB; b += blockDim.x) {
        __hip_atomic_exchange(&w.hcnt[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_exchange(&w.hfix[b], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
        __hip_atomic_exchange(&w.ctl->ccount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_exchange(&w.ctl->err, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w.ctl->levels = 0;
        w.ctl->radix = 0;
    }
}

__global__ void k_sel_read_stats(SelWS w, unsigned *out) {
    if (threadIdx.x == 0) {
        out[0] = __hip_atomic_fetch_or(&w.ctl->err, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[1] = w.ctl->levels;
        out[2] = w.ctl->radix;
    }
}

}  // namespace

int64_t sel_tmp_bytes(int64_t n) {
    const int64_t nn = std::max<int64_t>(n, 1);
    return align_up(NB * 4, 256) + align_up(NB * 8, 256) + 256 +
           align_up((int64_t)gather_blocks(n) * 8, 256) + 4 * align_up(nn * 8, 256) +
           2 * align_up(nn * 4, 256) + 256;
}

hipError_t launch_select_init(void *tmp, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(1024), 0, s, carve(tmp, n));
    return hipGetLastError();
}

hipError_t launch_select_stats(void *tmp, int64_t n, unsigned *out3, hipStream_t s) {
    hipLaunchKernelGGL(k_sel_read_stats, dim3(1), dim3(64), 0, s, carve(tmp, n), out3);
    return hipGetLastError();
}

hipError_t launch_select(const unsigned long long *key, const uint32_t *orig, const double *r,
                         int64_t n, double lam, const double *lam_dev, unsigned long long *range,
                         int64_t range_parts, void *tmp, IterState *st, const int *skip,
                         const LoopCtl *loop, int *host_flag, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const SelWS w = carve(tmp, n);
    hipLaunchKernelGGL(k_sel_hist, dim3(hist_blocks(n)), dim3(HT), 0, s, key, r, n, range,
                       range_parts, w, skip);
    hipLaunchKernelGGL(k_sel_bounds, dim3(1), dim3(HT), 0, s, w, n, lam, lam_dev,
                       (const unsigned long long *)range, skip);
    const int gb = gather_blocks(n);
    hipLaunchKernelGGL(k_sel_gather, dim3(gb), dim3(GT), 0, s, key, orig, r, n, w, skip);
    LoopCtl lc{};
    if (loop) lc = *loop;
    hipLaunchKernelGGL(k_sel_final, dim3(1), dim3(HT), 0, s, w, gb, n, lam, lam_dev, st, skip, lc,
                       loop ? 1 : 0, host_flag);
    return hipGetLastError();
}

}  // namespace ficp
