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
//                     stored per workgroup; k_sel_reduce adds the workgroups' copies.
//  2. k_sel_bounds  : one workgroup; prefix counts/sums over the buckets; U = the
//                     smallest FRMSD upper bound at any bucket end; candidate buckets
//                     [b0, b1] = those whose lower bound is <= U.  The true first
//                     minimum lies inside them.
//  3. k_sel_gather  : one pass: S_base = sum of r below b0 (fixed reduction tree, so
//                     bitwise deterministic), candidates (key, orig, r) appended.
//  4. k_sel_final   : one workgroup; (a) <= 4096 candidates: LDS bucket sort by
//                     (key, orig), exact prefix sums S_base + ..., FRMSD of every
//                     candidate k, first minimum (strict <, ficp.py:84); (b) more:
//                     refinement levels with 4096 sub-bins (exact integer sums of the
//                     rows that drop below, so still deterministic); (c) if that stalls
//                     (clustered or equal keys), an in-workgroup LSD radix sort.
// Level-0 bucket sums are bracketed exactly (truncated fixed point: [fx, fx + c) units);
// the bounds are compared in the log2 domain with a 1e-9 margin (see kMarg).  The decided
// k and threshold pair depend only on the exact, deterministic prefix sums.
// At C3 (1M x 1M) the candidate set holds 15-5000 rows, so step (a) is the normal case.
#include "ficp_internal.h"
#include "frmsd_bounds.h"

#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>

namespace ficp {

namespace {

typedef unsigned long long u64;
typedef unsigned __int128 u128;

// phase timestamps of the final kernel (tools/selcheck built with -DSEL_PROF only)
#ifdef SEL_PROF
__device__ unsigned long long g_selprof[40];
__device__ unsigned long long g_selclk[40];
#define SELPROF(i)                                       \
    do {                                                 \
        __syncthreads();                                 \
        if (threadIdx.x == 0) {                          \
            g_selprof[i] = wall_clock64();               \
            g_selclk[i] = clock64();                     \
        }                                                \
    } while (0)
// the first gather block's own stamps (no barrier: the other blocks are not perturbed)
#define GPROF(i)                                                        \
    do {                                                                \
        if (blk == 0 && threadIdx.x == 0) g_selprof[i] = wall_clock64(); \
    } while (0)
__device__ unsigned g_selcalls;
// thread 0 of workgroup B stamps slot i (no barrier)
#define BPROF(B, i)                                                         \
    do {                                                                    \
        if (blockIdx.x == (B) && threadIdx.x == 0) g_selprof[i] = wall_clock64(); \
    } while (0)
#else
#define BPROF(B, i) \
    do {            \
    } while (0)
#define SELPROF(i) \
    do {           \
    } while (0)
#define GPROF(i) \
    do {         \
    } while (0)
#endif

constexpr int NB = 8192;     // level-0 buckets
constexpr int NB_LOG = 13;
constexpr int HT = 512;      // threads of the bounds / final kernels (at 1024 they spilled)
constexpr int NWAVE = HT / 64;
constexpr int HHT = 1024;    // threads of the histogram kernel (33 VGPRs)
constexpr int CAP = 4096;    // candidates sorted in LDS with their r (the common case)
constexpr int CAP2 = 8192;   // candidates sorted in LDS with r left in global memory
constexpr int NSB = 2048;    // bins of the LDS bucket sort
constexpr int NSB_LOG = 11;
constexpr int NS = 4096;     // sub-bins of one refinement level
constexpr int NS_LOG = 12;
constexpr int MAXLEV = 4;
// window path (k_sel_win): rows a workgroup may hand over, coarse buckets per side of the
// window (4 per octave of distance), record words per workgroup, arrival counter stride
constexpr int NCS = fb::kWinNCS;
constexpr int NCB = 2 * NCS;
constexpr int WCTR = 64;
constexpr int SMALL_C = 160;  // final_small: above it the binned sort ranks faster (390: 5.8 vs 3.4 us)
#ifndef FICP_GT
#define FICP_GT 512
#endif
#ifndef FICP_GI
#define FICP_GI 8
#endif
constexpr int GT = FICP_GT;  // gather: threads per block
constexpr int GI = FICP_GI;  // gather: rows per thread (~1 block per CU at 1M rows; 512 x 8
                             // measured +1 % over 256 x 16 and 256 x 8)

// error bits of SelCtl::err (sticky; the host checks them after a run)
constexpr unsigned ERR_EMPTY = 1u;  // candidate set empty (cannot happen with finite r)
constexpr unsigned ERR_CAP = 2u;    // distributed run: a rank's candidates exceeded the capacity
constexpr unsigned ERR_SPIN = 4u;   // k_sel_bounds_gather: the bounds flag never came (bounded wait)

constexpr int NL = 2048, NF = 4096, NF_LOG = 12, NC_LOG = 11;
static_assert(NL + NF + NL == NB, "bucket map regions");
struct BMap {
    u64 kmin, kmax, wlo, whi;  // fine window [wlo, whi) (win)
    int s;                     // uniform shift (!win)
    int sl, sf, sh;            // shifts of the low / fine / high regions (win)
    int win, pad;
};

struct SelCtl {
    BMap map;              // level-0 bucket map of this call (k_sel_hist, block 0)
    int b0, b1;
    long long kbase;       // rows in buckets < b0
    double U;              // upper bound of h (log2 domain) at the minimum
    unsigned ccount;       // candidates appended (agent-scope atomics only)
    unsigned err;          // sticky error bits (agent-scope atomics only)
    unsigned levels;       // statistics: refinement levels run (plain, final kernel only)
    unsigned radix;        // statistics: radix fallbacks (plain, final kernel only)
    unsigned pad_;
    u64 bpub;              // k_sel_bounds_gather: (launch token << 32) | (b0 << 16) | b1
};
// the run's report copies {err, levels, radix} as three words from sel_err_word()
static_assert(offsetof(SelCtl, levels) == offsetof(SelCtl, err) + 4 &&
                  offsetof(SelCtl, radix) == offsetof(SelCtl, err) + 8,
              "SelCtl statistics words must follow err");

struct SelWS {
    unsigned *hcnt;  // [NB] reduced counts (plain stores, k_sel_reduce)
    double *hlo;     // [NB] bracket of each bucket's sum of r (plain stores, k_sel_reduce)
    double *hhi;
    unsigned *acnt;  // [NB / 16] per 16-bucket chunk: count and the two sums, in bucket order
    double *alo;     //   (k_sel_reduce; the bounds kernel's per-thread chunk totals)
    double *ahi;
    u64 *ppk;        // [HBMAX][NB] per-block (count << shift) + fixed-point sum (plain stores)
    SelCtl *ctl;
    double *parts;   // [gather blocks]
    double *fparts;  // [gather blocks][8] fit sums of the rows below the candidates
    u64 *ka, *kb;    // candidate ping-pong buffers (n each)
    uint32_t *oa, *ob;
    double *ra, *rb;
    uint32_t *pa, *pb;  // candidate row (work position): the fused fit reads its pair
    double *fpre;    // [CAP][4] fused fit: the pair of pack slots < CAP (gather)
    // the window path (k_sel_win):
    unsigned *gcc;   // [copies][NCB] coarse bucket counts (agent-scope atomics; the last
    u64 *gcf;        //   workgroup reads and zeroes them with exchanges) and fixed-point sums
    unsigned *wctr;  // arrival counters: top + 8 groups, WCTR words apart (atomics only)
    u64 *wacc;       // [copies][WACC] the workgroups' totals (atomics; the tail zeroes them)
    unsigned *wcnt;  // [copies][WCNT_S] window-row append counters (atomics, zeroed likewise)
    u64 *wk;         // [copies][CAP] the window rows appended: key, r, caller index and
    double *wr;      //   the fit pair (xs, ys, cx, cy)
    uint32_t *wo;
    double *wp;
};

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
inline int gather_blocks(int64_t n) { return (int)std::max<int64_t>(1, (n + GT * GI - 1) / (GT * GI)); }
// Histogram blocks: each writes its whole LDS histogram (12 B per bucket) with plain
// stores and k_sel_reduce sums them.  Global atomics execute at the memory side at one
// wave-instruction per ~50 ns per CU (MI355X_MICROARCH.md, global atomics), so flushing
// 8192 buckets with atomics cost ~15 us and reading + resetting them from one CU ~25 us.
#ifndef FICP_HIST_ROWS
#define FICP_HIST_ROWS 4096  // 256 x 4096 rows: +0.5 % at C3 over 128 x 8192 (tools/ab_bench.sh, round 3)
#endif
#ifndef FICP_HBMAX
#define FICP_HBMAX 256
#endif
constexpr int HBMAX = FICP_HBMAX;
constexpr int HROWS = FICP_HIST_ROWS;  // rows per histogram block (target)
inline int hist_blocks(int64_t n) { return (int)std::min<int64_t>(HBMAX, std::max<int64_t>(1, (n + HROWS - 1) / HROWS)); }

// One 64-bit LDS atomic per row: (1 << shift) + m, the count in the top cbits (a block
// holds at most `per` rows) and the fixed-point value m < 2^fixb below it with room for
// per of them.  fixb = 37 up to ~8K rows per block (relative truncation < 2^-35); the
// bracket [fx, fx + c) stays rigorous for any fixb, a smaller one only widens it.
struct HistPack {
    int shift, fixb;
};
inline HistPack hist_pack(int64_t n) {
    const int64_t nhb = hist_blocks(n);
    const int64_t per = (std::max<int64_t>(n, 1) + nhb - 1) / nhb;
    int cb = 1;
    while ((((int64_t)1) << cb) <= per) ++cb;
    HistPack h;
    h.shift = 64 - cb;
    h.fixb = std::min(37, h.shift - cb);
    return h;
}

// workspace layout; carve() and sel_tmp_bytes() share it
int64_t carve_bytes(int64_t n, SelWS *w, char *p0) {
    char *p = p0;
    auto take = [&](int64_t bytes) {
        char *q = p;
        p += align_up(bytes, 256);
        return q;
    };
    const int64_t nn = std::max<int64_t>(n, 1);
    SelWS x;
    x.hcnt = (unsigned *)take(NB * 4);
    x.hlo = (double *)take(NB * 8);
    x.hhi = (double *)take(NB * 8);
    x.acnt = (unsigned *)take(NB / 16 * 4);
    x.alo = (double *)take(NB / 16 * 8);
    x.ahi = (double *)take(NB / 16 * 8);
    x.ppk = (u64 *)take((int64_t)HBMAX * NB * 8);
    x.ctl = (SelCtl *)take(256);
    // the words kept zero by the kernels themselves (zeroed once, k_sel_init) sit at offsets
    // that do not depend on n: a context's workspace serves later runs of any smaller n
    x.gcc = (unsigned *)take(kWinCopies * NCB * 4);
    x.gcf = (u64 *)take(kWinCopies * NCB * 8);
    x.wctr = (unsigned *)take(9 * WCTR * 4);
    x.wacc = (u64 *)take(kWinCopies * 32 * 8);
    x.wcnt = (unsigned *)take(kWinCopies * 16 * 4);
    // the window rows: kWinCopies regions of CAP, appended
    const int64_t nwr = (int64_t)kWinCopies * CAP;
    x.wk = (u64 *)take(nwr * 8);
    x.wr = (double *)take(nwr * 8);
    x.wo = (uint32_t *)take(nwr * 4);
    x.wp = (double *)take(nwr * 32);
    x.parts = (double *)take((int64_t)gather_blocks(n) * 8);
    x.fparts = (double *)take((int64_t)gather_blocks(n) * 64);
    x.ka = (u64 *)take(nn * 8);
    x.kb = (u64 *)take(nn * 8);
    x.ra = (double *)take(nn * 8);
    x.rb = (double *)take(nn * 8);
    x.oa = (uint32_t *)take(nn * 4);
    x.ob = (uint32_t *)take(nn * 4);
    x.pa = (uint32_t *)take(nn * 4);
    x.pb = (uint32_t *)take(nn * 4);
    x.fpre = (double *)take(CAP * 32);
    if (w) *w = x;
    return (int64_t)(p - p0) + 256;
}

SelWS carve(void *tmp, int64_t n) {
    SelWS w;
    carve_bytes(n, &w, (char *)tmp);
    return w;
}

using fb::bits_of;
using fb::block_lb;
using fb::h_of;
using fb::kMarg;
using fb::lg2;
using fb::lo_r;

__device__ __forceinline__ int sel_shift(u64 kmin, u64 kmax) {
    const int b = bits_of(kmax > kmin ? kmax - kmin : 0ULL);
    return b > NB_LOG ? b - NB_LOG : 0;
}

// Bucket map of the level-0 histogram.  Uniform (a stage's first call): NB buckets of
// 2^s keys from kmin.  Windowed (the stage's later calls): the previous call's threshold
// key c gets NF fine buckets of 2^sf keys around it (half-width >= 64 uniform buckets and
// >= 4x the threshold's last move), the keys below and above the window NL coarse buckets
// each.  The threshold moves little from call to call (C3: < 1 uniform bucket after the
// third call), so the new candidate buckets fall in the fine part and hold ~1/32 of the
// rows.  Any monotone map keeps the bounds rigorous: each bucket's key range gives the
// lower r (lo_r of bucket_lo) and the fixed-point exponent (bucket_hi) of its rows.

// what the map needs from the previous call (loaded early by k_sel_hist)
struct BPrev {
    u64 tkey, tmove;
    int ok;
};
__device__ __forceinline__ BPrev bprev_of(const IterState *st) {
    BPrev v{0ULL, 0ULL, 0};
    if (st) {
        v.ok = st->phase == PH_LOOP && st->k > 0;
        v.tkey = st->tkey;
        v.tmove = st->tmove;
    }
    return v;
}

__device__ __forceinline__ BMap make_bmap(u64 kmin, u64 kmax, const BPrev &pv) {
    BMap m{};
    m.kmin = kmin;
    m.kmax = kmax;
    m.s = sel_shift(kmin, kmax);
    if (!pv.ok || m.s < 8) return m;
    const u64 c = pv.tkey;
    if (c < kmin || c > kmax) return m;
    const u64 mv = pv.tmove;
    u64 H = (u64)64 << m.s;
    if (mv < ((u64)1 << 60) && 4 * mv > H) H = 4 * mv;
    const int sf = max(0, bits_of(2 * H - 1) - NF_LOG);  // NF << sf >= 2 H
    if (sf > m.s - 3) return m;                          // not >= 8x finer: uniform
    const u64 W = (u64)NF << sf;
    u64 wlo = c - min(c - kmin, W / 2);
    if (kmax - wlo < W - 1) {
        if (kmax - kmin < W - 1) return m;
        wlo = kmax - (W - 1);
    }
    m.wlo = wlo;
    m.whi = wlo + W;
    m.sf = sf;
    m.sl = wlo > kmin ? max(0, bits_of(wlo - 1 - kmin) - NC_LOG) : 0;
    m.sh = m.whi <= kmax ? max(0, bits_of(kmax - m.whi) - NC_LOG) : 0;
    m.win = 1;
    return m;
}

__device__ __forceinline__ int bucket_of(const BMap &m, u64 k) {
    if (!m.win) return (int)((k - m.kmin) >> m.s);
    if (k < m.wlo) return (int)((k - m.kmin) >> m.sl);
    if (k < m.whi) return NL + (int)((k - m.wlo) >> m.sf);
    return NL + NF + (int)((k - m.whi) >> m.sh);
}

// lowest key of bucket b
__device__ __forceinline__ u64 bucket_lo(const BMap &m, int b) {
    if (!m.win) return m.kmin + ((u64)b << m.s);
    if (b < NL) return m.kmin + ((u64)b << m.sl);
    if (b < NL + NF) return m.wlo + ((u64)(b - NL) << m.sf);
    return m.whi + ((u64)(b - NL - NF) << m.sh);
}

// highest key of sub-bucket j (width 2^sh) from base, clipped to lim; (j + 1) << sh wraps
// to 0 only at 2^64 (j < 8192, sh <= 51), and then the clip applies
__device__ __forceinline__ u64 span_hi(u64 base, u64 lim, int j, int sh) {
    const u64 wdt = ((u64)(j + 1) << sh) - 1ULL;
    return wdt > lim - base ? lim : base + wdt;
}

// highest key any row of bucket b can have
__device__ __forceinline__ u64 bucket_hi(const BMap &m, int b) {
    if (!m.win) return span_hi(m.kmin, m.kmax, b, m.s);
    if (b < NL) return span_hi(m.kmin, m.wlo - 1, b, m.sl);
    if (b < NL + NF) return span_hi(m.wlo, min(m.whi - 1, m.kmax), b - NL, m.sf);
    return span_hi(m.whi, m.kmax, b - NL - NF, m.sh);
}

// exponent e_b with r < 2^e_b for every row of bucket b (1024: the bucket holds inf/NaN)
__device__ __forceinline__ int bucket_exp(const BMap &m, int b) {
    const u64 khi = bucket_hi(m, b);
    if (!(khi >> 63)) return 0;
    // from the bits of d_hi alone (no fp64 work): d < 2^(ex - 1022) for biased exponent ex,
    // so r = d^2 < 2^(2 ex - 2044); at most one bit looser than the exponent of d_hi^2
    const int ex = (int)((khi >> 52) & 0x7ffULL);
    return min(2 * ex - 2044, 1024);  // 1024: the bucket may hold inf / NaN or overflow
}

// Bounds work on h(k, S) (frmsd_bounds.h): no pow per bucket.

__device__ __forceinline__ bool better(double f, long long k, double bf, long long bk) {
    return f < bf || (f == bf && k < bk);
}

// ------------------------------------------------- block primitives (HT threads)
struct Scr {
    double f[8 * NWAVE];  // blk_sum8_add
    double d[NWAVE];
    long long l[NWAVE];
    u64 u[NWAVE];
    u64 v[NWAVE];
};

// deterministic: butterfly inside the wave (every lane ends with the same bits), wave
// partials in wave order
__device__ __forceinline__ double blk_sum(double x, Scr &s) {
    x = wave_sum63(x);
    if ((threadIdx.x & 63) == 63) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) t = t + s.d[w];
    __syncthreads();
    return t;
}

// acc8[e] += block sum of c[e] (thread 0 adds; fixed tree: wave butterfly, waves in order)
__device__ __forceinline__ void blk_sum8_add(double (&c)[8], double *acc8, Scr &s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = wave_sum63(c[e]);
    if ((threadIdx.x & 63) == 63)
#pragma unroll
        for (int e = 0; e < 8; ++e) s.f[8 * (threadIdx.x >> 6) + e] = c[e];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            double t = 0.0;
            for (int w = 0; w < NWAVE; ++w) t = t + s.f[8 * w + e];
            acc8[e] = acc8[e] + t;
        }
    }
    __syncthreads();
}

// fit contribution of work row i
__device__ __forceinline__ void fit_row(double (&c)[8], const FitSrc &fs, uint32_t i) {
    fit_add(c, fs.sx[i], fs.sy[i], fs.cx[i], fs.cy[i], fs.px, fs.py);
}

__device__ __forceinline__ double blk_min_d(double x, Scr &s) {
    x = wave_min63(x);
    if ((threadIdx.x & 63) == 63) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = s.d[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) t = fmin(t, s.d[w]);
    __syncthreads();
    return t;
}

__device__ __forceinline__ double blk_max_d(double x, Scr &s) {
    x = wave_max63(x);
    if ((threadIdx.x & 63) == 63) s.d[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = s.d[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) t = fmax(t, s.d[w]);
    __syncthreads();
    return t;
}

// {min, max} of two u64 quantities at once: returns min(a), max(b)
template <int NW = NWAVE>
__device__ __forceinline__ void blk_minmax_u64(u64 &a, u64 &b, u64 *su, u64 *sv) {
    // DPP steps (lane 63 ends with the wave's values; unwritten lanes read the neutral
    // values ~0 for the min and 0 for the max)
#define MINMAX_STEP(CTRL, ROWM)                                                       \
    {                                                                                 \
        const u64 xa = (u64)dpp::mov_ll<CTRL, ROWM>(-1LL, (long long)a);              \
        const u64 xb = (u64)dpp::mov_ll<CTRL, ROWM>(0, (long long)b);                 \
        a = xa < a ? xa : a;                                                          \
        b = xb > b ? xb : b;                                                          \
    }
    MINMAX_STEP(dpp::QP_XOR1, 0xf)
    MINMAX_STEP(dpp::QP_XOR2, 0xf)
    MINMAX_STEP(dpp::ROW_HALF_MIRROR, 0xf)
    MINMAX_STEP(dpp::ROW_MIRROR, 0xf)
    MINMAX_STEP(dpp::ROW_BCAST15, 0xA)
    MINMAX_STEP(dpp::ROW_BCAST31, 0xC)
#undef MINMAX_STEP
    if ((threadIdx.x & 63) == 63) {
        su[threadIdx.x >> 6] = a;
        sv[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    a = su[0];
    b = sv[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        a = su[w] < a ? su[w] : a;
        b = sv[w] > b ? sv[w] : b;
    }
    __syncthreads();
}

// min(a), max(b), min(c), max(d) in one reduction (one pair of barriers)
__device__ __forceinline__ void blk_minmax2_u64(u64 &a, u64 &b, u64 &c, u64 &d, Scr &s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u64 xa = __shfl_xor(a, o, 64), xb = __shfl_xor(b, o, 64);
        const u64 xc = __shfl_xor(c, o, 64), xd = __shfl_xor(d, o, 64);
        a = xa < a ? xa : a;
        b = xb > b ? xb : b;
        c = xc < c ? xc : c;
        d = xd > d ? xd : d;
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s.u[wv] = a;
        s.v[wv] = b;
        s.l[wv] = (long long)c;
        s.d[wv] = __longlong_as_double((long long)d);
    }
    __syncthreads();
    a = s.u[0];
    b = s.v[0];
    c = (u64)s.l[0];
    d = (u64)__double_as_longlong(s.d[0]);
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) {
        a = s.u[w] < a ? s.u[w] : a;
        b = s.v[w] > b ? s.v[w] : b;
        const u64 cw = (u64)s.l[w], dw = (u64)__double_as_longlong(s.d[w]);
        c = cw < c ? cw : c;
        d = dw > d ? dw : d;
    }
    __syncthreads();
}

__device__ __forceinline__ void blk_minmax_u64(u64 &a, u64 &b, Scr &s) {
    blk_minmax_u64<NWAVE>(a, b, s.u, s.v);
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
    const double x = wave_incl_scan_d(v);  // DPP (ficp_internal.h)
    if (lane == 63) s.d[wave] = x;
    const double ex = wave_shr1_d(x);
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
    const long long x = wave_incl_scan_ll(v);
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

// exclusive scans of a count and two sums at once (the same operations, in the same
// order, as blk_excl_scan_ll + two blk_excl_scan_d; one set of barriers)
__device__ __forceinline__ void blk_excl_scan3(long long &c, double &a, double &b, Scr &s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long xc = wave_incl_scan_ll(c);
    const double xa = wave_incl_scan_d(a), xb = wave_incl_scan_d(b);
    if (lane == 63) {
        s.l[wave] = xc;
        s.d[wave] = xa;
        s.u[wave] = (u64)__double_as_longlong(xb);
    }
    const double ea = wave_shr1_d(xa), eb = wave_shr1_d(xb);
    __syncthreads();
    long long oc = 0;
    double oa = 0.0, ob = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
        if (w < wave) {
            oc += s.l[w];
            oa = oa + s.d[w];
            ob = ob + __longlong_as_double((long long)s.u[w]);
        }
    }
    __syncthreads();
    c = oc + xc - c;
    a = wave ? oa + ea : ea;
    b = wave ? ob + eb : eb;
}

// block argmin of (f, k) with the first-minimum rule; result broadcast
__device__ __forceinline__ void blk_argmin(double &f, long long &k, Scr &s) {
    // DPP steps (fixed tree); a lane a step does not write keeps (inf, max): never better
#define ARGMIN_STEP(CTRL, ROWM)                                                      \
    {                                                                                \
        const double xf = dpp::mov_d<CTRL, ROWM>(INFINITY, f);                       \
        const long long xk = dpp::mov_ll<CTRL, ROWM>(0x7fffffffffffffffLL, k);       \
        if (better(xf, xk, f, k)) {                                                  \
            f = xf;                                                                  \
            k = xk;                                                                  \
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
__global__ __launch_bounds__(HHT) void k_sel_hist(const u64 *key, const double *r, int64_t n,
                                                 u64 *range, int64_t nparts, SelWS w,
                                                 const int *skip, HistPack hp,
                                                 const IterState *st) {
    BPROF(1, 30);
    const int sk = skip ? *skip : 0;  // checked after the first rows' loads have issued
    __shared__ u64 sp[NB];
    __shared__ u64 s_u[HHT / 64], s_v[HHT / 64];
#ifndef FICP_HIST_U
#define FICP_HIST_U 4
#endif
    constexpr int U = FICP_HIST_U;  // rows in flight per thread (8 measured -1 %)
    // this thread's first U rows and the previous call's threshold are loaded before the
    // range reduction, so their latency overlaps it
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * per, i1 = min(n, i0 + per);
    const int64_t ib = i0 + threadIdx.x;
    u64 kk[U];
    double rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t q = ib + (int64_t)u * HHT;
        kk[u] = (key && q < i1) ? key[q] : 0ULL;
        rv[u] = q < i1 ? r[q] : 0.0;
    }
    const BPrev pv = bprev_of(st);
    if (sk) return;
    for (int b = threadIdx.x; b < NB; b += HHT) sp[b] = 0ULL;
    u64 kmin, kmax;
    if (nparts > 0) {
        u64 a = 0, b = 0;
        // 4 parts in flight per thread (one load at a time serialised ~4 latencies)
        for (int64_t q0 = threadIdx.x; q0 < nparts; q0 += 4 * HHT) {
            ulonglong2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t q = q0 + (int64_t)u * HHT;
                v[u] = q < nparts ? *reinterpret_cast<const ulonglong2 *>(range + 2 + 2 * q)
                                  : ulonglong2{0ULL, 0ULL};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a = max(a, v[u].x);
                b = max(b, v[u].y);
            }
        }
        a = ~a;
        blk_minmax_u64<HHT / 64>(a, b, s_u, s_v);  // (its barriers also cover the LDS zeroing)
        kmin = a;
        kmax = b;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            range[0] = ~kmin;
            range[1] = kmax;
        }
    } else {
        kmin = ~range[0];
        kmax = range[1];
        __syncthreads();
    }
    // every block derives the same map; block 0 publishes it for the later kernels
    const BMap bm = make_bmap(kmin, kmax, pv);
    BPROF(1, 31);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        w.ctl->map = bm;
        // the candidate counter of this call starts at zero: reset here, a launch before
        // the gather's appends (k_sel_bounds_gather's block 0 then publishes the bounds
        // without first draining a reset of its own)
        __hip_atomic_exchange(&w.ctl->ccount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const u64 one = 1ULL << hp.shift;
    for (int64_t i = ib; i < i1; i += (int64_t)U * HHT) {
        if (i != ib) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = i + (int64_t)u * HHT;
                kk[u] = (key && q < i1) ? key[q] : 0ULL;
                rv[u] = q < i1 ? r[q] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + (int64_t)u * HHT < i1) {
                const int b = bucket_of(bm, key ? kk[u] : key_of_r(rv[u]));
                // r < 2^e for every row of the bucket, from the bucket's upper key bits
                // (a per-bucket LDS table cost its init and 16 KB: +1 % without it)
                const int e = bucket_exp(bm, b);
                const u64 m = (e < 1024 && rv[u] < INFINITY) ? (u64)ldexp(rv[u], hp.fixb - e) : 0ULL;
                atomicAdd(&sp[b], one + m);
            }
        }
    }
    __syncthreads();
    BPROF(1, 32);
    u64 *pp = w.ppk + (int64_t)blockIdx.x * NB;
    for (int b = threadIdx.x; b < NB; b += HHT) pp[b] = sp[b];
    BPROF(1, 33);
}

// sum of the per-block histograms (integer sums: exact, order-free).  RG thread groups
// per bucket each add a quarter of the copies, then LDS combines them: 32 copies per
// thread instead of 128 (the 32 workgroups of one thread per bucket were load-latency
// bound).
#ifndef FICP_SEL_RG
#define FICP_SEL_RG 16
#endif
constexpr int RG = FICP_SEL_RG;
constexpr int RBPB = 1024 / RG;  // buckets per workgroup
// the bucket's bracket and the 16-bucket chunk totals from its integer count and sum
// (lanes of one wave hold 64 consecutive buckets)
__device__ __forceinline__ void reduce_tail(const SelWS &w, int b, int bl, unsigned c, u64 f,
                                            const HistPack &hp);

__global__ __launch_bounds__(1024) void k_sel_reduce(SelWS w, int nhb, const int *skip,
                                                     HistPack hp, long long *iout) {
    const int sk = skip ? *skip : 0;  // checked after the copies' loads (no writes before)
    __shared__ unsigned s_c[RG][RBPB];
    __shared__ u64 s_f[RG][RBPB];
    const int bl = threadIdx.x % RBPB, g = threadIdx.x / RBPB;
    const int b = blockIdx.x * RBPB + bl;
    const u64 mask = (1ULL << hp.shift) - 1ULL;
    const int per = (nhb + RG - 1) / RG, q0 = g * per, q1 = min(nhb, q0 + per);
    unsigned c = 0;
    u64 f = 0;
    int q = q0;
    for (; q + 8 <= q1; q += 8) {
        u64 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = w.ppk[(int64_t)(q + u) * NB + b];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            c += (unsigned)(v[u] >> hp.shift);
            f += v[u] & mask;
        }
    }
    for (; q < q1; ++q) {
        const u64 v = w.ppk[(int64_t)q * NB + b];
        c += (unsigned)(v >> hp.shift);
        f += v & mask;
    }
    if (sk) return;
    s_c[g][bl] = c;
    s_f[g][bl] = f;
    __syncthreads();
    if (g != 0) return;
#pragma unroll
    for (int h = 1; h < RG; ++h) {
        c += s_c[h][bl];
        f += s_f[h][bl];
    }
    if (iout) {  // distributed run: this rank's integer totals, summed over ranks outside
        iout[b] = (long long)c;
        iout[NB + b] = (long long)f;
        return;
    }
    reduce_tail(w, b, bl, c, f, hp);
}

__device__ __forceinline__ void reduce_tail(const SelWS &w, int b, int bl, unsigned c, u64 f,
                                            const HistPack &hp) {
    // the bucket's sum bracketed by the truncated fixed-point sum (each row loses < 1
    // unit): f * 2^(e - fixb) <= sum < (f + c) * 2^(e - fixb); computed here, one bucket
    // per thread, instead of 16 per thread in the one-workgroup bounds kernel
    const int e = bucket_exp(w.ctl->map, b);
    double lo, hi;
    if (e >= 1024) {
        lo = hi = c ? INFINITY : 0.0;
    } else {
        lo = ldexp((double)f, e - hp.fixb);
        hi = ldexp((double)(f + c), e - hp.fixb);
    }
    w.hcnt[b] = c;
    w.hlo[b] = lo;
    w.hhi[b] = hi;
    // chunk totals of 16 consecutive buckets (lanes 16m..16m+15 of this wave), added in
    // bucket order by the chunk's first lane
    static_assert(RBPB == 64, "one wave of buckets per workgroup");
    const int l0 = bl & ~15;
    unsigned cs = 0;
    double ls = 0.0, hs = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        cs += (unsigned)__shfl((int)c, l0 + u, 64);
        ls = ls + __shfl(lo, l0 + u, 64);
        hs = hs + __shfl(hi, l0 + u, 64);
    }
    if ((bl & 15) == 0) {
        w.acnt[b >> 4] = cs;
        w.alo[b >> 4] = ls;
        w.ahi[b >> 4] = hs;
    }
}

// Bounds of the FRMSD curve over the level-0 buckets (one workgroup).  Per-thread
// chunks of PER consecutive buckets; the per-bucket work (two or four log2 each) runs
// only for the chunks that can hold the minimum, one bucket per lane (a chunk walked by
// its own thread serialised ~16 dependent evaluations: ~10 us at C3).
// an sc1 store (agent scope: written through for another workgroup of the same launch)
template <class T>
__device__ __forceinline__ void stc(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int MAXACT = HT / (NB / HT);  // active chunks evaluated one bucket per lane
// returns the candidate bucket range [b0, b1] packed as (b0 << 16) | b1 (every thread)
// (kBoundsSkipped when *skip: the launch is a no-op).  Every load that does not depend on
// another (skip flag, lambda, bucket map, chunk totals) issues before the first wait.
constexpr unsigned kBoundsSkipped = 0xffffffffu;
constexpr int BPER = NB / HT;
// bounds_body's LDS (its caller's: k_sel_bgf lays it over the final's buffer)
struct BoundsLds {
    Scr scr;
    int s_act[MAXACT];
    int s_nact;
    long long eC[MAXACT * BPER];  // rows before bucket j of active chunk a
    double eLo[MAXACT * BPER];    // lower sum before it
    double eHi[MAXACT * BPER];    // upper sum through it
    unsigned eN[MAXACT * BPER];   // its count
};
// The outputs (b0, b1, kbase, U) are stored sc1 and drained by the closing barrier, so a
// workgroup of the same launch that saw the published range may read them with sc1 loads
// (k_sel_bgf's final).
__device__ __forceinline__ unsigned bounds_body(SelWS w, int64_t N, double lam,
                                                const double *lam_dev, const int *skip,
                                                int fixb, BoundsLds &L, bool reset_ccount = true) {
    constexpr int PER = BPER;
    Scr &scr = L.scr;
    int *s_act = L.s_act;
    int &s_nact = L.s_nact;
    long long *eC = L.eC;
    double *eLo = L.eLo;
    double *eHi = L.eHi;
    unsigned *eN = L.eN;
    const int t = threadIdx.x;
    static_assert(PER == 16, "chunk totals of k_sel_reduce");
    // this thread's chunk of PER consecutive buckets: totals from k_sel_reduce; the
    // buckets themselves are loaded only by the chunks that stay active below
    const int sk = skip ? *skip : 0;
    const double lamv = lam_dev ? *lam_dev : lam;
    const BMap bm = w.ctl->map;
    const long long ct = w.acnt[t];
    const double tlo = w.alo[t], thi = w.ahi[t];
    unsigned cc[PER];
    double blo[PER], bhi[PER];
#ifndef FICP_BOUNDS_PRELOAD
#define FICP_BOUNDS_PRELOAD 0
#endif
    // FICP_BOUNDS_PRELOAD=1: every thread loads its 16 buckets with the chunk totals (one
    // round of loads, 160 KB) instead of only the active chunks after U1 (a second,
    // dependent round): 136 VGPRs for the gather blocks too, measured 4-5 % slower at C3
    // (8,140 vs 8,486-8,555 it/s, tools/ab_bench.sh, round 3)
    auto load_buckets = [&]() {
#pragma unroll
        for (int j = 0; j < PER; j += 4) {
            const uint4 c4 = *reinterpret_cast<const uint4 *>(w.hcnt + t * PER + j);
            const double2 l0 = *reinterpret_cast<const double2 *>(w.hlo + t * PER + j);
            const double2 l1 = *reinterpret_cast<const double2 *>(w.hlo + t * PER + j + 2);
            const double2 h0 = *reinterpret_cast<const double2 *>(w.hhi + t * PER + j);
            const double2 h1 = *reinterpret_cast<const double2 *>(w.hhi + t * PER + j + 2);
            cc[j] = c4.x;
            cc[j + 1] = c4.y;
            cc[j + 2] = c4.z;
            cc[j + 3] = c4.w;
            blo[j] = l0.x;
            blo[j + 1] = l0.y;
            blo[j + 2] = l1.x;
            blo[j + 3] = l1.y;
            bhi[j] = h0.x;
            bhi[j + 1] = h0.y;
            bhi[j + 2] = h1.x;
            bhi[j + 3] = h1.y;
        }
    };
    if (FICP_BOUNDS_PRELOAD) load_buckets();
    if (sk) return kBoundsSkipped;
    lam = lamv;
    SELPROF(8);
    if (t == 0) s_nact = 0;
    SELPROF(9);
    long long Cex = ct;
    double Plo = tlo, Phi = thi;
    blk_excl_scan3(Cex, Plo, Phi, scr);
    SELPROF(10);
    // U: the smallest upper bound of h at any bucket end.  Evaluated coarse to fine, with
    // the same result as evaluating every bucket: (1) U1 = the bound at each thread's
    // chunk end; (2) a chunk whose lower bound (its rows are all >= the first bucket's
    // lo_r) exceeds U1 can neither hold the minimising bucket end nor a candidate bucket;
    // (3) only the remaining chunks (a few, near the minimum) evaluate their buckets.
    const double p = 2.0 * lam + 1.0;
    const double Pend = Phi + thi;
    double U1 = ct ? h_of(Cex + ct, Pend, p) + kMarg : INFINITY;
    U1 = blk_min_d(U1, scr);
    SELPROF(11);
    // (the extra 1e-9 covers the fixed-point truncation of the per-bucket lower sums, so
    // that a chunk's bound never exceeds the bound of a bucket inside it)
    const bool active = ct && (!(block_lb(Cex, ct, Plo, lo_r(bucket_lo(bm, t * PER)), p) -
                                       1e-9 > U1) ||
                               !(p >= 1.0));
    if (active) {
        if (!FICP_BOUNDS_PRELOAD) load_buckets();
        const int a = atomicAdd(&s_nact, 1);
        if (a < MAXACT) {
            s_act[a] = t;
            long long C = Cex;
            double PL = Plo, PH = Phi;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                eC[a * PER + j] = C;
                eLo[a * PER + j] = PL;
                eN[a * PER + j] = cc[j];
                C += cc[j];
                PL = PL + blo[j];
                PH = PH + bhi[j];
                eHi[a * PER + j] = PH;
            }
        }
    }
    __syncthreads();
    const int nact = s_nact;
    double U = INFINITY;
    long long bmin = 0x7fffffffLL, bmax = -1, kb = 0;
    if (nact <= MAXACT) {
        // one bucket per lane: work item q = (active chunk q / PER, bucket q % PER)
        for (int q = t; q < nact * PER; q += HT) {
            const unsigned c = eN[q];
            if (c) U = fmin(U, h_of(eC[q] + c, eHi[q], p) + kMarg);
        }
        U = fmin(blk_min_d(U, scr), U1);
        SELPROF(12);
        for (int q = t; q < nact * PER; q += HT) {
            const int b = s_act[q / PER] * PER + (q % PER);
            const unsigned c = eN[q];
            if (c) {
                const double lb = block_lb(eC[q], c, eLo[q], lo_r(bucket_lo(bm, b)), p);
                if (!(lb > U) || !(p >= 1.0)) {
                    if (b < bmin) kb = eC[q];  // rows before this lane's first candidate
                    bmin = min(bmin, (long long)b);
                    bmax = max(bmax, (long long)b);
                }
            }
        }
    } else {  // many active chunks: every active thread walks its own buckets
        if (active) {
            long long C = Cex;
            double P = Phi;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                if (cc[j]) {
                    C += cc[j];
                    P = P + bhi[j];
                    U = fmin(U, h_of(C, P, p) + kMarg);
                }
            }
        }
        U = fmin(blk_min_d(U, scr), U1);
        SELPROF(12);
        if (active) {
            long long C = Cex;
            double P = Plo;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int b = t * PER + j;
                if (cc[j]) {
                    const double lb = block_lb(C, cc[j], P, lo_r(bucket_lo(bm, b)), p);
                    if (!(lb > U) || !(p >= 1.0)) {
                        if (bmax < 0) kb = C;  // rows before this thread's first candidate
                        bmin = min(bmin, (long long)b);
                        bmax = max(bmax, (long long)b);
                    }
                    C += cc[j];
                    P = P + blo[j];
                }
            }
        }
    }
    SELPROF(13);
    const long long my_bmin = bmin;
    {
        u64 a = (u64)bmin, z = (u64)(bmax + 1);  // min(bmin), max(bmax) in one reduction
        blk_minmax_u64(a, z, scr);
        bmin = (long long)a;
        bmax = (long long)z - 1;
    }
    if (bmax < 0) {  // no bucket qualifies (non-finite r): every row is a candidate
        bmin = 0;
        bmax = NB - 1;
        if (t == 0) __hip_atomic_store(&w.ctl->kbase, 0LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (my_bmin == bmin) {
        // rows in buckets < b0
        __hip_atomic_store(&w.ctl->kbase, (long long)kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) {
        __hip_atomic_store(&w.ctl->b0, (int)bmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&w.ctl->b1, (int)bmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&w.ctl->U, U, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (reset_ccount)
            __hip_atomic_exchange(&w.ctl->ccount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (every output drained before the caller publishes the range)
    SELPROF(14);
    return ((unsigned)bmin << 16) | (unsigned)bmax;
}

__global__ __launch_bounds__(HT) void k_sel_bounds(SelWS w, int64_t N, double lam,
                                                   const double *lam_dev, const int *skip,
                                                   int fixb) {
    __shared__ BoundsLds L;
    bounds_body(w, N, lam, lam_dev, skip, fixb, L);
}

// gen != 0: the candidate buckets come from block 0 of the same launch (k_sel_bounds_gather),
// published in ctl->bpub with the token gen; the rows' loads are issued before the wait
__device__ __forceinline__ void gather_body(const u64 *key, const uint32_t *orig, const double *r,
                                            int64_t n, SelWS w, FitSrc fs, int blk,
                                            unsigned gen, const int *skip) {
    GPROF(26);
    const int sk = skip ? *skip : 0;  // checked after the rows' loads have issued
    __shared__ double s_w[GT / 64];
    __shared__ double s_f[8 * (GT / 64)];
    __shared__ int s_b[2];
    const BMap bm = w.ctl->map;  // k_sel_hist's (an earlier launch)
    const int lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blk * (GT * GI) + threadIdx.x;
    // all loads first (no load waits behind the append's atomic).  With the fused fit the
    // rows' pairs load here too, before the bounds wait: which rows lie below the
    // candidates is known only after it, and loaded behind it the pairs cost ~7 us
    u64 kk[GI];
    double rr[GI];
    double fxs[GI], fys[GI], fxt[GI], fyt[GI];
#pragma unroll
    for (int q = 0; q < GI; ++q) {
        const int64_t i = base + (int64_t)q * GT;
        kk[q] = (key && i < n) ? key[i] : 0ULL;
        rr[q] = i < n ? r[i] : 0.0;
    }
    if (fs.on) {
#pragma unroll
        for (int q = 0; q < GI; ++q) {
            const int64_t i = base + (int64_t)q * GT;
            const bool ok = i < n;
            fxs[q] = ok ? fs.sx[i] : 0.0;
            fys[q] = ok ? fs.sy[i] : 0.0;
            fxt[q] = ok ? fs.cx[i] : 0.0;
            fyt[q] = ok ? fs.cy[i] : 0.0;
        }
    }
    if (sk) return;
    int b0, b1;
    if (gen) {
        if (threadIdx.x == 0) {
            // {gen, b0, b1} is one 8-B granule stored sc1 by block 0: an sc1 poll sees it
            // whole (MI355X_MICROARCH.md hand-off table), no acquire fence.  Bounded wait:
            // block 0 is dispatched first and never waits, so the flag comes; should it not
            // (2^20 polls, >= ~30 ms), raise ERR_SPIN (the host fails the run), no hang
            unsigned it = 0;
            u64 v;
            bool late = false;
            while (((v = __hip_atomic_load(&w.ctl->bpub, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)) >> 32) != gen) {
                if (++it == (1u << 20)) {
                    __hip_atomic_fetch_or(&w.ctl->err, ERR_SPIN, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            // a timed-out block takes an empty range: no row below, no candidate, so it
            // appends nothing at a ccount block 0 may not have reset yet (the run fails
            // with ERR_SPIN; k_sel_final ends the device loop)
            s_b[0] = late ? 0 : (int)((v >> 16) & 0xffffu);
            s_b[1] = late ? -1 : (int)(v & 0xffffu);
        }
        __syncthreads();
        b0 = s_b[0];
        b1 = s_b[1];
    } else {
        b0 = w.ctl->b0;
        b1 = w.ctl->b1;
    }
    GPROF(27);
    double acc = 0.0;
    unsigned inm = 0;   // bit q: row q is a candidate
    unsigned bel = 0;   // bit q: row q lies below the candidates (selected)
    unsigned wtot = 0;  // candidates of the wave
    u64 masks[GI];
#pragma unroll
    for (int q = 0; q < GI; ++q) {
        const int64_t i = base + (int64_t)q * GT;
        bool in = false;
        if (i < n) {
            if (!key) kk[q] = key_of_r(rr[q]);
            const int b = bucket_of(bm, kk[q]);
            if (b < b0) {
                acc = acc + rr[q];
                bel |= 1u << q;
            } else if (b <= b1) {
                in = true;
            }
        }
        masks[q] = __ballot(in);
        inm |= (in ? 1u : 0u) << q;
        wtot += (unsigned)__popcll(masks[q]);
    }
    // one append reservation per workgroup: a single word takes ~88 atomics/us, so one
    // per wave (~1800 at 1M rows) serialised this kernel at ~15 us
    __shared__ unsigned s_cnt[GT / 64], s_pos;
    const int wave = threadIdx.x >> 6;
    if (lane == 0) s_cnt[wave] = wtot;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
#pragma unroll
        for (int q = 0; q < GT / 64; ++q) tot += s_cnt[q];
        s_pos = tot ? __hip_atomic_fetch_add(&w.ctl->ccount, tot, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                    : 0u;
    }
    __syncthreads();
    if (wtot) {
        unsigned pos = s_pos;
        for (int q = 0; q < wave; ++q) pos += s_cnt[q];
        const u64 lt = (1ULL << lane) - 1ULL;
#pragma unroll
        for (int q = 0; q < GI; ++q) {
            if ((inm >> q) & 1u) {
                const int64_t i = base + (int64_t)q * GT;
                const unsigned p = pos + (unsigned)__popcll(masks[q] & lt);
                if ((int64_t)p >= n) continue;  // the buffers hold n candidates (never hit
                                                // unless ccount was stale: ERR_SPIN)
                // (sc1 stores: k_sel_bgf's final reads them in this launch)
                stc(w.ka + p, kk[q]);
                stc(w.oa + p, orig ? orig[i] : (uint32_t)i);
                stc(w.ra + p, rr[q]);
                stc(w.pa + p, (uint32_t)i);
                if (fs.on && p < (unsigned)CAP) {  // the final's pairs, no row lookup
                    stc(w.fpre + 4 * p, fxs[q]);
                    stc(w.fpre + 4 * p + 1, fys[q]);
                    stc(w.fpre + 4 * p + 2, fxt[q]);
                    stc(w.fpre + 4 * p + 3, fyt[q]);
                }
            }
            pos += (unsigned)__popcll(masks[q]);
        }
    }
    GPROF(28);
    // fused fit: the 8 sums of the rows below the candidates (all of them are selected)
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (fs.on) {
#pragma unroll
        for (int q = 0; q < GI; ++q)
            if ((bel >> q) & 1u) fit_add(c, fxs[q], fys[q], fxt[q], fyt[q], fs.px, fs.py);
    }
    // fixed tree: DPP wave sums (lane 63), then the waves in order
    acc = wave_sum63(acc);
    if (lane == 63) s_w[threadIdx.x >> 6] = acc;
    if (fs.on) {
#pragma unroll
        for (int e = 0; e < 8; ++e) c[e] = wave_sum63(c[e]);
        if (lane == 63)
#pragma unroll
            for (int e = 0; e < 8; ++e) s_f[8 * (threadIdx.x >> 6) + e] = c[e];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < GT / 64; ++q) t = t + s_w[q];
        stc(w.parts + blk, t);
    }
    if (fs.on && threadIdx.x < 8) {
        double t = 0.0;
        for (int q = 0; q < GT / 64; ++q) t = t + s_f[8 * q + threadIdx.x];
        stc(w.fparts + 8 * blk + threadIdx.x, t);
    }
    GPROF(29);
}

__global__ __launch_bounds__(GT) void k_sel_gather(const u64 *key, const uint32_t *orig,
                                                   const double *r, int64_t n, SelWS w,
                                                   const int *skip, FitSrc fs) {
    gather_body(key, orig, r, n, w, fs, blockIdx.x, 0u, skip);
}

// k_sel_bounds and k_sel_gather as one launch: block 0 computes the candidate buckets
// (bounds_body, GT == HT threads) and publishes [b0, b1] with the launch's token gen
// (unique per launch) in one 8-B sc1 store; blocks 1.. load their rows meanwhile, poll
// the word, then gather.  One launch boundary less per NN call, and the rows' loads overlap the bounds.
static_assert(GT == HT, "k_sel_bounds_gather: block 0 runs bounds_body with HT threads");
__global__ __launch_bounds__(GT) void k_sel_bounds_gather(const u64 *key, const uint32_t *orig,
                                                          const double *r, int64_t n, SelWS w,
                                                          double lam, const double *lam_dev,
                                                          const int *skip, int fixb, FitSrc fs,
                                                          unsigned gen, unsigned pub_gen) {
    if (blockIdx.x == 0) {
        // (ccount was reset by k_sel_hist, a launch earlier: nothing to drain before the
        // flag; b0, b1, U and kbase are read by k_sel_final, a later launch)
        __shared__ BoundsLds L;
        const unsigned bb = bounds_body(w, n, lam, lam_dev, skip, fixb, L, false);
        if (bb != kBoundsSkipped && threadIdx.x == 0) {
            // (pub_gen == gen except under the test-only fault injection FICP_FAULT_SPIN,
            // ficp_set_fault)
            __hip_atomic_store(&w.ctl->bpub, ((u64)pub_gen << 32) | bb, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    gather_body(key, orig, r, n, w, fs, blockIdx.x - 1, gen, skip);
}

// ---------------------------------------------------------- the final workgroup
// Every load of the gather's outputs (candidates, their pairs, the part sums) and of the
// bounds' outputs is sc1 (agent scope, past this CU's L1): k_sel_bgf runs the final in the
// gather's last workgroup, in the same launch as the sc1 stores that wrote them
// (MI355X_MICROARCH.md hand-off table; the same loads serve the separate k_sel_final).
template <class T>
__device__ __forceinline__ T ldc(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double2 ldc2(const double *p) { return make_double2(ldc(p), ldc(p + 1)); }
struct Cand {
    u64 *k;
    uint32_t *o;
    double *r;
    uint32_t *p;  // work row (fused fit)
};

struct FinalIn {
    long long N;
    double lam;
    double S0;      // exact (deterministic) sum of every row sorted before the candidates
    long long K0;   // number of those rows
    double U;
    FitSrc fs;      // fused fit (fs.on): rows whose sums go into fsum
    double *fsum;   // [8] in LDS, thread 0 accumulates in a fixed order
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
    // the threshold's move since the previous loop-body call of this stage (make_bmap)
    const bool prev = st->phase == PH_LOOP && st->k > 0 && bk != 0x7fffffffffffffffLL;
    st->tmove = prev ? (tkey > st->tkey ? tkey - st->tkey : st->tkey - tkey) : 0ULL;
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

// LDS layout of the final kernel's sort (bytes) for CAPT candidates, r in LDS or not
template <int CAPT, bool RL>
struct LdsLay {
    static constexpr int K = 0;                               // u64[CAPT]
    static constexpr int R = K + CAPT * 8;                    // f64[CAPT] (RL)
    static constexpr int O = R + (RL ? CAPT * 8 : 0);         // u32[CAPT]
    static constexpr int POS = O + CAPT * 4;                  // u16[CAPT]
    static constexpr int MEM = POS + CAPT * 2;                // u16[CAPT]
    static constexpr int BC = MEM + CAPT * 2;                 // u32[NSB] counts / fill
    static constexpr int BO = BC + NSB * 4;                   // u32[NSB] offsets
    static constexpr int END = BO + NSB * 4;
};
constexpr int L_END = LdsLay<CAP, true>::END > LdsLay<CAP2, false>::END ? LdsLay<CAP, true>::END
                                                                         : LdsLay<CAP2, false>::END;
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
static_assert(HT * 56 <= SMEM, "final_small's LDS (keys, r, orig, pos, fused-fit pairs)");

// (a) c <= CAPT candidates: bucket sort in LDS, exact prefix sums, first minimum.  RL:
// r is staged in LDS too (c <= CAP); otherwise (c <= CAP2) r is read from global memory
// in sorted order and the prefix sums overwrite the keys.  Flat FRMSD curves (lambda
// near 1) leave thousands of candidates that no bound separates: the in-workgroup radix
// sort took ~220 us for 5.4k of them, this path ~2x the small one.
// result of one sorted scan: first minimum (bf, bk; every thread), its threshold pair
// (tk, to; thread 0) and the sum of the scanned r (every thread)
struct ScanOut {
    double bf;
    long long bk;
    u64 tk;
    uint32_t to;
    double total;
};

// sort c <= CAPT candidates in LDS and scan them from (K0, S0): positions K0 + 1 .. K0 + c
template <int CAPT, bool RL, bool PRE = false>
__device__ ScanOut lds_sort_scan(const Cand &src, unsigned c, long long K0, double S0,
                                 const FinalIn &in, unsigned char *sm, Scr &scr) {
    using LY = LdsLay<CAPT, RL>;
    u64 *lk = (u64 *)(sm + LY::K);
    double *lr = (double *)(sm + LY::R);
    uint32_t *lo = (uint32_t *)(sm + LY::O);
    uint16_t *pos = (uint16_t *)(sm + LY::POS);
    uint16_t *mem = (uint16_t *)(sm + LY::MEM);
    unsigned *bc = (unsigned *)(sm + LY::BC);
    unsigned *bo = (unsigned *)(sm + LY::BO);
    const int t = threadIdx.x;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    for (unsigned i = t; i < c; i += HT) {
        // (PRE: the caller staged the candidates in LDS and passed a barrier)
        const u64 k = PRE ? lk[i] : ldc(src.k + (i));
        const uint32_t o = PRE ? lo[i] : ldc(src.o + (i));
        if (!PRE) {
            lk[i] = k;
            lo[i] = o;
            if (RL) lr[i] = ldc(src.r + (i));
        }
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
    }
    for (int b = t; b < NSB; b += HT) bc[b] = 0u;
    SELPROF(2);
    blk_minmax2_u64(kmn, kmx, omn, omx, scr);
    const Comp cmp = make_comp(kmn, kmx, (uint32_t)omn, (uint32_t)omx);
    const u64 vspan = cmp(kmx, (uint32_t)omx);
    const int vb = bits_of(vspan);
    const int sh = vb > NSB_LOG ? vb - NSB_LOG : 0;
    SELPROF(16);
    for (unsigned i = t; i < c; i += HT) atomicAdd(&bc[(int)(cmp(lk[i], lo[i]) >> sh)], 1u);
    __syncthreads();
    SELPROF(17);
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
    SELPROF(18);
    for (unsigned i = t; i < c; i += HT) {
        const int b = (int)(cmp(lk[i], lo[i]) >> sh);
        mem[bo[b] + atomicAdd(&bc[b], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    SELPROF(19);
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
    SELPROF(3);
    // exact prefix sums in sorted order, FRMSD of every candidate k
    constexpr int PP = CAPT / HT;  // positions per thread
    double v[PP];
    double tsum = 0.0;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        const unsigned p = (unsigned)(t * PP + q);
        v[q] = p < c ? (RL ? lr[pos[p]] : ldc(src.r + (pos[p]))) : 0.0;
        tsum = tsum + v[q];
    }
    double all;
    double run = blk_excl_scan_d(tsum, scr, all);
    // prefix sums by sorted position into LDS (over lr: its rows are in v[] now), then
    // FRMSD of every position with the positions dealt over all lanes (a thread's own
    // PP positions would run PP dependent pow() chains back to back)
    __syncthreads();
    double *ls = RL ? lr : (double *)lk;  // (!RL: the keys are read from global below)
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        const unsigned p = (unsigned)(t * PP + q);
        run = run + v[q];
        if (p < c) ls[p] = run;
    }
    __syncthreads();
    SELPROF(20);
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    for (unsigned p = t; p < c; p += HT) {
        const long long k = K0 + (long long)p + 1;
        const double f = frmsd_of(k, in.N, S0 + ls[p], in.lam);
        if (f < bf) {
            bf = f;
            bk = k;
        }
    }
    SELPROF(4);
    blk_argmin(bf, bk, scr);
    ScanOut r{bf, bk, 0, 0, all};
    if (t == 0 && bk != 0x7fffffffffffffffLL) {
        const unsigned e = pos[(unsigned)(bk - K0 - 1)];
        r.tk = RL ? lk[e] : ldc(src.k + (e));
        r.to = lo[e];
    }
    return r;
}

// (a) c <= CAPT candidates: one sorted scan, the fused fit's selected candidates, publish
// fpre (nullable): the pairs the gather stored by pack slot (the candidates not refined):
// 32 B per candidate from one 128-KB array instead of a work-row lookup and four loads
// into four 8-MB columns per candidate (C3's stage head, ~2,000 candidates: 10.5 us for
// the fit after the scan, TLB-bound)
template <int CAPT, bool RL>
__device__ void final_lds(const Cand &src, unsigned c, const FinalIn &in, unsigned char *sm,
                          Scr &scr, IterState *st, const double *fpre = nullptr) {
    const ScanOut r = lds_sort_scan<CAPT, RL>(src, c, in.K0, in.S0, in, sm, scr);
    if (in.fs.on && r.bk != 0x7fffffffffffffffLL) {  // fused fit: the selected candidates
        const uint16_t *pos = (const uint16_t *)(sm + LdsLay<CAPT, RL>::POS);
        const unsigned nsel = (unsigned)(r.bk - in.K0);
        double cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (fpre) {
            // positions t, t + HT, ... in increasing order, as the row lookup below; four
            // positions' loads issued together (clamped indices, the sums predicated)
            for (unsigned q0 = threadIdx.x; q0 < nsel; q0 += 4 * HT) {
                double2 a[4], b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const unsigned q = q0 + (unsigned)j * HT;
                    const unsigned e = pos[q < nsel ? q : q0];
                    a[j] = ldc2(fpre + 4 * e);
                    b[j] = ldc2(fpre + 4 * e + 2);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (q0 + (unsigned)j * HT < nsel) fit_add(cf, a[j].x, a[j].y, b[j].x, b[j].y, in.fs.px, in.fs.py);
            }
        } else {
            for (unsigned q = threadIdx.x; q < nsel; q += HT) fit_row(cf, in.fs, ldc(src.p + (pos[q])));
        }
        blk_sum8_add(cf, in.fsum, scr);
    }
    if (threadIdx.x == 0) publish(st, in, r.bf, r.bk, r.tk, r.to);
}

// (a0) c <= SMALL_C candidates (the windowed map's normal case: ~20-100 at C3): one candidate
// per thread, ranked by (key, orig) against all c in LDS (broadcast reads, no bins), one
// block scan of r in sorted order, FRMSD of every position, first minimum.  Fewer
// barriers than the binned sort of lds_sort_scan, whose fixed phases dominated at this c.
// Pre: thread t < c holds candidate t (pk, po, pr; with the fused fit also its pair in
// pf[4]), loaded in k_sel_final's prologue beside the state and S_base parts (they were a
// second dependent round trip after the candidate count).
struct CandPre {
    u64 k;
    uint32_t o;
    double r;
    double f[4];
};
__device__ void final_small(const CandPre &pre, unsigned c, const FinalIn &in, unsigned char *sm,
                            Scr &scr, IterState *st) {
    u64 *lk = (u64 *)sm;
    double *lr = (double *)(sm + HT * 8);
    uint32_t *lo = (uint32_t *)(sm + HT * 16);
    uint16_t *pos = (uint16_t *)(sm + HT * 20);
    double *lf = (double *)(sm + HT * 24);  // fused fit: the candidate's pair [4][HT]
    const unsigned t = threadIdx.x;
    u64 k = 0;
    uint32_t o = 0;
    if (t < c) {
        k = pre.k;
        o = pre.o;
        if (in.fs.on) {  // summed over LDS in sorted order below (deterministic)
            lf[t] = pre.f[0];
            lf[HT + t] = pre.f[1];
            lf[2 * HT + t] = pre.f[2];
            lf[3 * HT + t] = pre.f[3];
        }
        lk[t] = k;
        lo[t] = o;
        lr[t] = pre.r;
    }
    __syncthreads();
    SELPROF(21);
    if (t < c) {
        unsigned rank = 0;
        for (unsigned j = 0; j < c; ++j) rank += less_ko(lk[j], lo[j], k, o) ? 1u : 0u;
        pos[rank] = (uint16_t)t;
    }
    __syncthreads();
    SELPROF(22);
    const double v = t < c ? lr[pos[t]] : 0.0;
    double all;
    const double ex = blk_excl_scan_d(v, scr, all);
    SELPROF(23);
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    if (t < c) {
        const long long kk = in.K0 + (long long)t + 1;
        const double f = frmsd_of(kk, in.N, in.S0 + (ex + v), in.lam);
        if (f < bf) {
            bf = f;
            bk = kk;
        }
    }
    blk_argmin(bf, bk, scr);
    SELPROF(24);
    if (in.fs.on && bk != 0x7fffffffffffffffLL) {  // fused fit: the selected candidates
        double cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if ((long long)t < bk - in.K0) {
            const unsigned e = pos[t];
            fit_add(cf, lf[e], lf[HT + e], lf[2 * HT + e], lf[3 * HT + e], in.fs.px, in.fs.py);
        }
        blk_sum8_add(cf, in.fsum, scr);
    }
    SELPROF(25);
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

// (a') more than CAP2 candidates that refinement could not narrow (flat FRMSD curves at
// millions of rows, ties): counted into NS sub-bins of the (key, orig) order, moved into
// dst in sub-bin order, and scanned as consecutive groups of <= CAP2 (a group starts at
// the sub-bin holding every multiple of CAP2 / 2 of the prefix count, so no sub-bin may
// exceed CAP2 / 2),
// carrying k and the exact sum from group to group.  Returns false (nothing published)
// when a sub-bin is too large or there are too many groups: the radix path takes it.
constexpr int MAXGRP = 512;
__device__ bool final_chunked(const Cand &src, const Cand &dst, unsigned c, const FinalIn &in,
                              unsigned char *sm, Scr &scr, IterState *st, unsigned *g_beg) {
    constexpr unsigned H = CAP2 / 2;
    unsigned *cnt = (unsigned *)sm;        // [NS] (the sort area is free until the groups)
    unsigned *off = cnt + NS;              // [NS]
    unsigned *fil = off + NS;              // [NS]
    __shared__ unsigned s_ng, s_bad;
    const int t = threadIdx.x;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
    }
    for (int b = t; b < NS; b += HT) {
        cnt[b] = 0u;
        fil[b] = 0u;
    }
    if (t == 0) {
        s_ng = 0u;
        s_bad = 0u;
    }
    blk_minmax2_u64(kmn, kmx, omn, omx, scr);
    const Comp cmp = make_comp(kmn, kmx, (uint32_t)omn, (uint32_t)omx);
    const int vb = bits_of(cmp(kmx, (uint32_t)omx));
    const int sh = vb > NS_LOG ? vb - NS_LOG : 0;
    for (unsigned i = t; i < c; i += HT) atomicAdd(&cnt[(int)(cmp(ldc(src.k + (i)), ldc(src.o + (i))) >> sh)], 1u);
    __syncthreads();
    {
        constexpr int PB = NS / HT;
        unsigned v[PB];
        long long tot = 0;
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            v[j] = cnt[t * PB + j];
            tot += v[j];
        }
        long long all;
        long long ex = blk_excl_scan_ll(tot, scr, all);
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int b = t * PB + j;
            off[b] = (unsigned)ex;
            if (v[j] > H) atomicOr(&s_bad, 1u);
            // groups begin at offset 0 and at every sub-bin that holds a multiple m H
            // (m >= 1) of the prefix count: consecutive starts are < 2 H = CAP2 apart
            // because a sub-bin holds at most H rows
            const unsigned exu = (unsigned)ex, vv = v[j];
            bool start = false;
            if (vv) {
                const unsigned m = (exu + H - 1) / H;
                start = exu == 0 || m * H < exu + vv;
            }
            if (start) {
                const unsigned gi = atomicAdd(&s_ng, 1u);
                if (gi < (unsigned)MAXGRP) g_beg[gi] = exu;
            }
            ex += v[j];
        }
    }
    __syncthreads();
    const unsigned ng = s_ng;
    if (s_bad || ng > (unsigned)MAXGRP) return false;
    // group starts in ascending order (few: an insertion sort by thread 0)
    if (t == 0) {
        for (unsigned a = 1; a < ng; ++a) {
            const unsigned x = g_beg[a];
            unsigned b = a;
            while (b > 0 && g_beg[b - 1] > x) {
                g_beg[b] = g_beg[b - 1];
                --b;
            }
            g_beg[b] = x;
        }
        g_beg[ng] = c;
    }
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
        const int b = (int)(cmp(k, o) >> sh);
        const unsigned q = off[b] + atomicAdd(&fil[b], 1u);
        dst.k[q] = k;
        dst.o[q] = o;
        dst.r[q] = ldc(src.r + (i));
        dst.p[q] = ldc(src.p + (i));
    }
    __threadfence_block();
    __syncthreads();
    double carry = 0.0, bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    u64 tk = 0;
    uint32_t to = 0;
    for (unsigned gi = 0; gi < ng; ++gi) {
        const unsigned a = g_beg[gi], e = g_beg[gi + 1];
        const Cand sub{dst.k + a, dst.o + a, dst.r + a, dst.p + a};
        const ScanOut r = lds_sort_scan<CAP2, false>(sub, e - a, in.K0 + (long long)a,
                                                    in.S0 + carry, in, sm, scr);
        if (t == 0 && better(r.bf, r.bk, bf, bk)) {
            bf = r.bf;
            bk = r.bk;
            tk = r.tk;
            to = r.to;
        }
        carry = carry + r.total;
        __syncthreads();
    }
    if (t == 0) publish(st, in, bf, bk, tk, to);
    return true;
}

// (b) one refinement level over c > CAP candidates in global memory: returns false when
// it cannot shrink the set (the caller then sorts it)
// v * 2^56 truncated toward zero, two's complement in 128 bits (|v| < 2^70: fit terms of
// coordinates relative to the pivot, products of two of them)
__device__ __forceinline__ u128 fx56(double v) {
    const u64 b = (u64)__double_as_longlong(v);
    const int ex = (int)((b >> 52) & 0x7ff);
    if (ex == 0) return (u128)0;  // zero or subnormal: below the grid
    const u64 m = (b & 0xfffffffffffffULL) | (1ULL << 52);
    const int sft = ex - 1075 + 56;
    const u128 a = sft >= 0 ? ((u128)m << sft) : (sft > -64 ? (u128)(m >> (-sft)) : (u128)0);
    return (b >> 63) ? (u128)0 - a : a;
}

__device__ __forceinline__ double fx56_to_double(u128 s) {
    const bool neg = (s >> 127) != 0;
    const u128 a = neg ? (u128)0 - s : s;
    const double d = ldexp((double)(u64)(a >> 64), 64 - 56) + ldexp((double)(u64)a, -56);
    return neg ? -d : d;
}

// The fused fit's 8 sums of rows taken in an order that is not fixed (the candidate pack
// is filled by atomics): each term is accumulated exactly on the 2^-56 grid, so the sum
// is the same bits whatever the order; the block total goes into acc8 as a double.
__device__ void blk_sum_fx8_add(u128 (&a)[8], double *acc8) {
    __shared__ u64 s_fx[NWAVE * 8 * 2];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const u64 hi = __shfl_xor((u64)(a[e] >> 64), o, 64);
            const u64 lo = __shfl_xor((u64)a[e], o, 64);
            a[e] = a[e] + (((u128)hi << 64) | lo);
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            s_fx[(w * 8 + e) * 2] = (u64)(a[e] >> 64);
            s_fx[(w * 8 + e) * 2 + 1] = (u64)a[e];
        }
    __syncthreads();
    if (threadIdx.x < 8) {
        u128 t = 0;
        for (int q = 0; q < NWAVE; ++q)
            t = t + (((u128)s_fx[(q * 8 + threadIdx.x) * 2] << 64) | s_fx[(q * 8 + threadIdx.x) * 2 + 1]);
        acc8[threadIdx.x] = acc8[threadIdx.x] + fx56_to_double(t);
    }
    __syncthreads();
}

__device__ bool refine(Cand &src, Cand &dst, unsigned &c, FinalIn &in, unsigned char *sm,
                       Scr &scr) {
    unsigned *rc = (unsigned *)(sm + R_C);
    u64 *rs = (u64 *)(sm + R_S);
    unsigned *rn = (unsigned *)(sm + R_N);
    const int t = threadIdx.x;
    u64 kmn = ~0ULL, kmx = 0ULL, omn = ~0ULL, omx = 0ULL;
    double rmax = 0.0;
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
        rmax = fmax(rmax, ldc(src.r + (i)));
    }
    for (int b = t; b < NS; b += HT) {
        rc[b] = 0u;
        rs[b] = 0ULL;
    }
    if (t == 0) *rn = 0u;
    blk_minmax2_u64(kmn, kmx, omn, omx, scr);
    rmax = blk_max_d(rmax, scr);
    if (!(rmax < INFINITY)) return false;
    const Comp cmp = make_comp(kmn, kmx, (uint32_t)omn, (uint32_t)omx);
    const int vb = bits_of(cmp(kmx, (uint32_t)omx));
    if (vb == 0) return false;
    const int sh = vb > NS_LOG ? vb - NS_LOG : 0;
    // sub-bin sums of r as integers on the grid 2^Lq (floor per row), r < 2^(e+1): the
    // sums are the same whatever order the atomics run in (a double atomic sum was not,
    // and its last bits moved the bounds and so the split between the exact integer sum
    // below and the sorted scan: k flipped on flat FRMSD curves).  [lo, lo + cnt) units
    // bracket each sub-bin's true sum.
    const int e = rmax > 0.0 ? ilogb(rmax) : 0;
    const int Lq = e + 1 - (62 - bits_of((u64)c));
    for (unsigned i = t; i < c; i += HT) {
        const int b = (int)(cmp(ldc(src.k + (i)), ldc(src.o + (i))) >> sh);
        atomicAdd(&rc[b], 1u);
        atomicAdd(&rs[b], fx_floor(ldc(src.r + (i)), Lq));
    }
    __syncthreads();
    constexpr int PB = NS / HT;  // 4 sub-bins per thread
    unsigned cn[PB];
    double slo[PB], shi[PB];
    long long ct = 0;
    double stl = 0.0, sth = 0.0;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        cn[j] = rc[t * PB + j];
        const u64 f = rs[t * PB + j];
        slo[j] = ldexp((double)f, Lq);
        shi[j] = ldexp((double)(f + cn[j]), Lq);
        ct += cn[j];
        stl = stl + slo[j];
        sth = sth + shi[j];
    }
    long long ctot;
    double stot;
    const long long Cex = blk_excl_scan_ll(ct, scr, ctot);
    const double Plex = blk_excl_scan_d(stl, scr, stot);
    const double Phex = blk_excl_scan_d(sth, scr, stot);
    const double p = 2.0 * in.lam + 1.0;
    double U = in.U;
    {  // upper bound of h at each sub-bin end: the upper sums
        long long C = in.K0 + Cex;
        double P = in.S0 + Phex;
#pragma unroll
        for (int j = 0; j < PB; ++j)
            if (cn[j]) {
                C += cn[j];
                P = P + shi[j];
                U = fmin(U, h_of(C, P, p) + kMarg);
            }
    }
    U = blk_min_d(U, scr);
    long long bmin = 0x7fffffffLL, bmax = -1, nfirst = 0x7fffffffLL, nlast = -1;
    {  // lower bound inside each sub-bin: the lower sums
        long long C = in.K0 + Cex;
        double P = in.S0 + Plex;
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
                P = P + slo[j];
            }
        }
    }
    bmin = blk_min_ll(bmin, scr);
    bmax = blk_max_ll(bmax, scr);
    nfirst = blk_min_ll(nfirst, scr);
    nlast = blk_max_ll(nlast, scr);
    if (bmax < 0 || (bmin == nfirst && bmax == nlast)) return false;
    // rows that drop below the new range: exact integer sum on the grid 2^(e - 96); their
    // fused-fit terms exactly on the 2^-56 grid (the pack's order is not fixed)
    const int L = e - 96;
    u128 acc = 0;
    long long below = 0;
    u128 cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
        const double rv = ldc(src.r + (i));
        const int b = (int)(cmp(k, o) >> sh);
        if (b < bmin) {
            below += 1;
            if (in.fs.on) {
                const uint32_t wr = ldc(src.p + (i));
                double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                fit_add(v, in.fs.sx[wr], in.fs.sy[wr], in.fs.cx[wr], in.fs.cy[wr], in.fs.px,
                        in.fs.py);
#pragma unroll
                for (int q = 0; q < 8; ++q) cf[q] = cf[q] + fx56(v[q]);
            }
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
            dst.p[slot] = ldc(src.p + (i));
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
    if (in.fs.on) blk_sum_fx8_add(cf, in.fsum);
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
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
        omn = o < omn ? o : omn;
        omx = o > omx ? o : omx;
    }
    blk_minmax2_u64(kmn, kmx, omn, omx, scr);
    const int po = (bits_of(omx - omn) + 7) / 8, pk = (bits_of(kmx - kmn) + 7) / 8;
    const int np = po + pk;  // <= 4 + 8
    for (int j = t; j < 12 * 256; j += HT) hist[j] = 0u;
    __syncthreads();
    auto digit = [&](u64 k, uint32_t o, int p) -> unsigned {
        return p < po ? (unsigned)(((o - (uint32_t)omn) >> (8 * p)) & 0xffu)
                      : (unsigned)(((k - kmn) >> (8 * (p - po))) & 0xffu);
    };
    for (unsigned i = t; i < c; i += HT) {
        const u64 k = ldc(src.k + (i));
        const uint32_t o = ldc(src.o + (i));
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
            uint32_t o = 0, pw = 0;
            double rv = 0.0;
            unsigned d = 0;
            if (valid) {
                k = ldc(src.k + (i));
                o = ldc(src.o + (i));
                rv = ldc(src.r + (i));
                pw = ldc(src.p + (i));
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
                dst.p[q] = pw;
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
        const double v = i < c ? ldc(src.r + (i)) : 0.0;
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
    if (in.fs.on && bk != 0x7fffffffffffffffLL) {  // fused fit: the selected candidates
        double cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (unsigned q = t; q < (unsigned)(bk - in.K0); q += HT) fit_row(cf, in.fs, ldc(src.p + (q)));
        blk_sum8_add(cf, in.fsum, scr);
    }
    if (t == 0) {
        u64 tk = 0;
        uint32_t to = 0;
        if (bk != 0x7fffffffffffffffLL) {
            const unsigned e = (unsigned)(bk - in.K0 - 1);
            tk = ldc(src.k + (e));
            to = ldc(src.o + (e));
        }
        publish(st, in, bf, bk, tk, to);
    }
}

// With fuse_loop, thread 0 also runs the loop step of k_loop_update (ficp.py:122-154)
// and, with host_flag, stores the state's done flag to that (coherent pinned) host word.
// The final selection of one call (one HT-thread workgroup): k_sel_final, or the last
// gather workgroup of k_sel_bgf.  sm: SMEM bytes of LDS.
__device__ __forceinline__ void final_body(SelWS w, int nparts, int64_t N, double lam,
                                           const double *lam_dev, IterState *st, const int *skip,
                                           const LoopCtl &lc, int fuse_loop, int *host_flag,
                                           const FitSrc &fs, int64_t cap, unsigned char *sm) {
    // the independent loads (skip flag, lambda, the candidate count and the bounds'
    // outputs, and the first SMALL_C candidate slots whatever the count) issue together,
    // before the first wait
    const int sk = skip ? *skip : 0;
    const double lamv = lam_dev ? *lam_dev : lam;
    unsigned c = __hip_atomic_fetch_add(&w.ctl->ccount, 0u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    const unsigned errv = __hip_atomic_fetch_or(&w.ctl->err, 0u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    [[maybe_unused]] const unsigned c_in = c;
    const long long kbase = ldc(&w.ctl->kbase);
    const double Ub = ldc(&w.ctl->U);
    CandPre pre{};
    const bool pfc = (int64_t)threadIdx.x < cap && threadIdx.x < (unsigned)SMALL_C;
    if (pfc) {
        pre.k = ldc(w.ka + threadIdx.x);
        pre.o = ldc(w.oa + threadIdx.x);
        pre.r = ldc(w.ra + threadIdx.x);
        if (fs.on) {  // the gather stored the pairs of the first SMALL_C slots
            const double2 a01 = ldc2(w.fpre + 4 * threadIdx.x);
            const double2 a23 = ldc2(w.fpre + 4 * threadIdx.x + 2);
            pre.f[0] = a01.x;
            pre.f[1] = a01.y;
            pre.f[2] = a23.x;
            pre.f[3] = a23.y;
        }
    }
    if (sk) {
        if (host_flag && threadIdx.x == 0)
            __hip_atomic_store(host_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    lam = lamv;
    __shared__ Scr scr;
    __shared__ IterState s_st;  // thread 0's working copy of the state (one load, one store)
    __shared__ double s_fit[8];  // fused fit sums (thread 0)
    __shared__ unsigned s_gbeg[MAXGRP + 1];  // group starts of the chunked scan
    const int t = threadIdx.x;
    SELPROF(0);
    // the state copied word by word by all threads (thread 0 alone issued ~35 dependent
    // 16-B loads here and as many stores at the end: ~1 us each way)
    static_assert(sizeof(IterState) % 4 == 0, "IterState words");
    constexpr int SW = (int)(sizeof(IterState) / 4);
    for (int q = t; q < SW; q += HT) ((uint32_t *)&s_st)[q] = ((const uint32_t *)st)[q];
    if (t < 8) s_fit[t] = 0.0;
    double a = 0.0;
    for (int p = t; p < nparts; p += HT) a = a + ldc(w.parts + p);  // fixed order per thread
    FinalIn in;
    in.N = N;
    in.lam = lam;
    in.fs = fs;
    in.fsum = s_fit;
    in.S0 = blk_sum(a, scr);
    if (fs.on) {  // the gather blocks' sums of the rows below the candidates
        double cf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int p = t; p < nparts; p += HT)
#pragma unroll
            for (int e = 0; e < 8; ++e) cf[e] = cf[e] + ldc(w.fparts + 8 * p + e);
        blk_sum8_add(cf, s_fit, scr);
    }
    in.K0 = kbase;
    in.U = Ub;
    SELPROF(1);
    if (c == 0) {
        if (t == 0) {
            __hip_atomic_fetch_or(&w.ctl->err, ERR_EMPTY, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
            publish(&s_st, in, INFINITY, 0x7fffffffffffffffLL, 0, 0);
        }
    } else {
        Cand src{w.ka, w.oa, w.ra, w.pa}, dst{w.kb, w.ob, w.rb, w.pb};
        int lev = 0;
        bool stalled = false;
        while (c > (unsigned)CAP2 && lev < MAXLEV && !stalled) {
            stalled = !refine(src, dst, c, in, sm, scr);
            if (!stalled) ++lev;
            __threadfence_block();
            __syncthreads();
        }
        if (t == 0) w.ctl->levels += lev;
        if (c <= (unsigned)SMALL_C && lev == 0) {
            final_small(pre, c, in, sm, scr, &s_st);
        } else if (c <= (unsigned)SMALL_C) {  // after refinement: the candidates moved
            CandPre q{};
            if (t < c) {
                q.k = ldc(src.k + (t));
                q.o = ldc(src.o + (t));
                q.r = ldc(src.r + (t));
                if (fs.on) {
                    const uint32_t wr = ldc(src.p + (t));
                    q.f[0] = fs.sx[wr];
                    q.f[1] = fs.sy[wr];
                    q.f[2] = fs.cx[wr];
                    q.f[3] = fs.cy[wr];
                }
            }
            final_small(q, c, in, sm, scr, &s_st);
        } else if (c <= (unsigned)CAP) {
            final_lds<CAP, true>(src, c, in, sm, scr, &s_st, (lev == 0 && fs.on) ? w.fpre : nullptr);
        } else if (c <= (unsigned)CAP2) {
            final_lds<CAP2, false>(src, c, in, sm, scr, &s_st);
        } else if (!fs.on && final_chunked(src, dst, c, in, sm, scr, &s_st, s_gbeg)) {
            if (t == 0) w.ctl->levels += 1u << 16;  // statistics: chunked scans (high half)
        } else {
            if (t == 0) w.ctl->radix += 1;
            final_radix(src, dst, c, in, sm, scr, &s_st);
        }
    }
    SELPROF(5);
    if (t == 0) {
        // thread 0's step on a register copy (every field access of the LDS copy was a
        // dependent LDS round trip)
        IterState L = s_st;
        // the window path could not decide this call (k_sel_win): the NN launch queued
        // behind it was a no-op by nn_reuse, which the state machine restores here
        if (L.win_fail) {
            L.win_fail = 0;
            L.nn_reuse = 0;
        }
        if (fuse_loop) loop_step(&L, lc);
        // a sticky selection error (ERR_SPIN, ERR_CAP): this call's result is invalid, so
        // the device loop ends here and the host reports the flag (no further calls)
        if (fuse_loop && errv) {
            L.phase = PH_DONE;
            loop_set_flags(L);
        }
        // fused fit: T of the next loop body from this selection (k_fit_sums' work)
        if (fs.on && !L.no_fit && L.k > 0) fit_solve(s_fit, (double)L.k, fs.px, fs.py, fs.allow_refl, &L);
        s_st = L;
    }
    __syncthreads();
    for (int q = t; q < SW; q += HT) ((uint32_t *)st)[q] = ((const uint32_t *)&s_st)[q];
    if (t == 0 && host_flag)
        __hip_atomic_store(host_flag, s_st.done | (win_ok(s_st) ? kFlagWinNext : 0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    SELPROF(6);
#ifdef SEL_PROF
    // one line per 13 calls, in 10-ns ticks: bounds phases (block 0 of bounds_gather), the
    // first gather block (start vs bounds start, wait, append, sums), the final's phases
#ifndef SEL_PROF_EVERY
#define SEL_PROF_EVERY 13u
#endif
    if (t == 0 && (g_selcalls++ % SEL_PROF_EVERY) == 6u % SEL_PROF_EVERY) {
        const unsigned long long *g = g_selprof;
        printf("SELPROF c=%u->%u k=%lld lev=%u radix=%u hist %lld %lld %lld | b0 +%lld %lld %lld %lld %lld %lld %lld"
               " | gather +%lld bounds %lld app %lld sums %lld"
               " | gap %lld final pro %lld small %lld %lld %lld %lld %lld post %lld tail %lld\n", c_in, c,
               (long long)s_st.k, w.ctl->levels, w.ctl->radix,
               (long long)(g[31] - g[30]), (long long)(g[32] - g[31]), (long long)(g[33] - g[32]),
               (long long)(g[8] - g[33]), (long long)(g[9] - g[8]), (long long)(g[10] - g[9]),
               (long long)(g[11] - g[10]), (long long)(g[12] - g[11]), (long long)(g[13] - g[12]),
               (long long)(g[14] - g[13]),
               (long long)(g[26] - g[8]), (long long)(g[27] - g[26]), (long long)(g[28] - g[27]),
               (long long)(g[29] - g[28]), (long long)(g[0] - g[29]), (long long)(g[1] - g[0]),
               (long long)(g[21] - g[1]), (long long)(g[22] - g[21]), (long long)(g[23] - g[22]),
               (long long)(g[24] - g[23]), (long long)(g[25] - g[24]), (long long)(g[5] - g[25]),
               (long long)(g[6] - g[5]));
        if (c > (unsigned)SMALL_C)  // the binned LDS sort's phases (lds_sort_scan), then the fit
            printf("SELPROF_LDS load %lld minmax %lld count %lld scan %lld scatter %lld rank %lld "
                   "prefix %lld frmsd %lld argmin+fit %lld\n",
                   (long long)(g[2] - g[1]), (long long)(g[16] - g[2]), (long long)(g[17] - g[16]),
                   (long long)(g[18] - g[17]), (long long)(g[19] - g[18]), (long long)(g[3] - g[19]),
                   (long long)(g[20] - g[3]), (long long)(g[4] - g[20]), (long long)(g[5] - g[4]));
    }
#endif
}

__global__ __launch_bounds__(HT) void k_sel_final(SelWS w, int nparts, int64_t N, double lam,
                                                  const double *lam_dev, IterState *st,
                                                  const int *skip, LoopCtl lc, int fuse_loop,
                                                  int *host_flag, FitSrc fs, int64_t cap) {
    __shared__ __align__(16) unsigned char sm[SMEM];
    final_body(w, nparts, N, lam, lam_dev, st, skip, lc, fuse_loop, host_flag, fs, cap, sm);
}

// k_sel_bounds_gather and k_sel_final in one launch (round 5; three launches per full-path
// call instead of four): block 0 computes and publishes the candidate buckets, blocks 1..
// gather, and the last gather workgroup to arrive runs the final.  The hand-off is
// k_fit_sums' / k_sel_win's: the gather's outputs are sc1 stores, every storing wave drains
// them, one lane arrives at its group counter (blockIdx % 8) and the group's last at the
// top counter; the final reads them with sc1 loads.  Block 0's LDS is laid over the
// final's buffer (block 0 never runs the final).
static_assert(sizeof(BoundsLds) <= (size_t)SMEM, "bounds LDS inside the final's buffer");
__global__ __launch_bounds__(GT) void k_sel_bgf(const u64 *key, const uint32_t *orig, const double *r,
                                               int64_t n, SelWS w, double lam, const double *lam_dev,
                                               const int *skip, int fixb, FitSrc fs, unsigned gen,
                                               unsigned pub_gen, IterState *st, LoopCtl lc,
                                               int fuse_loop, int *host_flag, int64_t cap) {
    __shared__ __align__(16) unsigned char sm[SMEM];
    __shared__ int s_last;
    if (blockIdx.x == 0) {
        const unsigned bb = bounds_body(w, n, lam, lam_dev, skip, fixb, *reinterpret_cast<BoundsLds *>(sm), false);
        if (bb != kBoundsSkipped && threadIdx.x == 0)
            __hip_atomic_store(&w.ctl->bpub, ((u64)pub_gen << 32) | bb, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const unsigned ngb = gridDim.x - 1u, bid = blockIdx.x - 1u;
    gather_body(key, orig, r, n, w, fs, (int)bid, gen, skip);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned grp = bid & 7u, ng = min(ngb, 8u);
        const unsigned gsz = (ngb - grp + 7u) / 8u;
        unsigned *gc = w.wctr + WCTR * (1 + grp);
        bool last = false;
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
            __hip_atomic_exchange(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = __hip_atomic_fetch_add(w.wctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
            if (last) __hip_atomic_exchange(w.wctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    final_body(w, (int)ngb, n, lam, lam_dev, st, skip, lc, fuse_loop, host_flag, fs, cap, sm);
}

// ======================================================== window path (one launch)
// A later loop-body call of a stage (win_ok: C3 from the sixth call on) moves the
// threshold by a few to a few dozen rows, so one launch replaces hist / reduce / bounds +
// gather / final (~47 us of four launches at C3):
//  * every workgroup (HT threads x GI rows, the gather's shape) classifies its rows against
//    the key window [wlo, whi) of half-width H = 2^win_lh(tmove, wfloor) around the previous
//    threshold key: a row below it is selected whatever k is, so it adds to the count, the
//    sum of r and the 8 fit sums; a row inside is appended to the window rows (key, r,
//    caller index and its fit pair; one append counter per XCD); every row outside adds to
//    one of NCS coarse buckets per side, whose widths grow with the distance from the
//    window (H/4 units: 1, 1, 1, 1, then 4 per octave), counted with exact fixed-point sums
//    of r (LDS atomics, then agent-scope atomics into NCB words);
//  * the workgroup's totals go to the launch's accumulators with agent-scope atomics, in an
//    order-free exact form (round 5): counts as integers, the workgroup's fp64 sums of r
//    and of the fit terms (fixed trees inside the workgroup) as fixed-point integers on a
//    grid that holds them exactly (wfx_grid), split into 48-bit digits.  Any arrival order
//    gives the same total bits, so the last workgroup reads ~300 words instead of ~250
//    per-workgroup records (round 4: records + their fixed-order sums, ~5 us of its tail);
//  * the last workgroup to arrive (k_fit_sums' two-level hand-off) sorts the window rows
//    in LDS, scans them from (K0, S0) and takes the first FRMSD minimum inside the window,
//    then proves it global as k_sel_bounds does: every non-empty coarse bucket's lower
//    bound of h (block_lb: its rows are >= the bucket's lowest r) exceeds h at the
//    minimum + kMarg.  A bucket's width is at most ~1/4 of its distance from the window,
//    so its lower bound stays above the curve's rise there (fixed-width coarse buckets
//    next to the window were ~1e-3 loose in h at the window edge, where the curve rises
//    ~1e-7 above its minimum).  Then publish, the loop step, the fit of the next body
//    (the rows below the window + the selected window rows in sorted order) and the host
//    flag, as k_sel_final.
//  * Anything unproven (> CAP window rows, none, a non-finite r, a workgroup sum of r off
//    the grid, a bound <= U): the launch leaves the state alone except win_fail and
//    nn_reuse (the queued NN launch becomes a no-op) and stores kFlagRetry; the host
//    then enqueues launch_select for the same call.  The result never depends on which
//    path decided: both give the first minimum of the same exact curve (S sums differ in
//    their last bits only: k is pinned where the curve separates by > 1e-9).
using fb::WMap;
using fb::win_map;
using fb::win_cq;
using fb::win_cq_lo;
using fb::win_bucket_lo;
using fb::win_bucket_hi;
using fb::win_bucket_exp;

__device__ __forceinline__ void win_retry(IterState *st, int *host_flag) {
    st->nn_reuse = 1;  // the NN launch queued behind this one keeps the current outputs
    st->win_fail = 1;
    if (host_flag) __hip_atomic_store(host_flag, kFlagRetry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// c <= SMALL_C window rows (the normal case: tens): one row per thread, ranked
// by (key, orig) against all of them (LDS broadcast reads), one block scan in sorted order,
// FRMSD of every position, first minimum (final_small's arithmetic, on rows already in
// LDS).  s_aux receives S at the minimum and its threshold pair.
__device__ ScanOut win_scan_small(unsigned c, const FinalIn &in, const u64 *lk, const uint32_t *lo,
                                  const double *lr, uint16_t *pos, Scr &scr, u64 *s_aux) {
    const unsigned t = threadIdx.x;
    if (t < c) {
        const u64 k = lk[t];
        const uint32_t o = lo[t];
        unsigned rank = 0;
        // 8 rows' LDS loads in flight at a time (a plain loop waited for each in turn)
        const unsigned c8 = c & ~7u;
        for (unsigned j = 0; j < c8; j += 8) {
#pragma unroll
            for (unsigned u = 0; u < 8; ++u) rank += less_ko(lk[j + u], lo[j + u], k, o) ? 1u : 0u;
        }
        for (unsigned j = c8; j < c; ++j) rank += less_ko(lk[j], lo[j], k, o) ? 1u : 0u;
        pos[rank] = (uint16_t)t;
    }
    __syncthreads();
    const unsigned e = t < c ? pos[t] : 0u;
    const double v = t < c ? lr[e] : 0.0;
    double all;
    const double ex = blk_excl_scan_d(v, scr, all);
    const double S = in.S0 + (ex + v);
    double bf = INFINITY;
    long long bk = 0x7fffffffffffffffLL;
    if (t < c) {
        const long long kk = in.K0 + (long long)t + 1;
        const double f = frmsd_of(kk, in.N, S, in.lam);
        if (f < bf) {
            bf = f;
            bk = kk;
        }
    }
    blk_argmin(bf, bk, scr);
    if (t < c && in.K0 + (long long)t + 1 == bk) {
        s_aux[0] = (u64)__double_as_longlong(S);
        s_aux[1] = lk[e];
        s_aux[2] = (u64)lo[e];
    }
    __syncthreads();
    ScanOut r{bf, bk, 0, 0, all};
    if (bk != 0x7fffffffffffffffLL) {
        r.tk = s_aux[1];
        r.to = (uint32_t)s_aux[2];
    }
    return r;
}

// a word another workgroup of this launch stored (agent scope: past this CU's L1)
__device__ __forceinline__ double win_ld(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// --- order-free exact accumulation across workgroups
// v * 2^g truncated toward zero, two's complement in 128 bits (|v| 2^g < 2^126); *exact:
// whether no bit of v lies below the grid
__device__ __forceinline__ u128 wfx_grid(double v, int g, bool *exact) {
    const u64 b = (u64)__double_as_longlong(v);
    const int ex = (int)((b >> 52) & 0x7ff);
    if (ex == 0) {  // zero or subnormal
        *exact = (b << 1) == 0ULL;
        return (u128)0;
    }
    const u64 m = (b & 0xfffffffffffffULL) | (1ULL << 52);
    const int sft = ex - 1075 + g;
    u128 a;
    if (sft >= 0) {
        a = (u128)m << sft;
        *exact = true;
    } else if (sft > -64) {
        a = (u128)(m >> (-sft));
        *exact = (m & ((1ULL << (-sft)) - 1ULL)) == 0ULL;
    } else {
        a = (u128)0;
        *exact = false;
    }
    return (b >> 63) ? (u128)0 - a : a;
}
// the three 48-bit digits of a (the top one signed), each added with one atomic: the
// digit sums of up to 2^12 workgroups per word stay below 2^60
constexpr u64 kD48 = (1ULL << 48) - 1ULL;
__device__ __forceinline__ void wfx_add3(u64 *w3, u128 a) {
    __hip_atomic_fetch_add(&w3[0], (u64)a & kD48, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&w3[1], (u64)(a >> 48) & kD48, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&w3[2], (u64)((__int128)a >> 96), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the accumulated value (digit sums s0, s1 >= 0, s2 signed) / 2^g, rounded (a fixed
// formula: the same bits for the same digit sums).  The digits are recombined in integer
// arithmetic first (mod 2^128: exact, the total is below 2^127): a negative total has a
// large positive low part and a negative top digit, whose separate conversions cancelled.
__device__ __forceinline__ double wfx_total(u64 s0, u64 s1, u64 s2, int g) {
    const u128 v = (u128)s0 + ((u128)s1 << 48) + ((u128)s2 << 96);
    const bool neg = (v >> 127) != 0;
    const u128 a = neg ? (u128)0 - v : v;
    const double d = ldexp((double)(u64)(a >> 64), 64 - g) + ldexp((double)(u64)a, -g);
    return neg ? -d : d;
}
// the accumulator words of one copy (kWinCopies copies, blockIdx % kWinCopies)
constexpr int WA_BEL = 0;   // rows below the window
constexpr int WA_BAD = 1;   // non-finite rows + workgroup sums of r off the grid
constexpr int WA_S0 = 2;    // 3 digits: sum of r below the window, grid 2^(100 - e_below)
constexpr int WA_FIT = 5;   // 8 x 3 digits: the fit sums of the rows below it, grid 2^56
constexpr int WA_KMN = 29;  // max of ~key (the call's smallest finite key)
constexpr int WA_KMX = 30;  // max of key
constexpr int WA_SWIN = 31; // the window rows' fixed-point floor sum of r (unit 2^(e_win - fxb))
constexpr int WACC = 32;
constexpr int WFIT_G = 56;
constexpr int WCNT_S = 16;  // append counters 64 B apart (one per XCD copy)
static_assert(WACC == 32 && WCNT_S == 16, "carve_bytes' window words");
// r < 2^e for every row with a key <= khi (win_bucket_exp's rule)
__device__ __forceinline__ int win_key_exp(u64 khi) {
    if (!(khi >> 63)) return 0;
    const int ex = (int)((khi >> 52) & 0x7ffULL);
    return min(2 * ex - 2044, 1024);
}
__device__ __forceinline__ int win_s0_grid(const WMap &m) {
    // r < 2^e for every row below the window (the nearest coarse bucket's exponent); a
    // workgroup's sum < 2^(e + 12) lands below 2^112 on this grid
    const int e = win_bucket_exp(m, NCS - 1);
    return 100 - min(e, 900);
}

// window rows in LDS for lds_sort_scan<CAP, true, true> + where each one's pair lies
constexpr int W_ROW = LdsLay<CAP, true>::END;
constexpr int W_MAXWG = 2 * NSB - 1;  // workgroups of one launch (8M rows: 1954)
constexpr int W_SMEM = W_ROW + CAP * 4;
static_assert(W_SMEM <= 132 * 1024, "window path LDS");

#ifdef FICP_WIN_PROF
__device__ unsigned long long g_winp[8];
#define WINP_B(i)                                                         \
    do {                                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_winp[i] = wall_clock64(); \
    } while (0)
#define WINP_T(i)                                 \
    do {                                          \
        __syncthreads();                          \
        if (threadIdx.x == 0) wt_[i] = wall_clock64(); \
    } while (0)
#else
#define WINP_B(i) \
    do {          \
    } while (0)
#define WINP_T(i) \
    do {          \
    } while (0)
#endif

// The window path's decision (k_sel_win's last workgroup): the accumulators, the coarse
// buckets and the append counters (each read and zeroed), the window rows, the bounds.
__device__ __forceinline__ void win_tail(SelWS w, int64_t n, const WMap &m0, double lamv,
                                         IterState *st, const LoopCtl &lc, int *host_flag,
                                         const FitSrc &fs, int force_retry, Scr &scr) {
    const int t = threadIdx.x;
#ifdef FICP_WIN_PROF
    unsigned long long wt_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // (phase stamps, FICP_WIN_PROF)
#endif
    WINP_T(0);
    __shared__ __align__(16) unsigned char sm[W_SMEM];
    __shared__ IterState s_st;
    __shared__ double s_fit[8];
    __shared__ u64 s_tko[2];
    __shared__ u64 s_acc[kWinCopies * WACC];
    __shared__ unsigned s_wc[kWinCopies + 1];
    using LY = LdsLay<CAP, true>;
    // small windows (<= SMALL_C rows): the rows' fit pairs, also in the bin area (no bins)
    double4 *lpair = (double4 *)(sm + LY::BC);
    static_assert(SMALL_C * 32 <= 2 * NSB * 4, "the window pairs in the bin area");
    // one round of exchanges: the coarse buckets, the accumulators, the append counters
    unsigned cc = 0;
    u64 cf = 0;
    if (t < NCB) {
        unsigned cq[kWinCopies];
        u64 fq[kWinCopies];
#pragma unroll
        for (int q = 0; q < kWinCopies; ++q) {
            cq[q] = __hip_atomic_exchange(&w.gcc[q * NCB + t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fq[q] = __hip_atomic_exchange(&w.gcf[q * NCB + t], (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int q = 0; q < kWinCopies; ++q) {  // (integers: exact in any order)
            cc += cq[q];
            cf += fq[q];
        }
    }
    static_assert(kWinCopies * WACC <= HT, "one accumulator word per thread");
    const u64 av = t < kWinCopies * WACC
                       ? __hip_atomic_exchange(&w.wacc[t], (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0ULL;
    const unsigned wcv = (t >= HT - kWinCopies)
                             ? __hip_atomic_exchange(&w.wcnt[(t - (HT - kWinCopies)) * WCNT_S], 0u,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0u;
    constexpr int SW = (int)(sizeof(IterState) / 4);
    for (int q = t; q < SW; q += HT) ((uint32_t *)&s_st)[q] = ((const uint32_t *)st)[q];
    if (t < kWinCopies * WACC) s_acc[t] = av;
    if (t >= HT - kWinCopies) s_wc[t - (HT - kWinCopies)] = wcv;
    __syncthreads();
    WINP_T(6);
    // the copies combined (integers: any order), field by field
    __shared__ u64 s_tot[WACC];
    if (t < WACC) {
        u64 v = 0ULL;
        for (int q = 0; q < kWinCopies; ++q) {
            const u64 x = s_acc[q * WACC + t];
            v = (t == WA_KMN || t == WA_KMX) ? max(v, x) : v + x;
        }
        s_tot[t] = v;
    }
    if (t == WACC) {  // the append counters' prefix (region q: rows [s_wc[q], s_wc[q + 1]))
        unsigned run = 0;
        bool over = false;
        for (int q = 0; q < kWinCopies; ++q) {
            const unsigned c = s_wc[q];
            over = over || c > (unsigned)CAP;
            s_wc[q] = run;
            run += c;
        }
        s_wc[kWinCopies] = over ? (unsigned)(CAP + 1) : run;
    }
    __syncthreads();
    const long long Wt = (long long)s_wc[kWinCopies];  // (a region past CAP: the launch fails)
    const long long K0 = (long long)s_tot[WA_BEL];
    const long long bad = (long long)s_tot[WA_BAD];
    const int gs0 = win_s0_grid(m0);
    const double S0 = wfx_total(s_tot[WA_S0], s_tot[WA_S0 + 1], s_tot[WA_S0 + 2], gs0);
    // a lower bound of the window rows' sum (their floor sums: order-free, so the coarse
    // bounds above the window need not wait for the sorted scan)
    const double Swin_lo = ldexp((double)s_tot[WA_SWIN], win_key_exp(m0.whi - 1ULL) - m0.fxb);
    WMap m = m0;  // with the call's key range (the lowest coarse bucket's lowest r)
    m.kmin = ~s_tot[WA_KMN];
    m.kmax = s_tot[WA_KMX];
    if (t < 8)
        s_fit[t] = wfx_total(s_tot[WA_FIT + 3 * t], s_tot[WA_FIT + 3 * t + 1], s_tot[WA_FIT + 3 * t + 2], WFIT_G);
    bool fail = bad != 0 || Wt <= 0 || Wt > CAP;
    const double p = 2.0 * lamv + 1.0;
    u64 *lk = (u64 *)(sm + LY::K);
    double *lr = (double *)(sm + LY::R);
    uint32_t *lo = (uint32_t *)(sm + LY::O);
    uint32_t *lrow = (uint32_t *)(sm + W_ROW);  // where each LDS row's pair lies (slot)
    constexpr int EU = CAP / HT;
    const bool pin = Wt <= SMALL_C;  // the small windows' pairs go to LDS
    // every window row is a candidate; their loads first (the pairs of the first HT rows
    // too), the coarse bounds while they are in flight
    uint32_t sl[EU];
    u64 vk[EU];
    double vr[EU];
    uint32_t vo[EU];
    double4 vp = make_double4(0.0, 0.0, 0.0, 0.0);
    if (!fail) {
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const int e = t + u * HT;
            int q = 0;
#pragma unroll
            for (int j = 1; j < kWinCopies; ++j) q += (e >= (int)s_wc[j]) ? 1 : 0;
            sl[u] = (uint32_t)(q * CAP + (e - (int)s_wc[q]));
            if (e < Wt) {
                vk[u] = __hip_atomic_load(&w.wk[sl[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vr[u] = __hip_atomic_load(&w.wr[sl[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vo[u] = __hip_atomic_load(&w.wo[sl[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (u == 0 && pin && fs.on) {
                    const double *pp = w.wp + 4 * (int64_t)sl[0];
                    vp = make_double4(win_ld(pp), win_ld(pp + 1), win_ld(pp + 2), win_ld(pp + 3));
                }
            }
        }
    }
    // every coarse bucket's lower bound of h (k_sel_bounds' block_lb): rows before it = the
    // buckets before it (+ the window's rows above it); lower sum = the fixed-point brackets
    // before it (+ S0 and the window's floor sum above it)
    double lbv = INFINITY;
    bool lbok = true;
    {
        const int eb = t < NCB ? win_bucket_exp(m, t) : 0;
        const double lo_sum = (t < NCB && eb < 1024) ? ldexp((double)cf, eb - m.fxb) : 0.0;  // (exact)
        long long C0 = t < NCB ? (long long)cc : 0;
        double Pb = (t < NCS) ? lo_sum : 0.0;
        double Pa = (t >= NCS && t < NCB) ? lo_sum : 0.0;
        blk_excl_scan3(C0, Pb, Pa, scr);
        if (t == NCS - 1 && C0 + (long long)cc != K0) lbok = false;  // (a row lost: never)
        if (t < NCB && cc) {
            const bool below = t < NCS;
            lbv = block_lb(below ? C0 : C0 + Wt, (long long)cc, below ? Pb : (S0 + Swin_lo) + Pa,
                           lo_r(win_bucket_lo(m, t)), p);
        }
    }
    if (!fail) {
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const int e = t + u * HT;
            if (e < Wt) {
                lk[e] = vk[u];
                lr[e] = vr[u];
                lo[e] = vo[u];
                lrow[e] = sl[u];
                if (u == 0 && pin) lpair[e] = vp;
            }
        }
    }
    __syncthreads();
    WINP_T(2);
    FinalIn in;
    in.N = n;
    in.lam = lamv;
    in.S0 = S0;
    in.K0 = K0;
    in.U = 0.0;
    in.fs = fs;
    in.fsum = s_fit;
    ScanOut rs{INFINITY, 0x7fffffffffffffffLL, 0, 0, 0.0};
    __shared__ u64 s_aux[3];
    const bool small = Wt <= SMALL_C;  // (its rank loop is O(c) per row: 492 rows took 17.6 us)
    if (!fail) {
        if (small) {
            rs = win_scan_small((unsigned)Wt, in, lk, lo, lr, (uint16_t *)(sm + LY::POS), scr, s_aux);
        } else {
            const Cand none{nullptr, nullptr, nullptr, nullptr};
            rs = lds_sort_scan<CAP, true, true>(none, (unsigned)Wt, in.K0, in.S0, in, sm, scr);
        }
        fail = rs.bk == 0x7fffffffffffffffLL;
    }
    WINP_T(3);
    // the minimum is global: every coarse bucket's lower bound of h exceeds U
    double U = INFINITY;
    if (!fail) {
        // S at the minimum: s_aux (small) or lds_sort_scan's prefix sums by position in lr
        const double Sbk = small ? __longlong_as_double((long long)s_aux[0]) : in.S0 + lr[rs.bk - in.K0 - 1];
        U = h_of(rs.bk, Sbk, p) + kMarg;
        if (t == 0) {
            s_tko[0] = rs.tk;
            s_tko[1] = (u64)rs.to;
        }
    }
    const bool ok = lbok && (lbv > U);  // (empty buckets: lbv = inf)
    fail = fail || blk_max_ll(ok ? 0 : 1, scr) != 0 || force_retry;  // (its barriers publish s_tko)
    WINP_T(4);
#ifdef FICP_WIN_PROF
    if (fail && t == 0)
        printf("WINPROF W=%lld K0=%lld fail=1 | b0 load %llu cls %llu red %llu app %llu atom %llu wait %llu -> tail +%llu | acc %llu rows %llu sort %llu bounds %llu (10 ns)\n",
               Wt, K0, g_winp[1] - g_winp[0], g_winp[3] - g_winp[1], g_winp[4] - g_winp[3],
               g_winp[5] - g_winp[4], g_winp[2] - g_winp[5], g_winp[6] - g_winp[2], wt_[0] - g_winp[6],
               wt_[6] - wt_[0], wt_[2] - wt_[6], wt_[3] - wt_[2], wt_[4] - wt_[3]);
#endif
    if (fail) {
        if (t == 0) win_retry(st, host_flag);
        return;
    }
    // the fit of the selected candidates, in sorted order (positions t, t + HT, ...; a
    // fixed tree: deterministic): their pairs from LDS (small windows) or the pair array
    const uint32_t nsel = (uint32_t)(rs.bk - in.K0);
    if (fs.on) {
        const uint16_t *pos = (const uint16_t *)(sm + LY::POS);
        double cf8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t q = t; q < nsel; q += HT) {
            if (pin) {
                const double4 v = lpair[pos[q]];
                fit_add(cf8, v.x, v.y, v.z, v.w, fs.px, fs.py);
            } else {
                const double *pp = w.wp + 4 * (int64_t)lrow[pos[q]];
                fit_add(cf8, win_ld(pp), win_ld(pp + 1), win_ld(pp + 2), win_ld(pp + 3), fs.px, fs.py);
            }
        }
        blk_sum8_add(cf8, s_fit, scr);
    }
    WINP_T(8);
    if (t == 0) {
        IterState L = s_st;  // (thread 0's step on a register copy, as k_sel_final)
        publish(&L, in, rs.bf, rs.bk, s_tko[0], (uint32_t)s_tko[1]);
        // the next window's smallest half-width from this one's row count (2^lh keys)
        {
            const int f = win_floor(L.wfloor, n);
            if (Wt > 384) L.wfloor = max(kWinHMinLog, min(f, m.su + 2) - 1);
            else if (Wt < 48) L.wfloor = min(win_start_log(n), f + 1);
        }
        loop_step(&L, lc);
        if (fs.on && !L.no_fit && L.k > 0) fit_solve(s_fit, (double)L.k, fs.px, fs.py, fs.allow_refl, &L);
        s_st = L;
    }
    __syncthreads();
    WINP_T(9);
    for (int q = t; q < SW; q += HT) ((uint32_t *)st)[q] = ((const uint32_t *)&s_st)[q];
    if (t == 0 && host_flag)
        __hip_atomic_store(host_flag, s_st.done | (win_ok(s_st) ? kFlagWinNext : 0),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#ifdef FICP_WIN_PROF
    WINP_T(5);
    // (printed after the last stamp: a device printf is a host round trip)
    if (t == 0)
        printf("WINPROF W=%lld K0=%lld fail=0 | b0 load %llu cls %llu red %llu app %llu atom %llu wait %llu -> tail +%llu | acc %llu rows %llu sort %llu bounds %llu fit %llu step %llu store %llu (10 ns)\n",
               Wt, K0, g_winp[1] - g_winp[0], g_winp[3] - g_winp[1], g_winp[4] - g_winp[3],
               g_winp[5] - g_winp[4], g_winp[2] - g_winp[5], g_winp[6] - g_winp[2], wt_[0] - g_winp[6],
               wt_[6] - wt_[0], wt_[2] - wt_[6], wt_[3] - wt_[2], wt_[4] - wt_[3], wt_[8] - wt_[4],
               wt_[9] - wt_[8], wt_[5] - wt_[9]);
#endif
}

__global__ __launch_bounds__(HT) void k_sel_win(const double *r, const uint32_t *orig, int64_t n,
                                               const u64 *range, int64_t nparts, SelWS w,
                                               IterState *st, LoopCtl lc, int *host_flag,
                                               FitSrc fs, int force_retry) {
    constexpr int WI = GI;  // rows per thread (stride HT)
    static_assert(GT == HT, "k_sel_win: gather's workgroup shape");
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    __shared__ Scr scr;
    // coarse buckets in LDS, WREP copies by lane % WREP (most rows of a wave fall into a
    // few coarse buckets: one copy serialised up to 64 lanes per atomic), rows padded so
    // that a bucket's copies sit in different banks
    constexpr int WREP = 8, WRS = NCB + 1;
    __shared__ unsigned s_cc[WREP * WRS];
    __shared__ u64 s_cf[WREP * WRS];
    __shared__ double s_red[NWAVE][9];
    __shared__ u64 s_cnt[NWAVE];
    __shared__ int s_last;
    WINP_B(0);
    // every independent load first: the state's window inputs, the rows, the range parts
    const int sk = st->done;
    const int ph = st->phase, itv = st->it, stg = st->stage, wfl = st->wfloor;
    const long long kprev = st->k;
    const u64 tkey = st->tkey, tmove = st->tmove;
    const double lamv = st->lam_cur;
    // row q of this thread: pairs of consecutive rows per lane, so that every load is 16 B
    // (8-B lanes stream at 0.54-0.70x the 16-B rate, MI355X_MICROARCH.md)
    const int64_t base = (int64_t)blockIdx.x * (HT * WI) + 2 * t;
    auto row_of = [&](int q) -> int64_t { return base + (int64_t)(q >> 1) * (2 * HT) + (q & 1); };
    double rr[WI], xs[WI], ys[WI], xt[WI], yt[WI];
    uint32_t oo[WI];
#pragma unroll
    for (int q = 0; q < WI; q += 2) {
        // (i is even; the buffers hold n + 1 rows, so the pair of row n - 1 is readable; a
        // pair at or past n reads pair 0, whose values the row tests below ignore)
        const int64_t i = row_of(q) < n ? row_of(q) : 0;
        const double2 a = *reinterpret_cast<const double2 *>(r + i);
        const double2 b = *reinterpret_cast<const double2 *>(fs.sx + i);
        const double2 c = *reinterpret_cast<const double2 *>(fs.sy + i);
        const double2 d = *reinterpret_cast<const double2 *>(fs.cx + i);
        const double2 e = *reinterpret_cast<const double2 *>(fs.cy + i);
        const uint2 o = *reinterpret_cast<const uint2 *>(orig + i);
        rr[q] = a.x, rr[q + 1] = a.y;
        xs[q] = b.x, xs[q + 1] = b.y;
        ys[q] = c.x, ys[q + 1] = c.y;
        xt[q] = d.x, xt[q + 1] = d.y;
        yt[q] = e.x, yt[q + 1] = e.y;
        oo[q] = o.x, oo[q + 1] = o.y;
    }
    if (sk) {  // the run is over: the flag as k_sel_final's no-op
        if (blockIdx.x == 0 && t == 0 && host_flag)
            __hip_atomic_store(host_flag, kFlagDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    for (int b = t; b < WREP * WRS; b += HT) {
        s_cc[b] = 0u;
        s_cf[b] = 0ULL;
    }
    const WMap m0 = win_map(tkey, tmove, wfl, n);
    __shared__ int s_ce[NCB];  // each coarse bucket's fixed-point exponent
    if (t < NCB) s_ce[t] = win_bucket_exp(m0, t);
    // (uniform over the launch: every workgroup decides the same way, none arrives)
    if (!(ph == PH_LOOP && (itv >= 1 || win_first_body(itv, stg, tmove)) && kprev > 0 &&
          2.0 * lamv + 1.0 >= 1.0 && m0.ok)) {
        if (blockIdx.x == 0 && t == 0) win_retry(st, host_flag);
        return;
    }
    const int ewin = win_key_exp(m0.whi - 1ULL);  // r < 2^ewin in the window
    // an LDS-only barrier: __syncthreads() would also wait for every row's load
    // (vmcnt(0)); this way the rows are classified as their loads land
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    WINP_B(1);
    // classify the rows
    unsigned nbel = 0, nbad = 0;
    u64 kmn = ~0ULL, kmx = 0ULL;  // the finite rows' key range (the last workgroup's kmin)
    double sb = 0.0;
    double c8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u64 kk[WI];
    unsigned inw = 0;
    u64 swfx = 0;  // the window rows' floor sum of r (unit 2^(ewin - fxb): an order-free lower bound)
    unsigned *my_cc = s_cc + (lane % WREP) * WRS;
    u64 *my_cf = s_cf + (lane % WREP) * WRS;
#pragma unroll
    for (int q = 0; q < WI; ++q) {
        const int64_t i = row_of(q);
        kk[q] = 0ULL;
        if (i < n) {
            const double v = rr[q];
            if (!(v < INFINITY)) {  // inf / NaN: the full selection's special cases
                ++nbad;
                continue;
            }
            const u64 k = key_of_r(v);
            kk[q] = k;
            kmn = min(kmn, k);
            kmx = max(kmx, k);
            if (k < m0.wlo) {
                ++nbel;
                sb = sb + v;
                fit_add(c8, xs[q], ys[q], xt[q], yt[q], fs.px, fs.py);
                const int b = NCS - 1 - win_cq((m0.wlo - 1ULL - k) >> m0.su);
                const int e = s_ce[b];
                atomicAdd(&my_cc[b], 1u);
                atomicAdd(&my_cf[b], e < 1024 ? (u64)ldexp(v, m0.fxb - e) : 0ULL);
            } else if (k < m0.whi) {
                inw |= 1u << q;
                swfx += ewin < 1024 ? (u64)ldexp(v, m0.fxb - ewin) : 0ULL;
            } else {
                const int b = NCS + win_cq((k - m0.whi) >> m0.su);
                const int e = s_ce[b];
                atomicAdd(&my_cc[b], 1u);
                atomicAdd(&my_cf[b], e < 1024 ? (u64)ldexp(v, m0.fxb - e) : 0ULL);
            }
        }
    }
    WINP_B(3);
    // the window rows appended to this XCD copy's region (one atomic per wave that has
    // any; the tail orders them by (key, caller index), so the append order is free)
    const int cp = (int)(blockIdx.x % kWinCopies);
    u64 masks[WI];
    unsigned wtot = 0;
#pragma unroll
    for (int q = 0; q < WI; ++q) {
        masks[q] = __ballot((inw >> q) & 1u);
        wtot += (unsigned)__popcll(masks[q]);
    }
    {
        if (wtot) {  // (uniform per wave)
            unsigned wb = 0;
            if (lane == 0)
                wb = __hip_atomic_fetch_add(&w.wcnt[cp * WCNT_S], wtot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wb = __shfl(wb, 0);
            const u64 lt = (1ULL << lane) - 1ULL;
#pragma unroll
            for (int q = 0; q < WI; ++q) {
                if ((inw >> q) & 1u) {
                    const unsigned sidx = wb + (unsigned)__popcll(masks[q] & lt);
                    if (sidx < (unsigned)CAP) {  // (past CAP the tail fails the launch)
                        const int64_t s = (int64_t)cp * CAP + sidx;
                        __hip_atomic_store(&w.wk[s], kk[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wr[s], rr[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wo[s], oo[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wp[4 * s], xs[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wp[4 * s + 1], ys[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wp[4 * s + 2], xt[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&w.wp[4 * s + 3], yt[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                wb += (unsigned)__popcll(masks[q]);
            }
        }
    }
    // the workgroup's sums (fixed trees: DPP wave sums, then the waves in order)
    sb = wave_sum63(sb);
#pragma unroll
    for (int e = 0; e < 8; ++e) c8[e] = wave_sum63(c8[e]);
    const u64 cnt = wave_sum63_u64((u64)nbel | ((u64)nbad << 32));
    const u64 swv = wave_sum63_u64(swfx);
    __shared__ u64 s_swin[NWAVE];
    u64 pka = ~kmn, pkb = kmx;
    wave_range_reduce(pka, pkb);  // (max of ~kmin and of kmax, lane 63)
    __shared__ u64 s_kr[NWAVE][2];
    if (lane == 63) {
        s_kr[wave][0] = pka;
        s_kr[wave][1] = pkb;
        s_red[wave][0] = sb;
#pragma unroll
        for (int e = 0; e < 8; ++e) s_red[wave][1 + e] = c8[e];
        s_cnt[wave] = cnt;
        s_swin[wave] = swv;
    }
    __syncthreads();  // (the LDS atomics, the wave counts and sums are complete)
    WINP_B(4);
    // the coarse buckets first: their atomics complete while the rest is added
    if (t < NCB) {
        unsigned c = 0;
        u64 f = 0;
#pragma unroll
        for (int q = 0; q < WREP; ++q) {
            c += s_cc[q * WRS + t];
            f += s_cf[q * WRS + t];
        }
        if (c) {
            const int cb = cp * NCB + t;  // (the XCD's copy)
            __hip_atomic_fetch_add(&w.gcc[cb], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&w.gcf[cb], f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the workgroup's totals into the accumulators (the last wave: wave 0 flushed the
    // buckets): lane 0 the sum of r below (grid 2^g0), lanes 1-8 the fit sums (2^56),
    // lane 9 the counts, lane 10 the key range, lane 11 the window rows' floor sum
    if (wave == NWAVE - 1 && lane < 12) {
        u64 *acc = w.wacc + cp * WACC;
        if (lane < 9) {
            double v = s_red[0][lane];
            for (int q = 1; q < NWAVE; ++q) v = v + s_red[q][lane];
            bool exact = true;
            const u128 a = wfx_grid(v, lane == 0 ? win_s0_grid(m0) : WFIT_G, &exact);
            wfx_add3(acc + (lane == 0 ? WA_S0 : WA_FIT + 3 * (lane - 1)), a);
            // a sum of r off its grid cannot be carried exactly: the tail falls back
            if (lane == 0 && !exact)
                __hip_atomic_fetch_add(&acc[WA_BAD], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (lane == 9) {
            u64 cv = 0;
            for (int q = 0; q < NWAVE; ++q) cv += s_cnt[q];
            if (cv & 0xffffffffULL)
                __hip_atomic_fetch_add(&acc[WA_BEL], cv & 0xffffffffULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cv >> 32)
                __hip_atomic_fetch_add(&acc[WA_BAD], cv >> 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (lane == 11) {
            u64 sv = 0;
            for (int q = 0; q < NWAVE; ++q) sv += s_swin[q];
            if (sv) __hip_atomic_fetch_add(&acc[WA_SWIN], sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            u64 a = s_kr[0][0], b = s_kr[0][1];
            for (int q = 1; q < NWAVE; ++q) {
                a = max(a, s_kr[q][0]);
                b = max(b, s_kr[q][1]);
            }
            __hip_atomic_fetch_max(&acc[WA_KMN], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_max(&acc[WA_KMX], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    WINP_B(5);
    WINP_B(2);
    // hand-off (k_fit_sums' form): every storing wave waits for its stores and atomics,
    // then one lane arrives at its group counter and the group's last at the top counter
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    WINP_B(6);
    if (t == 0) {
        const unsigned grp = blockIdx.x & 7u, ng = min(gridDim.x, 8u);
        const unsigned gsz = (gridDim.x - grp + 7u) / 8u;
        unsigned *gc = w.wctr + WCTR * (1 + grp);
        bool last = false;
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
            __hip_atomic_exchange(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = __hip_atomic_fetch_add(w.wctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
            if (last) __hip_atomic_exchange(w.wctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    win_tail(w, n, m0, lamv, st, lc, host_flag, fs, force_retry, scr);
}

__global__ void k_sel_init(SelWS w) {
    if (threadIdx.x == 0) {
        __hip_atomic_exchange(&w.ctl->ccount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_exchange(&w.ctl->err, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w.ctl->levels = 0;
        w.ctl->radix = 0;
        __hip_atomic_store(&w.ctl->bpub, (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the window path's coarse buckets and arrival counters
    for (int b = threadIdx.x; b < kWinCopies * NCB; b += blockDim.x) {
        __hip_atomic_exchange(&w.gcc[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_exchange(&w.gcf[b], (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int b = threadIdx.x; b < 9 * WCTR; b += blockDim.x)
        __hip_atomic_exchange(&w.wctr[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int b = threadIdx.x; b < kWinCopies * WACC; b += blockDim.x)
        __hip_atomic_exchange(&w.wacc[b], (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int b = threadIdx.x; b < kWinCopies * WCNT_S; b += blockDim.x)
        __hip_atomic_exchange(&w.wcnt[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- distributed selection (source rows split over ranks) -------
// Every rank holds the NN results of its own rows.  The histogram's integer totals are
// summed over the ranks (exact, order-free), so every rank derives the same bounds and
// candidate buckets; each rank packs its candidates and the sum of its rows below them,
// the ranks' packs are gathered, and every rank runs the same final selection on the
// concatenation (the S_base parts added in rank order: identical k everywhere).
// Pack layout (int64 words): [0] count, [1] S_base bits, [2] overflow, [3] 0,
// then capd keys, capd caller indices, capd r bits.

// bracket + chunk totals from the ranks' summed integer histogram (64 buckets per block)
__global__ __launch_bounds__(64) void k_sel_finish(SelWS w, const long long *hist,
                                                   const int *skip, HistPack hp) {
    if (skip && *skip) return;
    const int bl = threadIdx.x, b = blockIdx.x * 64 + bl;
    reduce_tail(w, b, bl, (unsigned)hist[b], (u64)hist[NB + b], hp);
}

__global__ __launch_bounds__(HT) void k_sel_pack(SelWS w, int nparts, const int *skip,
                                                 long long *out, int capd) {
    if (skip && *skip) return;
    __shared__ Scr scr;
    const unsigned c = __hip_atomic_fetch_add(&w.ctl->ccount, 0u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    double a = 0.0;
    for (int p = threadIdx.x; p < nparts; p += HT) a = a + w.parts[p];  // fixed order per thread
    const double sb = blk_sum(a, scr);
    const unsigned cc = min(c, (unsigned)capd);
    if (threadIdx.x == 0) {
        out[0] = (long long)cc;
        out[1] = __double_as_longlong(sb);
        out[2] = c > (unsigned)capd ? 1 : 0;
        out[3] = 0;
    }
    for (unsigned j = threadIdx.x; j < cc; j += HT) {
        out[4 + j] = (long long)w.ka[j];
        out[4 + capd + j] = (long long)w.oa[j];
        out[4 + 2 * (int64_t)capd + j] = __double_as_longlong(w.ra[j]);
    }
}

__global__ __launch_bounds__(HT) void k_sel_unpack(SelWS w, const long long *all, int world,
                                                   int capd, const int *skip) {
    if (skip && *skip) return;
    const int64_t stride = 4 + 3 * (int64_t)capd;
    unsigned base = 0, over = 0;
    for (int q = 0; q < world; ++q) {
        const long long *pk = all + q * stride;
        const unsigned cq = (unsigned)pk[0];
        for (unsigned j = threadIdx.x; j < cq; j += HT) {
            w.ka[base + j] = (u64)pk[4 + j];
            w.oa[base + j] = (uint32_t)pk[4 + capd + j];
            w.ra[base + j] = __longlong_as_double(pk[4 + 2 * (int64_t)capd + j]);
            w.pa[base + j] = 0u;
        }
        if (threadIdx.x == 0) w.parts[q] = __longlong_as_double(pk[1]);
        over |= (unsigned)pk[2];
        base += cq;
    }
    if (threadIdx.x == 0) {
        __hip_atomic_exchange(&w.ctl->ccount, base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (over) __hip_atomic_fetch_or(&w.ctl->err, ERR_CAP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

int64_t sel_tmp_bytes(int64_t n) { return carve_bytes(n, nullptr, nullptr); }

unsigned *sel_err_word(void *tmp, int64_t n) { return &carve(tmp, n).ctl->err; }

int sel_hist_words() { return 2 * NB; }

hipError_t launch_select_dist_hist(const unsigned long long *key, const double *r, int64_t n,
                                   int64_t n_max, const unsigned long long *range, void *tmp,
                                   int64_t n_ws, const IterState *st, const int *skip,
                                   long long *hist_out, hipStream_t s) {
    const SelWS w = carve(tmp, n_ws);
    const HistPack hp = hist_pack(n_max);
    hipLaunchKernelGGL(k_sel_hist, dim3(hist_blocks(n_max)), dim3(HHT), 0, s, key, r, n,
                       const_cast<unsigned long long *>(range), (int64_t)0, w, skip, hp, st);
    hipLaunchKernelGGL(k_sel_reduce, dim3(NB / RBPB), dim3(1024), 0, s, w, hist_blocks(n_max), skip,
                       hp, hist_out);
    return hipGetLastError();
}

hipError_t launch_select_dist_gather(const unsigned long long *key, const uint32_t *orig,
                                     const double *r, int64_t n, int64_t n_total, int64_t n_max,
                                     const long long *hist, double lam, const double *lam_dev,
                                     void *tmp, int64_t n_ws, const int *skip, long long *pack,
                                     int capd, hipStream_t s) {
    const SelWS w = carve(tmp, n_ws);
    const HistPack hp = hist_pack(n_max);
    hipLaunchKernelGGL(k_sel_finish, dim3(NB / 64), dim3(64), 0, s, w, hist, skip, hp);
    hipLaunchKernelGGL(k_sel_bounds, dim3(1), dim3(HT), 0, s, w, n_total, lam, lam_dev, skip,
                       hp.fixb);
    const int gb = gather_blocks(n);
    if (n > 0)
        hipLaunchKernelGGL(k_sel_gather, dim3(gb), dim3(GT), 0, s, key, orig, r, n, w, skip,
                           FitSrc{});
    hipLaunchKernelGGL(k_sel_pack, dim3(1), dim3(HT), 0, s, w, n > 0 ? gb : 0, skip, pack, capd);
    return hipGetLastError();
}

hipError_t launch_select_dist_final(const long long *packs, int world, int capd, int64_t n_total,
                                    double lam, const double *lam_dev, void *tmp, int64_t n_ws,
                                    IterState *st, const int *skip, const LoopCtl *loop,
                                    int *host_flag, hipStream_t s) {
    const SelWS w = carve(tmp, n_ws);
    hipLaunchKernelGGL(k_sel_unpack, dim3(1), dim3(HT), 0, s, w, packs, world, capd, skip);
    LoopCtl lc{};
    if (loop) lc = *loop;
    hipLaunchKernelGGL(k_sel_final, dim3(1), dim3(HT), 0, s, w, world, n_total, lam, lam_dev, st,
                       skip, lc, loop ? 1 : 0, host_flag, FitSrc{}, std::max<int64_t>(n_ws, 1));
    return hipGetLastError();
}

bool select_win_fits(int64_t n) { return n > 0 && gather_blocks(n) <= W_MAXWG; }

hipError_t launch_select_win(const double *r, const uint32_t *orig, int64_t n,
                             const unsigned long long *range, int64_t range_parts, void *tmp,
                             IterState *st, const LoopCtl &loop, int *host_flag, hipStream_t s,
                             const FitSrc &fit, int fault) {
    // (the work order's caller indices; the tail's LDS holds the offsets of at most
    // W_MAXWG workgroups, select_win_fits)
    if (n <= 0 || !orig || !select_win_fits(n)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sel_win, dim3(gather_blocks(n)), dim3(HT), 0, s, r, orig, n, range,
                       range_parts, carve(tmp, n), st, loop, host_flag, fit,
                       (fault & FICP_FAULT_WIN) ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_select_init(void *tmp, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(1024), 0, s, carve(tmp, n));
    return hipGetLastError();
}

hipError_t launch_select(const unsigned long long *key, const uint32_t *orig, const double *r,
                         int64_t n, double lam, const double *lam_dev, unsigned long long *range,
                         int64_t range_parts, void *tmp, IterState *st, const int *skip,
                         const LoopCtl *loop, int *host_flag, hipStream_t s, const FitSrc *fit,
                         int fault) {
    if (n <= 0) return hipSuccess;
    const SelWS w = carve(tmp, n);
    const HistPack hp = hist_pack(n);
    hipLaunchKernelGGL(k_sel_hist, dim3(hist_blocks(n)), dim3(HHT), 0, s, key, r, n, range,
                       range_parts, w, skip, hp, (const IterState *)st);
    const int gb = gather_blocks(n);
    FitSrc fs{};
    if (fit && loop) fs = *fit;  // the fused fit needs the fused loop step (it runs after it)
    // launch tokens, unique per launch in this process; the start is salted per process so
    // that a token left in reused device memory by an earlier process cannot match
    static std::atomic<unsigned> s_gen{((unsigned)getpid() * 2654435761u) & 0x3fffffffu};
    unsigned gen = ++s_gen & 0x3fffffffu;
    if (gen == 0) gen = ++s_gen & 0x3fffffffu;  // 0 means "no flag"
    const unsigned pub = (fault & FICP_FAULT_SPIN) ? (gen ^ 0x40000000u) : gen;
    // Two forms of the bounds:
    //  * default: k_sel_bounds_gather -- block 0 of the gather computes the bounds and
    //    publishes them in-launch (relies on block 0 being dispatched first, raising
    //    ERR_SPIN instead of hanging should that order not hold) while the other blocks'
    //    row loads are in flight;
    //  * FICP_SEL_SPLIT=1: k_sel_bounds + k_sel_gather, no in-launch hand-off at all (the
    //    fallback should a dispatcher not keep blockIdx order; ~1.4 % slower at C3).
    const char *sp = getenv("FICP_SEL_SPLIT");
    const bool split = sp && atoi(sp) != 0;
    hipLaunchKernelGGL(k_sel_reduce, dim3(NB / RBPB), dim3(1024), 0, s, w, hist_blocks(n), skip,
                       hp, (long long *)nullptr);
    //  * round 5, the default: k_sel_bgf -- k_sel_bounds_gather with the final in its last
    //    gather workgroup (FICP_SEL_BGF=0: the final as its own launch).
    const char *bg = getenv("FICP_SEL_BGF");
    const bool bgf = !split && !(bg && atoi(bg) == 0);
    LoopCtl lc{};
    if (loop) lc = *loop;
    if (bgf) {
        hipLaunchKernelGGL(k_sel_bgf, dim3(gb + 1), dim3(GT), 0, s, key, orig, r, n, w, lam, lam_dev,
                           skip, hp.fixb, fs, gen, pub, st, lc, loop ? 1 : 0, host_flag,
                           std::max<int64_t>(n, 1));
        return hipGetLastError();
    }
    if (split) {
        hipLaunchKernelGGL(k_sel_bounds, dim3(1), dim3(HT), 0, s, w, n, lam, lam_dev, skip,
                           hp.fixb);
        hipLaunchKernelGGL(k_sel_gather, dim3(gb), dim3(GT), 0, s, key, orig, r, n, w, skip, fs);
    } else {
        hipLaunchKernelGGL(k_sel_bounds_gather, dim3(gb + 1), dim3(GT), 0, s, key, orig, r, n,
                           w, lam, lam_dev, skip, hp.fixb, fs, gen, pub);
    }
    hipLaunchKernelGGL(k_sel_final, dim3(1), dim3(HT), 0, s, w, gb, n, lam, lam_dev, st, skip, lc,
                       loop ? 1 : 0, host_flag, fs, std::max<int64_t>(n, 1));
    return hipGetLastError();
}

}  // namespace ficp
