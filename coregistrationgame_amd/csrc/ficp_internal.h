// ficp_internal.h -- shared types and kernel launchers of libficp (gfx950 only).
//
// Device data layout:
//   source  : SoA fp64 x[n], y[n], z[n] (z only when md == 3); x,y updated in place
//   target  : SoA fp64 tx[m], ty[m], tz[m] (original order, for corr gathers) and a
//             uniform XY grid: cell_start[ncells+1] + TPt pts[m] (cell-sorted AoS,
//             32 B per stem = two dwordx4 loads per candidate)
//   per call: idx[n] int32, dist[n] fp64, r[n] fp64 (= d^2), key[n] u64 (ordered
//             bits of dist), sorted val[n] (source index in selection order)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ficp {

constexpr int kWave = 64;

// order-preserving 64-bit key of a double (for d >= 0: the bits with the sign bit set)
__device__ __forceinline__ unsigned long long ordkey(double v) {
    unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

// the sort key of a row from its squared distance r: ordkey(sqrt(r)), bit for bit what the
// NN kernels store (write_out / cert_try).  The selection recomputes it from r when the NN
// did not store keys (C3 fused loop: 8 B per row less written by the NN and read by the
// histogram and the gather).
__device__ __forceinline__ unsigned long long key_of_r(double r) { return ordkey(sqrt(r)); }

// floor(r / 2^L) of an r >= 0 (finite): the fixed-point grid of order-free bucket sums
// (k_select.hip refine, k_batch.hip k_batch_select)
__device__ __forceinline__ unsigned long long fx_floor(double r, int L) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(r);
    const int ex = (int)((b >> 52) & 0x7ff);
    unsigned long long m = b & 0xfffffffffffffULL;
    int p2;
    if (ex == 0) {
        p2 = -1074;
    } else {
        m |= 1ULL << 52;
        p2 = ex - 1075;
    }
    const int sft = p2 - L;
    return sft >= 0 ? m << sft : (sft > -64 ? m >> (-sft) : 0ULL);
}

// ---- DPP wave reductions (GFX9 data-parallel primitives).  __shfl_xor compiles to
// ds_bpermute through the LDS crossbar (~60-100 cycles a step, 12 steps for a double
// butterfly); these take 6 VALU DPP steps.  The tree is fixed (quad, half-row, row, then
// rows 0+1 / 2+3 and the halves), so the sums are deterministic; the total lands in lane
// 63 only.  Every lane of the wave must be active.
namespace dpp {
constexpr int QP_XOR1 = 0xB1;          // quad_perm [1, 0, 3, 2]
constexpr int QP_XOR2 = 0x4E;          // quad_perm [2, 3, 0, 1]
constexpr int ROW_MIRROR = 0x140;      // lane i <- 15 - i within a row of 16
constexpr int ROW_HALF_MIRROR = 0x141; // lane i <- 7 - i within a half-row of 8
constexpr int ROW_BCAST15 = 0x142;     // lane 15 of each row -> the next row (row_mask selects)
constexpr int ROW_BCAST31 = 0x143;     // lane 31 -> rows 2 and 3 (row_mask selects)
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ double mov_d(double old, double x) {
    const long long ux = __double_as_longlong(x), uo = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)uo, (int)ux, CTRL, ROWM, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uo >> 32), (int)(ux >> 32), CTRL, ROWM, 0xf,
                                               false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ long long mov_ll(long long old, long long x) {
    const int lo = __builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWM, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(old >> 32), (int)(x >> 32), CTRL, ROWM, 0xf,
                                               false);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
}  // namespace dpp

// inclusive wave scans (every lane; fixed association: Hillis-Steele inside each row of
// 16 lanes by row_shr, then rows 0->1, 2->3 by row_bcast15 and rows 0-1 -> 2, 3 by
// row_bcast31), and the exclusive form by wave_shr:1 (lane 0 gets 0)
namespace dpp {
constexpr int ROW_SHR1 = 0x111, ROW_SHR2 = 0x112, ROW_SHR4 = 0x114, ROW_SHR8 = 0x118;
constexpr int WAVE_SHR1 = 0x138;
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ double movz_d(double x) {  // out-of-range source: 0
    const long long ux = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)ux, CTRL, ROWM, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(ux >> 32), CTRL, ROWM, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ long long movz_ll(long long x) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWM, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, ROWM, 0xf, true);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
}  // namespace dpp

__device__ __forceinline__ double wave_incl_scan_d(double x) {
    x = x + dpp::movz_d<dpp::ROW_SHR1>(x);
    x = x + dpp::movz_d<dpp::ROW_SHR2>(x);
    x = x + dpp::movz_d<dpp::ROW_SHR4>(x);
    x = x + dpp::movz_d<dpp::ROW_SHR8>(x);
    x = x + dpp::mov_d<dpp::ROW_BCAST15, 0xA>(0.0, x);
    x = x + dpp::mov_d<dpp::ROW_BCAST31, 0xC>(0.0, x);
    return x;
}
__device__ __forceinline__ long long wave_incl_scan_ll(long long x) {
    x += dpp::movz_ll<dpp::ROW_SHR1>(x);
    x += dpp::movz_ll<dpp::ROW_SHR2>(x);
    x += dpp::movz_ll<dpp::ROW_SHR4>(x);
    x += dpp::movz_ll<dpp::ROW_SHR8>(x);
    x += dpp::mov_ll<dpp::ROW_BCAST15, 0xA>(0, x);
    x += dpp::mov_ll<dpp::ROW_BCAST31, 0xC>(0, x);
    return x;
}
// the value of the lane below (lane 0: 0)
__device__ __forceinline__ double wave_shr1_d(double x) { return dpp::movz_d<dpp::WAVE_SHR1>(x); }
__device__ __forceinline__ long long wave_shr1_ll(long long x) { return dpp::movz_ll<dpp::WAVE_SHR1>(x); }

// wave sum, valid in lane 63
__device__ __forceinline__ double wave_sum63(double x) {
    x = x + dpp::mov_d<dpp::QP_XOR1>(0.0, x);
    x = x + dpp::mov_d<dpp::QP_XOR2>(0.0, x);
    x = x + dpp::mov_d<dpp::ROW_HALF_MIRROR>(0.0, x);
    x = x + dpp::mov_d<dpp::ROW_MIRROR>(0.0, x);
    x = x + dpp::mov_d<dpp::ROW_BCAST15, 0xA>(0.0, x);
    x = x + dpp::mov_d<dpp::ROW_BCAST31, 0xC>(0.0, x);
    return x;
}

// wave sum of integers, valid in lane 63
__device__ __forceinline__ unsigned long long wave_sum63_u64(unsigned long long x) {
    x += (unsigned long long)dpp::mov_ll<dpp::QP_XOR1>(0, (long long)x);
    x += (unsigned long long)dpp::mov_ll<dpp::QP_XOR2>(0, (long long)x);
    x += (unsigned long long)dpp::mov_ll<dpp::ROW_HALF_MIRROR>(0, (long long)x);
    x += (unsigned long long)dpp::mov_ll<dpp::ROW_MIRROR>(0, (long long)x);
    x += (unsigned long long)dpp::mov_ll<dpp::ROW_BCAST15, 0xA>(0, (long long)x);
    x += (unsigned long long)dpp::mov_ll<dpp::ROW_BCAST31, 0xC>(0, (long long)x);
    return x;
}

// lane 63's value in every lane (a scalar read, no LDS)
__device__ __forceinline__ double bcast63(double x) {
    const long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)u, 63);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), 63);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ unsigned long long bcast63_u64(unsigned long long x) {
    const int lo = __builtin_amdgcn_readlane((int)x, 63);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), 63);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// wave min / max, valid in lane 63
__device__ __forceinline__ double wave_min63(double x) {
    x = fmin(x, dpp::mov_d<dpp::QP_XOR1>(INFINITY, x));
    x = fmin(x, dpp::mov_d<dpp::QP_XOR2>(INFINITY, x));
    x = fmin(x, dpp::mov_d<dpp::ROW_HALF_MIRROR>(INFINITY, x));
    x = fmin(x, dpp::mov_d<dpp::ROW_MIRROR>(INFINITY, x));
    x = fmin(x, dpp::mov_d<dpp::ROW_BCAST15, 0xA>(INFINITY, x));
    x = fmin(x, dpp::mov_d<dpp::ROW_BCAST31, 0xC>(INFINITY, x));
    return x;
}
__device__ __forceinline__ double wave_max63(double x) {
    x = fmax(x, dpp::mov_d<dpp::QP_XOR1>(-INFINITY, x));
    x = fmax(x, dpp::mov_d<dpp::QP_XOR2>(-INFINITY, x));
    x = fmax(x, dpp::mov_d<dpp::ROW_HALF_MIRROR>(-INFINITY, x));
    x = fmax(x, dpp::mov_d<dpp::ROW_MIRROR>(-INFINITY, x));
    x = fmax(x, dpp::mov_d<dpp::ROW_BCAST15, 0xA>(-INFINITY, x));
    x = fmax(x, dpp::mov_d<dpp::ROW_BCAST31, 0xC>(-INFINITY, x));
    return x;
}

// wave-wide max of two u64 (all 64 lanes must be active)
// (DPP steps, like wave_sum63 below; a step's unwritten lanes read 0, neutral for max)
// -- the result is valid in lane 63 only
template <int CTRL, int ROWM>
__device__ __forceinline__ void range_step(unsigned long long &a, unsigned long long &b) {
    const int alo = __builtin_amdgcn_update_dpp(0, (int)a, CTRL, ROWM, 0xf, false);
    const int ahi = __builtin_amdgcn_update_dpp(0, (int)(a >> 32), CTRL, ROWM, 0xf, false);
    const int blo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWM, 0xf, false);
    const int bhi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWM, 0xf, false);
    const unsigned long long xa = ((unsigned long long)(unsigned)ahi << 32) | (unsigned)alo;
    const unsigned long long xb = ((unsigned long long)(unsigned)bhi << 32) | (unsigned)blo;
    a = xa > a ? xa : a;
    b = xb > b ? xb : b;
}
__device__ __forceinline__ void wave_range_reduce(unsigned long long &a, unsigned long long &b) {
    range_step<0xB1, 0xf>(a, b);   // quad_perm [1, 0, 3, 2]
    range_step<0x4E, 0xf>(a, b);   // quad_perm [2, 3, 0, 1]
    range_step<0x141, 0xf>(a, b);  // row_half_mirror
    range_step<0x140, 0xf>(a, b);  // row_mirror
    range_step<0x142, 0xA>(a, b);  // row_bcast15 -> rows 1, 3
    range_step<0x143, 0xC>(a, b);  // row_bcast31 -> rows 2, 3
}

// Key range of a sort input, produced without atomics: every producing workgroup stores
// its {max(~key), max(key)} to range[2 + 2 b .. 3 + 2 b] (plain stores, one lane), then
// one small reduction kernel writes range[0..1].  range_words(n) u64 words hold the parts
// of any producer that runs at most one workgroup per 256 keys.
inline int64_t range_words(int64_t n) { return 2 + 2 * ((n + 255) / 256 + 1); }

// block-wide {max(~key), max(key)} -> range[2 + 2 blockIdx.x ..] (all threads, 256/block)
__device__ __forceinline__ void block_range_store(unsigned long long *range, bool valid,
                                                  unsigned long long kmin_c,
                                                  unsigned long long kmax) {
    __shared__ unsigned long long s_ra[4], s_rb[4];
    unsigned long long a = valid ? kmin_c : 0ULL, b = valid ? kmax : 0ULL;
    wave_range_reduce(a, b);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 63) {
        s_ra[wave] = a;
        s_rb[wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = s_ra[0];
        b = s_rb[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            a = s_ra[w] > a ? s_ra[w] : a;
            b = s_rb[w] > b ? s_rb[w] : b;
        }
        range[2 + 2 * (int64_t)blockIdx.x] = a;
        range[3 + 2 * (int64_t)blockIdx.x] = b;
    }
}

// XCD-aware block order: the hardware deals workgroups round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, Workgroup dispatch), so block b runs on XCD b % 8.  Returning
// the logical block (b % 8) * q + min(b % 8, r) + b / 8 (q, r = nb / 8, nb % 8) hands each
// XCD one contiguous eighth of the work -- with a spatial work order, one compact region
// of the layer per XCD-private L2 -- and is a bijection on [0, nb).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t x = b & 7, q = nb >> 3, r = nb & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// squared distance in md dims in the reference's order, no contraction (cKDTree-identical
// bits): ((0 + dx*dx) + dy*dy) + dz*dz
template <int MD>
__device__ __forceinline__ double sq_dist(double qx, double qy, double qz, double px, double py,
                                          double pz) {
    double dx = qx - px;
    double dy = qy - py;
    double s = dx * dx;  // == 0 + dx*dx exactly
    s = s + dy * dy;
    if (MD == 3) {
        double dz = qz - pz;
        s = s + dz * dz;
    }
    return s;
}

struct alignas(32) TPt {
    double x, y, z;
    long long idx;
};

// Everything an NN kernel needs to search the static CHM grid.
// grid kernels address the cell-sorted stems (32 B each) through a buffer descriptor
constexpr int64_t kMaxGridStems = (int64_t)0x7fffffff / 32;

struct GridView {
    const TPt *pts;
    const int32_t *cell_start;  // ncells + 1
    double x0, y0, h, inv_h;
    double margin;              // conservative slack for the ring lower bound (m)
    int gx, gy;
    int64_t m;                  // stems (pts entries); m * 32 < 2^31 (buffer descriptor)
};

// The certified-reuse bound G per query (k_grid_nn.hip cert_try): fp32, rounded toward
// -inf, so the stored value stays a lower bound (4 B read + 4 B written per certified
// query instead of 8 + 8; C3 it/s unchanged against fp64 within noise, all -m gpu green).
typedef float gap_t;

// The window selection's cross-workgroup words (k_select.hip SelWS's window part: coarse
// buckets, accumulators, append counters) come in copies, one per XCD (blockIdx % 8):
// memory-side atomics on one word serialise (~88 per us), and 977 NN workgroups on 256
// words took ~11 us
#ifndef FICP_WIN_COPIES
#define FICP_WIN_COPIES 8
#endif
constexpr int kWinCopies = FICP_WIN_COPIES;
struct IterState;

// Per-launch NN arguments.
struct NNArgs {
    double *sx;                 // source x (updated in place when T != nullptr)
    double *sy;
    const double *sz;
    int64_t n;
    const double *T;            // pending 3x3 transform to apply before the query, or null
    const int *skip;            // device flag: kernel is a no-op when *skip != 0 (nullable)
    int32_t *idx;               // out
    double *dist;               // out (nullable)
    double *r;                  // out: d^2 (nullable)
    unsigned long long *key;    // out: order-preserving bits of dist (nullable)
    uint32_t *val;              // out: identity payload for the sort (nullable)
    double *cx;                 // out: XY of the matched stem (nullable)
    double *cy;
    const double *tx;           // original-order CHM layer (brute path gathers cx, cy)
    const double *ty;
    unsigned long long *range;  // out: key range parts (range_words(n) words; nullable)
    const int32_t *prev_bp;     // grid kernels: grid slot matched by this query in the previous
                                // call (warm start; nullable, entries < 0 ignored)
    int32_t *out_bp;            // grid kernels: out: grid slot matched (nullable; may alias)
    double *dz2;                // grid kernels: out: dz^2 of the match (nullable; md 3)
    gap_t *gap;                 // grid kernels: in/out: certified-reuse bound (nullable;
                                // needs cx, cy, dz2, out_bp; k_grid_nn.hip nn_query_cert)
    int cert_block;             // grid kernels, with gap and warm_c: > 0 packs each workgroup's
                                // uncertified queries onto its first lanes, up to this many
                                // lanes per query (1, 4 or 8) when they are few
    int multi;                  // grid kernel, certified calls: QPT queries per thread
                                // (k_nn_grid_q; the run loop's later calls)
    int warm_c;                 // grid kernels: start from the previous match held in
                                // (cx, cy, dz2): its d^2 to the moved query, no record reload
    const int *apply_flag;      // T is applied only while *apply_flag != 0 (nullable: always)
    const int *reuse;           // grid kernel: a no-op while *reuse != 0 -- the source has not
                                // moved since the previous call, whose outputs stand (nullable)
    // grid kernels, run loop: a launch that finds *skip set (the loop ended before it: the
    // launch queued behind the last selection) writes the caller-order XY instead,
    // fin_x[fin_orig[p]] = sx[p] (k_scatter_xy's work, no launch or host round trip of its own)
    const uint32_t *fin_orig;
    double *fin_x, *fin_y;
    // grid kernels with gap: the cold call stores no G and the first warm call loads none
    // (every G would be 0: that call scans every query with its cover anyway), 4 B per
    // query less written and read.  Set on both calls or on neither.
    int gap_cold;
};

// k_scatter_xy's work for rows [p0, p0 + cnt) of the work order
__device__ __forceinline__ void fin_scatter(const NNArgs &a, int64_t p0, int cnt) {
    for (int q = threadIdx.x; q < cnt; q += blockDim.x) {
        const int64_t p = p0 + q;
        if (p < a.n) {
            const uint32_t i = a.fin_orig[p];
            a.fin_x[i] = a.sx[p];
            a.fin_y[i] = a.sy[p];
        }
    }
}

// Device-resident state of one ICP stage (written by kernels, read back per iteration).
enum PlotPhase { PH_HEAD = 0, PH_LOOP = 1, PH_DONE = 2 };

struct alignas(16) IterState {
    double T[9];           // last fit
    double pad0;
    double frac;           // last fraction
    double frmsd;          // FRMSD at k
    long long k;           // selected k
    long long n_src;       // N
    double csx, csy, ctx, cty;  // centroids of the last fit (relative to the pivot)
    double H[4];
    // ---- device-resident ICP loop (k_loop_update: ficp.py:122-154 on the device)
    double Ttot[9];        // composite transform of the run
    double cur;            // current FRMSD (ficp.py:129, 144)
    double lam_cur;        // lambda of the stage in progress (read by the fraction kernels)
    double frmsd_last[2];  // last FRMSD of stages 1 and 2
    long long k_last;      // k of the last fraction call
    int phase;             // PlotPhase: HEAD (stage start), LOOP, DONE
    int stage, it;         // stage in progress, loop bodies completed in it
    int n_nn, n_fit;       // NN/fraction calls and fits so far
    int iters[2];          // loop bodies of stages 1 and 2
    int done;              // 1 once the run is over: NN, sort and scan are no-ops
    int no_fit;            // 1 unless a loop body is due: the fit is a no-op
    int apply;             // the NN call applies T (a fit ran in this iteration)
    int nn_reuse;          // a later stage's head: the source has not moved since the last NN
                           // call, whose outputs stand (ficp.py:151-153: _iterate() queries
                           // the same source again); the NN kernel is a no-op
    // selection threshold of the last fraction call (k_select.hip): the k-th pair of the
    // stable (key, orig) order; the fit selects {i : (key_i, orig_i) <= (tkey, torig)}
    unsigned long long tkey;
    long long torig;
    // |tkey - previous tkey| when both came from loop-body calls of one stage (else 0):
    // sizes the next call's fine bucket window (k_select.hip make_bmap)
    unsigned long long tmove;
    int n_reuse;           // NN calls answered by nn_reuse (ficp_stats::n_nn_reused)
    int win_fail;          // the window path (k_sel_win) could not decide this call: it set
                           // nn_reuse so the queued NN launch is a no-op, and the full
                           // selection of the same call (k_sel_final) clears both
    int wfloor;            // log2 of the window path's smallest half-width (keys): adapted
                           // by each window call to keep its window at ~48-384 rows (0:
                           // not yet, win_start_log)
    int pad3;
};

// The loop's done flag in pinned host memory (fused selection): bit 0 = the run is over;
// bit 1 = the next call may take the window path (win_ok below); kFlagRetry (alone) = the
// window path could not decide this call, the host enqueues the full selection for it.
constexpr int kFlagDone = 1, kFlagWinNext = 2, kFlagRetry = 4;
// window half-width 2^lh keys around the previous threshold key, lh = max(40, bits(tmove)
// + 2) <= 43 (k_select.hip k_sel_win)
// lh = max(wfloor, bits(tmove) + 1): at least twice the last move (C3's moves shrink
// ~3-10x per call); wfloor starts at 2^40 (C3 stage 1: ~40-160 rows) and follows the
// window's row count (stage 2's density put ~1,000 rows into 2^40)
// The floor starts at 2^(60 - bits(N)) keys (C3, 1M rows: 2^40; a 10k-row plot of C4 has
// 100x fewer rows per key: 2^46) and may grow 4 doublings above that (win_hmax_log).
// wfloor == 0: not adapted yet (the start).
constexpr int kWinHMinLog = 36, kWinHStartLog = 40;
__host__ __device__ __forceinline__ int win_start_log(long long n) {
    const int b = n > 0 ? 64 - __builtin_clzll((unsigned long long)n) : 0;
    const int v = 60 - b;
    return v < kWinHMinLog ? kWinHMinLog : (v > 48 ? 48 : v);
}
#ifndef FICP_WIN_HMAX_EXTRA
#define FICP_WIN_HMAX_EXTRA 4  // doublings of the window above its start (tools/build_variant.sh A/B)
#endif
__host__ __device__ __forceinline__ int win_hmax_log(long long n) {
    return win_start_log(n) + FICP_WIN_HMAX_EXTRA;
}
__host__ __device__ __forceinline__ int win_floor(int wfloor, long long n) {
    return wfloor > 0 ? wfloor : win_start_log(n);
}
// (tmove 0, no move known: the first loop body of a later stage, 2x the floor; C3's 73-row
// move there is ~2^39.6 keys)
__host__ __device__ __forceinline__ int win_lh(unsigned long long tmove, int wfloor) {
    if (!tmove) return wfloor + 1;
    const int b = 64 - __builtin_clzll(tmove);
    return b + 1 > wfloor ? b + 1 : wfloor;
}
// the next fraction call may take the window path: a loop body follows a loop body of the
// same stage (tkey and tmove from loop-body calls), or it is the first body of a later
// stage, whose head ran on the previous stage's converged source (C3: 73 rows moved there,
// inside 2x the floor; stage 1's first body moved 4,228 rows), the threshold moved less
// than 2^(win_hmax_log - 1) keys, p = 2 lambda + 1 >= 1 (the bounds' quasi-concavity)
__device__ __forceinline__ bool win_first_body(int it, int stage, unsigned long long tmove) {
    return it == 0 && stage >= 1 && tmove == 0;
}
__device__ __forceinline__ bool win_ok(const IterState &s) {
    return s.phase == PH_LOOP && !s.done && (s.it >= 1 || win_first_body(s.it, s.stage, s.tmove)) &&
           s.k > 0 &&
           win_lh(s.tmove, win_floor(s.wfloor, s.n_src)) <= win_hmax_log(s.n_src) &&
           2.0 * s.lam_cur + 1.0 >= 1.0;
}

// FRMSD(k) = (1 / (k/N)**lambda) * sqrt(S_k / k), in the reference's operation order
// (ficp.py:59-60, 81)
__device__ __forceinline__ double frmsd_of(long long k, long long N, double S, double lam) {
    const double frac = (double)k / (double)N;
    return (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
}

// one selected pair's contribution to the 8 fit sums (k_fit_sums' operations and order)
__device__ __forceinline__ void fit_add(double (&c)[8], double xs, double ys, double xt,
                                        double yt, double px, double py) {
    const double dxs = xs - px, dys = ys - py;
    const double dxt = xt - px, dyt = yt - py;
    c[0] = c[0] + dxs;
    c[1] = c[1] + dys;
    c[2] = c[2] + dxt;
    c[3] = c[3] + dyt;
    c[4] = c[4] + dxs * dxt;
    c[5] = c[5] + dxs * dyt;
    c[6] = c[6] + dys * dxt;
    c[7] = c[7] + dys * dyt;
}

// inputs of the fit fused into the selection (k_select.hip): the rows' positions and
// correspondences in work order, the pivot, and allow_reflection
struct FitSrc {
    const double *sx, *sy, *cx, *cy;
    double px, py;
    int on, allow_refl;
};

// The rigid fit from the 8 sums of the pivot-shifted pairs (s' = s - pivot, t' = t -
// pivot) over the k selected rows: sum s'x, s'y, t'x, t'y, s'x t'x, s'x t'y, s'y t'x,
// s'y t'y.  Closed-form 2-D Kabsch (ficp.py:89-110); writes T, the
// centroids and H into *st.
// the closed-form solve alone: T (row-major 3x3) from the 8 sums, centroids and H out
__device__ inline void fit_solve_T(const double c[8], double k, double px, double py,
                                   int allow_refl, double *T, double *cent4 = nullptr,
                                   double *H4 = nullptr);
__device__ inline void fit_solve(const double c[8], double k, double px, double py,
                                 int allow_refl, IterState *st) {
    fit_solve_T(c, k, px, py, allow_refl, st->T, &st->csx, st->H);
}
__device__ inline void fit_solve_T(const double c[8], double k, double px, double py,
                                   int allow_refl, double *T, double *cent4, double *H4) {
    // centroids of the pivot-shifted pairs, then H = sum s't'^T - k cs' ct'^T
    const double csx = c[0] / k, csy = c[1] / k, ctx = c[2] / k, cty = c[3] / k;
    double H[4];
    H[0] = c[4] - c[0] * ctx;
    H[1] = c[5] - c[0] * cty;
    H[2] = c[6] - c[1] * ctx;
    H[3] = c[7] - c[1] * cty;
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
    const double wsx = csx + px, wsy = csy + py;
    const double wtx = ctx + px, wty = cty + py;
    T[0] = R00;
    T[1] = R01;
    T[2] = wtx - (wsx * R00 + wsy * R01);
    T[3] = R10;
    T[4] = R11;
    T[5] = wty - (wsx * R10 + wsy * R11);
    T[6] = 0.0;
    T[7] = 0.0;
    T[8] = 1.0;
    if (cent4) {  // IterState: csx, csy, ctx, cty are consecutive
        cent4[0] = csx;
        cent4[1] = csy;
        cent4[2] = ctx;
        cent4[3] = cty;
    }
    if (H4)
        for (int e = 0; e < 4; ++e) H4[e] = H[e];
}

// Loop parameters and optional trace buffers of the device-resident loop.
struct LoopCtl {
    const double *lams;    // [nstages] on the device (read only past the first kLamIn)
    double lam_in[4];      // the first kLamIn lambdas, carried in the kernel arguments
    int nstages;
    int max_iter;
    double threshold;
    int max_trace;         // capacity of the trace buffers (NN calls), 0 = no trace
    int max_trace_idx;     // calls whose NN index is traced (<= max_trace; its buffer is n per call)
    int no_reuse_count;    // the NN step of this loop never honours nn_reuse (dist target mode):
                           // n_reuse stays 0
    int pad;
    long long *tk;         // [max_trace] k per call
    double *tf;            // [max_trace] FRMSD per call
    double *tl;            // [max_trace] lambda per call
    double *tT;            // [max_trace * 9] fits in order
};

constexpr int kLamIn = 4;
__host__ __device__ __forceinline__ double lam_of(const LoopCtl &c, int i) {
    return i < kLamIn ? c.lam_in[i] : c.lams[i];
}

// ---------------------------------------------- device-resident loop (k_loop.hip)
__device__ __forceinline__ void loop_set_flags(IterState &s) {
    s.done = s.phase == PH_DONE;
    s.no_fit = s.phase != PH_LOOP;
    s.apply = s.phase == PH_LOOP;
    s.nn_reuse = s.phase == PH_HEAD && s.n_nn > 0;
}

__device__ __forceinline__ void loop_end_stage(IterState &s, const LoopCtl &c) {
    // (constant indices: a caller's register copy of the state stays in registers)
    if (s.stage == 0) s.iters[0] = s.it;
    else if (s.stage == 1) s.iters[1] = s.it;
    s.stage += 1;
    s.it = 0;
    if (s.stage < c.nstages) {  // ficp.py:152-153: next lambda, next _iterate
        s.phase = PH_HEAD;
        s.lam_cur = lam_of(c, s.stage);
    } else {
        s.phase = PH_DONE;
    }
}

// one k_loop_update step on the state (thread 0 of one workgroup): the decisions of
// _iterate/run after an NN call + fraction (ficp.py:122-154)
__device__ __forceinline__ void loop_step(IterState *st, const LoopCtl &c) {
    IterState &s = *st;
    if (s.done) return;
    if (!c.no_reuse_count) s.n_reuse += s.nn_reuse;
    const int call = s.n_nn++;
    s.k_last = s.k;
    if (call < c.max_trace) {
        if (c.tk) c.tk[call] = s.k;
        if (c.tf) c.tf[call] = s.frmsd;
        if (c.tl) c.tl[call] = s.lam_cur;
    }
    if (s.phase == PH_HEAD) {  // ficp.py:123-129
        if (s.k == 0) {
            loop_end_stage(s, c);  // ficp.py:125-126: nothing selected, the stage returns
        } else {
            s.cur = s.frmsd;
            if (s.stage == 0) s.frmsd_last[0] = s.cur;
            else if (s.stage == 1) s.frmsd_last[1] = s.cur;
            s.phase = PH_LOOP;
            s.it = 0;
            if (c.max_iter <= 0) loop_end_stage(s, c);
        }
    } else {  // a loop body ran: fit -> apply -> NN -> fraction (ficp.py:132-140)
        if (s.n_fit < c.max_trace && c.tT)
            for (int e = 0; e < 9; ++e) c.tT[9 * s.n_fit + e] = s.T[e];
        s.n_fit += 1;
        double R[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                R[3 * i + j] = s.T[3 * i] * s.Ttot[j] + s.T[3 * i + 1] * s.Ttot[3 + j] +
                               s.T[3 * i + 2] * s.Ttot[6 + j];
        for (int e = 0; e < 9; ++e) s.Ttot[e] = R[e];
        const double nw = s.frmsd;
        if (s.stage == 0) s.frmsd_last[0] = nw;
        else if (s.stage == 1) s.frmsd_last[1] = nw;
        if (s.cur - nw <= c.threshold) {  // ficp.py:142 (the transform is already applied)
            loop_end_stage(s, c);
        } else {
            s.cur = nw;
            s.it += 1;
            if (s.it >= c.max_iter) loop_end_stage(s, c);
        }
    }
    loop_set_flags(s);
}

// ------------------------------------------- one small plot in one workgroup (k_small.hip)
// The Join button's size (app.py:630-661: 5-44 trees vs ~260 CHM stems): the whole run()
// in one launch, the CHM layer in LDS, one tree per thread.
constexpr int kSmallMaxN = 1024;            // trees (one per thread)
constexpr int kSmallMaxM = 4096;            // CHM stems staged in LDS (96 KB at md 3)
constexpr int64_t kSmallMaxPairs = 1 << 18; // brute-force pairs per NN call (~10 us in one CU)
struct SmallArgs {
    const double *rows;         // trees as the caller's (n x ld) rows on the device (nullable:
    int64_t ld;                 //   then the SoA columns below are read)
    double *sx, *sy;            // trees (caller order), SoA; moved in place (nullable with rows)
    const double *sz;
    int n;
    const double *tx, *ty, *tz; // CHM layer (original order)
    int m;
    int allow_refl;
    IterState *st;              // out: the final loop state (stats, T_total), device
    int32_t *tidx;              // out (nullable): NN index per call [max_trace][n]
    // pinned host report (nullable): the final XY interleaved, the state, the device clock
    // at start and end, then *host_flag = 1 (system scope) -- no copy or report launch
    double *host_xy;
    IterState *host_st;
    unsigned long long *host_t; // [2]
    int *host_flag;
};
bool small_run_fits(int64_t n, int64_t m);
hipError_t launch_small_run(const SmallArgs &a, int md, const LoopCtl &lc, hipStream_t s);

// ----------------------------------------------------------------- launchers
// device -> coherent pinned host copies + a completion flag the host polls (k_loop.hip)
struct ReportSeg {
    const void *src;  // device, 4-B aligned
    void *dst;        // coherent pinned host memory
    int words;        // 32-bit words (0: unused)
};
hipError_t launch_report(const ReportSeg &a, const ReportSeg &b, const ReportSeg &c, int *flag,
                         unsigned long long *t_end, hipStream_t s);
// zero the sort timeout flag and stamp the device clock (100 MHz) into *t0 (host); with lc,
// also initialise the loop state *st (the work of launch_loop_init, one launch less)
hipError_t launch_run_start(uint32_t *tflag, unsigned long long *t0, hipStream_t s,
                            unsigned *selerr = nullptr, IterState *st = nullptr,
                            const LoopCtl *lc = nullptr);

// grid build (k_grid_nn.hip)
// bbox of (x, y) -> out4 {xmin, xmax, ymin, ymax}; with ox, also copies x, y (z) there
hipError_t launch_minmax2(const double *x, const double *y, int64_t m, double *partials,
                          double *out4, hipStream_t s, const double *z = nullptr,
                          double *ox = nullptr, double *oy = nullptr, double *oz = nullptr);
hipError_t launch_grid_count(const double *x, const double *y, int64_t m, double x0, double y0,
                             double inv_h, int gx, int gy, int32_t *cell_of, int32_t *counts,
                             hipStream_t s);
hipError_t launch_grid_scatter(const double *x, const double *y, const double *z, int64_t m,
                               const int32_t *cell_of, const int32_t *cell_start,
                               int32_t *fill, TPt *pts, hipStream_t s);
hipError_t launch_grid_sort_cells(TPt *pts, const int32_t *cell_start, int64_t ncells,
                                  hipStream_t s);
// The NN launchers finish with launch_range_reduce when a.range is set, unless
// reduce_range is false (then the caller launches it, over nn_range_parts workgroups).
// ev_start/ev_stop (nullable): events carried by the NN dispatch itself (kernel timing)
hipError_t launch_nn_grid(const NNArgs &a, const GridView &g, int md, hipStream_t s,
                          bool reduce_range = true, hipEvent_t ev_start = nullptr,
                          hipEvent_t ev_stop = nullptr);
int64_t nn_range_parts(int64_t n, int64_t m, bool grid);
// first NN call index of a run that takes k_nn_grid_q (k_grid_nn.hip FICP_NN_QPT_FROM)
int nn_qpt_from();
int64_t brute_chunk_count(int64_t n, int64_t m);  // target chunks of the brute kernel
hipError_t launch_nn_brute(const NNArgs &a, const double *tx, const double *ty,
                           const double *tz, int64_t m, int md, double *part_d2,
                           int32_t *part_idx, hipStream_t s, bool reduce_range = true);
hipError_t launch_deinterleave(const double *rows, int64_t n, int64_t ld, int ncols,
                               double *c0, double *c1, double *c2, hipStream_t s);
hipError_t launch_put_xy_rows(const double *x, const double *y, int64_t n, int64_t ld, double *rows,
                              hipStream_t s);
hipError_t launch_interleave_xy(const double *x, const double *y, int64_t n, double *out_xy,
                                hipStream_t s);
// n16 16-B words from src to dst (device buffers, 16-B aligned, not overlapping)
hipError_t launch_copy16(const void *src, void *dst, int64_t n16, hipStream_t s);
// Two-level bucket sort of points by a grid key (k_bsort.hip).  mode 0: key = cell id
// cy * gx + cx (grid layout: TPt records + cell_start); mode 1: 8x8-supertile order
// (work order: SoA coordinates + caller index).  Order: (key, point index).
struct PlotGrid;
struct BSortGeom {
    double x0, y0, inv_h;
    int gx, gy;
    int mode;                // 2: many plots (C4): key = cell_base + cell of the point's plot
                             // 3: many plots' trees: key = wbase + the supertile-order key of
                             //    the point in its plot's grid (the batch work order)
    const int32_t *plot;     // modes 2, 3: plot of each point
    const PlotGrid *grids;   // modes 2, 3: per-plot geometry
};
struct BSortPlan {
    int fs;         // fine bits (key & ((1 << fs) - 1))
    int nbk;        // coarse buckets (key >> fs)
    int nb1;        // slices of the count / scatter kernels
    int bcap;       // points ordered in LDS by one k_bs_bucket workgroup
    int64_t per;    // points per slice
    int64_t nkeys;
};
struct BSortOut {
    TPt *pts;             // mode 0: records in key order
    int32_t *cell_start;  // mode 0: [nkeys + 1]
    double *wx, *wy, *wz; // mode 1 (wz nullable)
    uint32_t *worig;      // mode 1
};
// one sort job of k_bsort.hip: inputs, geometry, plan, outputs and its carved scratch
struct BSJob {
    const double *x, *y, *z;
    int64_t n;
    BSortGeom g;
    BSortPlan p;
    BSortOut o;
    uint32_t *counts, *totals, *base;
    TPt *rec;
    uint64_t *gcomp;
    uint32_t *gpos;
};
struct BSPair {
    BSJob a, b;
    int split[4];  // workgroups of job a in each of the four kernels
};
BSortPlan bsort_plan(int64_t n, int64_t nkeys);
bool bsort_supported(int64_t n, int64_t nkeys);
int64_t bsort_tmp_bytes(int64_t n, int64_t nkeys);
BSJob bsort_job(const double *x, const double *y, const double *z, int64_t n, const BSortGeom &g,
                int64_t nkeys, const BSortOut &o, void *tmp);
// two jobs in the same four launches (b.n == 0: job a alone); both must be supported
hipError_t launch_bsort2(const BSJob &a, const BSJob &b, hipStream_t s);
hipError_t launch_bsort(const double *x, const double *y, const double *z, int64_t n,
                        const BSortGeom &g, int64_t nkeys, const BSortOut &o, void *tmp,
                        hipStream_t s);
// spatial work order of a source layer: key64 = (8x8-supertile cell order << 32) | i
hipError_t launch_src_cellkey(const double *sx, const double *sy, int64_t n, const GridView &g,
                              unsigned long long *key, hipStream_t s);
// w*[p] = s*[perm[p]], worig[p] = perm[p]
hipError_t launch_gather_work(const uint32_t *perm, const double *sx, const double *sy,
                              const double *sz, int64_t n, double *wx, double *wy, double *wz,
                              uint32_t *worig, hipStream_t s);
// s*[worig[p]] = w*[p]
hipError_t launch_scatter_xy(const uint32_t *worig, const double *wx, const double *wy, int64_t n,
                             double *sx, double *sy, hipStream_t s);
hipError_t launch_scatter_i32(const uint32_t *worig, const int32_t *w, int64_t n, int32_t *out,
                              hipStream_t s);

// scans / sort (k_sort.hip)
// Exclusive scan of n int32; out[n] = total. tmp >= scan_tmp_elems(n).  atomic_in: the
// input was accumulated with atomics and is read with atomic RMWs.
int64_t scan_tmp_elems(int64_t n);
hipError_t launch_scan_i32(const int32_t *in, int32_t *out, int64_t n, int32_t *tmp,
                           bool atomic_in, hipStream_t s);
// Memory-model rule of this library: a word that any kernel updates with
// device-scope atomics is reset with atomics (these kernels, never hipMemset or plain
// stores) and read with atomic RMWs.
hipError_t launch_atomic_zero32(uint32_t *p, int64_t n, hipStream_t s);
hipError_t launch_atomic_zero64(unsigned long long *p, int64_t n, hipStream_t s);
// Stable argsort: order[j] = position (0..n-1) of the j-th smallest (key64, orig) pair
// (orig == null: orig = position).  range[0..1] = {max(~key), max(key)} of the keys (from
// the NN launchers or launch_key_range, see range_words).  r/rs (nullable):
// rs[j] = r[order[j]].  Scratch: sort_tmp_bytes(n).
int64_t sort_tmp_bytes(int64_t n);
// sticky flag set when a look-back wait timed out (results of that sort are invalid)
uint32_t *sort_timeout_flag(void *tmp, int64_t n);
hipError_t launch_key_range(const unsigned long long *key, int64_t n, unsigned long long *range,
                            hipStream_t s);
// range[0..1] from the nparts parts a producer stored (see block_range_store)
hipError_t launch_range_reduce(unsigned long long *range, int64_t nparts, hipStream_t s);
hipError_t launch_sort(const unsigned long long *key64, const uint32_t *orig, int64_t n,
                       unsigned long long *range, uint32_t *order, const double *r, double *rs,
                       void *tmp, const int *skip, hipStream_t s);
hipError_t launch_keys_from_doubles(const double *d, int64_t n, unsigned long long *key,
                                    uint32_t *val, hipStream_t s);

// FRMSD-optimal fraction by bucketed selection (k_select.hip): st->k, frac, frmsd and the
// threshold pair (tkey, torig) of the k-th (key, orig) entry, without sorting every row.
// Requires n == N (the run loop).  range = the NN call's key range.  orig nullable.
int64_t sel_tmp_bytes(int64_t n);
hipError_t launch_select_init(void *tmp, int64_t n, hipStream_t s);
// out3 (device): {sticky error bits, refinement levels run, radix fallbacks}
// range_parts > 0: range holds the producer's unreduced parts (block_range_store); the
// histogram kernel reduces them (no launch_range_reduce needed) and stores range[0..1].
// loop (nullable): the last kernel also runs the k_loop_update step; host_flag (nullable,
// coherent pinned host memory): receives st->done after that step.
hipError_t launch_select(const unsigned long long *key, const uint32_t *orig, const double *r,
                         int64_t n, double lam, const double *lam_dev, unsigned long long *range,
                         int64_t range_parts, void *tmp, IterState *st, const int *skip,
                         const LoopCtl *loop, int *host_flag, hipStream_t s,
                         const FitSrc *fit = nullptr, int fault = 0);
// the selection's sticky error word inside its workspace (k_run_start resets it per run),
// followed by its statistics words levels and radix (the report reads all three)
unsigned *sel_err_word(void *tmp, int64_t n);
// the window path (k_select.hip k_sel_win): one launch for a later loop-body call of a
// stage (the host takes it when the previous call's flag had kFlagWinNext); on success the
// same outputs as launch_select with loop and fit, on failure kFlagRetry (state unchanged
// but win_fail / nn_reuse)
hipError_t launch_select_win(const double *r, const uint32_t *orig, int64_t n,
                             const unsigned long long *range, int64_t range_parts, void *tmp,
                             IterState *st, const LoopCtl &loop, int *host_flag, hipStream_t s,
                             const FitSrc &fit, int fault = 0);
// whether one k_sel_win launch can decide n rows (its records hold <= W_MAXWG workgroups;
// larger layers would fail every window call and pay a retry round trip)
bool select_win_fits(int64_t n);
// test-only fault injection (ficp_set_fault): block 0 of k_sel_bounds_gather publishes a
// wrong token, so every gather block times out (ERR_SPIN)
constexpr int FICP_FAULT_SPIN = 1;
// test-only: k_sel_win reports kFlagRetry after doing its work (the fallback path)
constexpr int FICP_FAULT_WIN = 2;

// selection + fit + apply (k_select_fit.hip)
int64_t frac_tmp_bytes(int64_t n);
// r_i = sum_md (src_i - corr_i)^2 on SoA inputs
hipError_t launch_residuals(const double *sx, const double *sy, const double *sz,
                            const double *cx, const double *cy, const double *cz, int64_t n,
                            int md, double *r, hipStream_t s);
// argmin_k FRMSD(k) over r in selection order (rs) -> st->k, st->frac, st->frmsd
// partitioned target (C5): shard idx offset; merged (d2, idx) -> key, r, cx, cy, range
hipError_t launch_add_offset(int32_t *idx, int64_t n, int64_t off, hipStream_t s);
hipError_t launch_fill_inf(double *d2, int32_t *idx, int64_t n, hipStream_t s);
// remove_matches: the KNN_K best (distance, stem index) of queries [q0, n) in cdist order
// (d = sqrt(d2), then index), skipping stems with removed[idx] != 0 (nullable)
constexpr int KNN_K = 8;
hipError_t launch_knn_grid(const double *sx, const double *sy, const double *sz, int64_t q0,
                           int64_t n, const GridView &g, int md, const uint8_t *removed,
                           int32_t *out_id, double *out_d, hipStream_t s);
hipError_t launch_corr_from_merge(const double *d2, const int32_t *idx, const double *tx,
                                  const double *ty, int64_t n, unsigned long long *key, double *r,
                                  double *cx, double *cy, unsigned long long *range,
                                  hipStream_t s);
// device-resident ICP loop (k_loop.hip)
hipError_t launch_loop_init(IterState *st, const LoopCtl &c, hipStream_t s);
hipError_t launch_loop_update(IterState *st, const LoopCtl &c, hipStream_t s);
hipError_t launch_trace_idx(const IterState *st, const int32_t *idx, const uint32_t *worig,
                            int64_t n, int32_t *out, int max_trace, hipStream_t s);
hipError_t launch_fraction(const double *rs, int64_t n, int64_t n_src, double lambda_val,
                           const double *lam_dev,
                           void *tmp, IterState *st, const int *skip, hipStream_t s);
// Rigid fit of source (sx, sy) onto its correspondences (cx, cy).  With key != null the
// selected rows are the first st->k entries of the stable order (order, key) -- with
// order == null the threshold pair is st->(tkey, torig) from launch_select; with
// key == null every one of the n rows is used.
struct FitIn {
    const double *sx, *sy, *cx, *cy;
    const unsigned long long *key;
    const uint32_t *order;
    const uint32_t *orig;   // caller index of each position (tie order; null = identity)
    int64_t n;
    double px, py;          // pivot subtracted before summation
    const IterState *st;
};
int64_t fit_tmp_bytes(int64_t n);
// byte offset past the fit's arrival counters: free scratch for other reductions
int64_t fit_scratch_offset();
// zero the scratch's arrival counter: once per (re)allocation of the scratch
hipError_t launch_fit_init(void *tmp, hipStream_t s);
hipError_t launch_fit(const FitIn &a, int allow_reflection, void *tmp, IterState *st,
                      const int *skip, hipStream_t s);
// distributed runs (capi_dist.hip): this rank's 8 fit sums; the solve on the ranks' sums
hipError_t launch_fit_sums(const FitIn &a, void *tmp, const int *skip, double *out8,
                           hipStream_t s);
hipError_t launch_fit_solve_ranks(const double *sums, int world, double px, double py,
                                  int allow_refl, IterState *st, const int *skip, hipStream_t s);
// distributed selection (k_select.hip): local histogram -> integer totals (int64[2 * 8192]);
// from the summed totals: bounds, local candidates packed (int64[4 + 3 capd]); from the
// gathered packs: the final selection with the fused loop step
int sel_hist_words();
hipError_t launch_select_dist_hist(const unsigned long long *key, const double *r, int64_t n,
                                   int64_t n_max, const unsigned long long *range, void *tmp,
                                   int64_t n_ws, const IterState *st, const int *skip,
                                   long long *hist_out, hipStream_t s);
hipError_t launch_select_dist_gather(const unsigned long long *key, const uint32_t *orig,
                                     const double *r, int64_t n, int64_t n_total, int64_t n_max,
                                     const long long *hist, double lam, const double *lam_dev,
                                     void *tmp, int64_t n_ws, const int *skip, long long *pack,
                                     int capd, hipStream_t s);
hipError_t launch_select_dist_final(const long long *packs, int world, int capd, int64_t n_total,
                                    double lam, const double *lam_dev, void *tmp, int64_t n_ws,
                                    IterState *st, const int *skip, const LoopCtl *loop,
                                    int *host_flag, hipStream_t s);
hipError_t launch_apply_xy(double *x, double *y, int64_t n, const double *T, hipStream_t s);
// apply T while !*skip and *apply_flag (device flags of the loop state)
hipError_t launch_apply_xy_flags(double *x, double *y, int64_t n, const double *T, const int *skip,
                                 const int *apply_flag, hipStream_t s);
hipError_t launch_sum_sq_diff(const double *sx, const double *sy, const double *sz,
                              const double *cx, const double *cy, const double *cz, int64_t k,
                              int md, void *tmp, double *out, hipStream_t s);

// ------------------------------------------------------------- batch of plots (C4)
// Plot p owns source rows [so[p], so[p+1]) and CHM rows [to[p], to[p+1]) of the
// concatenated layers; every kernel below works on all plots at once.
struct PlotGrid {
    double x0, y0, h, inv_h, margin, px, py;  // grid geometry; (px, py) = fit pivot
    long long cell_base;                     // first cell of this plot in cell_start
    int gx, gy;
    int m;                                   // CHM stems of the plot (0: plot is skipped)
    int pad;
    long long wbase;                         // first work-order key of the plot's trees
                                             // (k_bsort.hip mode 3: 8x8-supertile order)
};


// Device-resident per-plot ICP state (the _iterate loop of ficp.py:122-147 per plot).
struct alignas(16) PlotState {
    double T[9];       // transform to apply before the next NN (when apply != 0)
    double Ttot[9];    // composite transform of the run
    double cur;        // current FRMSD (ficp.py:129, 144)
    double frmsd;      // FRMSD of the last fraction call
    double frac;
    long long k;       // k of the last fraction call
    int phase;         // PlotPhase
    int stage;         // 0, 1
    int it;            // loop bodies completed in this stage
    int apply;
    int n_nn, n_fit, iters0, iters1;
    unsigned long long tkey;  // selection threshold: rows with (key, row) <= (tkey, trow)
    long long trow;           // (global row index) are the k selected ones
    unsigned long long tmove; // |tkey - previous tkey| between two loop-body calls (else 0)
    int wfloor;               // the window path's smallest half-width, log2 keys (adapted)
    int pad;
};

// per-plot bbox of the CHM layer: bb[4p..4p+3] = xmin, xmax, ymin, ymax
hipError_t launch_batch_bbox(const double *tx, const double *ty, const int64_t *to, int nplots,
                             double *bb, hipStream_t s);
hipError_t launch_fill_plot_ids(const int64_t *off, int nplots, int32_t *plot_of, hipStream_t s);
hipError_t launch_batch_grid_count(const double *tx, const double *ty, int64_t m,
                                   const int32_t *tplot, const PlotGrid *grids, int32_t *cell_of,
                                   int32_t *counts, hipStream_t s);
// NN of every live plot's trees against its own CHM grid; idx = index in the concatenated
// CHM layer.  Applies states[p].T first where states[p].apply.  call: the batch iteration
// (0 = the cold call; the first warm calls scan most queries and run one query per thread)
hipError_t launch_nn_grid_batch(const NNArgs &a, const int32_t *plot_of, const PlotGrid *grids,
                                const TPt *pts, int64_t m, const int32_t *cell_start,
                                const PlotState *st, int md, hipStream_t s, int64_t call = 0);
// k_batch_init: the offsets and lambdas from coherent pinned staging (so_h, to_h, lam_h)
// into their device copies, the arrival counters zeroed, every plot's state initialised
struct BatchInitArgs {
    const int64_t *so_h, *to_h;
    const double *lam_h;
    int64_t *so, *to;
    double *lams;
    unsigned long long *arrive;
    int nplots, nstages, nl, narrive;
    PlotState *st;
};
hipError_t launch_batch_init(const BatchInitArgs &a, hipStream_t s);
// Per-plot LDS counting sort (k_batch.hip k_plot_sort): mode 0 the batch grid (TPt records
// + cell_start, as k_bsort.hip mode 2), mode 1 the batch work order (wx, wy, wz, worig, as
// mode 3), the same (key, row) order; one workgroup per plot and job (b: a second job).
struct PlotSortJob {
    const double *x, *y, *z;  // the points' columns (z nullable), plots concatenated
    const int64_t *off;       // [nplots + 1] (device)
    int mode;
    TPt *pts;
    int32_t *cell_start;
    double *wx, *wy, *wz;
    uint32_t *worig;
};
bool plot_sort_fits(int64_t max_points, int64_t max_keys);
// the work order's XY back into caller order, one workgroup per plot (plots that fit the
// plot sort): sx[worig[w]] = wx[w] within each plot's rows
hipError_t launch_plot_scatter_xy(const uint32_t *worig, const double *wx, const double *wy,
                                  const int64_t *off, int nplots, double *sx, double *sy,
                                  hipStream_t s);
hipError_t launch_plot_sort(const PlotSortJob &a, const PlotSortJob *b, const PlotGrid *grids,
                            int nplots, hipStream_t s);
// plot chunks of the batch fit (k_batch_fit) for plots of at most max_rows rows
int batch_fit_chunks(int64_t max_rows);
// part: nplots * batch_fit_chunks(max_rows) * 8 doubles; ctr: nplots arrival counters
// (atomics only: zero them once per allocation with launch_batch_fit_ctr_zero)
// key == nullptr: each row's key is derived from r (key_of_r)
hipError_t launch_batch_fit(const double *sx, const double *sy, const double *cx,
                            const double *cy, const unsigned long long *key, const double *r,
                            const int64_t *so, const PlotGrid *grids, int nplots, int64_t max_rows,
                            int allow_refl, PlotState *st, double *part, unsigned *ctr, hipStream_t s,
                            const uint32_t *worig = nullptr);
hipError_t launch_batch_fit_ctr_zero(unsigned *ctr, int n, hipStream_t s);
// Per-plot FRMSD-optimal fraction (ficp.py:73-86), one workgroup per live plot: bucket
// histogram of the plot's keys, bounds, exact sort of the candidate window only; sets
// k, frac, frmsd and the threshold pair (tkey, trow).  Scratch: 3 x n words of 8 B and
// 2 x n of 4 B (indexed by global row).  max_rows: the largest plot.
struct BatchSelScratch {
    unsigned long long *wkey, *skey;
    uint32_t *wrow, *srow;
    double *wr, *sr;
    // the caller's row of each work row (the batch work order, k_bsort.hip mode 3; nullable:
    // the rows are in caller order): the selection's tie-break at equal keys
    const uint32_t *worig;
};
// the loop step and the next body's rigid fit inside the selection (nullable: the separate
// k_batch_fit and k_batch_update launches)
struct BatchStepArgs {
    const double *sx, *sy, *cx, *cy;
    const PlotGrid *grids;
    int allow_refl, nstages, max_iter;
    double threshold;
    // non-null: the selection's workgroups count their plots' arrivals here (zero before
    // the first launch; the last one resets it) and the last stores the live count in *flag
    // (no k_batch_live launch)
    unsigned long long *arrive = nullptr;
    int *flag = nullptr;
    long long *trace = nullptr;  // per-call k trace rows of this launch's plots (nullable)
    int max_trace = 0;
    const uint32_t *worig = nullptr;  // the fit's tie-break at the threshold key (as above)
};
hipError_t launch_batch_live(int nplots, const PlotState *st, int *flag, hipStream_t s);
// key == nullptr: the keys are derived from r (key_of_r), as the NN that stored r computed them
hipError_t launch_batch_select(const unsigned long long *key, const double *r, const int64_t *so,
                               int nplots, int64_t max_rows, const double *lambdas,
                               PlotState *st, BatchSelScratch ws, hipStream_t s,
                               const BatchStepArgs *step = nullptr);
// *flag (coherent pinned host memory) <- number of plots still running
hipError_t launch_batch_update(int nplots, int nstages, double threshold, int max_iter,
                               PlotState *st, int *flag, hipStream_t s, long long *trace = nullptr,
                               int max_trace = 0);

}  // namespace ficp
