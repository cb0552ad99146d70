// k_sort.hip -- the fractional-trim residual sort (ficp.py:63,78: argsort(distances))
// and the int32 exclusive scan used by the grid build.
//
// Contract: `order` = work positions sorted by (key64, orig) lexicographically, where
// key64 is the order-preserving bit pattern of the distance and orig the caller's index
// of that position -- i.e. numpy's argsort(dist, kind="stable") in caller indices.
//
// Method, one launch per 8-bit digit, no global prefix-sum kernels:
//  0. k_os_hist: derives a 32-bit key (key64 - kmin) >> s from the key range (kmin/kmax
//     reduced from per-workgroup parts of the NN kernel or of k_key_range), scatters
//     (key32, position) into ORIG order -- so LSD stability alone orders exact ties by orig -- and builds the
//     four digit histograms at once (they do not depend on the order).
//  1-3. per 8-bit digit, reduce-then-scan: k_rs_count (per-tile digit counts),
//     k_rs_rowscan (exclusive offsets per digit over the tiles), k_os_pass (stable scatter:
//     items ranked with 64-lane ballot matching and per-wave LDS counters, digit runs
//     written coalesced from an LDS staging copy).  No communication between the
//     workgroups of a launch.  The last pass also emits r in selection order.
//  5. k_os_fixup: runs of equal key32 (distinct distances closer than 2^s ulps: rare)
//     are re-ordered by key64 with a stable insertion sort.
#include "ficp_internal.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace ficp {

namespace {

constexpr int OB = 256;              // threads per pass block (4 waves)
constexpr int OIPT = 8;              // items per thread
constexpr int OTILE = OB * OIPT;     // 2048 items per tile
constexpr int SCAN_I = 16;
constexpr int SCAN_TILE = 256 * SCAN_I;

// Derived key width and pass count: (key64 - kmin) >> s keeps the top KEY_BITS bits of
// the key range; runs of equal derived keys (distinct distances closer than 2^s ulps:
// 27 % of the elements in short runs, longest 7, at C3) are ordered by k_os_fixup.
constexpr int KEY_BITS = 24;
constexpr int NPASS = KEY_BITS / 8;

struct SortWS {
    uint32_t *kA, *kB, *vB;      // key ping-pong, val pong (ping = the caller's order)
    uint2 *pairs;                // (key, position) in orig order from k_os_hist (aliases kB, vB)
    uint32_t *hist;              // [4][256]
    uint32_t *status;            // [4][ntiles][256]
    uint32_t *tickets;           // [4] tile tickets + [1] spin-timeout flag
    uint32_t *counts;            // [256][ntiles] (reduce-then-scan mode, plain stores only)
    int ntiles;
};

// range[0..1] = {max(~key), max(key)}: written by k_range_reduce (plain stores) in an
// earlier kernel of the stream
__device__ __forceinline__ void load_range(const unsigned long long *range,
                                           unsigned long long &kmin, unsigned long long &kmax) {
    kmin = ~range[0];
    kmax = range[1];
}

__device__ __forceinline__ int key_shift(unsigned long long kmin, unsigned long long kmax) {
    const unsigned long long span = kmax > kmin ? kmax - kmin : 0ULL;
    const int bits = span ? 64 - __clzll((long long)span) : 0;
    return bits > KEY_BITS ? bits - KEY_BITS : 0;
}

template <typename T>
__device__ __forceinline__ T block_excl_scan256(T v, T *s_w /* [4] */, T &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    T pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_w[w];
    total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return pre + x - v;
}

// key range for callers without a fused producer (API paths): per-workgroup parts
__global__ __launch_bounds__(256) void k_key_range(const unsigned long long *key, int64_t n,
                                                   unsigned long long *range) {
    unsigned long long a = 0, b = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const unsigned long long k = key[i];
        a = max(a, ~k);
        b = max(b, k);
    }
    block_range_store(range, true, a, b);
}

// one workgroup: range[0..1] = max over the nparts parts (plain loads and stores)
__global__ __launch_bounds__(1024) void k_range_reduce(unsigned long long *range, int64_t nparts) {
    __shared__ unsigned long long s_a[16], s_b[16];
    unsigned long long a = 0, b = 0;
    const unsigned long long *part = range + 2;
    for (int64_t p = threadIdx.x; p < nparts; p += 1024) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(part + 2 * p);
        a = max(a, v.x);
        b = max(b, v.y);
    }
    wave_range_reduce(a, b);  // (lane 63)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 63) {
        s_a[wave] = a;
        s_b[wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = s_a[0];
        b = s_b[0];
        for (int w = 1; w < 16; ++w) {
            a = max(a, s_a[w]);
            b = max(b, s_b[w]);
        }
        range[0] = a;
        range[1] = b;
    }
}

__device__ __forceinline__ void wave_hist_add(uint32_t *h, uint32_t d, bool valid) {
    // aggregate equal digits of the wave (ballot match) -> one LDS atomic per distinct digit
    const int lane = threadIdx.x & 63;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    if (valid && __popcll(peers & ((1ULL << lane) - 1ULL)) == 0)
        atomicAdd(&h[d], (uint32_t)__popcll(peers));
}

__global__ __launch_bounds__(256) void k_os_hist(const unsigned long long *key64,
                                                 const uint32_t *orig, int64_t n,
                                                 const unsigned long long *range, SortWS ws,
                                                 int64_t status_words, const int *skip) {
    if (skip && *skip) return;
    __shared__ uint32_t s_h[NPASS][256];
    for (int e = threadIdx.x; e < NPASS * 256; e += 256) (&s_h[0][0])[e] = 0;
    // zero the look-back status words and the tickets for the passes that follow; they
    // are only ever touched by device-scope atomics (plain stores to words that other
    // kernels update atomically are not reliably ordered with those atomics)
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < status_words;
         e += (int64_t)gridDim.x * 256)
        __hip_atomic_exchange(&ws.status[e], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x < 4)  // [4] is the sticky error flag
        __hip_atomic_exchange(&ws.tickets[threadIdx.x], 0u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    __shared__ unsigned long long s_rng[2];
    if (threadIdx.x == 0) load_range(range, s_rng[0], s_rng[1]);
    __syncthreads();
    const unsigned long long kmin = s_rng[0];
    const int s = key_shift(kmin, s_rng[1]);
    const int64_t nround = (n + 255) / 256;
    for (int64_t q = blockIdx.x; q < nround; q += gridDim.x) {  // block-uniform trip count
        const int64_t p = q * 256 + threadIdx.x;
        const bool valid = p < n;
        uint32_t k = 0;
        if (valid) {
            k = (uint32_t)((key64[p] - kmin) >> s);
            const int64_t o = orig ? (int64_t)orig[p] : p;
            ws.pairs[o] = make_uint2(k, (uint32_t)p);  // one 8-B store per element
        }
#pragma unroll
        for (int d = 0; d < NPASS; ++d) wave_hist_add(s_h[d], (k >> (8 * d)) & 255u, valid);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NPASS * 256; e += 256) {
        const uint32_t c = (&s_h[0][0])[e];
        if (c) atomicAdd(&ws.hist[e], c);
    }
}

// tile = blockIdx.x; global offsets from excl_tab[digit][tile] (k_rs_count + k_rs_rowscan)
template <int PASS, bool PIN = false>
__global__ __launch_bounds__(OB) void k_os_pass(const uint32_t *kin, const uint32_t *vin,
                                                uint32_t *kout, uint32_t *vout, int64_t n,
                                                SortWS ws, const uint32_t *excl_tab,
                                                const double *r, double *rs, const int *skip) {
    if (skip && *skip) return;
    constexpr int SH = 8 * PASS;
    __shared__ uint32_t s_k[OTILE];
    __shared__ uint32_t s_v[OTILE];
    __shared__ uint32_t s_cnt[4][256];
    __shared__ uint32_t s_loc[256];
    __shared__ uint32_t s_gb[256];
    __shared__ uint32_t s_w[4];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = (int)blockIdx.x;
#pragma unroll
    for (int w = 0; w < 4; ++w) s_cnt[w][tid] = 0;
    // digit base = exclusive scan of this pass's global histogram (built by atomics:
    // read it at the memory side too)
    uint32_t htot;
    const uint32_t hv = __hip_atomic_fetch_or(&ws.hist[PASS * 256 + tid], 0u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t dbase = block_excl_scan256<uint32_t>(hv, s_w, htot);
    const int t = s_tile;  // the scan's barriers published s_tile and s_cnt
    if (t >= ws.ntiles) {  // cannot happen with reset tickets; never write out of bounds
        if (tid == 0) atomicOr(&ws.tickets[4], 4u);
        return;
    }
    const int64_t t0 = (int64_t)t * OTILE;
    const int cnt = (int)min((int64_t)OTILE, n - t0);

    // ---- load + rank (stable) without block barriers
    uint32_t k[OIPT], v[OIPT], rk[OIPT];
    const unsigned long long lt = (1ULL << lane) - 1ULL;
#pragma unroll
    for (int j = 0; j < OIPT; ++j) {
        const int li = wave * (OIPT * 64) + j * 64 + lane;
        const bool valid = li < cnt;
        if (PIN) {  // first pass: the (key, position) pairs k_os_hist stored in orig order
            const uint2 q = valid ? ws.pairs[t0 + li] : make_uint2(0u, 0u);
            k[j] = q.x;
            v[j] = q.y;
        } else {
            k[j] = valid ? kin[t0 + li] : 0u;
            v[j] = valid ? vin[t0 + li] : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < OIPT; ++j) {
        const int li = wave * (OIPT * 64) + j * 64 + lane;
        const bool valid = li < cnt;
        const uint32_t d = (k[j] >> SH) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t old = s_cnt[wave][d];
        const int lr = __popcll(peers & lt);
        rk[j] = old + (uint32_t)lr;
        if (valid && lr == 0) s_cnt[wave][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // ---- per digit (thread = digit): wave offsets, tile count, look-back
    const uint32_t c0 = s_cnt[0][tid], c1 = s_cnt[1][tid], c2 = s_cnt[2][tid], c3 = s_cnt[3][tid];
    const uint32_t mine = c0 + c1 + c2 + c3;
    const uint32_t excl = excl_tab[(int64_t)tid * ws.ntiles + t];
    s_gb[tid] = dbase + excl;
    s_cnt[0][tid] = 0;
    s_cnt[1][tid] = c0;
    s_cnt[2][tid] = c0 + c1;
    s_cnt[3][tid] = c0 + c1 + c2;
    uint32_t ltot;
    // the scan's barriers publish s_gb and s_cnt; s_loc is written after them and needs
    // a barrier of its own before any thread reads another digit's entry
    s_loc[tid] = block_excl_scan256<uint32_t>(mine, s_w, ltot);
    __syncthreads();
    // ---- stage the tile in LDS in output order, then write digit runs coalesced
#pragma unroll
    for (int j = 0; j < OIPT; ++j) {
        const int li = wave * (OIPT * 64) + j * 64 + lane;
        if (li < cnt) {
            const uint32_t d = (k[j] >> SH) & 255u;
            const uint32_t pos = s_loc[d] + s_cnt[wave][d] + rk[j];
            s_k[pos] = k[j];
            s_v[pos] = v[j];
        }
    }
    __syncthreads();
    for (int p = tid; p < cnt; p += OB) {
        const uint32_t kk = s_k[p];
        const uint32_t d = (kk >> SH) & 255u;
        const uint32_t g = s_gb[d] + ((uint32_t)p - s_loc[d]);
        const uint32_t vv = s_v[p];
        if (g >= (uint64_t)n || vv >= (uint64_t)n) {  // inconsistent offsets: flag, never fault
            atomicOr(&ws.tickets[4], 8u);
            continue;
        }
        kout[g] = kk;
        vout[g] = vv;
        if (rs) rs[g] = r[vv];
    }
}

// reduce-then-scan: per-tile digit counts of pass PASS -> counts[digit][tile]
template <int PASS, bool PIN = false>
__global__ __launch_bounds__(OB) void k_rs_count(const uint32_t *kin, const uint2 *pin, int64_t n,
                                                 uint32_t *counts, int ntiles, const int *skip) {
    if (skip && *skip) return;
    constexpr int SH = 8 * PASS;
    __shared__ uint32_t s_h[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    s_h[tid] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * OTILE;
    const int cnt = (int)min((int64_t)OTILE, n - t0);
#pragma unroll
    for (int j = 0; j < OIPT; ++j) {
        const int li = wave * (OIPT * 64) + j * 64 + lane;
        const bool valid = li < cnt;
        const uint32_t k = valid ? (PIN ? pin[t0 + li].x : kin[t0 + li]) : 0u;
        wave_hist_add(s_h, (k >> SH) & 255u, valid);
    }
    __syncthreads();
    counts[(int64_t)tid * ntiles + blockIdx.x] = s_h[tid];
}

// one block per digit: exclusive scan over the tiles, in place
__global__ __launch_bounds__(256) void k_rs_rowscan(uint32_t *counts, int ntiles, const int *skip) {
    if (skip && *skip) return;
    __shared__ uint32_t s_w[4];
    uint32_t *row = counts + (int64_t)blockIdx.x * ntiles;
    const int per = (ntiles + 255) / 256;
    const int b0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (int b = b0; b < min(ntiles, b0 + per); ++b) sum += row[b];
    uint32_t total;
    uint32_t pre = block_excl_scan256<uint32_t>(sum, s_w, total);
    for (int b = b0; b < min(ntiles, b0 + per); ++b) {
        const uint32_t c = row[b];
        row[b] = pre;
        pre += c;
    }
}


// Runs of equal key32 hold distinct distances closer than 2^s ulps: order them by the
// full key (stable: equal key64 keep their orig order).
__global__ __launch_bounds__(256) void k_os_fixup(const uint32_t *k32, uint32_t *val,
                                                  const unsigned long long *key64,
                                                  const double *r, double *rs, int64_t n,
                                                  const int *skip) {
    if (skip && *skip) return;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= n) return;
    const uint32_t kj = k32[j];
    if (k32[j + 1] != kj) return;
    if (j > 0 && k32[j - 1] == kj) return;  // not the head of the run
    int64_t e = j + 1;
    while (e < n && k32[e] == kj) ++e;
    bool moved = false;  // stable insertion sort of the run by key64
    for (int64_t a = j + 1; a < e; ++a) {
        const uint32_t v = val[a];
        const unsigned long long kv = key64[v];
        int64_t b = a - 1;
        while (b >= j) {
            const uint32_t vb = val[b];
            if (key64[vb] > kv) {
                val[b + 1] = vb;
                --b;
                moved = true;
            } else {
                break;
            }
        }
        val[b + 1] = v;
    }
    if (rs && moved)
        for (int64_t a = j; a < e; ++a) rs[a] = r[val[a]];
}

// Resets of words that kernels update with atomics (histograms, counters, key ranges,
// flags): done with atomics, never with memset or plain stores.
__global__ __launch_bounds__(256) void k_atomic_zero32(uint32_t *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        __hip_atomic_exchange(&p[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_atomic_zero64(unsigned long long *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        __hip_atomic_exchange(&p[i], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_keys_from_doubles(const double *d, int64_t n,
                                                           unsigned long long *key,
                                                           uint32_t *val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ordkey(d[i]);
    if (val) val[i] = (uint32_t)i;
}

// ------------------------------------------------------------- int32 exclusive scan
template <bool ATOMIC_IN>
__device__ __forceinline__ int32_t scan_load(const int32_t *in, int64_t i) {
    if (ATOMIC_IN)
        return __hip_atomic_fetch_or(const_cast<int32_t *>(in) + i, 0, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    return in[i];
}

template <bool ATOMIC_IN>
__global__ __launch_bounds__(256) void k_scan_partial(const int32_t *in, int64_t n, int32_t *bsum) {
    __shared__ int32_t s_w[4];
    const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int32_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_I; ++q)
        if (t0 + q < n) s += scan_load<ATOMIC_IN>(in, t0 + q);
    int32_t total;
    block_excl_scan256<int32_t>(s, s_w, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_bsums(int32_t *bsum, int nb) {
    __shared__ int32_t s_w[4];
    const int per = (nb + 255) / 256;
    const int b0 = threadIdx.x * per;
    int32_t s = 0;
    for (int b = b0; b < min(nb, b0 + per); ++b) s += bsum[b];
    int32_t total;
    int32_t pre = block_excl_scan256<int32_t>(s, s_w, total);
    for (int b = b0; b < min(nb, b0 + per); ++b) {
        const int32_t c = bsum[b];
        bsum[b] = pre;
        pre += c;
    }
    if (threadIdx.x == 0) bsum[nb] = total;
}

template <bool ATOMIC_IN>
__global__ __launch_bounds__(256) void k_scan_final(const int32_t *in, int32_t *out, int64_t n,
                                                    const int32_t *bsum, int nb) {
    __shared__ int32_t s_w[4];
    const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int32_t v[SCAN_I];
    int32_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_I; ++q) {
        v[q] = (t0 + q < n) ? scan_load<ATOMIC_IN>(in, t0 + q) : 0;
        s += v[q];
    }
    int32_t total;
    int32_t pre = block_excl_scan256<int32_t>(s, s_w, total) + bsum[blockIdx.x];
#pragma unroll
    for (int q = 0; q < SCAN_I; ++q) {
        if (t0 + q < n) out[t0 + q] = pre;
        pre += v[q];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = bsum[nb];
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }
inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

SortWS carve(void *tmp, int64_t n) {
    SortWS w{};
    w.ntiles = (int)((n + OTILE - 1) / OTILE);
    char *p = (char *)tmp;
    w.kA = (uint32_t *)p;
    p += align_up(n * 4, 256);
    w.kB = (uint32_t *)p;
    p += align_up(n * 4, 256);
    w.vB = (uint32_t *)p;
    p += align_up(n * 4, 256);
    w.pairs = (uint2 *)w.kB;  // 8n bytes over kB and vB (contiguous; both free until pass 1)
    w.hist = (uint32_t *)p;
    p += 4 * 256 * 4;
    w.tickets = (uint32_t *)p;
    p += 256;
    w.status = (uint32_t *)p;
    p += align_up(4LL * w.ntiles * 256 * 4, 256);
    w.counts = (uint32_t *)p;
    return w;
}

}  // namespace

int64_t scan_tmp_elems(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_scan_i32(const int32_t *in, int32_t *out, int64_t n, int32_t *tmp,
                           bool atomic_in, hipStream_t s) {
    const int nb = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (nb == 0) return hipMemsetAsync(out, 0, sizeof(int32_t), s);
    if (atomic_in)
        hipLaunchKernelGGL(k_scan_partial<true>, dim3(nb), dim3(256), 0, s, in, n, tmp);
    else
        hipLaunchKernelGGL(k_scan_partial<false>, dim3(nb), dim3(256), 0, s, in, n, tmp);
    hipLaunchKernelGGL(k_scan_bsums, dim3(1), dim3(256), 0, s, tmp, nb);
    if (atomic_in)
        hipLaunchKernelGGL(k_scan_final<true>, dim3(nb), dim3(256), 0, s, in, out, n, tmp, nb);
    else
        hipLaunchKernelGGL(k_scan_final<false>, dim3(nb), dim3(256), 0, s, in, out, n, tmp, nb);
    return hipGetLastError();
}

hipError_t launch_atomic_zero32(uint32_t *p, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int nb = (int)std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_atomic_zero32, dim3(nb), dim3(256), 0, s, p, n);
    return hipGetLastError();
}

hipError_t launch_atomic_zero64(unsigned long long *p, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int nb = (int)std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_atomic_zero64, dim3(nb), dim3(256), 0, s, p, n);
    return hipGetLastError();
}

uint32_t *sort_timeout_flag(void *tmp, int64_t n) { return carve(tmp, n).tickets + 4; }

int64_t sort_tmp_bytes(int64_t n) {
    const int64_t nt = (n + OTILE - 1) / OTILE;
    return 3 * align_up(n * 4, 256) + 4 * 256 * 4 + 256 + align_up(4 * nt * 256 * 4, 256) +
           nt * 256 * 4 + 256;
}

hipError_t launch_range_reduce(unsigned long long *range, int64_t nparts, hipStream_t s) {
    hipLaunchKernelGGL(k_range_reduce, dim3(1), dim3(1024), 0, s, range, nparts);
    return hipGetLastError();
}

hipError_t launch_key_range(const unsigned long long *key, int64_t n, unsigned long long *range,
                            hipStream_t s) {
    const int nb = (int)std::min<int64_t>(512, std::max<int64_t>(1, (n + 255) / 256));
    hipLaunchKernelGGL(k_key_range, dim3(nb), dim3(256), 0, s, key, n, range);
    return launch_range_reduce(range, nb, s);
}

hipError_t launch_sort(const unsigned long long *key64, const uint32_t *orig, int64_t n,
                       unsigned long long *range, uint32_t *order, const double *r, double *rs,
                       void *tmp, const int *skip, hipStream_t s) {
    if (n == 0) return hipSuccess;
    SortWS w = carve(tmp, n);
    hipLaunchKernelGGL(k_atomic_zero32, dim3(NPASS), dim3(256), 0, s, w.hist,
                       (int64_t)(NPASS * 256));
    const int64_t status_words = 0;
    const int hb = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (n + 2047) / 2048));
    hipLaunchKernelGGL(k_os_hist, dim3(hb), dim3(256), 0, s, key64, orig, n,
                       (const unsigned long long *)range, w, status_words, skip);
    // pairs -> (kA, order) -> (kB, vB) -> (kA, order); the last pass also gathers rs
    static_assert(NPASS == 3, "pass chain below is written for three 8-bit digits");
    const dim3 g(w.ntiles), b(OB);
    const uint32_t *nul = nullptr;
#define FICP_PASS(P, PIN, KIN, VIN, KOUT, VOUT, R, RS)                                        \
    hipLaunchKernelGGL((k_rs_count<P, PIN>), g, b, 0, s, KIN, (const uint2 *)w.pairs, n,       \
                       w.counts, w.ntiles, skip);                                             \
    hipLaunchKernelGGL(k_rs_rowscan, dim3(256), dim3(256), 0, s, w.counts, w.ntiles, skip);     \
    hipLaunchKernelGGL((k_os_pass<P, PIN>), g, b, 0, s, KIN, VIN, KOUT, VOUT, n, w,             \
                       (const uint32_t *)w.counts, R, RS, skip);
    const double *rnul = nullptr;
    double *rsnul = nullptr;
    FICP_PASS(0, true, nul, nul, w.kA, order, rnul, rsnul)
    FICP_PASS(1, false, w.kA, order, w.kB, w.vB, rnul, rsnul)
    FICP_PASS(2, false, w.kB, w.vB, w.kA, order, r, rs)
#undef FICP_PASS
    hipLaunchKernelGGL(k_os_fixup, dim3(nblk(n)), dim3(256), 0, s, w.kA, order, key64, r, rs, n,
                       skip);
    return hipGetLastError();
}

hipError_t launch_keys_from_doubles(const double *d, int64_t n, unsigned long long *key,
                                    uint32_t *val, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keys_from_doubles, dim3(nblk(n)), dim3(256), 0, s, d, n, key, val);
    return hipGetLastError();
}

}  // namespace ficp
