// k_sort.hip -- the fractional-trim residual sort (ficp.py:63,78: argsort(distances))
// and the int32 exclusive scan used by the grid build.
//
// Sort contract: stable order of (key, val) pairs by the 64-bit order-preserving key of
// the distance, val = source index, input in index order -> ties end up ordered by
// index.  Method:
//   1. stable LSD radix sort of the TOP 32 key bits (4 passes x 8-bit digits; per pass
//      a tile histogram, a per-digit scan over tiles and a stable scatter that ranks the
//      tile in LDS with 64-lane ballot matching and writes digit runs coalesced);
//   2. fix-up: each run of equal top-32 bits is re-ordered by the full 64-bit key with
//      an insertion sort by the run's first lane (runs are short: the top 32 bits of a
//      double carry 20 mantissa bits; equal full keys are already in index order).
// Top-32 + fix-up moves 20 B per item per pass instead of 32 B and halves the passes of
// a full 64-bit LSD sort.
#include "ficp_internal.h"

namespace ficp {

namespace {

constexpr int SB = 256;             // threads per sort block
constexpr int SI = 16;              // items per thread
constexpr int STILE = SB * SI;      // items per tile
constexpr int SCAN_I = 16;
constexpr int SCAN_TILE = 256 * SCAN_I;

__device__ __forceinline__ unsigned long long ordkey(double v) {
    unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

// exclusive scan of one uint32 per thread over a 256-thread block (4 waves)
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

template <bool FROM64>
__device__ __forceinline__ uint32_t load_key(const void *kin, int64_t i) {
    if (FROM64) return (uint32_t)(((const unsigned long long *)kin)[i] >> 32);
    return ((const uint32_t *)kin)[i];
}

template <bool FROM64>
__global__ __launch_bounds__(SB) void k_radix_hist(const void *kin, int64_t n, int shift,
                                                   uint32_t *counts, int nb, const int *skip) {
    if (skip && *skip) return;
    __shared__ uint32_t s_h[256];
    s_h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * STILE;
    const int cnt = (int)min((int64_t)STILE, n - t0);
    for (int li = threadIdx.x; li < cnt; li += SB) {
        const uint32_t k = load_key<FROM64>(kin, t0 + li);
        atomicAdd(&s_h[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * nb + blockIdx.x] = s_h[threadIdx.x];
}

// one block per digit: exclusive scan of counts[d][0..nb) in place, rowtot[d] = total
__global__ __launch_bounds__(SB) void k_radix_rowscan(uint32_t *counts, int nb, uint32_t *rowtot,
                                                      const int *skip) {
    if (skip && *skip) return;
    __shared__ uint32_t s_w[4];
    uint32_t *row = counts + (int64_t)blockIdx.x * nb;
    const int per = (nb + SB - 1) / SB;
    const int b0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (int b = b0; b < min(nb, b0 + per); ++b) sum += row[b];
    uint32_t total;
    uint32_t pre = block_excl_scan256<uint32_t>(sum, s_w, total);
    for (int b = b0; b < min(nb, b0 + per); ++b) {
        const uint32_t c = row[b];
        row[b] = pre;
        pre += c;
    }
    if (threadIdx.x == 0) rowtot[blockIdx.x] = total;
}

template <bool FROM64>
__global__ __launch_bounds__(SB) void k_radix_scatter(const void *kin, const uint32_t *vin,
                                                      int64_t n, int shift,
                                                      const uint32_t *counts,
                                                      const uint32_t *rowtot, int nb,
                                                      uint32_t *kout, uint32_t *vout,
                                                      const double *rin, double *rout,
                                                      const int *skip) {
    if (skip && *skip) return;
    __shared__ uint32_t s_k[STILE];
    __shared__ uint32_t s_v[STILE];
    __shared__ uint32_t s_base[256];
    __shared__ uint32_t s_loc[256];
    __shared__ uint32_t s_run[256];
    __shared__ uint32_t s_wc[4][256];
    __shared__ uint32_t s_w[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * STILE;
    const int cnt = (int)min((int64_t)STILE, n - t0);

    const uint32_t tot = rowtot[tid];
    const uint32_t mine = counts[(int64_t)tid * nb + blockIdx.x];
    const uint32_t nxt = (blockIdx.x + 1 < (unsigned)nb) ? counts[(int64_t)tid * nb + blockIdx.x + 1] : tot;
    uint32_t dummy;
    const uint32_t ex_tot = block_excl_scan256<uint32_t>(tot, s_w, dummy);
    const uint32_t ex_loc = block_excl_scan256<uint32_t>(nxt - mine, s_w, dummy);
    s_base[tid] = ex_tot + mine;
    s_loc[tid] = ex_loc;
    s_run[tid] = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) s_wc[w][tid] = 0;
    __syncthreads();

    const unsigned long long lt = (1ULL << lane) - 1ULL;
    for (int r = 0; r < SI; ++r) {
        const int li = r * SB + tid;
        const bool valid = li < cnt;
        uint32_t k = 0, v = 0;
        int d = 0;
        if (valid) {
            k = load_key<FROM64>(kin, t0 + li);
            v = vin ? vin[t0 + li] : (uint32_t)(t0 + li);
            d = (k >> shift) & 255;
        }
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const int lrank = __popcll(peers & lt);
        if (valid && lrank == 0) s_wc[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pre = s_run[d];
            for (int w = 0; w < wave; ++w) pre += s_wc[w][d];
            const uint32_t pos = s_loc[d] + pre + (uint32_t)lrank;
            s_k[pos] = k;
            s_v[pos] = v;
        }
        __syncthreads();
        s_run[tid] += s_wc[0][tid] + s_wc[1][tid] + s_wc[2][tid] + s_wc[3][tid];
#pragma unroll
        for (int w = 0; w < 4; ++w) s_wc[w][tid] = 0;
        __syncthreads();
    }
    for (int li = tid; li < cnt; li += SB) {
        const uint32_t k = s_k[li];
        const int d = (k >> shift) & 255;
        const uint32_t g = s_base[d] + ((uint32_t)li - s_loc[d]);
        kout[g] = k;
        vout[g] = s_v[li];
        if (rout) rout[g] = rin[s_v[li]];  // last pass: residuals in selection order
    }
}

// runs of equal top-32 bits: order by the full key (stable insertion sort by the run head)
__global__ __launch_bounds__(256) void k_sort_fixup(const uint32_t *k32, uint32_t *val,
                                                    const unsigned long long *key64,
                                                    const double *rin, double *rout, int64_t n,
                                                    const int *skip) {
    if (skip && *skip) return;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= n) return;
    const uint32_t kj = k32[j];
    if (k32[j + 1] != kj) return;
    if (j > 0 && k32[j - 1] == kj) return;  // not the head of the run
    int64_t e = j + 1;
    while (e < n && k32[e] == kj) ++e;
    for (int64_t a = j + 1; a < e; ++a) {
        const uint32_t v = val[a];
        const unsigned long long kv = key64[v];
        int64_t b = a - 1;
        while (b >= j) {
            const uint32_t vb = val[b];
            const unsigned long long kb = key64[vb];
            if (kb > kv || (kb == kv && vb > v)) {
                val[b + 1] = vb;
                --b;
            } else {
                break;
            }
        }
        val[b + 1] = v;
    }
    if (rout)
        for (int64_t a = j; a < e; ++a) rout[a] = rin[val[a]];
}

__global__ __launch_bounds__(256) void k_keys_from_doubles(const double *d, int64_t n,
                                                           unsigned long long *key,
                                                           uint32_t *val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ordkey(d[i]);
    val[i] = (uint32_t)i;
}

// ------------------------------------------------------------- int32 exclusive scan
__global__ __launch_bounds__(256) void k_scan_partial(const int32_t *in, int64_t n, int32_t *bsum) {
    __shared__ int32_t s_w[4];
    const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int32_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_I; ++q)
        if (t0 + q < n) s += in[t0 + q];
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

__global__ __launch_bounds__(256) void k_scan_final(const int32_t *in, int32_t *out, int64_t n,
                                                    const int32_t *bsum, int nb) {
    __shared__ int32_t s_w[4];
    const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int32_t v[SCAN_I];
    int32_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_I; ++q) {
        v[q] = (t0 + q < n) ? in[t0 + q] : 0;
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

}  // namespace

int64_t scan_tmp_elems(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_scan_i32(const int32_t *in, int32_t *out, int64_t n, int32_t *tmp,
                           hipStream_t s) {
    const int nb = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (nb == 0) {
        hipMemsetAsync(out, 0, sizeof(int32_t), s);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_scan_partial, dim3(nb), dim3(256), 0, s, in, n, tmp);
    hipLaunchKernelGGL(k_scan_bsums, dim3(1), dim3(256), 0, s, tmp, nb);
    hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(256), 0, s, in, out, n, tmp, nb);
    return hipGetLastError();
}

static inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

int64_t sort_tmp_bytes(int64_t n) {
    const int64_t nb = (n + STILE - 1) / STILE;
    return 3 * align_up(n * 4, 256) + align_up(256 * nb * 4, 256) + 256 * 4 + 256;
}

hipError_t launch_sort_pairs(const unsigned long long *key, const uint32_t *val_in, int64_t n,
                             uint32_t *val_out, const double *r_in, double *r_sorted, void *tmp,
                             const int *skip, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int nb = (int)((n + STILE - 1) / STILE);
    char *p = (char *)tmp;
    uint32_t *kA = (uint32_t *)p;
    p += align_up(n * 4, 256);
    uint32_t *kB = (uint32_t *)p;
    p += align_up(n * 4, 256);
    uint32_t *vB = (uint32_t *)p;
    p += align_up(n * 4, 256);
    uint32_t *counts = (uint32_t *)p;
    p += align_up((int64_t)256 * nb * 4, 256);
    uint32_t *rowtot = (uint32_t *)p;
    // pass 0: from the u64 keys (bits 32..39) into B; then B->A(val_out), A->B, B->A
    const void *kin = key;
    const uint32_t *vin = val_in;
    uint32_t *kouts[4] = {kB, kA, kB, kA};
    uint32_t *vouts[4] = {vB, val_out, vB, val_out};
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 8 * pass;
        if (pass == 0) {
            hipLaunchKernelGGL(k_radix_hist<true>, dim3(nb), dim3(SB), 0, s, kin, n, shift, counts,
                               nb, skip);
        } else {
            hipLaunchKernelGGL(k_radix_hist<false>, dim3(nb), dim3(SB), 0, s, kin, n, shift,
                               counts, nb, skip);
        }
        hipLaunchKernelGGL(k_radix_rowscan, dim3(256), dim3(SB), 0, s, counts, nb, rowtot, skip);
        if (pass == 0) {
            hipLaunchKernelGGL(k_radix_scatter<true>, dim3(nb), dim3(SB), 0, s, kin, vin, n, shift,
                               counts, rowtot, nb, kouts[pass], vouts[pass],
                               (const double *)nullptr, (double *)nullptr, skip);
        } else {
            hipLaunchKernelGGL(k_radix_scatter<false>, dim3(nb), dim3(SB), 0, s, kin, vin, n,
                               shift, counts, rowtot, nb, kouts[pass], vouts[pass],
                               pass == 3 ? r_in : (const double *)nullptr,
                               pass == 3 ? r_sorted : (double *)nullptr, skip);
        }
        kin = kouts[pass];
        vin = vouts[pass];
    }
    hipLaunchKernelGGL(k_sort_fixup, dim3(nblk(n)), dim3(256), 0, s, kA, val_out, key, r_in,
                       r_sorted, n, skip);
    return hipGetLastError();
}

hipError_t launch_keys_from_doubles(const double *d, int64_t n, unsigned long long *key,
                                    uint32_t *val, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keys_from_doubles, dim3(nblk(n)), dim3(256), 0, s, d, n, key, val);
    return hipGetLastError();
}

}  // namespace ficp
