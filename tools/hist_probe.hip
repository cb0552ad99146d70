// hist_probe.hip -- cost of building the selection's level-0 histogram (8192 packed u64
// buckets) with one device-scope atomic per row, on C3-like residual keys (tools only).
// Build: hipcc -O3 --offload-arch=gfx950 tools/hist_probe.hip -o tools/hist_probe
// Prints microseconds per pass (median of 30) for 1M rows:
//   direct   : one global 64-bit atomic add per row (bucket from the key bits)
//   waveagg  : lanes of a wave with the same bucket combined first (match + one atomic)
//   ldsflush : per-256-row-block LDS histogram, nonzero buckets flushed with atomics
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s: %s\n", #x, hipGetErrorString(e));                        \
            return 1;                                                            \
        }                                                                        \
    } while (0)

typedef unsigned long long u64;
constexpr int NB = 8192;

__global__ void k_direct(const u64 *key, const double *r, int n, u64 kmin, int s, u64 *h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)min((key[i] - kmin) >> s, (u64)(NB - 1));
    const u64 v = (1ULL << 43) + (u64)ldexp(r[i], 10);
    __hip_atomic_fetch_add(&h[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_waveagg(const u64 *key, const double *r, int n, u64 kmin, int s, u64 *h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = i < n;
    const int b = ok ? (int)min((key[i] - kmin) >> s, (u64)(NB - 1)) : -1;
    u64 v = ok ? (1ULL << 43) + (u64)ldexp(r[i], 10) : 0;
    // lanes sharing a bucket: the lowest lane adds the group's sum
    const int lane = threadIdx.x & 63;
    u64 pend = __ballot(ok);
    while (pend) {
        const int l0 = __ffsll((long long)pend) - 1;
        const int b0 = __shfl(b, l0);
        const u64 same = __ballot(b == b0);
        u64 x = (b == b0) ? v : 0;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if (lane == l0) __hip_atomic_fetch_add(&h[b0], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend &= ~same;
        if (__popcll(same) < 4) break;  // the rest direct
    }
    if (pend >> lane & 1)
        __hip_atomic_fetch_add(&h[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_ldsflush(const u64 *key, const double *r, int n, u64 kmin, int s, u64 *h) {
    __shared__ u64 sh[NB];
    for (int j = threadIdx.x; j < NB; j += blockDim.x) sh[j] = 0;
    __syncthreads();
    const int per = 4;
    int bs[per];
    for (int q = 0; q < per; ++q) {
        const int i = (blockIdx.x * per + q) * blockDim.x + threadIdx.x;
        bs[q] = -1;
        if (i < n) {
            const int b = (int)min((key[i] - kmin) >> s, (u64)(NB - 1));
            atomicAdd(&sh[b], (1ULL << 43) + (u64)ldexp(r[i], 10));
            bs[q] = b;
        }
    }
    __syncthreads();
    // flush: each row's bucket once (the first row that sees a nonzero value takes it)
    for (int q = 0; q < per; ++q) {
        if (bs[q] >= 0) {
            const u64 v = atomicExch(&sh[bs[q]], 0ULL);
            if (v) __hip_atomic_fetch_add(&h[bs[q]], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

static u64 hkey(double v) {
    u64 u;
    memcpy(&u, &v, 8);
    return u | 0x8000000000000000ULL;
}

int main() {
    const int n = 1 << 20;
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    std::vector<u64> key(n);
    std::vector<double> r(n);
    for (int i = 0; i < n; ++i) {
        double d2;
        if (ud(rng) < 0.6) {
            const double a = nd(rng), b = nd(rng), c = nd(rng);
            d2 = 0.09 * (a * a + b * b) + c * c * 0.01;
        } else {
            const double d = 2.0 * sqrt(-2.0 * log(1.0 - ud(rng)));
            d2 = d * d;
        }
        r[i] = d2;
        key[i] = hkey(sqrt(d2));
    }
    const u64 kmin = *std::min_element(key.begin(), key.end());
    const u64 kmax = *std::max_element(key.begin(), key.end());
    int bits = 64 - __builtin_clzll(kmax - kmin);
    const int s = bits > 13 ? bits - 13 : 0;
    std::vector<int> cnt(NB, 0);
    for (int i = 0; i < n; ++i) cnt[std::min<u64>((key[i] - kmin) >> s, NB - 1)]++;
    printf("hottest bucket %d rows, nonzero buckets %ld\n", *std::max_element(cnt.begin(), cnt.end()),
           (long)std::count_if(cnt.begin(), cnt.end(), [](int c) { return c > 0; }));
    // work order: rows in a spatial order, keys random -> shuffle like the NN output
    u64 *dk;
    double *dr;
    u64 *dh;
    CK(hipMalloc(&dk, n * 8));
    CK(hipMalloc(&dr, n * 8));
    CK(hipMalloc(&dh, NB * 8));
    CK(hipMemcpy(dk, key.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, r.data(), n * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[3] = {"direct", "waveagg", "ldsflush"};
    for (int v = 0; v < 3; ++v) {
        std::vector<float> t;
        for (int rep = 0; rep < 30; ++rep) {
            CK(hipMemset(dh, 0, NB * 8));
            CK(hipEventRecord(e0));
            if (v == 0) hipLaunchKernelGGL(k_direct, dim3(n / 256), dim3(256), 0, 0, dk, dr, n, kmin, s, dh);
            if (v == 1) hipLaunchKernelGGL(k_waveagg, dim3(n / 256), dim3(256), 0, 0, dk, dr, n, kmin, s, dh);
            if (v == 2) hipLaunchKernelGGL(k_ldsflush, dim3(n / 1024), dim3(256), 0, 0, dk, dr, n, kmin, s, dh);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1000.f);
        }
        std::vector<u64> hh(NB);
        CK(hipMemcpy(hh.data(), dh, NB * 8, hipMemcpyDeviceToHost));
        u64 tot = 0;
        for (u64 x : hh) tot += x >> 43;
        std::sort(t.begin(), t.end());
        printf("%-10s %8.2f us (min %.2f) rows %llu\n", names[v], t[15], t[0], tot);
    }
    return 0;
}
