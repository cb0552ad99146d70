// Microbenchmark: cost of the per-element histogram forms a bucketed residual selection
// could use (1M elements, random bucket ids).  Prints microseconds per pass (median of 20).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_direct(const uint32_t *b, const double *r, int n, uint32_t *cnt, double *sum) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t q = b[i];
    __hip_atomic_fetch_add(&cnt[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsafeAtomicAdd(&sum[q], r[i]);
}
__global__ void k_direct_u64(const uint32_t *b, const double *r, int n, unsigned long long *acc) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t q = b[i];
    unsigned long long v = (1ULL << 44) | (unsigned long long)(r[i] * 1048576.0);
    __hip_atomic_fetch_add(&acc[q], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_count_only(const uint32_t *b, int n, uint32_t *cnt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    __hip_atomic_fetch_add(&cnt[b[i]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int NB>
__global__ __launch_bounds__(1024) void k_lds(const uint32_t *b, const double *r, int n, int per, uint32_t *cnt, double *sum) {
    __shared__ uint32_t sc[NB];
    __shared__ double ss[NB];
    for (int j = threadIdx.x; j < NB; j += blockDim.x) { sc[j] = 0; ss[j] = 0.0; }
    __syncthreads();
    int i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        uint32_t q = b[i] & (NB - 1);
        atomicAdd(&sc[q], 1u);
        atomicAdd(&ss[q], r[i]);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < NB; j += blockDim.x) {
        if (sc[j]) {
            __hip_atomic_fetch_add(&cnt[j], sc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsafeAtomicAdd(&sum[j], ss[j]);
        }
    }
}
__global__ void k_stream(const uint32_t *b, const double *r, int n, double *out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = r[i] + (double)b[i];
    if (v == -1.0) out[0] = v;
}

int main() {
    const int n = 1 << 20, NB = 65536;
    std::vector<uint32_t> hb(n);
    std::vector<double> hr(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        // bell-shaped occupancy like the residual buckets: sum of two uniforms
        uint32_t a = (s >> 33) & 0x7fff, c = (s >> 17) & 0x7fff;
        hb[i] = (a + c) & (NB - 1);
        hr[i] = (double)((s >> 40) & 0xffff) * 1e-3;
    }
    uint32_t *b, *cnt; double *r, *sum, *out; unsigned long long *acc;
    CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&r, n * 8)); CK(hipMalloc(&cnt, NB * 4));
    CK(hipMalloc(&sum, NB * 8)); CK(hipMalloc(&acc, NB * 8)); CK(hipMalloc(&out, 8));
    CK(hipMemcpy(b, hb.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(r, hr.data(), n * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn) {
        std::vector<float> t;
        for (int it = 0; it < 25; ++it) {
            hipEventRecord(e0); fn(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (it >= 5) t.push_back(ms * 1000.f);
        }
        std::sort(t.begin(), t.end());
        printf("%-28s %8.2f us (min %.2f)\n", name, t[t.size() / 2], t[0]);
    };
    const int g = (n + 255) / 256;
    timeit("stream read 12B/elt", [&] { k_stream<<<g, 256>>>(b, r, n, out); });
    timeit("count only u32 64K", [&] { k_count_only<<<g, 256>>>(b, n, cnt); });
    timeit("direct u32+f64 64K", [&] { k_direct<<<g, 256>>>(b, r, n, cnt, sum); });
    timeit("direct u64 packed 64K", [&] { k_direct_u64<<<g, 256>>>(b, r, n, acc); });
    timeit("lds 4096 x 256 WG", [&] { k_lds<4096><<<256, 1024>>>(b, r, n, n / 256, cnt, sum); });
    timeit("lds 4096 x 64 WG", [&] { k_lds<4096><<<64, 1024>>>(b, r, n, n / 64, cnt, sum); });
    timeit("lds 8192 x 128 WG", [&] { k_lds<8192><<<128, 1024>>>(b, r, n, n / 128, cnt, sum); });
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
