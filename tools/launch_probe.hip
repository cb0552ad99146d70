// launch_probe.hip -- back-to-back dispatch cost of dependent kernels on one stream
// (tools only): 1000 launches of an empty kernel at several grid shapes, and a chain of
// 1000 kernels where each reads what the previous one wrote.  Prints us per launch.
// Build: hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                         \
    do {                                                              \
        hipError_t e = (x);                                           \
        if (e != hipSuccess) {                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                 \
        }                                                             \
    } while (0)

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0 && *p == 12345) *p = 0;
}

__global__ void k_chain(int *p) {
    __shared__ int s;
    if (threadIdx.x == 0) s = p[blockIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) p[blockIdx.x] = s + 1;
}

__global__ void k_lds64k(int *p) {
    __shared__ double big[8192];
    big[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0 && big[5] == 12345.0) *p = 0;
}

int main() {
    int *d;
    CK(hipMalloc(&d, 1 << 20));
    CK(hipMemset(d, 0, 1 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg {
        const char *name;
        int kind, grid, block;
    } cfgs[] = {{"empty 1x64", 0, 1, 64},          {"empty 1x512", 0, 1, 512},
                {"empty 128x1024", 0, 128, 1024},  {"empty 4096x256", 0, 4096, 256},
                {"chain 1x512", 1, 1, 512},        {"chain 128x256", 1, 128, 256},
                {"lds64k 128x1024", 2, 128, 1024}, {"lds64k 1x512", 2, 1, 512}};
    for (const Cfg &c : cfgs) {
        for (int rep = 0; rep < 2; ++rep) {
            const int N = 1000;
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < N; ++i) {
                if (c.kind == 0) hipLaunchKernelGGL(k_empty, dim3(c.grid), dim3(c.block), 0, s, d);
                if (c.kind == 1) hipLaunchKernelGGL(k_chain, dim3(c.grid), dim3(c.block), 0, s, d);
                if (c.kind == 2) hipLaunchKernelGGL(k_lds64k, dim3(c.grid), dim3(c.block), 0, s, d);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) printf("%-18s %7.2f us per launch\n", c.name, ms * 1000.f / N);
        }
    }
    // the same dependent chain captured into hipGraphs: one graph of 1000 kernels, and a
    // graph of 7 (one loop body) launched 1000 / 7 times
    for (int len : {1000, 7}) {
        for (int grid : {1, 128}) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int i = 0; i < len; ++i)
                hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, d);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            const int reps = 1000 / len;
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipEventRecord(e0, s));
                for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep)
                    printf("graph of %4d, chain %dx256 %7.2f us per kernel\n", len, grid,
                           ms * 1000.f / (reps * len));
            }
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    return 0;
}
