// gap_probe.hip -- idle gap after a kernel that leaves much dirty data in L2 (tools only):
// pairs (writer of B bytes, small reader) on one stream; run under
// rocprofv3 --kernel-trace and read the gap between each writer's end and the next start.
// Build: hipcc -O3 --offload-arch=gfx950 tools/gap_probe.hip -o tools/gap_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_write(double *p, long long n, double v) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long long j = i; j < n; j += (long long)gridDim.x * blockDim.x) p[j] = v + (double)j;
}
__global__ void k_write_nt(double *p, long long n, double v) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long long j = i; j < n; j += (long long)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(v + (double)j, p + j);
}
__global__ void k_small(double *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = p[1] + 1.0;
}

int main() {
    double *d;
    const long long maxn = 64LL << 20;  // 512 MB
    if (hipMalloc(&d, maxn * 8) != hipSuccess) return 1;
    hipStream_t s;
    hipStreamCreate(&s);
    for (long long mb : {1LL, 8LL, 32LL, 64LL}) {
        const long long n = mb << 17;  // doubles
        for (int r = 0; r < 20; ++r) {
            hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, s, d, n, (double)r);
            hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d);
        }
        for (int r = 0; r < 20; ++r) {
            hipLaunchKernelGGL(k_write_nt, dim3(4096), dim3(256), 0, s, d, n, (double)r);
            hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d);
        }
    }
    hipStreamSynchronize(s);
    printf("done\n");
    return 0;
}
