// k_loop.hip -- the ICP loop of ficp.py:122-154 as a device-resident state machine.
//
// One "iteration" of the host's launch sequence is {fit -> NN (+apply) -> sort -> FRMSD
// scan -> k_loop_update}; k_loop_update takes the decisions of _iterate/run on the
// device (stage head, convergence test `current - new <= threshold` (ficp.py:142),
// max_iterations, the lambda switch of ficp.py:152) and sets the skip flags the next
// iteration's kernels read, so the host only enqueues iterations and watches one flag
// a few iterations behind instead of synchronising on every NN call.
#include "ficp_internal.h"

#include <math.h>
#include <string.h>

namespace ficp {

namespace {

__device__ void loop_init(IterState *st, const LoopCtl &c) {
    IterState &s = *st;
    for (int e = 0; e < 9; ++e) s.Ttot[e] = (e % 4 == 0) ? 1.0 : 0.0;
    s.cur = INFINITY;
    s.frmsd_last[0] = s.frmsd_last[1] = INFINITY;
    s.k_last = 0;
    s.stage = 0;
    s.it = 0;
    s.n_nn = s.n_fit = 0;
    s.n_reuse = 0;
    s.win_fail = 0;
    s.wfloor = 0;  // (win_start_log of the plot's rows)
    s.iters[0] = s.iters[1] = 0;
    s.phase = c.nstages > 0 ? PH_HEAD : PH_DONE;
    s.lam_cur = c.nstages > 0 ? lam_of(c, 0) : 0.0;
    loop_set_flags(s);
}

__global__ void k_loop_init(IterState *st, LoopCtl c) {
    if (threadIdx.x == 0) loop_init(st, c);
}

__global__ void k_loop_update(IterState *st, LoopCtl c) {
    if (threadIdx.x != 0) return;
    IterState s = *st;  // one batch of loads instead of a chain of dependent round trips
    loop_step(&s, c);
    *st = s;
}

// idx of this call, in the caller's row order, into the trace (before k_loop_update)
__global__ __launch_bounds__(256) void k_trace_idx(const IterState *st, const int32_t *idx,
                                                   const uint32_t *worig, int64_t n,
                                                   int32_t *out, int max_trace) {
    if (st->done) return;
    const int call = st->n_nn;
    if (call >= max_trace) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[(int64_t)call * n + (worig ? (int64_t)worig[i] : i)] = idx[i];
}

}  // namespace

// Copies up to three device segments into coherent pinned host memory and then raises
// *flag (system scope, after a system fence): the host polls the flag instead of a
// stream synchronisation plus one hipMemcpyAsync per segment (those cost 40-50 us of idle
// device each at C3, profiles/r1sel trace).
// run start: zero the sort's timeout flag and stamp the device clock (100 MHz) into
// coherent host memory; the report kernel stamps the end (ficp_stats::gpu_ms without
// event records, each of which left ~5 us of idle queue); with st, the loop state's
// initialisation too (one launch less per run)
__global__ void k_run_start(uint32_t *tflag, unsigned long long *t0, unsigned *selerr,
                            IterState *st, LoopCtl lc) {
    if (threadIdx.x == 0) {
        if (st) loop_init(st, lc);
        __hip_atomic_exchange(tflag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the selection's sticky error bits are per run (a failed run leaves no poison)
        if (selerr) __hip_atomic_exchange(selerr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(t0, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_run_start(uint32_t *tflag, unsigned long long *t0, hipStream_t s,
                            unsigned *selerr, IterState *st, const LoopCtl *lc) {
    const LoopCtl c = lc ? *lc : LoopCtl{};
    hipLaunchKernelGGL(k_run_start, dim3(1), dim3(64), 0, s, tflag, t0, selerr, lc ? st : nullptr,
                       c);
    return hipGetLastError();
}

__global__ void k_report(ReportSeg a, ReportSeg b, ReportSeg c, int *flag,
                         unsigned long long *t_end) {
    const ReportSeg sg[3] = {a, b, c};
    for (int q = 0; q < 3; ++q) {
        const uint32_t *src = (const uint32_t *)sg[q].src;
        uint32_t *dst = (uint32_t *)sg[q].dst;
        const int nw = sg[q].words;
        // 16-B words where both ends allow (the batch's per-plot states, ~240 KB at 1,024
        // plots: 4-B stores into host memory from 256 threads took ~55 us)
        const bool v4 = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
        const int n4 = v4 ? nw / 4 : 0;
        for (int w = threadIdx.x; w < n4; w += blockDim.x)
            reinterpret_cast<uint4 *>(dst)[w] = reinterpret_cast<const uint4 *>(src)[w];
        for (int w = 4 * n4 + threadIdx.x; w < nw; w += blockDim.x) dst[w] = src[w];
    }
    if (t_end && threadIdx.x == 0)
        __hip_atomic_store(t_end, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_report(const ReportSeg &a, const ReportSeg &b, const ReportSeg &c, int *flag,
                         unsigned long long *t_end,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_report, dim3(1), dim3(1024), 0, s, a, b, c, flag, t_end);
    return hipGetLastError();
}

hipError_t launch_loop_init(IterState *st, const LoopCtl &c, hipStream_t s) {
    hipLaunchKernelGGL(k_loop_init, dim3(1), dim3(64), 0, s, st, c);
    return hipGetLastError();
}

hipError_t launch_loop_update(IterState *st, const LoopCtl &c, hipStream_t s) {
    hipLaunchKernelGGL(k_loop_update, dim3(1), dim3(64), 0, s, st, c);
    return hipGetLastError();
}

hipError_t launch_trace_idx(const IterState *st, const int32_t *idx, const uint32_t *worig,
                            int64_t n, int32_t *out, int max_trace, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_trace_idx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, st, idx,
                       worig, n, out, max_trace);
    return hipGetLastError();
}

}  // namespace ficp
