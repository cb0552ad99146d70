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

__device__ __forceinline__ void set_flags(IterState &s) {
    s.done = s.phase == PH_DONE;
    s.no_fit = s.phase != PH_LOOP;
    s.apply = s.phase == PH_LOOP;
}

__global__ void k_loop_init(IterState *st, LoopCtl c) {
    if (threadIdx.x != 0) return;
    IterState &s = *st;
    for (int e = 0; e < 9; ++e) s.Ttot[e] = (e % 4 == 0) ? 1.0 : 0.0;
    s.cur = INFINITY;
    s.frmsd_last[0] = s.frmsd_last[1] = INFINITY;
    s.k_last = 0;
    s.stage = 0;
    s.it = 0;
    s.n_nn = s.n_fit = 0;
    s.iters[0] = s.iters[1] = 0;
    s.phase = c.nstages > 0 ? PH_HEAD : PH_DONE;
    s.lam_cur = c.nstages > 0 ? c.lams[0] : 0.0;
    set_flags(s);
}

__device__ __forceinline__ void end_stage(IterState &s, const LoopCtl &c) {
    if (s.stage < 2) s.iters[s.stage] = s.it;
    s.stage += 1;
    s.it = 0;
    if (s.stage < c.nstages) {  // ficp.py:152-153: next lambda, next _iterate
        s.phase = PH_HEAD;
        s.lam_cur = c.lams[s.stage];
    } else {
        s.phase = PH_DONE;
    }
}

__global__ void k_loop_update(IterState *st, LoopCtl c) {
    if (threadIdx.x != 0) return;
    IterState &s = *st;
    if (s.done) return;
    const int call = s.n_nn++;
    s.k_last = s.k;
    if (call < c.max_trace) {
        if (c.tk) c.tk[call] = s.k;
        if (c.tf) c.tf[call] = s.frmsd;
        if (c.tl) c.tl[call] = s.lam_cur;
    }
    if (s.phase == PH_HEAD) {  // ficp.py:123-129
        if (s.k == 0) {
            end_stage(s, c);  // ficp.py:125-126: nothing selected, the stage returns
        } else {
            s.cur = s.frmsd;
            if (s.stage < 2) s.frmsd_last[s.stage] = s.cur;
            s.phase = PH_LOOP;
            s.it = 0;
            if (c.max_iter <= 0) end_stage(s, c);
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
        if (s.stage < 2) s.frmsd_last[s.stage] = nw;
        if (s.cur - nw <= c.threshold) {  // ficp.py:142 (the transform is already applied)
            end_stage(s, c);
        } else {
            s.cur = nw;
            s.it += 1;
            if (s.it >= c.max_iter) end_stage(s, c);
        }
    }
    set_flags(s);
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
