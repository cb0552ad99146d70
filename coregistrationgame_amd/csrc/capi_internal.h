// capi_internal.h -- state shared by the C ABI translation units (capi.hip, capi_batch.hip).
#pragma once

#include "../../include/ficp.h"
#include "ficp_internal.h"

#include <emmintrin.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ficp_capi {

using namespace ficp;


extern thread_local std::string g_err;  // defined in capi.hip

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(FICP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
    } while (0)

#define CHK(expr)                     \
    do {                              \
        int r_ = (expr);              \
        if (r_ != FICP_OK) return r_; \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned gen = 0;  // bumped on every (re)allocation
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return FICP_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(FICP_ENOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        ++gen;
        return FICP_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T *as() const {
        return (T *)p;
    }
};

// Pinned host staging (capacity-cached like DevBuf).  A D2H copy into pageable memory ran
// at ~8 GB/s on the box (24 MB in 3 ms, tools/host_probe.py); into pinned memory at the
// link rate, so results come back through this buffer.  (H2D from pageable memory already
// ran at the pinned rate, 24 MB in 0.44 ms, and is left direct.)
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: kernels store into it
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return FICP_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(FICP_ENOMEM, "hipHostMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        return FICP_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T *as() const {
        return (T *)p;
    }
};

enum ProfClass { P_NN = 1, P_SORT = 2, P_FRAC = 4, P_FIT = 8, P_GRID = 16, P_MISC = 32 };

struct ProfRec {
    const char *name;
    hipEvent_t a, b;
};

}  // namespace ficp_capi

using namespace ficp_capi;

struct BatchBufs;  // capi_batch.hip
constexpr int kLoopRing = 16;  // in-flight iterations of the device ICP loop (>= lookahead + 1)
void batch_release(BatchBufs *b);

// coherent pinned block the report kernel writes (capi.hip report_wait)
struct HostReport {
    IterState st;
    unsigned misc[4];  // sort flag, selection {error bits, levels, radix fallbacks}
    double bb[4];      // CHM bbox
    unsigned long long t[2];  // device clock (100 MHz) at run start / at the final report
    int flag;          // -1 while pending, 1 when the segments have landed
    int bflag;         // the same for set_target_device's early bbox report (bb)
};

struct ficp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int nn_mode = 0;
    int fault = 0;  // test-only fault injection mask (ficp_set_fault)
    int64_t runs_small = 0;  // runs taken by the one-workgroup path (k_small.hip)

    // target (CHM layer)
    bool has_target = false;
    int64_t m = 0;
    int md = 2;
    DevBuf tx, ty, tz;
    bool grid_ready = false, bbox_ready = false;
    double bb[4] = {0, 0, 0, 0};
    DevBuf cell_of, counts, cell_start, fill, pts, scan_tmp, mm_part, mm_out;
    GridView gv{};
    int64_t ncells = 0;
    double pivot_x = 0.0, pivot_y = 0.0;

    // per-call buffers (work order)
    DevBuf sx, sy, sz, idx, dist, r, key, val, order, sort_tmp, frac_tmp, fit_tmp, bd2, bidx;
    DevBuf ccx, ccy, rs, range;      // matched XY, r in selection order, key range
    DevBuf wx, wy, wz, worig, tidx;  // spatial work order of the source
    DevBuf stage, stage2, cx, cy, cz, state_dev;
    DevBuf bp;  // grid slot of each query's last match (warm start of the next NN call)
    DevBuf dz2; // dz^2 of each query's last match (warm start from (ccx, ccy, dz2))
    bool bbox_dev = false;  // the bbox is in mm_out already (set_target_device), not read yet
    bool bbox_pending = false;  // set_target_device's bbox report is queued (h_rep->bflag)
    DevBuf gap; // certified-reuse bound of each query's match (k_grid_nn.hip nn_query_cert)
    DevBuf lams, tr_k, tr_f, tr_l, tr_T, tr_idx;  // device loop: lambdas and traces
    DevBuf sel_tmp, sel_stats;  // bucketed fraction selection (k_select.hip)
    DevBuf bs_tmp, bs_tmp2;     // two-level bucket sort scratch (k_bsort.hip): grid, work order
    unsigned sel_init_gen = 0;  // sel_tmp allocation whose atomic words are initialised
    unsigned fit_init_gen = 0;  // fit_tmp allocation whose arrival counter is zeroed
    unsigned sel_levels = 0, sel_radix = 0;  // selection statistics (cumulative)
    int64_t win_calls = 0, win_retries = 0;  // window-path fraction calls / fallbacks
    int *h_flags = nullptr;                        // pinned ring of per-iteration done flags
    unsigned *h_misc = nullptr;                    // pinned: sort flag, selection stats
    HostReport *h_rep = nullptr;                   // coherent pinned (report kernel)
    hipEvent_t loop_ev[kLoopRing] = {};
    IterState *h_state = nullptr;  // pinned

    // profiling
    int prof_mask = 0;
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> ev_pool;
    std::map<std::string, std::pair<int64_t, double>> prof_acc;

    hipEvent_t ev0 = nullptr, ev1 = nullptr;

    BatchBufs *batch = nullptr;  // capi_batch.hip

    // distributed run of one plot over several ranks (capi.hip, ficp_dist_*)
    hipStream_t own_stream = nullptr;  // the context's stream while a caller's stream is set
    int dist_mode = 0;                 // 0 none, 1 target-partitioned, 2 source-partitioned
    int64_t dist_n = 0, dist_ntot = 0, dist_nmax = 0, dist_nws = 0;
    int64_t dist_calls = 0;            // NN steps enqueued in this run (the first is cold)
    double dist_px = 0.0, dist_py = 0.0;
    int dist_refl = 0;
    double *dist_x = nullptr, *dist_y = nullptr;  // the caller's rows (device)
    const double *dist_z = nullptr;
    LoopCtl dist_lc{};
    DevBuf gorig;                      // caller index (row0 + local) of each work-order row
    DevBuf drange;                     // int64 range words of the local rows (top bit flipped)

    PinBuf pin;  // pinned staging of results on their way to the caller's (pageable) arrays
    PinBuf pin_xy{nullptr, 0, hipHostMallocCoherent};  // k_small_run's XY, stored by the kernel
    PinBuf pin_up;             // bounce buffer of small target uploads (ficp_set_target)
    hipEvent_t up_ev = nullptr;  // the last upload from pin_up
    // per-call k trace of the batch runs (ficp_set_batch_trace): host rows of max_trace
    int64_t *btrace_host = nullptr;
    int32_t btrace_max = 0;
    DevBuf btrace;
};
constexpr size_t kBounceBytes = 1 << 20;  // ficp_set_target layers up to 1 MB bounce (no sync)

namespace ficp_capi {

inline hipEvent_t ev_get(ficp_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Events carried by one kernel's own dispatch (hipExtLaunchKernelGGL): they time exactly
// that kernel and add no marker packets (a hipEventRecord pair around a launch costs
// ~5.7 us of idle queue time per event at C3, measured in profiles/r1sel trace).
struct KernelEvents {
    ficp_ctx *c;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    KernelEvents(ficp_ctx *c_, int cls, const char *n) : c(c_), name(n) {
        if (c->prof_mask & cls) {
            a = ev_get(c);
            b = ev_get(c);
        }
    }
    ~KernelEvents() {
        if (a) c->recs.push_back({name, a, b});
    }
};

struct ProfScope {
    ficp_ctx *c;
    const char *name;
    hipStream_t s;
    hipEvent_t a = nullptr;
    // (stream: the launches' stream when not the context's, e.g. a batch sub-stream)
    ProfScope(ficp_ctx *c_, int cls, const char *n, hipStream_t stream = nullptr)
        : c(c_), name(n), s(stream ? stream : c_->stream) {
        if (c->prof_mask & cls) {
            a = ev_get(c);
            (void)hipEventRecord(a, s);
        }
    }
    ~ProfScope() {
        if (a) {
            hipEvent_t b = ev_get(c);
            (void)hipEventRecord(b, s);
            c->recs.push_back({name, a, b});
        }
    }
};

inline int set_device(ficp_ctx *c) {
    HIPCHK(hipSetDevice(c->device));
    return FICP_OK;
}

inline int sync(ficp_ctx *c) {
    HIPCHK(hipStreamSynchronize(c->stream));
    return FICP_OK;
}

// host (n x ld) rows -> device SoA columns (first ncols)
// Uniform grid over the bbox [x0,x1] x [y0,y1] of m stems: about one stem per cell (the
// disk-clipped row scan measured best at 1 vs 0.25/0.5/2 at C3), at most 4m + 64 cells;
// margin = the search bounds' rounding allowance.
inline void plan_grid(double x0, double x1, double y0, double y1, int64_t m, double &h,
                      int64_t &gx, int64_t &gy, double &margin) {
    const char *pc = getenv("FICP_GRID_PER_CELL");   // read per plan (tests switch it)
    const double kPerCell = pc && atof(pc) > 0.0 ? atof(pc) : 1.0;
    const double sxr = x1 - x0, syr = y1 - y0;
    if (m <= 1 || (sxr <= 0.0 && syr <= 0.0)) h = 1.0;
    else if (sxr > 0.0 && syr > 0.0) h = sqrt(sxr * syr * kPerCell / (double)m);
    else h = std::max(sxr, syr) * kPerCell / (double)m;
    if (!(h > 0.0)) h = 1.0;
    for (;;) {
        gx = (int64_t)floor(sxr / h) + 1;
        gy = (int64_t)floor(syr / h) + 1;
        if (gx * gy <= 4 * m + 64 && gx < (1 << 24) && gy < (1 << 24)) break;
        h *= 1.5;
    }
    margin = 64.0 * 2.220446049250313e-16 * (fabs(x0) + fabs(y0) + sxr + syr + h);
}

inline int upload_rows(ficp_ctx *c, const double *rows, int64_t n, int64_t ld, int ncols, DevBuf &c0,
                DevBuf &c1, DevBuf *c2) {
    CHK(c0.ensure(n * 8));
    CHK(c1.ensure(n * 8));
    if (c2) CHK(c2->ensure(n * 8));
    if (n == 0) return FICP_OK;
    CHK(c->stage.ensure(n * ld * 8));
    HIPCHK(hipMemcpyAsync(c->stage.p, rows, n * ld * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_deinterleave(c->stage.as<double>(), n, ld, ncols, c0.as<double>(),
                               c1.as<double>(), c2 ? c2->as<double>() : nullptr, c->stream));
    return FICP_OK;
}
// f(i0, i1) over [0, n) on the caller and a persistent pool of host threads (large host
// copies: the constructor's layer copies, staged results).  Spawning threads per call cost
// ~20-40 us each; the pool's workers sleep on a condition variable between calls.
// FICP_HOST_THREADS (default 16, the GPU box's per-job CPU share) caps the threads; a call
// made while another one owns the pool runs on its caller alone.
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();  // never destroyed: workers outlive exit paths
        return *p;
    }
    int threads() const { return nthreads_; }
    // false: the pool is busy (run serially)
    bool run(int parts, const std::function<void(int)> &job) {
        std::unique_lock<std::mutex> own(busy_, std::try_to_lock);
        if (!own.owns_lock()) return false;
        unsigned long long gen;
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &job;
            parts_ = parts;
            left_ = parts;
            gen = ++gen_;
            claim_.store((gen & 0xffffffffULL) << 32);  // (generation, next part): a late worker claims nothing
        }
        cv_.notify_all();
        work(&job, gen, parts);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return left_ == 0; });
        job_ = nullptr;
        return true;
    }

  private:
    HostPool() {
        const char *e = getenv("FICP_HOST_THREADS");
        nthreads_ = std::max(1, std::min(64, e ? atoi(e) : 16));
        for (int t = 1; t < nthreads_; ++t) std::thread([this] { loop(); }).detach();
    }
    // claims parts of generation gen until none is left (or a newer generation began)
    void work(const std::function<void(int)> *j, unsigned long long gen, int parts) {
        for (;;) {
            unsigned long long c = claim_.load();
            int i;
            do {
                if ((c >> 32) != (gen & 0xffffffffULL) || (int)(c & 0xffffffffULL) >= parts) return;
                i = (int)(c & 0xffffffffULL);
            } while (!claim_.compare_exchange_weak(c, c + 1));
            (*j)(i);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_all();
        }
    }
    void loop() {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)> *j;
            unsigned long long gen;
            int parts;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen && job_ != nullptr; });
                seen = gen = gen_;
                j = job_;
                parts = parts_;
            }
            work(j, gen, parts);
        }
    }
    int nthreads_ = 1;
    std::mutex busy_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int parts_ = 0, left_ = 0;
    std::atomic<unsigned long long> claim_{0};
    unsigned long long gen_ = 0;
};

// memcpy with non-temporal 16-B stores (SSE2, baseline x86-64) into a 16-B aligned
// destination: no read-for-ownership of the destination lines, which a large copy into a
// fresh pinned block would otherwise pay (3 memory transfers per byte instead of 2)
inline void stream_copy(char *d, const char *s, size_t bytes) {
    size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > bytes) head = bytes;
    memcpy(d, s, head);
    d += head;
    s += head;
    bytes -= head;
    const size_t nv = bytes / 64;
    for (size_t i = 0; i < nv; ++i) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(s + 64 * i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(s + 64 * i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i *)(s + 64 * i + 32));
        const __m128i e = _mm_loadu_si128((const __m128i *)(s + 64 * i + 48));
        _mm_stream_si128((__m128i *)(d + 64 * i), a);
        _mm_stream_si128((__m128i *)(d + 64 * i + 16), b);
        _mm_stream_si128((__m128i *)(d + 64 * i + 32), c);
        _mm_stream_si128((__m128i *)(d + 64 * i + 48), e);
    }
    _mm_sfence();
    memcpy(d + 64 * nv, s + 64 * nv, bytes - 64 * nv);
}

template <typename F>
inline void host_parallel(int64_t n, F f) {
    const int64_t per_min = 1 << 17;
    HostPool &hp = HostPool::get();
    const int nt = (int)std::min<int64_t>(hp.threads(), std::max<int64_t>(1, n / per_min));
    if (nt <= 1) {
        f((int64_t)0, n);
        return;
    }
    const int64_t per = (n + nt - 1) / nt;
    const std::function<void(int)> job = [&](int t) {
        const int64_t a = std::min(n, t * per), b = std::min(n, a + per);
        if (b > a) f(a, b);
    };
    if (!hp.run(nt, job)) f((int64_t)0, n);
}

// page-locked host memory the DMA engines reach directly (hipHostMalloc'd blocks, e.g.
// the Python host pool's); pageable memory is reported as not pinned
inline bool host_pinned(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// device bytes -> the caller's host memory through the pinned staging buffer
inline int d2h_staged(ficp_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!bytes) return FICP_OK;
    CHK(c->pin.ensure(bytes));
    HIPCHK(hipMemcpyAsync(c->pin.p, src, bytes, hipMemcpyDeviceToHost, c->stream));
    CHK(sync(c));
    const char *s = c->pin.as<const char>();
    char *d = (char *)dst;
    host_parallel((int64_t)bytes, [&](int64_t a, int64_t b) { memcpy(d + a, s + a, (size_t)(b - a)); });
    return FICP_OK;
}

// interleaved device XY (n x 2) -> columns 0 and 1 of the caller's (n x ld) rows; every
// other column is left untouched (ficp.py:114-118)
inline int d2h_xy_columns(ficp_ctx *c, const double *xy_dev, int64_t n, double *dst, int64_t ld) {
    if (n <= 0) return FICP_OK;
    CHK(c->pin.ensure((size_t)n * 16));
    HIPCHK(hipMemcpyAsync(c->pin.p, xy_dev, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    CHK(sync(c));
    const double *xy = c->pin.as<const double>();
    host_parallel(n, [&](int64_t a, int64_t b) {
        if (ld == 2) {
            memcpy(dst + 2 * a, xy + 2 * a, (size_t)(b - a) * 16);
            return;
        }
        for (int64_t i = a; i < b; ++i) {
            dst[i * ld] = xy[2 * i];
            dst[i * ld + 1] = xy[2 * i + 1];
        }
    });
    return FICP_OK;
}

// Wait for a flag that a kernel stores (system scope) into coherent pinned memory; -1 =
// not yet written.  Ends with an error when the stream fails or drains without it.
int poll_flag(ficp_ctx *c, int *flag, int &v);

}  // namespace ficp_capi
