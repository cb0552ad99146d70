// capi.hip -- the C ABI of include/ficp.h: context, buffers, the ICP driver loop.
//
// The loop is the reference's _iterate (ficp.py:122-147) with every array operation on
// the device; per iteration the host reads back one small IterState (k, FRMSD, T) to
// take the convergence decision `current - new <= threshold` (ficp.py:142).
#include "../../include/ficp.h"
#include "capi_internal.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <chrono>

#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <vector>

using namespace ficp;

using namespace ficp_capi;

namespace ficp_capi {
thread_local std::string g_err;

// Wait for a done flag that a kernel stores into coherent pinned memory (-1 = not yet
// written).  After 20 ms of waiting the stream is queried now and then, so that a device
// error or a drained stream without the store ends the wait instead of spinning forever.
// Not earlier: each hipStreamQuery left a ~6 us idle gap in the queue (one per loop
// iteration at C3, between the NN launch and the next selection; rocprofv3 runtime +
// kernel trace).
int poll_flag(ficp_ctx *c, int *flag, int &v) {
    std::chrono::steady_clock::time_point t0{};
    for (uint64_t spin = 1;; ++spin) {
        v = __atomic_load_n(flag, __ATOMIC_ACQUIRE);
        if (v != -1) return FICP_OK;
        if ((spin & 1023) == 0) {
            const auto now = std::chrono::steady_clock::now();
            if (spin == 1024) t0 = now;
            if (now - t0 < std::chrono::milliseconds(20)) {
                __builtin_ia32_pause();
                continue;
            }
            const hipError_t e = hipStreamQuery(c->stream);
            if (e == hipSuccess) {
                v = __atomic_load_n(flag, __ATOMIC_ACQUIRE);
                if (v != -1) return FICP_OK;
                return fail(FICP_EHIP, "device loop flag was not written");
            }
            if (e != hipErrorNotReady) return fail(FICP_EHIP, "device loop: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
}
}  // namespace ficp_capi

namespace {

// the selection's sticky error bits (k_select.hip ERR_*) by name
std::string sel_err_text(unsigned e) {
    std::string s = "fraction selection raised error flag " + std::to_string(e) + " (results invalid):";
    if (e & 1u) s += " ERR_EMPTY (no candidate row)";
    if (e & 2u) s += " ERR_CAP (a rank's candidates exceeded the pack capacity)";
    if (e & 4u) s += " ERR_SPIN (the bounds hand-off of k_sel_bounds_gather never arrived)";
    return s;
}

// bounding box of the CHM layer (grid geometry and the fit's pivot), once per target
// Run the report kernel (device segments -> coherent pinned host memory) and poll its
// flag: one short host wait instead of hipMemcpyAsync + hipStreamSynchronize.
int report_wait(ficp_ctx *c, const ReportSeg &a, const ReportSeg &b, const ReportSeg &d,
                unsigned long long *t_end = nullptr) {
    __atomic_store_n(&c->h_rep->flag, -1, __ATOMIC_RELAXED);
    HIPCHK(launch_report(a, b, d, &c->h_rep->flag, t_end, c->stream));
    int v = 0;
    return poll_flag(c, &c->h_rep->flag, v);
}

// set_target_device queues the bbox's report right behind the bbox kernel, so it lands
// while the caller queues its other work (C3's bench: the source's reset copy and
// k_run_start) instead of after it; ensure_bbox then finds it landed or nearly.  A second
// set_target* collects a pending one first, so a report never lands over a later one's.
int bbox_collect(ficp_ctx *c) {
    if (!c->bbox_pending) return FICP_OK;
    int v = 0;
    CHK(poll_flag(c, &c->h_rep->bflag, v));
    c->bbox_pending = false;
    return FICP_OK;
}

int ensure_bbox(ficp_ctx *c) {
    if (c->bbox_ready) return FICP_OK;
    if (c->bbox_pending) {
        CHK(bbox_collect(c));
    } else {
        CHK(c->mm_part.ensure(1024 * 4 * 8));
        CHK(c->mm_out.ensure(4 * 8));
        if (!c->bbox_dev)
            HIPCHK(launch_minmax2(c->tx.as<double>(), c->ty.as<double>(), c->m,
                                  c->mm_part.as<double>(), c->mm_out.as<double>(), c->stream));
        CHK(report_wait(c, ReportSeg{c->mm_out.p, c->h_rep->bb, 8}, ReportSeg{}, ReportSeg{}));
    }
    c->bbox_dev = false;
    memcpy(c->bb, c->h_rep->bb, sizeof c->bb);
    const double *bb = c->bb;
    if (!(std::isfinite(bb[0]) && std::isfinite(bb[1]) && std::isfinite(bb[2]) &&
          std::isfinite(bb[3])))
        return fail(FICP_EINVAL, "target coordinates must be finite");
    c->pivot_x = bb[0] + 0.5 * (bb[1] - bb[0]);
    c->pivot_y = bb[2] + 0.5 * (bb[3] - bb[2]);
    c->bbox_ready = true;
    return FICP_OK;
}

// job: with the bucket-sort path, the build is returned as a job (launched by the caller
// together with the work order) instead of being launched here
int ensure_grid(ficp_ctx *c, BSJob *job = nullptr) {
    if (c->grid_ready) return FICP_OK;
    const int64_t m = c->m;
    ProfScope ps(c, P_GRID, "grid_build");
    CHK(ensure_bbox(c));
    const double x0 = c->bb[0], x1 = c->bb[1], y0 = c->bb[2], y1 = c->bb[3];
    double h, margin;
    int64_t gx, gy;
    plan_grid(x0, x1, y0, y1, m, h, gx, gy, margin);
    c->ncells = gx * gy;
    GridView g{};
    g.x0 = x0;
    g.y0 = y0;
    g.h = h;
    g.inv_h = 1.0 / h;
    g.gx = (int)gx;
    g.gy = (int)gy;
    g.margin = margin;
    CHK(c->cell_start.ensure((c->ncells + 1) * 4));
    CHK(c->pts.ensure(m * sizeof(TPt)));
    if (bsort_supported(m, c->ncells) && !getenv("FICP_GRID_ATOMIC")) {
        // two-level bucket sort of the stems by cell (k_bsort.hip)
        CHK(c->bs_tmp.ensure(bsort_tmp_bytes(m, c->ncells)));
        const BSortGeom bg{x0, y0, g.inv_h, g.gx, g.gy, 0};
        BSortOut bo{};
        bo.pts = c->pts.as<TPt>();
        bo.cell_start = c->cell_start.as<int32_t>();
        if (job && m > 0)
            *job = bsort_job(c->tx.as<double>(), c->ty.as<double>(),
                             c->md == 3 ? c->tz.as<double>() : nullptr, m, bg, c->ncells, bo,
                             c->bs_tmp.p);
        else
            HIPCHK(launch_bsort(c->tx.as<double>(), c->ty.as<double>(),
                                c->md == 3 ? c->tz.as<double>() : nullptr, m, bg, c->ncells, bo,
                                c->bs_tmp.p, c->stream));
        g.pts = c->pts.as<TPt>();
        g.cell_start = c->cell_start.as<int32_t>();
        g.m = m;
        c->gv = g;
        c->grid_ready = true;
        return FICP_OK;
    }
    // counting sort of the stems by cell with global atomics (grids bsort cannot plan)
    CHK(c->cell_of.ensure(m * 4));
    CHK(c->counts.ensure((c->ncells + 1) * 4));
    CHK(c->fill.ensure((c->ncells + 1) * 4));
    CHK(c->cell_start.ensure((c->ncells + 1) * 4));
    CHK(c->pts.ensure(m * sizeof(TPt)));
    CHK(c->scan_tmp.ensure(scan_tmp_elems(c->ncells) * 4 + 64));
    // counts/fill are updated with atomics: reset them with atomics
    HIPCHK(launch_atomic_zero32((uint32_t *)c->counts.p, c->ncells + 1, c->stream));
    HIPCHK(launch_atomic_zero32((uint32_t *)c->fill.p, c->ncells + 1, c->stream));
    HIPCHK(launch_grid_count(c->tx.as<double>(), c->ty.as<double>(), m, g.x0, g.y0, g.inv_h, g.gx,
                             g.gy, c->cell_of.as<int32_t>(), c->counts.as<int32_t>(), c->stream));
    HIPCHK(launch_scan_i32(c->counts.as<int32_t>(), c->cell_start.as<int32_t>(), c->ncells,
                           c->scan_tmp.as<int32_t>(), true, c->stream));
    HIPCHK(launch_grid_scatter(c->tx.as<double>(), c->ty.as<double>(),
                               c->md == 3 ? c->tz.as<double>() : nullptr, m,
                               c->cell_of.as<int32_t>(), c->cell_start.as<int32_t>(),
                               c->fill.as<int32_t>(), c->pts.as<TPt>(), c->stream));
    HIPCHK(launch_grid_sort_cells(c->pts.as<TPt>(), c->cell_start.as<int32_t>(), c->ncells,
                                  c->stream));
    g.pts = c->pts.as<TPt>();
    g.cell_start = c->cell_start.as<int32_t>();
    g.m = m;
    c->gv = g;
    c->grid_ready = true;
    return FICP_OK;
}

bool use_grid(ficp_ctx *c, int64_t n) {
    if (c->nn_mode == 1 || c->m > kMaxGridStems) return false;  // grid limit: brute force
    if (c->nn_mode == 2) return true;
    return (double)n * (double)c->m > 4.0e6;
}

// fit scratch of n rows; a fresh allocation gets its arrival counter zeroed
int ensure_fit(ficp_ctx *c, int64_t n) {
    CHK(c->fit_tmp.ensure(fit_tmp_bytes(n)));
    if (c->fit_tmp.gen != c->fit_init_gen) {
        HIPCHK(launch_fit_init(c->fit_tmp.p, c->stream));
        c->fit_init_gen = c->fit_tmp.gen;
    }
    return FICP_OK;
}

int ensure_work(ficp_ctx *c, int64_t n) {
    CHK(c->idx.ensure(n * 4));
    CHK(c->dist.ensure(n * 8));
    CHK(c->r.ensure((n + 1) * 8));  // (+1: k_sel_win's 16-B row-pair loads)
    CHK(c->key.ensure(n * 8));
    CHK(c->val.ensure(n * 4));
    CHK(c->order.ensure(n * 4));
    CHK(c->sort_tmp.ensure(sort_tmp_bytes(n)));
    CHK(c->frac_tmp.ensure(frac_tmp_bytes(n)));
    CHK(ensure_fit(c, n));
    CHK(c->state_dev.ensure(sizeof(IterState)));
    CHK(c->ccx.ensure((n + 1) * 8));
    CHK(c->ccy.ensure((n + 1) * 8));
    CHK(c->rs.ensure(n * 8));
    CHK(c->range.ensure(range_words(n) * 8));
    CHK(c->sel_tmp.ensure(sel_tmp_bytes(n)));
    CHK(c->sel_stats.ensure(16));
    if (c->sel_tmp.gen != c->sel_init_gen) {  // fresh allocation: zero its atomic words
        HIPCHK(launch_select_init(c->sel_tmp.p, n, c->stream));
        c->sel_init_gen = c->sel_tmp.gen;
    }
    return FICP_OK;
}

unsigned long long *range_ptr(ficp_ctx *c) { return c->range.as<unsigned long long>(); }

// NN of the device source (sx, sy, sz) against the target; optional pending transform.
// With want_keys the sort inputs (key, range, r, matched XY) are produced too (and dist
// is not).  warm: 0 = cold search, 1 = record the matched grid slots, 2 = also start
// every query from its previous match (grid mode, same work order within one run).
int nn_call(ficp_ctx *c, double *sx, double *sy, const double *sz, int64_t n, const double *T,
            bool want_keys, int warm = 0, const int *skip = nullptr,
            const int *apply_flag = nullptr, bool reduce_range = true, bool want_idx = true,
            const int *reuse = nullptr, bool store_key = true, bool multi = false,
            const uint32_t *fin_orig = nullptr, double *fin_x = nullptr, double *fin_y = nullptr,
            bool gap_cold = false) {
    NNArgs a{};
    a.fin_orig = fin_orig;
    a.fin_x = fin_x;
    a.fin_y = fin_y;
    a.sx = sx;
    a.sy = sy;
    a.sz = sz;
    a.n = n;
    a.T = T;
    a.skip = skip;
    a.apply_flag = apply_flag;
    a.reuse = reuse;
    a.multi = multi ? 1 : 0;
    a.idx = want_idx ? c->idx.as<int32_t>() : nullptr;  // the run loop reads idx only for traces
    a.dist = want_keys ? nullptr : c->dist.as<double>();
    a.r = c->r.as<double>();
    a.key = (want_keys && store_key) ? c->key.as<unsigned long long>() : nullptr;
    a.val = nullptr;
    a.cx = want_keys ? c->ccx.as<double>() : nullptr;
    a.cy = want_keys ? c->ccy.as<double>() : nullptr;
    a.tx = c->tx.as<double>();
    a.ty = c->ty.as<double>();
    a.range = want_keys ? range_ptr(c) : nullptr;
    if (use_grid(c, n)) {
        CHK(ensure_grid(c));
        if (warm && a.cx) {
            // warm start from the previous call's match: (cx, cy) and dz^2 per query
            CHK(c->dz2.ensure(n * 8));
            a.dz2 = c->dz2.as<double>();
            a.warm_c = warm == 2 ? 1 : 0;
            // certified reuse of the match (nn_query_cert): the bound G and the match slot;
            // a workgroup's uncertified queries packed, up to 8 lanes per query
            CHK(c->gap.ensure(n * sizeof(gap_t)));
            CHK(c->bp.ensure(n * 4));
            a.gap = c->gap.as<gap_t>();
            a.out_bp = c->bp.as<int32_t>();
            a.cert_block = 8;
            a.gap_cold = gap_cold ? 1 : 0;
        }
        {
            KernelEvents ke(c, P_NN, "nn_grid");  // the NN kernel alone (bench roofline)
            HIPCHK(launch_nn_grid(a, c->gv, c->md, c->stream, false, ke.a, ke.b));
        }
        if (a.range && reduce_range)
            HIPCHK(launch_range_reduce(a.range, nn_range_parts(n, c->m, true), c->stream));
    } else {
        const int64_t nch = brute_chunk_count(n, c->m);
        if (nch > 1) {
            CHK(c->bd2.ensure(nch * n * 8));
            CHK(c->bidx.ensure(nch * n * 4));
        }
        {
            ProfScope ps(c, P_NN, "nn_brute");
            HIPCHK(launch_nn_brute(a, c->tx.as<double>(), c->ty.as<double>(),
                                   c->md == 3 ? c->tz.as<double>() : nullptr, c->m, c->md,
                                   c->bd2.as<double>(), c->bidx.as<int32_t>(), c->stream, false));
        }
        if (a.range && reduce_range)
            HIPCHK(launch_range_reduce(a.range, nn_range_parts(n, c->m, false), c->stream));
    }
    return FICP_OK;
}

// sort (key, orig) of the last NN call, then the FRMSD fraction scan
int sort_and_select(ficp_ctx *c, int64_t n, int64_t N, double lam, const uint32_t *orig,
                    const int *skip = nullptr, const double *lam_dev = nullptr) {
    {
        ProfScope ps(c, P_SORT, "sort");
        HIPCHK(launch_sort(c->key.as<unsigned long long>(), orig, n, range_ptr(c),
                           c->order.as<uint32_t>(), c->r.as<double>(), c->rs.as<double>(),
                           c->sort_tmp.p, skip, c->stream));
    }
    {
        ProfScope ps(c, P_FRAC, "fraction");
        HIPCHK(launch_fraction(c->rs.as<double>(), n, N, lam, lam_dev, c->frac_tmp.p,
                               c->state_dev.as<IterState>(), skip, c->stream));
    }
    return FICP_OK;
}

int read_state(ficp_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->h_state, c->state_dev.p, sizeof(IterState), hipMemcpyDeviceToHost,
                          c->stream));
    return sync(c);
}

// Spatial work order: the source permuted into 8x8-cell supertile order of the CHM grid
// (ties by index), so each wave's queries scan neighbouring cells.
// job: as in ensure_grid (the bucket-sort path returns its job instead of launching)
int build_work_order(ficp_ctx *c, const double *sx, const double *sy, const double *sz,
                     int64_t n, BSJob *job = nullptr) {
    CHK(c->wx.ensure((n + 1) * 8));  // (+1: k_sel_win's 16-B row-pair loads)
    CHK(c->wy.ensure((n + 1) * 8));
    if (sz) CHK(c->wz.ensure(n * 8));
    CHK(c->worig.ensure((n + 1) * 4));
    ProfScope ps(c, P_MISC, "work_order");
    const GridView &g = c->gv;
    const int64_t nkeys = (int64_t)((g.gx + 7) / 8) * (int64_t)((g.gy + 7) / 8) * 64;
    if (bsort_supported(n, nkeys) && !getenv("FICP_WORK_RADIX")) {
        // run_core launches it with the grid build as one two-job bucket sort (it ran on a
        // side stream beside the build before: fork/join events and four more launches)
        CHK(c->bs_tmp2.ensure(bsort_tmp_bytes(n, nkeys)));
        const BSortGeom bg{g.x0, g.y0, g.inv_h, g.gx, g.gy, 1};
        BSortOut bo{};
        bo.wx = c->wx.as<double>();
        bo.wy = c->wy.as<double>();
        bo.wz = sz ? c->wz.as<double>() : nullptr;
        bo.worig = c->worig.as<uint32_t>();
        if (job) {
            *job = bsort_job(sx, sy, sz, n, bg, nkeys, bo, c->bs_tmp2.p);
            return FICP_OK;
        }
        HIPCHK(launch_bsort(sx, sy, sz, n, bg, nkeys, bo, c->bs_tmp2.p, c->stream));
        return FICP_OK;
    }
    HIPCHK(launch_src_cellkey(sx, sy, n, c->gv, c->key.as<unsigned long long>(), c->stream));
    HIPCHK(launch_key_range(c->key.as<unsigned long long>(), n, range_ptr(c), c->stream));
    HIPCHK(launch_sort(c->key.as<unsigned long long>(), nullptr, n, range_ptr(c),
                       c->order.as<uint32_t>(), nullptr, nullptr, c->sort_tmp.p, nullptr,
                       c->stream));
    HIPCHK(launch_gather_work(c->order.as<uint32_t>(), sx, sy, sz, n, c->wx.as<double>(),
                              c->wy.as<double>(), sz ? c->wz.as<double>() : nullptr,
                              c->worig.as<uint32_t>(), c->stream));
    return FICP_OK;
}

// A small plot's whole run in one workgroup (k_small.hip): the Join button's size
// (app.py:630-661).  One launch, then the state and traces come back as in run_core.
// rows (device, n x ld, nullable): the trees as uploaded (else the SoA sx, sy, sz); with
// host_xy the kernel reports straight into coherent pinned memory (the XY, the state, the
// clock stamps and a flag the host polls): one launch and one poll per run()
int run_small(ficp_ctx *c, const double *rows, int64_t ld, double *sx, double *sy,
              const double *sz, int64_t n, int32_t nstages, const double *lambdas,
              double threshold, int32_t max_iter, int32_t allow_refl, ficp_stats *st,
              double **host_xy) {
    CHK(c->state_dev.ensure(sizeof(IterState)));
    LoopCtl lc{};
    lc.nstages = nstages;
    lc.max_iter = max_iter;
    lc.threshold = threshold;
    for (int e = 0; e < kLamIn; ++e) lc.lam_in[e] = e < nstages ? lambdas[e] : 0.0;
    if (nstages > kLamIn) {
        CHK(c->lams.ensure((size_t)nstages * 8));
        HIPCHK(hipMemcpyAsync(c->lams.p, lambdas, (size_t)nstages * 8, hipMemcpyHostToDevice,
                              c->stream));
        lc.lams = c->lams.as<double>();
    }
    const int mt = (st && st->max_trace > 0) ? st->max_trace : 0;
    int32_t *tidx = nullptr;
    if (mt > 0) {
        lc.max_trace = mt;
        CHK(c->tr_k.ensure((size_t)mt * 8));
        CHK(c->tr_f.ensure((size_t)mt * 8));
        CHK(c->tr_l.ensure((size_t)mt * 8));
        CHK(c->tr_T.ensure((size_t)mt * 72));
        lc.tk = c->tr_k.as<long long>();
        lc.tf = c->tr_f.as<double>();
        lc.tl = c->tr_l.as<double>();
        lc.tT = c->tr_T.as<double>();
        if (st->trace_idx) {
            lc.max_trace_idx = st->max_trace_idx > 0 ? std::min(st->max_trace_idx, mt) : mt;
            CHK(c->tr_idx.ensure((size_t)lc.max_trace_idx * (size_t)n * 4));
            tidx = c->tr_idx.as<int32_t>();
        }
    }
    SmallArgs a{};
    a.rows = rows;
    a.ld = ld;
    a.sx = sx;
    a.sy = sy;
    a.sz = c->md == 3 ? sz : nullptr;
    a.n = (int)n;
    a.tx = c->tx.as<double>();
    a.ty = c->ty.as<double>();
    a.tz = c->md == 3 ? c->tz.as<double>() : nullptr;
    a.m = (int)c->m;
    a.allow_refl = allow_refl;
    a.st = c->state_dev.as<IterState>();
    a.tidx = tidx;
    if (host_xy) {
        CHK(c->pin_xy.ensure((size_t)n * 16));
        a.host_xy = c->pin_xy.as<double>();
        a.host_st = &c->h_rep->st;
        a.host_t = c->h_rep->t;
        a.host_flag = &c->h_rep->flag;
        __atomic_store_n(&c->h_rep->flag, -1, __ATOMIC_RELAXED);
        HIPCHK(launch_small_run(a, c->md, lc, c->stream));
        int v = 0;
        CHK(poll_flag(c, &c->h_rep->flag, v));
        *host_xy = c->pin_xy.as<double>();
    } else {
        CHK(c->sel_stats.ensure(16));
        HIPCHK(launch_run_start(c->sel_stats.as<uint32_t>(), &c->h_rep->t[0], c->stream));
        HIPCHK(launch_small_run(a, c->md, lc, c->stream));
        CHK(report_wait(c, ReportSeg{c->state_dev.p, &c->h_rep->st, (int)(sizeof(IterState) / 4)},
                        ReportSeg{}, ReportSeg{}, &c->h_rep->t[1]));
    }
    const IterState &h = c->h_rep->st;
    if (!h.done) return fail(FICP_EHIP, "small-plot ICP kernel did not finish");
    c->runs_small += 1;
    if (!st) return FICP_OK;
    st->path = 1;
    st->n_nn_calls = h.n_nn;
    st->n_nn_reused = h.n_reuse;
    st->n_fits = h.n_fit;
    st->iters[0] = h.iters[0];
    st->iters[1] = h.iters[1];
    st->k_last = h.k_last;
    st->frmsd_last[0] = h.frmsd_last[0];
    st->frmsd_last[1] = h.frmsd_last[1];
    memcpy(st->T_total, h.Ttot, sizeof st->T_total);
    const int nc = std::min(h.n_nn, mt), nf = std::min(h.n_fit, mt);
    if (nc > 0 || nf > 0) {
        if (nc > 0 && st->trace_k)
            HIPCHK(hipMemcpyAsync(st->trace_k, c->tr_k.p, nc * 8, hipMemcpyDeviceToHost, c->stream));
        if (nc > 0 && st->trace_frmsd)
            HIPCHK(hipMemcpyAsync(st->trace_frmsd, c->tr_f.p, nc * 8, hipMemcpyDeviceToHost, c->stream));
        if (nc > 0 && st->trace_lambda)
            HIPCHK(hipMemcpyAsync(st->trace_lambda, c->tr_l.p, nc * 8, hipMemcpyDeviceToHost, c->stream));
        if (nc > 0 && tidx)
            HIPCHK(hipMemcpyAsync(st->trace_idx, tidx, (size_t)std::min(nc, lc.max_trace_idx) * (size_t)n * 4,
                                  hipMemcpyDeviceToHost, c->stream));
        if (nf > 0 && st->trace_T)
            HIPCHK(hipMemcpyAsync(st->trace_T, c->tr_T.p, (size_t)nf * 72, hipMemcpyDeviceToHost, c->stream));
        CHK(sync(c));
    }
    st->gpu_ms = (double)(c->h_rep->t[1] - c->h_rep->t[0]) * 1e-5;  // 100 MHz ticks
    return FICP_OK;
}

// the one-workgroup path takes the run (auto NN mode, FICP_SMALL != 0)
bool use_small(ficp_ctx *c, int64_t n) {
    if (c->nn_mode != 0 || !small_run_fits(n, c->m)) return false;
    const char *e = getenv("FICP_SMALL");
    return !(e && atoi(e) == 0);
}

// the device-resident ICP: stages of ficp.py:122-147
int run_core(ficp_ctx *c, double *sx, double *sy, const double *sz, int64_t n, int32_t nstages,
             const double *lambdas, double threshold, int32_t max_iter, int32_t allow_refl,
             ficp_stats *st) {
    if (st) {
        st->n_nn_calls = 0;
        st->n_nn_reused = 0;
        st->n_fits = 0;
        st->iters[0] = st->iters[1] = 0;
        st->k_last = 0;
        st->frmsd_last[0] = st->frmsd_last[1] = INFINITY;
        for (int e = 0; e < 9; ++e) st->T_total[e] = (e % 4 == 0) ? 1.0 : 0.0;
        st->gpu_ms = 0.0;
        for (double &h : st->host_ms) h = 0.0;
        st->path = 0;
    }
    if (n == 0 || c->m == 0) return FICP_OK;  // ficp.py:66-68 + 125-126: nothing moves
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large (max 2^30 - 1)");
    if (use_small(c, n))
        return run_small(c, nullptr, 0, sx, sy, sz, n, nstages, lambdas, threshold, max_iter,
                         allow_refl, st, nullptr);
    CHK(ensure_work(c, n));
    uint32_t *tflag = sort_timeout_flag(c->sort_tmp.p, n);
    IterState *dst = c->state_dev.as<IterState>();
    // loop parameters and traces live on the device (k_loop.hip)
    LoopCtl lc{};
    lc.nstages = nstages;
    lc.max_iter = max_iter;
    lc.threshold = threshold;
    // the first kLamIn lambdas travel in the kernel arguments (a pageable H2D copy left
    // ~15 us of idle device before the loop); more stages read the device array
    for (int e = 0; e < kLamIn; ++e) lc.lam_in[e] = e < nstages ? lambdas[e] : 0.0;
    if (nstages > kLamIn) {
        CHK(c->lams.ensure((size_t)nstages * 8));
        HIPCHK(hipMemcpyAsync(c->lams.p, lambdas, (size_t)nstages * 8, hipMemcpyHostToDevice,
                              c->stream));
        lc.lams = c->lams.as<double>();
    }
    const int mt = (st && st->max_trace > 0) ? st->max_trace : 0;
    int32_t *tidx = nullptr;
    if (mt > 0) {
        lc.max_trace = mt;
        CHK(c->tr_k.ensure((size_t)mt * 8));
        CHK(c->tr_f.ensure((size_t)mt * 8));
        CHK(c->tr_l.ensure((size_t)mt * 8));
        CHK(c->tr_T.ensure((size_t)mt * 72));
        lc.tk = c->tr_k.as<long long>();
        lc.tf = c->tr_f.as<double>();
        lc.tl = c->tr_l.as<double>();
        lc.tT = c->tr_T.as<double>();
        if (st->trace_idx) {
            lc.max_trace_idx = st->max_trace_idx > 0 ? std::min(st->max_trace_idx, mt) : mt;
            if ((double)lc.max_trace_idx * (double)n * 4.0 > 8e9)
                return fail(FICP_EINVAL, "trace_idx of %d calls x %lld rows is too large",
                            lc.max_trace_idx, (long long)n);
            CHK(c->tr_idx.ensure((size_t)lc.max_trace_idx * (size_t)n * 4));
            tidx = c->tr_idx.as<int32_t>();
        }
    }
    // selection path without traces: the selection's last kernel also runs the loop step
    // and stores the done flag straight into the pinned ring (and, fuse_fit, the rigid fit
    // of the next iteration: gather + final, no k_fit_sums pass).
    const bool fused = !tidx;
    // the rigid fit fused into the selection (gather: the rows below the candidates, their
    // pairs loaded before the bounds wait; final: the selected candidates, prefetched in its
    // prologue) instead of a k_fit_sums pass: +1.5-2.5 % at C3 (tools/ab_bench.sh, 2 x 40
    // steps: 8,067 / 8,140 vs 7,965 / 7,933 it/s).  FICP_FUSE_FIT=0: the separate pass.
    const char *ff = getenv("FICP_FUSE_FIT");
    const bool fuse_fit = !(ff && atoi(ff) == 0);
    // with the fused loop and fit every consumer of the sort key (histogram, gather) derives
    // it from r (key_of_r): the NN stores 8 B per row less.  FICP_NN_KEYS=1: stored keys.
    const char *nk = getenv("FICP_NN_KEYS");
    const bool keys_from_r = fused && fuse_fit && !(nk && atoi(nk) != 0);
    // the window path (k_sel_win, one launch instead of four) for the calls whose previous
    // flag carried kFlagWinNext; FICP_SEL_WIN=0 turns it off.  It needs the work order (its
    // arrays: library buffers, 16-B aligned for the window pass's loads).
    const char *wv = getenv("FICP_SEL_WIN");
    const bool use_win = fused && fuse_fit && keys_from_r && use_grid(c, n) && select_win_fits(n) &&
                         !(wv && atoi(wv) == 0);
    HIPCHK(launch_run_start(tflag, &c->h_rep->t[0], c->stream, sel_err_word(c->sel_tmp.p, n), dst,
                            &lc));
    // the CHM layer's bbox (grid plan, pivot) after k_run_start: that launch is queued
    // before the host waits for the bbox instead of after it
    CHK(ensure_bbox(c));
    double *wx = sx, *wy = sy;
    const double *wz = sz;
    const uint32_t *worig = nullptr;
    if (use_grid(c, n)) {
        // the grid build and the work order: one bucket sort of two jobs (four launches)
        BSJob gj{}, wj{};
        CHK(ensure_grid(c, &gj));
        CHK(build_work_order(c, sx, sy, sz, n, &wj));
        if (gj.n > 0 || wj.n > 0)
            HIPCHK(launch_bsort2(gj.n > 0 ? gj : wj, gj.n > 0 ? wj : BSJob{}, c->stream));
        wx = c->wx.as<double>();
        wy = c->wy.as<double>();
        wz = sz ? c->wz.as<double>() : nullptr;
        worig = c->worig.as<uint32_t>();
    }
    FitIn fa{wx, wy, c->ccx.as<double>(), c->ccy.as<double>(), c->key.as<unsigned long long>(),
             nullptr, worig, n, c->pivot_x, c->pivot_y, dst};
    const FitSrc fsrc{wx, wy, c->ccx.as<double>(), c->ccy.as<double>(), c->pivot_x, c->pivot_y, 1,
                      allow_refl};
    // Iterations are enqueued `la` ahead of the one whose done flag the host reads, so
    // the device never waits for the host; the iterations enqueued past the end are
    // no-ops (every kernel tests the flags k_loop_update set).  la = 1 with the fused
    // selection runs the half-step form below; it needs the fit + NN of an iteration to
    // outlast the host's wake-up and five launches (~20 us): from 64k rows (C2 100k:
    // equal to la = 2; C3: +1.5 % over whole-iteration lookahead).
    const int la = n >= (1 << 16) ? 1 : 2;
    const int64_t cap = (int64_t)nstages * ((int64_t)std::max(max_iter, 0) + 1);
    int64_t j = 0;
    bool finished = nstages <= 0;
    // the calls from this index on take k_nn_grid_q (mostly certified queries);
    // FICP_NN_QPT_FROM overrides (a large value: never)
    const char *qf = getenv("FICP_NN_QPT_FROM");
    const int64_t nn_multi_from = qf ? atoll(qf) : nn_qpt_from();
    // part A of iteration i: the fit and the NN call; part B: the selection (and, not
    // fused, the loop step and the flag copy)
    int64_t last_a = -1;  // the last iteration whose fit + NN were enqueued
    auto enq_a = [&](int64_t i) -> int {
        if (!(fused && fuse_fit)) {
            ProfScope ps(c, P_FIT, "fit");
            HIPCHK(launch_fit(fa, allow_refl, c->fit_tmp.p, dst, &dst->no_fit, c->stream));
        }
        // (a later stage's head reuses the previous call's outputs: dst->nn_reuse)
        // (a launch queued behind the loop's end writes the caller-order XY: fin_*)
        CHK(nn_call(c, wx, wy, wz, n, dst->T, true, i == 0 ? 1 : 2, &dst->done, &dst->apply,
                    false, tidx != nullptr, &dst->nn_reuse, !keys_from_r, i >= nn_multi_from,
                    worig, sx, sy, i <= 1));
        last_a = i;
        return FICP_OK;
    };
    auto enq_b = [&](int64_t i, bool win) -> int {
        const int slot = (int)(i % kLoopRing);
        if (fused) __atomic_store_n(&c->h_flags[slot], -1, __ATOMIC_RELAXED);
        if (win) {
            ProfScope ps(c, P_SORT, "select");
            HIPCHK(launch_select_win(c->r.as<double>(), worig, n, range_ptr(c),
                                     nn_range_parts(n, c->m, use_grid(c, n)), c->sel_tmp.p, dst, lc,
                                     &c->h_flags[slot], c->stream, fsrc, c->fault));
            return FICP_OK;
        }
        {
            ProfScope ps(c, P_SORT, "select");
            HIPCHK(launch_select(keys_from_r ? nullptr : c->key.as<unsigned long long>(), worig,
                                 c->r.as<double>(), n, 0.0,
                                 &dst->lam_cur, range_ptr(c), nn_range_parts(n, c->m, use_grid(c, n)),
                                 c->sel_tmp.p, dst, &dst->done, fused ? &lc : nullptr,
                                 fused ? &c->h_flags[slot] : nullptr, c->stream,
                                 (fused && fuse_fit) ? &fsrc : nullptr, c->fault));
        }
        if (!fused) {
            if (tidx)
                HIPCHK(launch_trace_idx(dst, c->idx.as<int32_t>(), worig, n, tidx, lc.max_trace_idx,
                                        c->stream));
            HIPCHK(launch_loop_update(dst, lc, c->stream));
            HIPCHK(hipMemcpyAsync(&c->h_flags[slot], &dst->done, 4, hipMemcpyDeviceToHost,
                                  c->stream));
            // (fused: the final kernel stores the flag itself and the host polls the
            // pinned word; no event record, each one costs an idle gap in the queue)
            HIPCHK(hipEventRecord(c->loop_ev[slot], c->stream));
        }
        return FICP_OK;
    };
    int flag_v = 0;  // the last flag read (fused): kFlagDone | kFlagWinNext, or kFlagRetry
    int64_t fin_j = INT64_MAX;  // the call whose flag ended the loop
    auto wait_flag = [&](int64_t i) -> int {
        const int old = (int)(i % kLoopRing);
        if (fused) {
            int v = 0;
            CHK(poll_flag(c, &c->h_flags[old], v));
            flag_v = v;
            finished = (v & kFlagDone) != 0;
        } else {
            HIPCHK(hipEventSynchronize(c->loop_ev[old]));
            finished = c->h_flags[old] != 0;
        }
        if (finished) fin_j = i;
        return FICP_OK;
    };
    if (fused && la == 1) {
        // half-step lookahead: iteration i's selection, then i+1's fit and NN, then wait
        // for i's flag.  The device runs that fit + NN (>= 30 us) while the host wakes and
        // enqueues the next selection, and a finished run leaves two no-op launches
        // queued instead of a whole iteration's seven
        // With the window path: a call whose previous flag allowed it takes k_sel_win; if
        // that cannot decide (kFlagRetry: the NN launch behind it was a no-op), the full
        // selection of the same call and the NN launch are enqueued again.
        if (!finished && cap > 0) CHK(enq_a(0));
        bool win = false;
        for (; j < cap && !finished; ++j) {
            CHK(enq_b(j, win));
            if (j + 1 < cap) CHK(enq_a(j + 1));
            CHK(wait_flag(j));
            if (flag_v & kFlagRetry) {
                c->win_retries += 1;
                CHK(enq_b(j, false));
                if (j + 1 < cap) CHK(enq_a(j + 1));
                CHK(wait_flag(j));
                if (flag_v & kFlagRetry) return fail(FICP_EHIP, "selection retry did not decide");
            } else if (win) {
                c->win_calls += 1;
            }
            win = use_win && (flag_v & kFlagWinNext) != 0;
        }
    } else {
        for (; j < cap && !finished; ++j) {
            CHK(enq_a(j));
            CHK(enq_b(j, false));
            if (j >= la) CHK(wait_flag(j - la));
        }
    }
    // one host round trip for everything the run reports: the caller-order XY, the loop
    // state, the sort's timeout flag and the selection's statistics (each separate sync
    // cost ~40 us of idle device at C3)
    // the caller-order XY: written by an NN launch queued behind the loop's last call
    // (fin_scatter: it found the done flag), else here
    if (worig && !(last_a > fin_j)) HIPCHK(launch_scatter_xy(worig, wx, wy, n, sx, sy, c->stream));
    c->h_rep->misc[1] = c->h_rep->misc[2] = c->h_rep->misc[3] = 0u;
    CHK(report_wait(c, ReportSeg{c->state_dev.p, &c->h_rep->st, (int)(sizeof(IterState) / 4)},
                    ReportSeg{tflag, &c->h_rep->misc[0], 1},
                    ReportSeg{sel_err_word(c->sel_tmp.p, n), &c->h_rep->misc[1], 3},
                    &c->h_rep->t[1]));
    memcpy(c->h_state, &c->h_rep->st, sizeof(IterState));
    memcpy(c->h_misc, c->h_rep->misc, sizeof c->h_rep->misc);
    if (!c->h_state->done) return fail(FICP_EHIP, "device ICP loop did not finish");
    if (st) {
        const IterState &h = *c->h_state;
        st->n_nn_calls = h.n_nn;
        st->n_nn_reused = h.n_reuse;
        st->n_fits = h.n_fit;
        st->iters[0] = h.iters[0];
        st->iters[1] = h.iters[1];
        st->k_last = h.k_last;
        st->frmsd_last[0] = h.frmsd_last[0];
        st->frmsd_last[1] = h.frmsd_last[1];
        memcpy(st->T_total, h.Ttot, sizeof st->T_total);
        const int nc = std::min(h.n_nn, mt), nf = std::min(h.n_fit, mt);
        if (nc > 0 || nf > 0) {
            if (nc > 0 && st->trace_k)
                HIPCHK(hipMemcpyAsync(st->trace_k, c->tr_k.p, nc * 8, hipMemcpyDeviceToHost, c->stream));
            if (nc > 0 && st->trace_frmsd)
                HIPCHK(hipMemcpyAsync(st->trace_frmsd, c->tr_f.p, nc * 8, hipMemcpyDeviceToHost,
                                      c->stream));
            if (nc > 0 && st->trace_lambda)
                HIPCHK(hipMemcpyAsync(st->trace_lambda, c->tr_l.p, nc * 8, hipMemcpyDeviceToHost,
                                      c->stream));
            if (nc > 0 && tidx)
                HIPCHK(hipMemcpyAsync(st->trace_idx, tidx,
                                      (size_t)std::min(nc, lc.max_trace_idx) * (size_t)n * 4,
                                      hipMemcpyDeviceToHost, c->stream));
            if (nf > 0 && st->trace_T)
                HIPCHK(hipMemcpyAsync(st->trace_T, c->tr_T.p, (size_t)nf * 72, hipMemcpyDeviceToHost,
                                      c->stream));
            CHK(sync(c));
        }
        st->gpu_ms = (double)(c->h_rep->t[1] - c->h_rep->t[0]) * 1e-5;  // 100 MHz ticks
    }
    if (c->h_misc[0])
        return fail(FICP_EHIP, "residual sort raised error flag %u (results invalid)", c->h_misc[0]);
    c->sel_levels = c->h_misc[2];
    c->sel_radix = c->h_misc[3];
    if (c->h_misc[1]) return fail(FICP_EHIP, "%s", sel_err_text(c->h_misc[1]).c_str());
    return FICP_OK;
}

int check_ctx(ficp_ctx *c) {
    if (!c) return fail(FICP_EINVAL, "null context");
    return set_device(c);
}

int check_md(int32_t md) {
    if (md != 2 && md != 3) return fail(FICP_EINVAL, "md must be 2 or 3 (got %d)", md);
    return FICP_OK;
}

// ---- distributed runs (ficp_dist_*): small glue kernels
constexpr unsigned long long kFlip = 0x8000000000000000ULL;
constexpr int kDistTrace = 4096;  // k trace capacity of a distributed run (NN calls)

// the key range {~kmin, kmax} of the local rows as int64 words whose signed order is the
// unsigned order (top bit flipped): the caller's MAX all-reduce gives the global range
__global__ void k_dist_range_out(const unsigned long long *range, long long *out,
                                 const int *skip) {
    if ((skip && *skip) || threadIdx.x != 0) return;
    out[0] = (long long)(range[0] ^ kFlip);
    out[1] = (long long)(range[1] ^ kFlip);
}

__global__ void k_dist_range_in(const long long *in, unsigned long long *range, const int *skip) {
    if ((skip && *skip) || threadIdx.x != 0) return;
    range[0] = (unsigned long long)in[0] ^ kFlip;
    range[1] = (unsigned long long)in[1] ^ kFlip;
}

__global__ void k_dist_gorig(const uint32_t *worig, int64_t n, int64_t row0, uint32_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)(row0 + (worig ? (int64_t)worig[i] : i));
}

int check_dist(ficp_ctx *c, int mode) {
    CHK(check_ctx(c));
    if (c->dist_mode != mode)
        return fail(FICP_ESTATE, "no %s-partitioned run begun on this context",
                    mode == 1 ? "target" : "source");
    return FICP_OK;
}

void reset_target(ficp_ctx *c, int64_t m, int md) {
    c->has_target = true;
    c->grid_ready = false;
    c->bbox_ready = false;
    c->bbox_dev = false;
    c->m = m;
    c->md = md;
}

}  // namespace

// ===================================================================== C ABI
extern "C" {

int ficp_version(void) { return 100; }

const char *ficp_last_error(void) { return g_err.c_str(); }

int ficp_device_count(int *count) {
    if (!count) return fail(FICP_EINVAL, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(FICP_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return FICP_OK;
}

int ficp_create(int device, ficp_ctx **out) {
    if (!out) return fail(FICP_EINVAL, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(FICP_ENODEV, "no HIP device");
    if (device < 0 || device >= n)
        return fail(FICP_EINVAL, "device %d out of range [0,%d)", device, n);
    ficp_ctx *c = new ficp_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipHostMalloc((void **)&c->h_state, sizeof(IterState), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess)
        e = hipHostMalloc((void **)&c->h_flags, kLoopRing * sizeof(int), hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_misc, 16 * sizeof(unsigned), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_rep, sizeof(HostReport), hipHostMallocCoherent);
    for (int k = 0; k < kLoopRing && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&c->loop_ev[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        delete c;
        return fail(FICP_EHIP, "context setup: %s", hipGetErrorString(e));
    }
    *out = c;
    return FICP_OK;
}

void ficp_destroy(ficp_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->own_stream) c->stream = c->own_stream;  // a caller's stream is not ours to destroy
    c->gorig.release();
    c->drange.release();
    DevBuf *bufs[] = {&c->tx,     &c->ty,         &c->tz,       &c->cell_of,  &c->counts,
                      &c->cell_start, &c->fill,   &c->pts,      &c->scan_tmp, &c->mm_part,
                      &c->mm_out, &c->sx,         &c->sy,       &c->sz,       &c->idx,
                      &c->dist,   &c->r,          &c->key,      &c->val,      &c->order,
                      &c->sort_tmp, &c->frac_tmp, &c->fit_tmp,  &c->bd2,      &c->bidx,
                      &c->ccx,    &c->ccy,        &c->rs,       &c->range,    &c->wx,
                      &c->wy,     &c->wz,         &c->worig,    &c->tidx,     &c->stage,
                      &c->stage2, &c->cx,         &c->cy,       &c->cz,       &c->state_dev,
                      &c->btrace,
                      &c->bp,     &c->dz2,        &c->gap,      &c->lams,       &c->tr_k,     &c->tr_f,     &c->tr_l,
                      &c->tr_T,   &c->tr_idx,     &c->sel_tmp,  &c->sel_stats, &c->bs_tmp, &c->bs_tmp2};
    for (DevBuf *b : bufs) b->release();
    c->pin.release();
    c->pin_xy.release();
    c->pin_up.release();
    if (c->up_ev) (void)hipEventDestroy(c->up_ev);
    batch_release(c->batch);
    c->batch = nullptr;
    for (auto &r : c->recs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    if (c->h_misc) (void)hipHostFree(c->h_misc);
    if (c->h_rep) (void)hipHostFree(c->h_rep);
    for (hipEvent_t &e : c->loop_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int ficp_set_fault(ficp_ctx *c, int32_t mask) {
    if (!c) return fail(FICP_EINVAL, "null context");
    c->fault = mask;
    return FICP_OK;
}

int ficp_set_nn_mode(ficp_ctx *c, int32_t mode) {
    if (!c) return fail(FICP_EINVAL, "null context");
    if (mode < 0 || mode > 2) return fail(FICP_EINVAL, "nn mode must be 0, 1 or 2");
    c->nn_mode = mode;
    return FICP_OK;
}

int ficp_profile_enable(ficp_ctx *c, int32_t mask) {
    if (!c) return fail(FICP_EINVAL, "null context");
    c->prof_mask = mask;
    return FICP_OK;
}

int ficp_path_stats(ficp_ctx *c, int64_t out[4]) {
    CHK(check_ctx(c));
    if (!out) return fail(FICP_EINVAL, "null out");
    out[0] = c->win_calls;
    out[1] = c->win_retries;
    out[2] = (int64_t)c->sel_levels;
    out[3] = (int64_t)c->sel_radix;
    return FICP_OK;
}

// wall-clock length of the union of intervals (ms): records on concurrent streams (the batch
// sub-batches) overlap, so their summed durations overstate the time the kernels held the GPU
static double union_ms(std::vector<std::pair<double, double>> iv) {
    std::sort(iv.begin(), iv.end());
    double tot = 0.0, a = 0.0, b = 0.0;
    bool open = false;
    for (const auto &x : iv) {
        if (!open || x.first > b) {
            if (open) tot += b - a;
            a = x.first;
            b = x.second;
            open = true;
        } else {
            b = std::max(b, x.second);
        }
    }
    return open ? tot + (b - a) : 0.0;
}

int ficp_profile_report(ficp_ctx *c, char *buf, int64_t buflen) {
    CHK(check_ctx(c));
    CHK(sync(c));
    // every record's interval as offsets from the first record's start event (signed)
    std::map<std::string, std::vector<std::pair<double, double>>> ivs;
    std::vector<std::pair<double, double>> all;
    const hipEvent_t ref = c->recs.empty() ? nullptr : c->recs.front().a;
    for (auto &r : c->recs) {
        float ms = 0.f, oa = 0.f, ob = 0.f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        (void)hipEventElapsedTime(&oa, ref, r.a);
        (void)hipEventElapsedTime(&ob, ref, r.b);
        auto &acc = c->prof_acc[r.name];
        acc.first += 1;
        acc.second += ms;
        ivs[r.name].push_back({(double)oa, (double)ob});
        all.push_back({(double)oa, (double)ob});
        c->ev_pool.push_back(r.a);
        c->ev_pool.push_back(r.b);
    }
    c->recs.clear();
    std::string s = "{";
    bool first = true;
    for (auto &kv : c->prof_acc) {
        char item[320];
        const auto it = ivs.find(kv.first);
        const double wall = it == ivs.end() ? 0.0 : union_ms(it->second);
        snprintf(item, sizeof item, "%s\"%s\": {\"count\": %lld, \"ms\": %.6f, \"wall_ms\": %.6f}",
                 first ? "" : ", ", kv.first.c_str(), (long long)kv.second.first, kv.second.second, wall);
        s += item;
        first = false;
    }
    if (!all.empty()) {  // every recorded interval together
        char item[160];
        snprintf(item, sizeof item, "%s\"_all\": {\"count\": %lld, \"wall_ms\": %.6f}", first ? "" : ", ",
                 (long long)all.size(), union_ms(all));
        s += item;
    }
    s += "}";
    c->prof_acc.clear();
    if (!buf || buflen <= 0) return fail(FICP_EINVAL, "null buffer");
    if ((int64_t)s.size() + 1 > buflen)
        return fail(FICP_EINVAL, "buffer too small (%zu)", s.size() + 1);
    memcpy(buf, s.c_str(), s.size() + 1);
    return FICP_OK;
}

int ficp_set_target(ficp_ctx *c, const double *tgt, int64_t m, int64_t ld, int32_t md) {
    CHK(check_ctx(c));
    CHK(check_md(md));
    if (m < 0 || (m > 0 && (!tgt || ld < md))) return fail(FICP_EINVAL, "bad target shape");
    if (m > 0x7fffffff) return fail(FICP_EINVAL, "target too large");
    CHK(bbox_collect(c));
    reset_target(c, m, md);
    const size_t bytes = (size_t)m * (size_t)ld * 8;
    if (m > 0 && bytes <= kBounceBytes) {
        // a small layer (the Join button's ~260 stems) goes through a pinned bounce buffer:
        // the caller's array is free as soon as this returns and the upload runs stream-
        // ordered before the next run, with no host round trip (the previous upload from
        // the bounce buffer is waited for first; it is long done by then)
        CHK(c->pin_up.ensure(kBounceBytes));
        if (c->up_ev) HIPCHK(hipEventSynchronize(c->up_ev));
        else HIPCHK(hipEventCreateWithFlags(&c->up_ev, hipEventDisableTiming));
        memcpy(c->pin_up.p, tgt, bytes);
        CHK(upload_rows(c, c->pin_up.as<double>(), m, ld, md, c->tx, c->ty, &c->tz));
        HIPCHK(hipEventRecord(c->up_ev, c->stream));
        return FICP_OK;
    }
    CHK(upload_rows(c, tgt, m, ld, md, c->tx, c->ty, &c->tz));
    return sync(c);
}

int ficp_set_target_device(ficp_ctx *c, const double *x, const double *y, const double *z,
                           int64_t m, int32_t md) {
    CHK(check_ctx(c));
    CHK(check_md(md));
    if (m < 0 || (m > 0 && (!x || !y || (md == 3 && !z))))
        return fail(FICP_EINVAL, "bad target");
    if (m > 0x7fffffff) return fail(FICP_EINVAL, "target too large");
    CHK(bbox_collect(c));
    reset_target(c, m, md);
    CHK(c->tx.ensure(m * 8));
    CHK(c->ty.ensure(m * 8));
    CHK(c->tz.ensure(m * 8));
    if (m > 0) {
        // one kernel copies the columns and reduces the bbox (three copies + the bbox
        // pass were four launches); ensure_bbox reads the result
        CHK(c->mm_part.ensure(1024 * 4 * 8));
        CHK(c->mm_out.ensure(4 * 8));
        HIPCHK(launch_minmax2(x, y, m, c->mm_part.as<double>(), c->mm_out.as<double>(), c->stream,
                              md == 3 ? z : nullptr, c->tx.as<double>(), c->ty.as<double>(),
                              md == 3 ? c->tz.as<double>() : nullptr));
        c->bbox_dev = true;
        __atomic_store_n(&c->h_rep->bflag, -1, __ATOMIC_RELAXED);
        HIPCHK(launch_report(ReportSeg{c->mm_out.p, c->h_rep->bb, 8}, ReportSeg{}, ReportSeg{},
                             &c->h_rep->bflag, nullptr, c->stream));
        c->bbox_pending = true;
    }
    return FICP_OK;  // stream-ordered; the grid is built on first use
}

int ficp_nn(ficp_ctx *c, const double *src, int64_t n, int64_t ld, int32_t *idx, double *dist) {
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (n < 0 || (n > 0 && (!src || !idx || !dist || ld < c->md)))
        return fail(FICP_EINVAL, "bad source");
    if (n == 0 || c->m == 0) return FICP_OK;
    CHK(upload_rows(c, src, n, ld, c->md, c->sx, c->sy, &c->sz));
    CHK(ensure_work(c, n));
    CHK(nn_call(c, c->sx.as<double>(), c->sy.as<double>(), c->sz.as<double>(), n, nullptr,
                false));
    CHK(d2h_staged(c, idx, c->idx.p, (size_t)n * 4));
    return d2h_staged(c, dist, c->dist.p, (size_t)n * 8);
}

int ficp_optimal_fraction(ficp_ctx *c, const double *src, int64_t lds, const double *corr,
                          int64_t ldc, const double *dist, int64_t n, int64_t n_source,
                          int32_t md, double lambda_val, double *frac, int64_t *k) {
    CHK(check_ctx(c));
    CHK(check_md(md));
    if (!frac || !k) return fail(FICP_EINVAL, "null output");
    *frac = 0.0;
    *k = 0;
    if (n_source == 0 || n == 0) return FICP_OK;  // ficp.py:76-77
    if (n < 0 || n_source < 0 || !src || !corr || !dist || lds < md || ldc < md)
        return fail(FICP_EINVAL, "bad arguments");
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large");
    CHK(ensure_work(c, n));
    CHK(upload_rows(c, src, n, lds, md, c->sx, c->sy, &c->sz));
    CHK(upload_rows(c, corr, n, ldc, md, c->cx, c->cy, &c->cz));
    CHK(c->stage2.ensure(n * 8));
    HIPCHK(hipMemcpyAsync(c->stage2.p, dist, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_residuals(c->sx.as<double>(), c->sy.as<double>(), c->sz.as<double>(),
                            c->cx.as<double>(), c->cy.as<double>(), c->cz.as<double>(), n, md,
                            c->r.as<double>(), c->stream));
    HIPCHK(launch_keys_from_doubles(c->stage2.as<double>(), n, c->key.as<unsigned long long>(),
                                    nullptr, c->stream));
    HIPCHK(launch_key_range(c->key.as<unsigned long long>(), n, range_ptr(c), c->stream));
    CHK(sort_and_select(c, n, n_source, lambda_val, nullptr));
    CHK(read_state(c));
    *k = c->h_state->k;
    *frac = c->h_state->frac;
    return FICP_OK;
}

int ficp_frmsd(ficp_ctx *c, const double *src, int64_t lds, const double *corr, int64_t ldc,
               int64_t rows, int64_t num_elements, int32_t md, double fraction,
               double lambda_val, double *out) {
    CHK(check_ctx(c));
    CHK(check_md(md));
    if (!out) return fail(FICP_EINVAL, "null output");
    if (num_elements == 0) {  // ficp.py:56-57
        *out = INFINITY;
        return FICP_OK;
    }
    const int64_t k = rows;
    if (k < 0 || (k > 0 && (!src || !corr || lds < md || ldc < md)))
        return fail(FICP_EINVAL, "bad arguments");
    CHK(upload_rows(c, src, k, lds, md, c->sx, c->sy, &c->sz));
    CHK(upload_rows(c, corr, k, ldc, md, c->cx, c->cy, &c->cz));
    CHK(ensure_fit(c, std::max<int64_t>(k, 4096)));
    CHK(c->stage2.ensure(64));
    HIPCHK(launch_sum_sq_diff(c->sx.as<double>(), c->sy.as<double>(), c->sz.as<double>(),
                              c->cx.as<double>(), c->cy.as<double>(), c->cz.as<double>(), k, md,
                              (char *)c->fit_tmp.p + fit_scratch_offset(), c->stage2.as<double>(),
                              c->stream));
    double S = 0.0;
    HIPCHK(hipMemcpyAsync(&S, c->stage2.p, 8, hipMemcpyDeviceToHost, c->stream));
    CHK(sync(c));
    *out = (1.0 / pow(fraction, lambda_val)) * sqrt(S / (double)num_elements);  // ficp.py:59-60
    return FICP_OK;
}

int ficp_argsort(ficp_ctx *c, const double *d, int64_t n, int64_t *order) {
    CHK(check_ctx(c));
    if (n < 0 || (n > 0 && (!d || !order))) return fail(FICP_EINVAL, "bad arguments");
    if (n == 0) return FICP_OK;
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large");
    CHK(ensure_work(c, n));
    CHK(c->stage2.ensure(n * 8));
    HIPCHK(hipMemcpyAsync(c->stage2.p, d, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_keys_from_doubles(c->stage2.as<double>(), n, c->key.as<unsigned long long>(),
                                    nullptr, c->stream));
    uint32_t *tflag = sort_timeout_flag(c->sort_tmp.p, n);
    HIPCHK(launch_atomic_zero32(tflag, 1, c->stream));
    HIPCHK(launch_key_range(c->key.as<unsigned long long>(), n, range_ptr(c), c->stream));
    HIPCHK(launch_sort(c->key.as<unsigned long long>(), nullptr, n, range_ptr(c),
                       c->order.as<uint32_t>(), nullptr, nullptr, c->sort_tmp.p, nullptr,
                       c->stream));
    CHK(c->pin.ensure((size_t)n * 4 + 64));
    uint32_t *tmp = c->pin.as<uint32_t>();
    uint32_t *tf = tmp + ((n + 15) & ~(int64_t)15);
    HIPCHK(hipMemcpyAsync(tf, tflag, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(tmp, c->order.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    CHK(sync(c));
    if (*tf) return fail(FICP_EHIP, "sort look-back timed out (results invalid)");
    host_parallel(n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) order[i] = tmp[i];
    });
    return FICP_OK;
}

int ficp_fit_rigid2d(ficp_ctx *c, const double *src, int64_t lds, const double *tgt,
                     int64_t ldt, int64_t k, int32_t allow_reflection, double T[9]) {
    CHK(check_ctx(c));
    if (!T || k <= 0 || !src || !tgt || lds < 2 || ldt < 2)
        return fail(FICP_EINVAL, "bad arguments (k must be >= 1)");
    CHK(upload_rows(c, src, k, lds, 2, c->sx, c->sy, nullptr));
    CHK(upload_rows(c, tgt, k, ldt, 2, c->cx, c->cy, nullptr));
    CHK(ensure_fit(c, k));
    CHK(c->state_dev.ensure(sizeof(IterState)));
    // pivot: the first source point keeps the sums well conditioned for any offset
    double p[2] = {0.0, 0.0};
    HIPCHK(hipMemcpyAsync(&p[0], c->sx.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&p[1], c->sy.p, 8, hipMemcpyDeviceToHost, c->stream));
    CHK(sync(c));
    FitIn fa{c->sx.as<double>(), c->sy.as<double>(), c->cx.as<double>(), c->cy.as<double>(),
             nullptr, nullptr, nullptr, k, p[0], p[1], c->state_dev.as<IterState>()};
    HIPCHK(launch_fit(fa, allow_reflection, c->fit_tmp.p, c->state_dev.as<IterState>(), nullptr,
                      c->stream));
    CHK(read_state(c));
    memcpy(T, c->h_state->T, 9 * sizeof(double));
    return FICP_OK;
}

int ficp_apply_xy(ficp_ctx *c, const double *pts, int64_t n, int64_t ld, const double T[9],
                  double *out_xy) {
    CHK(check_ctx(c));
    if (n < 0 || (n > 0 && (!pts || !out_xy || ld < 2)) || !T)
        return fail(FICP_EINVAL, "bad arguments");
    if (n == 0) return FICP_OK;
    CHK(upload_rows(c, pts, n, ld, 2, c->sx, c->sy, nullptr));
    CHK(c->stage2.ensure(std::max<int64_t>(n * 16, 128)));
    CHK(c->state_dev.ensure(sizeof(IterState)));
    double *dT = c->state_dev.as<IterState>()->T;
    HIPCHK(hipMemcpyAsync(dT, T, 9 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_apply_xy(c->sx.as<double>(), c->sy.as<double>(), n, dT, c->stream));
    HIPCHK(launch_interleave_xy(c->sx.as<double>(), c->sy.as<double>(), n, c->stage2.as<double>(),
                                c->stream));
    return d2h_staged(c, out_xy, c->stage2.p, (size_t)n * 16);
}

int ficp_run(ficp_ctx *c, double *src, int64_t n, int64_t ld, int32_t nstages,
             const double *lambdas, double threshold, int32_t max_iterations,
             int32_t allow_reflection, ficp_stats *stats) {
    return ficp_run_into(c, src, src, n, ld, nstages, lambdas, threshold, max_iterations,
                         allow_reflection, stats);
}

int ficp_run_into(ficp_ctx *c, const double *src, double *out, int64_t n, int64_t ld,
                  int32_t nstages, const double *lambdas, double threshold,
                  int32_t max_iterations, int32_t allow_reflection, ficp_stats *stats) {
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (n < 0 || (n > 0 && (!src || !out || ld < c->md)) || nstages < 0 || (nstages > 0 && !lambdas))
        return fail(FICP_EINVAL, "bad arguments");
    auto copy_rows = [&]() {  // out = src: the columns the run leaves alone
        if (out != src) ficp_host_copy(out, src, n * ld * 8);
    };
    if (n == 0 || c->m == 0) {
        copy_rows();
        return run_core(c, nullptr, nullptr, nullptr, 0, nstages, lambdas, threshold,
                        max_iterations, allow_reflection, stats);
    }
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = clk::now();
    if (use_small(c, n) && n <= 0x3fffffff) {
        // the Join button's size: one H2D of the rows, one launch that reports straight
        // into pinned memory, one poll (k_small.hip)
        CHK(c->stage.ensure((size_t)n * ld * 8));
        HIPCHK(hipMemcpyAsync(c->stage.p, src, (size_t)n * ld * 8, hipMemcpyHostToDevice, c->stream));
        const auto t1 = clk::now();
        double *xy = nullptr;
        CHK(run_small(c, c->stage.as<double>(), ld, nullptr, nullptr, nullptr, n, nstages, lambdas,
                      threshold, max_iterations, allow_reflection, stats, &xy));
        const auto t2 = clk::now();
        copy_rows();
        for (int64_t i = 0; i < n; ++i) {  // columns 0, 1 only (ficp.py:114-118)
            out[i * ld] = xy[2 * i];
            out[i * ld + 1] = xy[2 * i + 1];
        }
        if (stats) {
            stats->host_ms[0] = ms(t0, t1);
            stats->host_ms[1] = ms(t1, t2);
            stats->host_ms[2] = ms(t2, clk::now());
            stats->host_ms[3] = 0.0;
        }
        return FICP_OK;
    }
    // the rows stay in c->stage (upload_rows) for the whole run: at the end the moved XY
    // replace their columns 0, 1 there and the rows come back in one D2H, straight into
    // `out` when it is page-locked (the library's pooled blocks) -- no host-side column
    // write-back, and the caller needs no copy of the rows for the run to move
    CHK(upload_rows(c, src, n, ld, c->md, c->sx, c->sy, &c->sz));
    const auto t1 = clk::now();
    CHK(run_core(c, c->sx.as<double>(), c->sy.as<double>(),
                 c->md == 3 ? c->sz.as<double>() : nullptr, n, nstages, lambdas, threshold,
                 max_iterations, allow_reflection, stats));
    const auto t2 = clk::now();
    const bool pinned = host_pinned(out);
    if (out == src && !pinned) {
        // in place into pageable rows (ficp_run): only the moved XY come back (16 B per
        // row through the pinned staging), the caller's other columns are already right
        HIPCHK(launch_interleave_xy(c->sx.as<double>(), c->sy.as<double>(), n, c->stage.as<double>(),
                                    c->stream));
        CHK(d2h_xy_columns(c, c->stage.as<double>(), n, out, ld));
        if (stats) {
            stats->host_ms[0] = ms(t0, t1);
            stats->host_ms[1] = ms(t1, t2);
            stats->host_ms[2] = ms(t2, clk::now());
            stats->host_ms[3] = 0.0;
        }
        return FICP_OK;
    }
    HIPCHK(launch_put_xy_rows(c->sx.as<double>(), c->sy.as<double>(), n, ld, c->stage.as<double>(),
                              c->stream));
    const size_t bytes = (size_t)n * (size_t)ld * 8;
    if (pinned) {
        HIPCHK(hipMemcpyAsync(out, c->stage.p, bytes, hipMemcpyDeviceToHost, c->stream));
        CHK(sync(c));
    } else {
        CHK(d2h_staged(c, out, c->stage.p, bytes));
    }
    if (stats) {
        stats->host_ms[0] = ms(t0, t1);
        stats->host_ms[1] = ms(t1, t2);
        stats->host_ms[2] = ms(t2, clk::now());
        stats->host_ms[3] = 0.0;
    }
    return FICP_OK;
}

int ficp_run_device(ficp_ctx *c, double *x, double *y, const double *z, int64_t n,
                    int32_t nstages, const double *lambdas, double threshold,
                    int32_t max_iterations, int32_t allow_reflection, ficp_stats *stats) {
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (n < 0 || (n > 0 && (!x || !y || (c->md == 3 && !z))) || nstages < 0 ||
        (nstages > 0 && !lambdas))
        return fail(FICP_EINVAL, "bad arguments");
    return run_core(c, x, y, c->md == 3 ? z : nullptr, n, nstages, lambdas, threshold,
                    max_iterations, allow_reflection, stats);
}

// ---- CHMPlot.remove_matches (chm_plot.py:223-285), SURVEY.md §8(f1)
int ficp_remove_matches(ficp_ctx *c, const double *plot, int64_t n, int64_t ld,
                        const double *thresh, int32_t *removed, int64_t *n_removed) {
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (!n_removed || n < 0 || (n > 0 && (!plot || !thresh || !removed || ld < c->md)))
        return fail(FICP_EINVAL, "bad arguments");
    *n_removed = 0;
    const int64_t m = c->m;
    if (n == 0 || m == 0) return FICP_OK;
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large (max 2^30 - 1)");
    if (m > kMaxGridStems) return fail(FICP_EINVAL, "CHM layer too large for the grid");
    CHK(ensure_grid(c));
    CHK(upload_rows(c, plot, n, ld, c->md, c->sx, c->sy, &c->sz));
    CHK(c->bidx.ensure((size_t)n * KNN_K * 4));  // the K candidates of every plot tree
    CHK(c->bd2.ensure((size_t)n * KNN_K * 8));
    CHK(c->tidx.ensure((size_t)m));  // the removed-stem mask (one byte per stem)
    std::vector<int32_t> kid((size_t)n * KNN_K);
    std::vector<double> kd((size_t)n * KNN_K);
    std::vector<uint8_t> rem((size_t)m, 0);
    auto query = [&](int64_t q0, bool masked) -> int {
        if (masked)
            HIPCHK(hipMemcpyAsync(c->tidx.p, rem.data(), (size_t)m, hipMemcpyHostToDevice,
                                  c->stream));
        HIPCHK(launch_knn_grid(c->sx.as<double>(), c->sy.as<double>(), c->sz.as<double>(), q0, n,
                               c->gv, c->md, masked ? (const uint8_t *)c->tidx.p : nullptr,
                               c->bidx.as<int32_t>(), c->bd2.as<double>(), c->stream));
        const size_t off = (size_t)q0 * KNN_K, cnt = (size_t)(n - q0) * KNN_K;
        HIPCHK(hipMemcpyAsync(kid.data() + off, c->bidx.as<int32_t>() + off, cnt * 4,
                              hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(kd.data() + off, c->bd2.as<double>() + off, cnt * 8,
                              hipMemcpyDeviceToHost, c->stream));
        return sync(c);
    };
    CHK(query(0, false));
    // The greedy walk of the reference, in plot-tree order: each tree takes its nearest
    // remaining stem (first of its K candidates not yet removed).  When all K of a tree
    // are gone, the trees from it on are queried again with the removed stems masked.
    int64_t remaining = m, cnt = 0;
    for (int64_t i = 0; i < n && remaining > 0;) {
        int j = -1;
        for (int u = 0; u < KNN_K; ++u) {
            const int32_t id = kid[(size_t)i * KNN_K + u];
            if (id == 0x7fffffff) break;  // fewer than K stems left for this tree
            if (!rem[(size_t)id]) {
                j = u;
                break;
            }
        }
        if (j < 0) {
            CHK(query(i, true));
            if (kid[(size_t)i * KNN_K] == 0x7fffffff) break;  // nothing left at all
            continue;
        }
        const int32_t id = kid[(size_t)i * KNN_K + j];
        if (kd[(size_t)i * KNN_K + j] < thresh[i]) {  // chm_plot.py:249, 282
            rem[(size_t)id] = 1;
            removed[cnt++] = id;
            --remaining;
        }
        ++i;
    }
    *n_removed = cnt;
    return FICP_OK;
}

// ---- partitioned target: NN against this context's shard, the
// caller merges the shards (all-reduce of d2, then of the masked idx), then the
// selection + fit on the merged correspondences.
int ficp_nn_device(ficp_ctx *c, const double *x, const double *y, const double *z, int64_t n,
                   int64_t idx_offset, double *d2, int32_t *idx) {
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (n < 0 || (n > 0 && (!x || !y || (c->md == 3 && !z) || !d2 || !idx)))
        return fail(FICP_EINVAL, "bad arguments");
    if (n == 0) return FICP_OK;
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large (max 2^30 - 1)");
    if (idx_offset < 0 || idx_offset + c->m > 0x7fffffff) return fail(FICP_EINVAL, "bad idx_offset");
    if (c->m == 0) {  // empty shard: never the minimum of the merge
        HIPCHK(launch_fill_inf(d2, idx, n, c->stream));
        return sync(c);
    }
    CHK(ensure_work(c, n));
    NNArgs a{};
    a.sx = const_cast<double *>(x);
    a.sy = const_cast<double *>(y);
    a.sz = c->md == 3 ? z : nullptr;
    a.n = n;
    a.idx = idx;
    a.r = d2;
    a.tx = c->tx.as<double>();
    a.ty = c->ty.as<double>();
    if (use_grid(c, n)) {
        CHK(ensure_grid(c));
        ProfScope ps(c, P_NN, "nn_grid");
        HIPCHK(launch_nn_grid(a, c->gv, c->md, c->stream, false));
    } else {
        const int64_t nch = brute_chunk_count(n, c->m);
        if (nch > 1) {
            CHK(c->bd2.ensure(nch * n * 8));
            CHK(c->bidx.ensure(nch * n * 4));
        }
        ProfScope ps(c, P_NN, "nn_brute");
        HIPCHK(launch_nn_brute(a, c->tx.as<double>(), c->ty.as<double>(),
                               c->md == 3 ? c->tz.as<double>() : nullptr, c->m, c->md,
                               c->bd2.as<double>(), c->bidx.as<int32_t>(), c->stream, false));
    }
    HIPCHK(launch_add_offset(idx, n, idx_offset, c->stream));
    return sync(c);
}

int ficp_select_fit_device(ficp_ctx *c, const double *x, const double *y, int64_t n,
                           const double *d2, const int32_t *idx, const double *tx,
                           const double *ty, int64_t n_source, double lambda_val,
                           int32_t allow_reflection, double pivot_x, double pivot_y, int64_t *k,
                           double *frmsd, double T[9]) {
    CHK(check_ctx(c));
    if (!k || !frmsd || !T) return fail(FICP_EINVAL, "null output");
    if (n < 0 || (n > 0 && (!x || !y || !d2 || !idx || !tx || !ty)) || n_source < n)
        return fail(FICP_EINVAL, "bad arguments");
    for (int e = 0; e < 9; ++e) T[e] = (e % 4 == 0) ? 1.0 : 0.0;
    *k = 0;
    *frmsd = INFINITY;
    if (n == 0) return FICP_OK;
    if (n > 0x3fffffff) return fail(FICP_EINVAL, "n too large (max 2^30 - 1)");
    CHK(ensure_work(c, n));
    uint32_t *tflag = sort_timeout_flag(c->sort_tmp.p, n);
    HIPCHK(launch_atomic_zero32(tflag, 1, c->stream));
    HIPCHK(launch_corr_from_merge(d2, idx, tx, ty, n, c->key.as<unsigned long long>(),
                                  c->r.as<double>(), c->ccx.as<double>(), c->ccy.as<double>(),
                                  range_ptr(c), c->stream));
    const bool sel = n == n_source;
    if (sel) {
        HIPCHK(launch_select(c->key.as<unsigned long long>(), nullptr, c->r.as<double>(), n,
                             lambda_val, nullptr, range_ptr(c), 0, c->sel_tmp.p,
                             c->state_dev.as<IterState>(), nullptr, nullptr, nullptr, c->stream));
    } else {
        CHK(sort_and_select(c, n, n_source, lambda_val, nullptr));
    }
    CHK(read_state(c));
    *k = c->h_state->k;
    *frmsd = c->h_state->frmsd;
    if (*k > 0) {
        IterState *dst = c->state_dev.as<IterState>();
        FitIn fa{x, y, c->ccx.as<double>(), c->ccy.as<double>(), c->key.as<unsigned long long>(),
                 sel ? nullptr : c->order.as<uint32_t>(), nullptr, n, pivot_x, pivot_y, dst};
        HIPCHK(launch_fit(fa, allow_reflection, c->fit_tmp.p, dst, nullptr, c->stream));
        CHK(read_state(c));
        memcpy(T, c->h_state->T, 9 * sizeof(double));
    }
    uint32_t tf = 0;
    HIPCHK(hipMemcpy(&tf, tflag, 4, hipMemcpyDeviceToHost));
    if (tf) return fail(FICP_EHIP, "residual sort raised error flag %u (results invalid)", tf);
    if (sel) {
        unsigned ss[3] = {0, 0, 0};
        HIPCHK(hipMemcpyAsync(ss, sel_err_word(c->sel_tmp.p, n), 12, hipMemcpyDeviceToHost,
                              c->stream));
        CHK(sync(c));
        c->sel_levels = ss[1];
        c->sel_radix = ss[2];
        if (ss[0]) return fail(FICP_EHIP, "%s", sel_err_text(ss[0]).c_str());
    }
    return FICP_OK;
}

int ficp_apply_device(ficp_ctx *c, double *x, double *y, int64_t n, const double T[9]) {
    CHK(check_ctx(c));
    if (n < 0 || (n > 0 && (!x || !y)) || !T) return fail(FICP_EINVAL, "bad arguments");
    if (n == 0) return FICP_OK;
    CHK(c->state_dev.ensure(sizeof(IterState)));
    double *dT = c->state_dev.as<IterState>()->T;
    HIPCHK(hipMemcpyAsync(dT, T, 9 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_apply_xy(x, y, n, dT, c->stream));
    return sync(c);
}

int ficp_dev_alloc(ficp_ctx *c, int64_t bytes, void **ptr) {
    CHK(check_ctx(c));
    if (!ptr || bytes < 0) return fail(FICP_EINVAL, "bad arguments");
    HIPCHK(hipMalloc(ptr, std::max<int64_t>(bytes, 1)));
    return FICP_OK;
}

int ficp_dev_free(ficp_ctx *c, void *ptr) {
    CHK(check_ctx(c));
    HIPCHK(hipFree(ptr));
    return FICP_OK;
}

int ficp_host_alloc(int64_t bytes, void **ptr) {
    if (!ptr || bytes < 0) return fail(FICP_EINVAL, "bad arguments");
    *ptr = nullptr;
    HIPCHK(hipHostMalloc(ptr, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return FICP_OK;
}

int ficp_host_free(void *ptr) {
    if (ptr) HIPCHK(hipHostFree(ptr));
    return FICP_OK;
}

int ficp_host_copy(void *dst, const void *src, int64_t bytes) {
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return fail(FICP_EINVAL, "bad arguments");
    char *d = (char *)dst;
    const char *s = (const char *)src;
    // 2 MiB pieces per thread at least (host_parallel); each piece with streaming stores when
    // the destination is 16-B aligned: a plain memcpy of a ~1.5 MiB piece stays under
    // glibc's non-temporal threshold and reads every destination line first (FICP_HOST_NT=0:
    // plain memcpy)
    static const bool nt = !(getenv("FICP_HOST_NT") && atoi(getenv("FICP_HOST_NT")) == 0);
    host_parallel((bytes + 15) / 16, [&](int64_t a, int64_t b) {
        const int64_t lo = a * 16, hi = std::min<int64_t>(b * 16, bytes);
        if (hi <= lo) return;
        if (nt) stream_copy(d + lo, s + lo, (size_t)(hi - lo));
        else memcpy(d + lo, s + lo, (size_t)(hi - lo));
    });
    return FICP_OK;
}

int ficp_memcpy_h2d(ficp_ctx *c, void *dst, const void *src, int64_t bytes) {
    CHK(check_ctx(c));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return sync(c);
}

int ficp_memcpy_d2h(ficp_ctx *c, void *dst, const void *src, int64_t bytes) {
    CHK(check_ctx(c));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return sync(c);
}

int ficp_memcpy_d2d(ficp_ctx *c, void *dst, const void *src, int64_t bytes) {
    CHK(check_ctx(c));
    if (bytes < 0) return fail(FICP_EINVAL, "negative size");
    // aligned, disjoint buffers: one copy kernel (C3's 16 MB x, y reset: 7.5 us against
    // 9.3 us for the runtime's blit; the step rate is within noise either way);
    // FICP_D2D_KERNEL=0: hipMemcpyAsync
    static const bool kern = [] {
        const char *e = getenv("FICP_D2D_KERNEL");
        return !(e && atoi(e) == 0);
    }();
    const uintptr_t d = (uintptr_t)dst, s = (uintptr_t)src;
    if (kern && bytes >= 16 && ((d | s | (uintptr_t)bytes) & 15) == 0 &&
        (d + (uintptr_t)bytes <= s || s + (uintptr_t)bytes <= d)) {
        HIPCHK(launch_copy16(src, dst, bytes / 16, c->stream));
        return FICP_OK;
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    return FICP_OK;
}

int ficp_synchronize(ficp_ctx *c) {
    CHK(check_ctx(c));
    return sync(c);
}


// ===================================================================== distributed runs
// One plot over several ranks, every step enqueued on the context's
// stream -- the caller's stream after ficp_set_stream, on which it also runs its
// collectives -- so no step waits for the host; the host reads one done flag per
// iteration (ficp_dist_wait), one iteration behind.
int ficp_set_stream(ficp_ctx *c, void *stream) {
    CHK(check_ctx(c));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (!c->own_stream) c->own_stream = c->stream;
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    if (c->stream == c->own_stream) c->own_stream = nullptr;
    return FICP_OK;
}

int ficp_dist_begin(ficp_ctx *c, int32_t mode, double *x, double *y, const double *z,
                    int64_t n_local, int64_t n_total, int64_t n_max, int64_t row0,
                    int32_t nstages, const double *lambdas, double threshold,
                    int32_t max_iterations, int32_t allow_reflection, double pivot_x,
                    double pivot_y, int32_t world, int32_t capd) {
    CHK(check_ctx(c));
    if (mode != 1 && mode != 2) return fail(FICP_EINVAL, "mode must be 1 (target) or 2 (source)");
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    if (n_local <= 0 || n_local > 0x3fffffff || n_total < n_local || n_max < n_local ||
        row0 < 0 || row0 + n_local > n_total || n_total > 0x7fffffff || !x || !y ||
        (c->md == 3 && !z) || nstages < 0 || nstages > kLamIn || (nstages > 0 && !lambdas) ||
        world < 1 || capd < 1)
        return fail(FICP_EINVAL, "bad arguments");
    if (mode == 1 && n_local != n_total) return fail(FICP_EINVAL, "target mode replicates the rows");
    if (c->m > kMaxGridStems) return fail(FICP_EINVAL, "the distributed run needs the grid NN");
    c->nn_mode = 2;  // the steps below are written for the grid kernels (any layer size)
    c->dist_mode = 0;
    c->dist_n = n_local;
    c->dist_ntot = n_total;
    c->dist_nmax = n_max;
    c->dist_nws = std::max<int64_t>(n_local, (int64_t)world * capd);
    c->dist_calls = 0;
    c->dist_px = pivot_x;
    c->dist_py = pivot_y;
    c->dist_refl = allow_reflection;
    c->dist_x = x;
    c->dist_y = y;
    c->dist_z = c->md == 3 ? z : nullptr;
    CHK(ensure_work(c, n_local));
    CHK(c->sel_tmp.ensure(sel_tmp_bytes(c->dist_nws)));
    if (c->sel_tmp.gen != c->sel_init_gen) {
        HIPCHK(launch_select_init(c->sel_tmp.p, c->dist_nws, c->stream));
        c->sel_init_gen = c->sel_tmp.gen;
    }
    CHK(c->drange.ensure(16));
    if (mode == 2) {  // this rank's rows in the spatial work order of the whole layer's grid
        CHK(ensure_bbox(c));
        BSJob gj{}, wj{};
        CHK(ensure_grid(c, &gj));
        CHK(build_work_order(c, x, y, c->dist_z, n_local, &wj));
        if (gj.n > 0 || wj.n > 0)
            HIPCHK(launch_bsort2(gj.n > 0 ? gj : wj, gj.n > 0 ? wj : BSJob{}, c->stream));
    }
    CHK(c->gorig.ensure(n_local * 4));
    hipLaunchKernelGGL(k_dist_gorig, dim3((unsigned)((n_local + 255) / 256)), dim3(256), 0,
                       c->stream, mode == 2 ? c->worig.as<uint32_t>() : nullptr, n_local, row0,
                       c->gorig.as<uint32_t>());
    HIPCHK(hipGetLastError());
    LoopCtl lc{};
    lc.nstages = nstages;
    lc.max_iter = max_iterations;
    lc.threshold = threshold;
    for (int e = 0; e < kLamIn; ++e) lc.lam_in[e] = e < nstages ? lambdas[e] : 0.0;
    // k of every call (one store per call by the loop step): ficp_dist_end's trace_k
    CHK(c->tr_k.ensure((size_t)kDistTrace * 8));
    lc.max_trace = kDistTrace;
    lc.tk = c->tr_k.as<long long>();
    // the target mode's shard NN never skips a call (its index offset is added per call),
    // so n_nn_reused stays 0 there
    lc.no_reuse_count = mode == 1;
    c->dist_lc = lc;
    HIPCHK(launch_loop_init(c->state_dev.as<IterState>(), lc, c->stream));
    c->dist_mode = mode;
    return FICP_OK;
}

/* the fit of ficp.py:134 from the previous selection, this rank's rows: 8 sums (device) */
int ficp_dist_fit_sums(ficp_ctx *c, double *sums8) {
    CHK(check_ctx(c));
    if (!c->dist_mode || !sums8) return fail(c->dist_mode ? FICP_EINVAL : FICP_ESTATE, "bad call");
    IterState *st = c->state_dev.as<IterState>();
    const bool src = c->dist_mode == 2;
    FitIn fa{src ? c->wx.as<double>() : c->dist_x, src ? c->wy.as<double>() : c->dist_y,
             c->ccx.as<double>(), c->ccy.as<double>(), c->key.as<unsigned long long>(), nullptr,
             c->gorig.as<uint32_t>(), c->dist_n, c->dist_px, c->dist_py, st};
    HIPCHK(launch_fit_sums(fa, c->fit_tmp.p, &st->no_fit, sums8, c->stream));
    return FICP_OK;
}

/* the solve on the ranks' sums (world x 8, added in rank order); target mode also
   applies T to the replicated rows here (source mode applies it in the NN step) */
int ficp_dist_fit_solve(ficp_ctx *c, const double *sums, int32_t world) {
    CHK(check_ctx(c));
    if (!c->dist_mode || !sums || world < 1) return fail(c->dist_mode ? FICP_EINVAL : FICP_ESTATE, "bad call");
    IterState *st = c->state_dev.as<IterState>();
    HIPCHK(launch_fit_solve_ranks(sums, world, c->dist_px, c->dist_py, c->dist_refl, st,
                                  &st->no_fit, c->stream));
    if (c->dist_mode == 1)
        HIPCHK(launch_apply_xy_flags(c->dist_x, c->dist_y, c->dist_n, st->T, &st->done, &st->apply,
                                     c->stream));
    return FICP_OK;
}

/* target mode: NN of the replicated rows against this context's shard (as ficp_nn_device),
   a no-op once the controller's run is over */
int ficp_dist_nn_shard(ficp_ctx *c, ficp_ctx *ctrl, int64_t idx_offset, double *d2, int32_t *idx) {
    CHK(check_dist(ctrl, 1));
    CHK(check_ctx(c));
    if (!c->has_target) return fail(FICP_ESTATE, "no target set");
    const int64_t n = ctrl->dist_n;
    if (!d2 || !idx || idx_offset < 0 || idx_offset + c->m > 0x7fffffff)
        return fail(FICP_EINVAL, "bad arguments");
    if (c->stream != ctrl->stream) return fail(FICP_ESTATE, "shard and controller streams differ");
    if (c->m == 0) {
        HIPCHK(launch_fill_inf(d2, idx, n, c->stream));
        return FICP_OK;
    }
    CHK(ensure_work(c, n));
    NNArgs a{};
    a.sx = ctrl->dist_x;
    a.sy = ctrl->dist_y;
    a.sz = c->md == 3 ? ctrl->dist_z : nullptr;
    a.n = n;
    a.idx = idx;
    a.r = d2;
    a.tx = c->tx.as<double>();
    a.ty = c->ty.as<double>();
    a.skip = &ctrl->state_dev.as<IterState>()->done;
    if (c->m > kMaxGridStems) return fail(FICP_EINVAL, "the distributed run needs the grid NN");
    c->nn_mode = 2;
    CHK(ensure_bbox(c));
    CHK(ensure_grid(c));
    HIPCHK(launch_nn_grid(a, c->gv, c->md, c->stream, false));
    HIPCHK(launch_add_offset(idx, n, idx_offset, c->stream));
    return FICP_OK;
}

/* target mode: the merged (d2, idx) -> selection + loop step (ficp.py:73-86, 122-154);
   the iteration's done flag goes to slot `iteration` of the pinned ring */
int ficp_dist_select_merged(ficp_ctx *c, const double *d2, const int32_t *idx, const double *tx,
                            const double *ty, int64_t iteration) {
    CHK(check_dist(c, 1));
    if (!d2 || !idx || !tx || !ty || iteration < 0) return fail(FICP_EINVAL, "bad arguments");
    const int64_t n = c->dist_n;
    IterState *st = c->state_dev.as<IterState>();
    HIPCHK(launch_corr_from_merge(d2, idx, tx, ty, n, c->key.as<unsigned long long>(),
                                  c->r.as<double>(), c->ccx.as<double>(), c->ccy.as<double>(),
                                  range_ptr(c), c->stream));
    const int slot = (int)(iteration % kLoopRing);
    __atomic_store_n(&c->h_flags[slot], -1, __ATOMIC_RELAXED);
    HIPCHK(launch_select(c->key.as<unsigned long long>(), nullptr, c->r.as<double>(), n, 0.0,
                         &st->lam_cur, range_ptr(c), (n + 255) / 256, c->sel_tmp.p, st, &st->done,
                         &c->dist_lc, &c->h_flags[slot], c->stream, nullptr));
    c->dist_calls += 1;
    return FICP_OK;
}

/* source mode: NN of this rank's rows (T applied first, certified reuse from the second
   call) against the whole layer; range2 (int64[2], device) = the rows' key range words
   for the caller's MAX all-reduce */
int ficp_dist_nn_local(ficp_ctx *c, int64_t *range2) {
    CHK(check_dist(c, 2));
    if (!range2) return fail(FICP_EINVAL, "bad arguments");
    IterState *st = c->state_dev.as<IterState>();
    CHK(nn_call(c, c->wx.as<double>(), c->wy.as<double>(), c->md == 3 ? c->wz.as<double>() : nullptr,
                c->dist_n, st->T, true, c->dist_calls == 0 ? 1 : 2, &st->done, &st->apply, true,
                false, &st->nn_reuse));
    hipLaunchKernelGGL(k_dist_range_out, dim3(1), dim3(64), 0, c->stream, range_ptr(c),
                       (long long *)range2, &st->done);
    HIPCHK(hipGetLastError());
    return FICP_OK;
}

/* source mode: the local histogram under the global range (int64[2] from the MAX
   all-reduce) -> hist (int64[2 * 8192], device) for the caller's SUM all-reduce */
int ficp_dist_hist(ficp_ctx *c, const int64_t *range2, int64_t *hist) {
    CHK(check_dist(c, 2));
    if (!range2 || !hist) return fail(FICP_EINVAL, "bad arguments");
    IterState *st = c->state_dev.as<IterState>();
    hipLaunchKernelGGL(k_dist_range_in, dim3(1), dim3(64), 0, c->stream, (const long long *)range2,
                       range_ptr(c), &st->done);
    HIPCHK(hipGetLastError());
    HIPCHK(launch_select_dist_hist(c->key.as<unsigned long long>(), c->r.as<double>(), c->dist_n,
                                   c->dist_nmax, range_ptr(c), c->sel_tmp.p, c->dist_nws, st,
                                   &st->done, (long long *)hist, c->stream));
    return FICP_OK;
}

int ficp_dist_hist_words(void) { return sel_hist_words(); }

/* source mode: bounds from the summed histogram, this rank's candidates packed into
   pack (int64[4 + 3 capd], device) for the caller's all-gather */
int ficp_dist_candidates(ficp_ctx *c, const int64_t *hist, int64_t *pack, int32_t capd) {
    CHK(check_dist(c, 2));
    if (!hist || !pack || capd < 1) return fail(FICP_EINVAL, "bad arguments");
    IterState *st = c->state_dev.as<IterState>();
    HIPCHK(launch_select_dist_gather(c->key.as<unsigned long long>(), c->gorig.as<uint32_t>(),
                                     c->r.as<double>(), c->dist_n, c->dist_ntot, c->dist_nmax,
                                     (const long long *)hist, 0.0, &st->lam_cur, c->sel_tmp.p,
                                     c->dist_nws, &st->done, (long long *)pack, capd, c->stream));
    return FICP_OK;
}

/* source mode: the final selection on the gathered packs (world x (4 + 3 capd), rank
   order) + the loop step; the done flag goes to slot `iteration` of the pinned ring */
int ficp_dist_final(ficp_ctx *c, const int64_t *packs, int32_t world, int32_t capd,
                    int64_t iteration) {
    CHK(check_dist(c, 2));
    if (!packs || world < 1 || capd < 1 || (int64_t)world * capd > c->dist_nws || iteration < 0)
        return fail(FICP_EINVAL, "bad arguments");
    IterState *st = c->state_dev.as<IterState>();
    const int slot = (int)(iteration % kLoopRing);
    __atomic_store_n(&c->h_flags[slot], -1, __ATOMIC_RELAXED);
    HIPCHK(launch_select_dist_final((const long long *)packs, world, capd, c->dist_ntot, 0.0,
                                    &st->lam_cur, c->sel_tmp.p, c->dist_nws, st, &st->done,
                                    &c->dist_lc, &c->h_flags[slot], c->stream));
    c->dist_calls += 1;
    return FICP_OK;
}

/* host: wait for iteration `iteration`'s done flag (*done = 1: the run is over) */
int ficp_dist_wait(ficp_ctx *c, int64_t iteration, int32_t *done) {
    CHK(check_ctx(c));
    if (!c->dist_mode || !done || iteration < 0) return fail(FICP_EINVAL, "bad call");
    int v = 0;
    CHK(poll_flag(c, &c->h_flags[iteration % kLoopRing], v));
    *done = (v & kFlagDone) != 0;
    return FICP_OK;
}

/* end of the run: source mode writes this rank's XY back to the caller's rows; stats as
   ficp_run's (without traces) */
int ficp_dist_end(ficp_ctx *c, ficp_stats *st) {
    CHK(check_ctx(c));
    if (!c->dist_mode) return fail(FICP_ESTATE, "no distributed run begun");
    const int mode = c->dist_mode;
    c->dist_mode = 0;
    if (mode == 2)
        HIPCHK(launch_scatter_xy(c->worig.as<uint32_t>(), c->wx.as<double>(), c->wy.as<double>(),
                                 c->dist_n, c->dist_x, c->dist_y, c->stream));
    c->h_rep->misc[1] = c->h_rep->misc[2] = c->h_rep->misc[3] = 0u;
    CHK(report_wait(c, ReportSeg{c->state_dev.p, &c->h_rep->st, (int)(sizeof(IterState) / 4)},
                    ReportSeg{sel_err_word(c->sel_tmp.p, c->dist_nws), &c->h_rep->misc[1], 3},
                    ReportSeg{}));
    const IterState &h = c->h_rep->st;
    if (!h.done) return fail(FICP_EHIP, "distributed ICP loop did not finish");
    if (c->h_rep->misc[1] & 2u)
        return fail(FICP_EHIP, "ERR_CAP: a rank's selection candidates exceeded the pack capacity");
    if (c->h_rep->misc[1]) return fail(FICP_EHIP, "%s", sel_err_text(c->h_rep->misc[1]).c_str());
    if (st) {
        st->n_nn_calls = h.n_nn;
        st->n_nn_reused = h.n_reuse;
        st->n_fits = h.n_fit;
        st->iters[0] = h.iters[0];
        st->iters[1] = h.iters[1];
        st->k_last = h.k_last;
        st->frmsd_last[0] = h.frmsd_last[0];
        st->frmsd_last[1] = h.frmsd_last[1];
        memcpy(st->T_total, h.Ttot, sizeof st->T_total);
        st->gpu_ms = 0.0;
        for (double &hm : st->host_ms) hm = 0.0;
        st->path = 0;
        const int nc = std::min(std::min(h.n_nn, st->max_trace), kDistTrace);
        if (nc > 0 && st->trace_k) {
            HIPCHK(hipMemcpyAsync(st->trace_k, c->tr_k.p, (size_t)nc * 8, hipMemcpyDeviceToHost,
                                  c->stream));
            CHK(sync(c));
        }
    }
    return FICP_OK;
}

}  // extern "C"
