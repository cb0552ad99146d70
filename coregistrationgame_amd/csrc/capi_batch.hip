// capi_batch.hip -- ficp_run_batch / ficp_run_batch_device: many independent plots per
// device pass (BASELINE config C4, 1024 plots x 10k trees vs 10k CHM stems).
//
// The reference joins plots one at a time (App.join_plot, app.py:630-661, one
// FractionalICP(...).run() per plot).  Here every plot's CHM grid lives in one set of
// arrays (per-plot geometry, global cell ids), and one batch iteration advances every
// live plot by one step of ficp.py:122-147:
//
//   batch_fit    (LOOP plots: fit on the plot's selection, T kept in the plot's state)
//   -> nn_grid_batch (applies T, exact 1-NN against the plot's own grid, keys + r)
//   -> batch_select  (one workgroup per plot: FRMSD-optimal k + selection threshold)
//   -> batch_update  (per-plot convergence test ficp.py:142, stage switch ficp.py:152)
//
// The update kernel stores the number of plots still running into a ring of coherent
// pinned words; the host enqueues batch iteration i + 1 before it polls iteration i's
// word, so the device never idles on the host.  A finished batch leaves one iteration
// of no-op launches queued (every kernel skips converged plots).
#include "capi_internal.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

struct BatchBufs {
    DevBuf so, to, plot_of, tplot, grids, st, bb, lams;
    DevBuf cell_of, counts, fill, cell_start, pts, scan_tmp, bs_tmp;
    DevBuf key, gap, r, ccx, ccy, bp, dz2, wkey, skey, wrow, srow, wr, sr;
    DevBuf sx, sy, sz, tx, ty, tz, stage;  // staging of the host entry point
    DevBuf wx, wy, wz, worig;              // the trees in the batch work order (k_bsort mode 3)
    DevBuf fpart, fctr;                    // batch fit: per-chunk sums, per-plot arrivals
    DevBuf arrive;                         // fused step: per sub-batch arrival/live counter
    unsigned fctr_init_gen = 0;            // fctr allocation whose counters are zeroed
    int *h_flag = nullptr;                 // coherent pinned ring: plots still running
    PinBuf up{nullptr, 0, hipHostMallocCoherent};  // the small per-run uploads (k_batch_init reads them)
    PinBuf rep{nullptr, 0, hipHostMallocCoherent};  // report kernel target: states + flag
    static constexpr int kSubMax = 4;
    hipStream_t ss[kSubMax] = {};          // sub-batch streams 1.. (0 is the context's)
    hipEvent_t fork = nullptr, join[kSubMax] = {};
};
constexpr int kBatchRing = 4;
constexpr int kMaxSub = BatchBufs::kSubMax;  // sub-batches on their own streams (h_flag: kMaxSub rings)

void batch_release(BatchBufs *b) {
    if (!b) return;
    DevBuf *bufs[] = {&b->so,       &b->to,      &b->plot_of,  &b->tplot, &b->grids, &b->st,
                      &b->bb,      &b->lams,     &b->cell_of, &b->counts,
                      &b->fill,     &b->cell_start, &b->pts,   &b->scan_tmp, &b->key, &b->gap,
                      &b->r,        &b->ccx,     &b->ccy,      &b->wkey,  &b->skey,  &b->wrow,
                      &b->srow,     &b->wr,      &b->sr,       &b->sx,    &b->sy,    &b->sz,
                      &b->tx,       &b->ty,      &b->tz,       &b->stage, &b->bp,
                      &b->dz2,      &b->bs_tmp,  &b->fpart,   &b->fctr, &b->arrive,
                      &b->wx,       &b->wy,      &b->wz,      &b->worig};
    for (DevBuf *d : bufs) d->release();
    b->up.release();
    b->rep.release();
    for (int q = 0; q < kMaxSub; ++q) {
        if (b->ss[q]) (void)hipStreamDestroy(b->ss[q]);
        if (b->join[q]) (void)hipEventDestroy(b->join[q]);
    }
    if (b->fork) (void)hipEventDestroy(b->fork);
    if (b->h_flag) (void)hipHostFree(b->h_flag);
    delete b;
}

namespace {

int check_offsets(const int64_t *off, int32_t nplots, const char *what, int64_t &total) {
    if (!off) return fail(FICP_EINVAL, "null %s offsets", what);
    if (off[0] != 0) return fail(FICP_EINVAL, "%s offsets must start at 0", what);
    for (int32_t p = 0; p < nplots; ++p)
        if (off[p + 1] < off[p]) return fail(FICP_EINVAL, "%s offsets must be non-decreasing", what);
    total = off[nplots];
    return FICP_OK;
}

BatchBufs *batch_of(ficp_ctx *c) {
    if (!c->batch) c->batch = new BatchBufs();
    return c->batch;
}

// The trees of a batch job: their columns, count and (device) plot of every tree.
struct BatchTrees {
    const double *x, *y, *z;
    int64_t n;
    const int32_t *plot;
    const int64_t *off_h, *off_d;  // per-plot row offsets (host, device)
};

// per-plot CHM grids in one set of arrays (cells of plot p: cell_base_p .. +gx*gy-1) and,
// with trees.n > 0, the batch work order of the trees in the same four bucket-sort launches
// (k_bsort.hip modes 2 and 3: plot, then 8x8-cell supertile of the plot's grid, then cell,
// then caller row) into b.wx / wy / wz / worig.  Returns in *work whether it was built.
int build_batch_grids(ficp_ctx *c, BatchBufs &b, int32_t nplots, const int64_t *to_h,
                      const double *tx, const double *ty, const double *tz, int64_t m, int md,
                      std::vector<PlotGrid> &grids, const BatchTrees &trees, bool *work) {
    *work = false;
    CHK(b.bb.ensure((size_t)nplots * 4 * 8));
    HIPCHK(launch_batch_bbox(tx, ty, b.to.as<int64_t>(), nplots, b.bb.as<double>(), c->stream));
    // the bboxes through the report kernel into coherent pinned memory and a polled flag
    // (a pageable D2H copy + stream sync cost more idle device)
    const size_t bbytes = (size_t)nplots * 4 * 8;
    CHK(b.rep.ensure(std::max<size_t>(bbytes, (size_t)nplots * sizeof(PlotState)) + 64));
    int *bflag = (int *)(b.rep.as<char>() + bbytes + 32);
    __atomic_store_n(bflag, -1, __ATOMIC_RELAXED);
    HIPCHK(launch_report(ReportSeg{b.bb.p, b.rep.p, (int)(bbytes / 4)}, ReportSeg{}, ReportSeg{},
                         bflag, nullptr, c->stream));
    {
        int v = 0;
        CHK(poll_flag(c, bflag, v));
    }
    const double *bb = b.rep.as<const double>();
    grids.assign(nplots, PlotGrid{});
    int64_t ncells = 0, nwkeys = 0;
    int64_t ps_pts = 0, ps_keys = 0;  // the per-plot sort's largest plot (points, keys)
    for (int32_t p = 0; p < nplots; ++p) {
        PlotGrid &g = grids[p];
        const int64_t mp = to_h[p + 1] - to_h[p];
        g.m = (int)mp;
        g.cell_base = ncells;
        g.wbase = nwkeys;
        // (every plot's trees, those of plots without stems included, fit the plot sort or not)
        if (trees.n > 0) ps_pts = std::max<int64_t>(ps_pts, trees.off_h[p + 1] - trees.off_h[p]);
        if (mp == 0) {  // no CHM stems: the plot never runs (ficp.py:66-68, 125-126)
            g.x0 = g.y0 = g.px = g.py = 0.0;
            g.h = g.inv_h = 1.0;
            g.gx = g.gy = 1;
            ncells += 1;
            nwkeys += 64;
            continue;
        }
        const double x0 = bb[4 * p], x1 = bb[4 * p + 1], y0 = bb[4 * p + 2], y1 = bb[4 * p + 3];
        if (!(std::isfinite(x0) && std::isfinite(x1) && std::isfinite(y0) && std::isfinite(y1)))
            return fail(FICP_EINVAL, "plot %d: target coordinates must be finite", (int)p);
        double h, margin;
        int64_t gx, gy;
        plan_grid(x0, x1, y0, y1, mp, h, gx, gy, margin);
        g.x0 = x0;
        g.y0 = y0;
        g.h = h;
        g.inv_h = 1.0 / h;
        g.margin = margin;
        g.gx = (int)gx;
        g.gy = (int)gy;
        g.px = x0 + 0.5 * (x1 - x0);  // fit pivot: the plot's CHM bbox centre
        g.py = y0 + 0.5 * (y1 - y0);
        ncells += gx * gy;
        nwkeys += ((gx + 7) / 8) * ((gy + 7) / 8) * 64;  // (k_bsort.hip st_key's range)
        ps_keys = std::max<int64_t>(ps_keys, ((gx + 7) / 8) * ((gy + 7) / 8) * 64);  // (>= gx * gy)
        ps_pts = std::max<int64_t>(ps_pts, mp);
    }
    if (ncells > 0x7ffffffe) return fail(FICP_EINVAL, "batch grid too large");
    CHK(b.grids.ensure((size_t)nplots * sizeof(PlotGrid)));
    HIPCHK(hipMemcpyAsync(b.grids.p, grids.data(), (size_t)nplots * sizeof(PlotGrid),
                          hipMemcpyHostToDevice, c->stream));
    CHK(b.cell_start.ensure((ncells + 1) * 4));
    CHK(b.pts.ensure(m * sizeof(TPt)));
    // Plots that fit one workgroup (C4: 10k stems and trees): the per-plot LDS sort of both
    // jobs in one launch (k_batch.hip k_plot_sort, the same order as the bucket sort below).
    // FICP_PLOT_SORT=0: the bucket sort.
    const char *pse = getenv("FICP_PLOT_SORT");
    if (plot_sort_fits(ps_pts, ps_keys) && !(pse && atoi(pse) == 0) && !getenv("FICP_GRID_ATOMIC")) {
        PlotSortJob gjob{};
        gjob.x = tx;
        gjob.y = ty;
        gjob.z = md == 3 ? tz : nullptr;
        gjob.off = b.to.as<int64_t>();
        gjob.mode = 0;
        gjob.pts = b.pts.as<TPt>();
        gjob.cell_start = b.cell_start.as<int32_t>();
        PlotSortJob wjob{};
        if (trees.n > 0) {
            CHK(b.wx.ensure(trees.n * 8));
            CHK(b.wy.ensure(trees.n * 8));
            if (md == 3) CHK(b.wz.ensure(trees.n * 8));
            CHK(b.worig.ensure(trees.n * 4));
            wjob.x = trees.x;
            wjob.y = trees.y;
            wjob.z = md == 3 ? trees.z : nullptr;
            wjob.off = trees.off_d;
            wjob.mode = 1;
            wjob.wx = b.wx.as<double>();
            wjob.wy = b.wy.as<double>();
            wjob.wz = md == 3 ? b.wz.as<double>() : nullptr;
            wjob.worig = b.worig.as<uint32_t>();
        }
        HIPCHK(launch_plot_sort(gjob, trees.n > 0 ? &wjob : nullptr, b.grids.as<PlotGrid>(), nplots, c->stream));
        *work = trees.n > 0;
        return FICP_OK;
    }
    // the bucket sort and the atomic grid build key the stems by their plot
    CHK(b.tplot.ensure(m * 4));
    HIPCHK(launch_fill_plot_ids(b.to.as<int64_t>(), nplots, b.tplot.as<int32_t>(), c->stream));
    // the work order's job (mode 3), when the bucket sort can plan it
    const bool want_work = trees.n > 0 && bsort_supported(trees.n, nwkeys);
    BSortGeom wg{};
    BSortOut wo{};
    if (want_work) {
        CHK(b.wx.ensure(trees.n * 8));
        CHK(b.wy.ensure(trees.n * 8));
        if (md == 3) CHK(b.wz.ensure(trees.n * 8));
        CHK(b.worig.ensure(trees.n * 4));
        wg.mode = 3;
        wg.plot = trees.plot;
        wg.grids = b.grids.as<PlotGrid>();
        wo.wx = b.wx.as<double>();
        wo.wy = b.wy.as<double>();
        wo.wz = md == 3 ? b.wz.as<double>() : nullptr;
        wo.worig = b.worig.as<uint32_t>();
    }
    const int64_t wtmp = want_work ? bsort_tmp_bytes(trees.n, nwkeys) : 0;
    if (bsort_supported(m, ncells) && !getenv("FICP_GRID_ATOMIC")) {
        // the two-level bucket sort of the single-plot grid (k_bsort.hip) keyed by the
        // global cell id of each stem's plot grid: 1.3 -> ~0.25 ms per 1024-plot batch;
        // the trees' work order rides in the same four launches (as the single plot's)
        const int64_t gtmp = bsort_tmp_bytes(m, ncells);
        CHK(b.bs_tmp.ensure(gtmp + wtmp));
        BSortGeom bg{};
        bg.mode = 2;
        bg.plot = b.tplot.as<int32_t>();
        bg.grids = b.grids.as<PlotGrid>();
        BSortOut bo{};
        bo.pts = b.pts.as<TPt>();
        bo.cell_start = b.cell_start.as<int32_t>();
        const BSJob gj = bsort_job(tx, ty, md == 3 ? tz : nullptr, m, bg, ncells, bo, b.bs_tmp.p);
        const BSJob wj = want_work ? bsort_job(trees.x, trees.y, md == 3 ? trees.z : nullptr, trees.n, wg,
                                               nwkeys, wo, b.bs_tmp.as<char>() + gtmp)
                                   : BSJob{};
        HIPCHK(launch_bsort2(gj, wj, c->stream));
        *work = want_work;
        return FICP_OK;
    }
    if (want_work) {
        CHK(b.bs_tmp.ensure(wtmp));
        HIPCHK(launch_bsort(trees.x, trees.y, md == 3 ? trees.z : nullptr, trees.n, wg, nwkeys, wo,
                            b.bs_tmp.p, c->stream));
        *work = true;
    }
    // counting sort with global atomics (grids the bucket sort cannot plan)
    CHK(b.cell_of.ensure(m * 4));
    CHK(b.counts.ensure((ncells + 1) * 4));
    CHK(b.fill.ensure((ncells + 1) * 4));
    CHK(b.scan_tmp.ensure(scan_tmp_elems(ncells) * 4 + 64));
    HIPCHK(launch_atomic_zero32((uint32_t *)b.counts.p, ncells + 1, c->stream));
    HIPCHK(launch_atomic_zero32((uint32_t *)b.fill.p, ncells + 1, c->stream));
    HIPCHK(launch_batch_grid_count(tx, ty, m, b.tplot.as<int32_t>(), b.grids.as<PlotGrid>(),
                                   b.cell_of.as<int32_t>(), b.counts.as<int32_t>(), c->stream));
    HIPCHK(launch_scan_i32(b.counts.as<int32_t>(), b.cell_start.as<int32_t>(), ncells,
                           b.scan_tmp.as<int32_t>(), true, c->stream));
    HIPCHK(launch_grid_scatter(tx, ty, md == 3 ? tz : nullptr, m, b.cell_of.as<int32_t>(),
                               b.cell_start.as<int32_t>(), b.fill.as<int32_t>(), b.pts.as<TPt>(),
                               c->stream));
    HIPCHK(launch_grid_sort_cells(b.pts.as<TPt>(), b.cell_start.as<int32_t>(), ncells, c->stream));
    return FICP_OK;
}

int batch_core(ficp_ctx *c, int32_t nplots, const int64_t *so_h, double *sx, double *sy,
               const double *sz, const int64_t *to_h, const double *tx, const double *ty,
               const double *tz, int md, int32_t nstages, const double *lambdas,
               double threshold, int32_t max_iter, int32_t allow_refl,
               ficp_plot_stats *per_plot) {
    const int64_t n = so_h[nplots], m = to_h[nplots];
    BatchBufs &b = *batch_of(c);
    if (!b.h_flag)
        HIPCHK(hipHostMalloc((void **)&b.h_flag, kMaxSub * kBatchRing * sizeof(int),
                             hipHostMallocCoherent));
    CHK(b.so.ensure((size_t)(nplots + 1) * 8));
    CHK(b.to.ensure((size_t)(nplots + 1) * 8));
    CHK(b.st.ensure((size_t)nplots * sizeof(PlotState)));
    CHK(b.lams.ensure((size_t)std::max(nstages, 1) * 8));
    CHK(b.arrive.ensure(kMaxSub * 8));
    {
        // offsets and lambdas through coherent pinned staging, read by k_batch_init itself
        // (three staged copies were three runtime blit launches); the previous run of this
        // context has finished with it
        const size_t off = (size_t)(nplots + 1) * 8, nl = (size_t)std::max(nstages, 0) * 8;
        CHK(b.up.ensure(2 * off + nl + 64));
        char *u = b.up.as<char>();
        memcpy(u, so_h, off);
        memcpy(u + off, to_h, off);
        if (nl) memcpy(u + 2 * off, lambdas, nl);
        BatchInitArgs ia{};
        ia.so_h = (const int64_t *)u;
        ia.to_h = (const int64_t *)(u + off);
        ia.lam_h = (const double *)(u + 2 * off);
        ia.so = b.so.as<int64_t>();
        ia.to = b.to.as<int64_t>();
        ia.lams = b.lams.as<double>();
        // the fused step's arrival counters start at zero (each launch's last workgroup
        // resets its own); zeroed here, so an earlier failed run leaves none
        ia.arrive = b.arrive.as<unsigned long long>();
        ia.nplots = nplots;
        ia.nstages = nstages;
        ia.nl = (int)(nl / 8);
        ia.narrive = kMaxSub;
        ia.st = b.st.as<PlotState>();
        HIPCHK(launch_batch_init(ia, c->stream));
    }
    bool work = false;  // the trees run in the batch work order (b.wx, wy, wz, worig)
    if (n > 0 && m > 0 && nstages > 0) {
        std::vector<PlotGrid> grids;
        CHK(b.plot_of.ensure(n * 4));
        HIPCHK(launch_fill_plot_ids(b.so.as<int64_t>(), nplots, b.plot_of.as<int32_t>(),
                                    c->stream));
        {
            // FICP_BATCH_WORK=0: the trees stay in caller order
            const char *we = getenv("FICP_BATCH_WORK");
            const bool want = !(we && atoi(we) == 0);
            const BatchTrees trees{sx, sy, md == 3 ? sz : nullptr, want ? n : 0, b.plot_of.as<int32_t>(),
                                   so_h, b.so.as<int64_t>()};
            ProfScope ps(c, P_GRID, "batch_grid_build");
            CHK(build_batch_grids(c, b, nplots, to_h, tx, ty, tz, m, md, grids, trees, &work));
        }
        // the columns the batch iterations read and move: the work order's, or the caller's
        double *qx = work ? b.wx.as<double>() : sx;
        double *qy = work ? b.wy.as<double>() : sy;
        const double *qz = (md == 3) ? (work ? b.wz.as<double>() : sz) : nullptr;
        const uint32_t *worig = work ? b.worig.as<uint32_t>() : nullptr;
        CHK(b.gap.ensure(n * sizeof(gap_t)));
        CHK(b.dz2.ensure(n * 8));
        CHK(b.r.ensure(n * 8));
        CHK(b.ccx.ensure(n * 8));
        CHK(b.ccy.ensure(n * 8));
        CHK(b.bp.ensure(n * 4));
        CHK(b.wkey.ensure(n * 8));
        CHK(b.skey.ensure(n * 8));
        CHK(b.wrow.ensure(n * 4));
        CHK(b.srow.ensure(n * 4));
        CHK(b.wr.ensure(n * 8));
        CHK(b.sr.ensure(n * 8));
        const BatchSelScratch ws{b.wkey.as<unsigned long long>(), b.skey.as<unsigned long long>(),
                                 b.wrow.as<uint32_t>(), b.srow.as<uint32_t>(), b.wr.as<double>(),
                                 b.sr.as<double>(), worig};
        int64_t max_rows = 0;
        for (int32_t p = 0; p < nplots; ++p) max_rows = std::max(max_rows, so_h[p + 1] - so_h[p]);
        NNArgs a{};
        a.sx = qx;
        a.sy = qy;
        a.sz = qz;
        a.n = n;
        a.idx = nullptr;  // the batch returns XY and per-plot records, not the NN index
        a.r = b.r.as<double>();
        // the NN stores no sort keys: the selection and the fit derive each from its row's r
        // (key_of_r, the NN's own operations), 8 B per tree and call less written and read.
        // FICP_BATCH_KEYS=1: stored keys.
        const char *bke = getenv("FICP_BATCH_KEYS");
        const bool keys_stored = bke && atoi(bke) != 0;
        a.key = nullptr;
        a.cx = b.ccx.as<double>();
        a.cy = b.ccy.as<double>();
        a.tx = tx;
        a.ty = ty;
        a.range = nullptr;
        a.out_bp = b.bp.as<int32_t>();
        if (keys_stored) {
            CHK(b.key.ensure(n * 8));
            a.key = b.key.as<unsigned long long>();
        }
        // certified reuse of each query's match (k_grid_nn.hip cert_try): the first call
        // of the batch is cold (every plot starts there), the rest are warm
        a.gap = b.gap.as<gap_t>();
        a.dz2 = md == 3 ? b.dz2.as<double>() : nullptr;
        a.cert_block = 8;
        PlotState *st = b.st.as<PlotState>();
        CHK(b.fpart.ensure((size_t)nplots * (size_t)batch_fit_chunks(max_rows) * 64));
        CHK(b.fctr.ensure((size_t)nplots * 4));
        if (b.fctr.gen != b.fctr_init_gen) {  // fresh allocation: zero its atomic words
            HIPCHK(launch_batch_fit_ctr_zero(b.fctr.as<unsigned>(), nplots, c->stream));
            b.fctr_init_gen = b.fctr.gen;
        }
        // every plot makes at most nstages * (max_iter + 1) NN calls
        const int64_t cap = (int64_t)nstages * ((int64_t)std::max(max_iter, 0) + 1) + 1;
        // From 64 plots on: two sub-batches, each on its own stream, so one half's
        // latency-bound selection (one workgroup per plot) runs beside the other half's
        // NN.  The plots are independent (app.py:658-660), so the split changes no result.
        // Measured with the fused step (tools/batch_ab.sh, plot-it/s): 128 plots 846k vs
        // 834k, 512 1,082k vs 1,019k, 1024 1,119k vs 1,061k.  FICP_BATCH_STREAMS=1..4
        // forces the count.
        int nsub = nplots >= 64 ? 2 : 1;
        if (const char *e = getenv("FICP_BATCH_STREAMS")) nsub = std::max(1, std::min(kMaxSub, atoi(e)));
        // (the fused step's arrival counters were zeroed by k_batch_init, before the fork)
        // the per-call k trace is cleared here too, before the fork: the sub-streams write
        // their plots' rows as soon as the fork event lets them run
        long long *trace = nullptr;  // per-call k of every plot (ficp_set_batch_trace), -1 = none
        if (c->btrace_host && c->btrace_max > 0) {
            const size_t tb = (size_t)nplots * (size_t)c->btrace_max * 8;
            CHK(c->btrace.ensure(tb));
            HIPCHK(hipMemsetAsync(c->btrace.p, 0xff, tb, c->stream));
            trace = c->btrace.as<long long>();
        }
        // Joins the sub-batch streams back into the context's stream on EVERY exit of this
        // scope, error returns included: kernels still queued on a sub-stream must finish
        // before the next run's uploads and memsets on c->stream reuse their buffers.
        struct JoinGuard {
            BatchBufs &b;
            hipStream_t main;
            int forked = 0;  // sub-streams 1 .. forked-1 wait on the fork
            ~JoinGuard() {
                for (int q = 1; q < forked; ++q) {
                    if (b.join[q] && hipEventRecord(b.join[q], b.ss[q]) == hipSuccess &&
                        hipStreamWaitEvent(main, b.join[q], 0) == hipSuccess)
                        continue;
                    (void)hipStreamSynchronize(b.ss[q]);  // cannot join by event: drain it
                }
            }
        } joins{b, c->stream};
        if (nsub > 1) {
            if (!b.fork) HIPCHK(hipEventCreateWithFlags(&b.fork, hipEventDisableTiming));
            HIPCHK(hipEventRecord(b.fork, c->stream));  // the grids, states and offsets are ready
            for (int q = 1; q < nsub; ++q) {
                if (!b.ss[q]) HIPCHK(hipStreamCreateWithFlags(&b.ss[q], hipStreamNonBlocking));
                if (!b.join[q]) HIPCHK(hipEventCreateWithFlags(&b.join[q], hipEventDisableTiming));
                HIPCHK(hipStreamWaitEvent(b.ss[q], b.fork, 0));
                joins.forked = q + 1;
            }
        }
        struct Sub {
            int p0, np;
            int64_t r0, nr;
            hipStream_t s;
            int *ring;
            bool finished;
        };
        Sub subs[kMaxSub];
        for (int q = 0; q < nsub; ++q) {
            Sub &u = subs[q];
            u.p0 = (int)((int64_t)nplots * q / nsub);
            u.np = (int)((int64_t)nplots * (q + 1) / nsub) - u.p0;
            u.r0 = so_h[u.p0];
            u.nr = so_h[u.p0 + u.np] - u.r0;
            u.s = q == 0 ? c->stream : b.ss[q];
            u.ring = b.h_flag + q * kBatchRing;
            u.finished = u.np == 0;
        }
        const size_t fch = (size_t)batch_fit_chunks(max_rows) * 8;  // fit partial doubles per plot
        // the loop step and the next body's fit run inside the selection (one workgroup per
        // plot, its rows L2-hot): two launches per batch iteration fewer.  FICP_BATCH_FUSE=0:
        // the separate k_batch_fit and k_batch_update launches.
        const char *bf = getenv("FICP_BATCH_FUSE");
        const bool bfuse = !(bf && atoi(bf) == 0);
        BatchStepArgs step{qx, qy, b.ccx.as<double>(), b.ccy.as<double>(), b.grids.as<PlotGrid>(),
                           allow_refl, nstages, max_iter, threshold};
        if (trace) step.max_trace = c->btrace_max;
        step.worig = worig;
        auto enqueue = [&](Sub &u, int64_t bit) -> int {
            const int qi = (int)(&u - subs);
            int *flag = &u.ring[bit % kBatchRing];
            __atomic_store_n(flag, -1, __ATOMIC_RELEASE);
            // kernel timing: every sub-batch's launches, with events on its own stream (the
            // NN roofline divides every plot's NN bytes by the sum of the launch times)
            const bool prof = true;
            PlotState *su = st + u.p0;
            const int64_t *sou = b.so.as<int64_t>() + u.p0;
            const PlotGrid *gu = b.grids.as<PlotGrid>() + u.p0;
            if (!bfuse) {
                ProfScope ps(c, prof ? P_FIT : 0, "batch_fit", u.s);
                HIPCHK(launch_batch_fit(qx, qy, b.ccx.as<double>(), b.ccy.as<double>(),
                                        a.key, b.r.as<double>(), sou, gu, u.np, max_rows,
                                        allow_refl, su, b.fpart.as<double>() + (size_t)u.p0 * fch,
                                        b.fctr.as<unsigned>() + u.p0, u.s, worig));
            }
            NNArgs au = a;  // this sub-batch's trees: the per-tree arrays from its first row
            au.warm_c = bit > 0 ? 1 : 0;
            au.gap_cold = bit <= 1 ? 1 : 0;  // (every plot's calls 0 and 1 are batch iterations 0 and 1)
            au.sx = qx + u.r0;
            au.sy = qy + u.r0;
            au.sz = a.sz ? a.sz + u.r0 : nullptr;
            au.n = u.nr;
            au.r = a.r + u.r0;
            au.key = a.key ? a.key + u.r0 : nullptr;
            au.cx = a.cx + u.r0;
            au.cy = a.cy + u.r0;
            au.out_bp = a.out_bp + u.r0;
            au.gap = a.gap + u.r0;
            au.dz2 = a.dz2 ? a.dz2 + u.r0 : nullptr;
            {
                ProfScope ps(c, prof ? P_NN : 0, "nn_grid_batch", u.s);
                HIPCHK(launch_nn_grid_batch(au, b.plot_of.as<int32_t>() + u.r0, b.grids.as<PlotGrid>(),
                                            b.pts.as<TPt>(), m, b.cell_start.as<int32_t>(), st,
                                            md, u.s, bit));
            }
            BatchStepArgs su_step = step;  // this sub-batch's grids, counter, flag and trace
            su_step.grids = gu;  // indexed by the plot within the sub-batch (fit pivot)
            su_step.trace = trace ? trace + (size_t)u.p0 * (size_t)step.max_trace : nullptr;
            su_step.arrive = b.arrive.as<unsigned long long>() + qi;
            su_step.flag = flag;
            {
                ProfScope ps(c, prof ? P_FRAC : 0, "batch_select", u.s);
                HIPCHK(launch_batch_select(a.key, b.r.as<double>(), sou, u.np,
                                           max_rows, b.lams.as<double>(), su, ws, u.s,
                                           bfuse ? &su_step : nullptr));
            }
            // (fused: the selection's last workgroup stores the live count, k_batch.hip
            // batch_arrive -- the k_batch_live launch cost ~5-8 us per batch iteration)
            if (!bfuse)
                HIPCHK(launch_batch_update(u.np, nstages, threshold, max_iter, su, flag, u.s, su_step.trace,
                                           step.max_trace));
            return FICP_OK;
        };
        for (int q = 0; q < nsub; ++q)
            if (!subs[q].finished) CHK(enqueue(subs[q], 0));
        for (int64_t w = 0; w < cap; ++w) {
            bool all = true;
            for (int q = 0; q < nsub; ++q)  // one batch iteration ahead, per sub-batch
                if (!subs[q].finished && w + 1 < cap) CHK(enqueue(subs[q], w + 1));
            for (int q = 0; q < nsub; ++q) {
                Sub &u = subs[q];
                if (u.finished) continue;
                int live = 0;
                CHK(poll_flag(c, &u.ring[w % kBatchRing], live));
                u.finished = live == 0;
                all = all && u.finished;
            }
            if (all) break;
        }
        for (int q = 0; q < nsub; ++q)
            if (!subs[q].finished) return fail(FICP_EHIP, "batch did not converge within its bound");
    }  // JoinGuard: the sub-streams join c->stream here
    // the moved XY back into the caller's rows (sx[worig[w]] = wx[w]): per plot through LDS
    // when the plots fit one workgroup, else k_scatter_xy
    if (work) {
        int64_t max_rows = 0;
        for (int32_t p = 0; p < nplots; ++p) max_rows = std::max(max_rows, so_h[p + 1] - so_h[p]);
        if (plot_sort_fits(max_rows, 0))
            HIPCHK(launch_plot_scatter_xy(b.worig.as<uint32_t>(), b.wx.as<double>(), b.wy.as<double>(),
                                          b.so.as<int64_t>(), nplots, sx, sy, c->stream));
        else
            HIPCHK(launch_scatter_xy(b.worig.as<uint32_t>(), b.wx.as<double>(), b.wy.as<double>(), n, sx,
                                     sy, c->stream));
    }
    // one report kernel copies the plot states into coherent pinned memory and raises a
    // flag the host polls (a pageable D2H copy + stream sync left ~40 us of idle device)
    const size_t sbytes = (size_t)nplots * sizeof(PlotState);
    CHK(b.rep.ensure(sbytes + 64));
    int *rflag = (int *)(b.rep.as<char>() + sbytes + 32);
    __atomic_store_n(rflag, -1, __ATOMIC_RELAXED);
    HIPCHK(launch_report(ReportSeg{b.st.p, b.rep.p, per_plot ? (int)(sbytes / 4) : 0}, ReportSeg{},
                         ReportSeg{}, rflag, nullptr, c->stream));
    {
        int v = 0;
        CHK(poll_flag(c, rflag, v));
    }
    if (c->btrace_host && c->btrace_max > 0) {
        const size_t tb = (size_t)nplots * (size_t)c->btrace_max * 8;
        if (n > 0 && m > 0 && nstages > 0) {
            HIPCHK(hipMemcpyAsync(c->btrace_host, c->btrace.p, tb, hipMemcpyDeviceToHost, c->stream));
            CHK(sync(c));
        } else {
            memset(c->btrace_host, 0xff, tb);  // no call ran
        }
    }
    if (per_plot) {
        const PlotState *hs = b.rep.as<const PlotState>();
        for (int32_t p = 0; p < nplots; ++p) {
            const PlotState &s = hs[p];
            ficp_plot_stats &o = per_plot[p];
            memcpy(o.T_total, s.Ttot, sizeof o.T_total);
            o.frmsd_last = s.frmsd;
            o.k_last = s.k;
            o.n_nn_calls = s.n_nn;
            o.n_fits = s.n_fit;
            o.iters[0] = s.iters0;
            o.iters[1] = s.iters1;
        }
    }
    return FICP_OK;  // the report's flag follows every kernel of the run on the stream
}

int check_batch_args(int32_t nplots, int32_t md, int32_t nstages, const double *lambdas) {
    if (nplots <= 0 || nplots > 65535)
        return fail(FICP_EINVAL, "nplots must be in [1, 65535] (got %d)", (int)nplots);
    if (md != 2 && md != 3) return fail(FICP_EINVAL, "md must be 2 or 3 (got %d)", (int)md);
    if (nstages < 0 || (nstages > 0 && !lambdas)) return fail(FICP_EINVAL, "bad stages");
    return FICP_OK;
}

}  // namespace

extern "C" {

int ficp_set_batch_trace(ficp_ctx *c, int64_t *trace_k, int32_t max_calls) {
    if (!c) return fail(FICP_EINVAL, "null context");
    if (max_calls < 0 || (max_calls > 0 && !trace_k)) return fail(FICP_EINVAL, "bad trace arguments");
    c->btrace_host = max_calls > 0 ? trace_k : nullptr;
    c->btrace_max = max_calls;
    return FICP_OK;
}

int ficp_run_batch(ficp_ctx *c, int32_t nplots, const int64_t *src_off, double *src,
                   int64_t lds, const int64_t *tgt_off, const double *tgt, int64_t ldt,
                   int32_t md, int32_t nstages, const double *lambdas, double threshold,
                   int32_t max_iterations, int32_t allow_reflection, ficp_plot_stats *per_plot) {
    if (!c) return fail(FICP_EINVAL, "null context");
    CHK(set_device(c));
    CHK(check_batch_args(nplots, md, nstages, lambdas));
    int64_t n = 0, m = 0;
    CHK(check_offsets(src_off, nplots, "source", n));
    CHK(check_offsets(tgt_off, nplots, "target", m));
    if (n > 0x3fffffff || m > kMaxGridStems) return fail(FICP_EINVAL, "batch too large");
    if ((n > 0 && (!src || lds < md)) || (m > 0 && (!tgt || ldt < md)))
        return fail(FICP_EINVAL, "bad source/target arrays");
    BatchBufs &b = *batch_of(c);
    CHK(upload_rows(c, src, n, lds, md, b.sx, b.sy, &b.sz));
    CHK(upload_rows(c, tgt, m, ldt, md, b.tx, b.ty, &b.tz));
    CHK(batch_core(c, nplots, src_off, b.sx.as<double>(), b.sy.as<double>(), b.sz.as<double>(),
                   tgt_off, b.tx.as<double>(), b.ty.as<double>(), b.tz.as<double>(), md, nstages,
                   lambdas, threshold, max_iterations, allow_reflection, per_plot));
    if (n == 0) return FICP_OK;
    CHK(b.stage.ensure(n * 16));
    HIPCHK(launch_interleave_xy(b.sx.as<double>(), b.sy.as<double>(), n, b.stage.as<double>(),
                                c->stream));
    return d2h_xy_columns(c, b.stage.as<double>(), n, src, lds);
}

int ficp_run_batch_device(ficp_ctx *c, int32_t nplots, const int64_t *src_off, double *x,
                          double *y, const double *z, const int64_t *tgt_off, const double *tx,
                          const double *ty, const double *tz, int32_t md, int32_t nstages,
                          const double *lambdas, double threshold, int32_t max_iterations,
                          int32_t allow_reflection, ficp_plot_stats *per_plot) {
    if (!c) return fail(FICP_EINVAL, "null context");
    CHK(set_device(c));
    CHK(check_batch_args(nplots, md, nstages, lambdas));
    int64_t n = 0, m = 0;
    CHK(check_offsets(src_off, nplots, "source", n));
    CHK(check_offsets(tgt_off, nplots, "target", m));
    if (n > 0x3fffffff || m > kMaxGridStems) return fail(FICP_EINVAL, "batch too large");
    if ((n > 0 && (!x || !y || (md == 3 && !z))) || (m > 0 && (!tx || !ty || (md == 3 && !tz))))
        return fail(FICP_EINVAL, "bad device arrays");
    return batch_core(c, nplots, src_off, x, y, z, tgt_off, tx, ty, tz, md, nstages, lambdas,
                      threshold, max_iterations, allow_reflection, per_plot);
}

}  // extern "C"
