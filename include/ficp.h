/*
 * ficp.h -- C ABI of the MI355X-native Fractional ICP engine (libficp.so).
 *
 * Drop-in boundary: the reference has no native boundary of its own; its
 * interface is the Python class `FractionalICP` (ficp.py:5-154), imported by
 * the Join caller (app.py:20, app.py:658-660) and by the tests
 * (tests/test_ficp.py:9, tests/test_rigid_2d_operations.py:8).  The Python
 * facade coregistrationgame_amd/ficp.py keeps that class surface and binds
 * these entry points with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Host arrays are row-major C-contiguous fp64 with a leading dimension `ld`
 *    (columns); only the first `md` columns (2 or 3) are read, only columns 0,1
 *    are ever written.  The library never keeps a host pointer after a call
 *    returns.
 *  - `*_device` entry points take SoA device pointers (x[], y[], z[]) on the
 *    context's device; they are the "inputs already resident in HBM" path.
 *  - Return value: FICP_OK (0) or a negative FICP_E* code; ficp_last_error()
 *    returns a thread-local message for the last failure.
 *  - A context is not thread-safe; distinct contexts are independent.  All
 *    work of a context runs on one HIP stream of its device.
 *  - Parity rules: squared distance ((0+dx^2)+dy^2)+dz^2 in
 *    fp64 without FMA contraction, argmin on it, dist = sqrt; exact ties go to
 *    the lowest target index; selection order = stable sort of dist.
 */
#ifndef FICP_H
#define FICP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FICP_OK 0
#define FICP_EINVAL (-1)  /* bad argument (shape, md, null pointer)          */
#define FICP_EHIP (-2)    /* HIP runtime error                                */
#define FICP_ENOMEM (-3)  /* device allocation failed                         */
#define FICP_ESTATE (-4)  /* call order (e.g. no target set)                  */
#define FICP_ENODEV (-5)  /* no usable GPU                                    */

typedef struct ficp_ctx ficp_ctx;

/* Per-run statistics and optional traces (caller-owned arrays, nullable).
 * The caller must zero-initialise the struct (`ficp_stats st = {0};` / ctypes default)
 * and then set the "in" fields: max_trace, the trace pointers and max_trace_idx are read
 * by every run, and garbage there truncates or overruns the traces. */
typedef struct ficp_stats {
    int32_t n_nn_calls;      /* out: NN correspondence calls (both stages)            */
    int32_t n_fits;          /* out: fits applied = ICP loop bodies (ficp.py:132-145) */
    int32_t iters[2];        /* out: loop bodies per stage                            */
    int64_t k_last;          /* out: k of the last fraction call                      */
    double frmsd_last[2];    /* out: last FRMSD of each stage                         */
    double T_total[9];       /* out: composite transform of the whole run (row-major) */
    double gpu_ms;           /* out: wall time of the run on the device stream        */
    int32_t max_trace;       /* in : capacity of the trace arrays (NN calls)          */
    int32_t n_nn_reused;     /* out: NN calls answered by the previous call's outputs (a
                                later stage's head: the source has not moved since)   */
    int64_t *trace_k;        /* [max_trace]      k per NN/fraction call               */
    double *trace_frmsd;     /* [max_trace]      FRMSD at that k                      */
    double *trace_lambda;    /* [max_trace]      lambda in force                      */
    double *trace_T;         /* [max_trace * 9]  fits, in order                       */
    int32_t *trace_idx;      /* [max_trace * n]  NN target index per call             */
    double host_ms[4];       /* out: host wall time of ficp_run's phases: [0] source
                                upload, [1] device loop (enqueue + waits, incl. gpu_ms),
                                [2] result download + column write-back, [3] 0         */
    int32_t path;            /* out: 0 = the multi-kernel device loop, 1 = the whole run in
                                one workgroup (small plots, auto NN mode: k_small.hip)   */
    int32_t max_trace_idx;   /* in : calls whose NN index goes to trace_idx (0: max_trace);
                                trace_idx then holds min(this, max_trace) * n entries    */
} ficp_stats;

/* --- library / context ------------------------------------------------- */
int ficp_version(void);                       /* ABI version, e.g. 100 */
const char *ficp_last_error(void);
int ficp_device_count(int *count);
int ficp_create(int device, ficp_ctx **out);
void ficp_destroy(ficp_ctx *ctx);
/* NN algorithm: 0 = auto, 1 = brute force (LDS-tiled), 2 = uniform grid. */
int ficp_set_nn_mode(ficp_ctx *ctx, int32_t mode);
/* Test-only fault injection (no reference counterpart): mask 1 makes the selection's
   bounds hand-off never arrive, so the run must fail with the ERR_SPIN flag (4) instead of
   hanging or writing out of bounds; mask 2 makes every window-path fraction call report
   that it could not decide, so the run takes the full selection for each of them (the
   fallback's test).  0 = off (the default). */
int ficp_set_fault(ficp_ctx *ctx, int32_t mask);
/* Kernel timing with HIP events on the context stream: mask bit per kernel class
   (1 = nn, 2 = sort, 4 = scan/fraction, 8 = fit, 16 = grid build); 0 = off. */
int ficp_profile_enable(ficp_ctx *ctx, int32_t mask);
/* JSON {"kernel": {"count": c, "ms": total}, ...} of the timings so far; resets them. */
int ficp_profile_report(ficp_ctx *ctx, char *buf, int64_t buflen);
/* Selection path counters of this context since its creation (no reference counterpart;
   diagnostics of find_optimal_fraction, ficp.py:73-86, inside ficp_run): out[0] = fraction
   calls decided by the one-launch window path, out[1] = window-path calls that fell back to
   the full bucketed selection, out[2] = refinement levels, out[3] = radix fallbacks (the
   last two: the last run). */
int ficp_path_stats(ficp_ctx *ctx, int64_t out[4]);

/* --- static CHM layer (target) ----------------------------------------- */
/* Replaces the per-call cKDTree(target) of ficp.py:69: uploads the target once and
   builds its uniform grid; reused by every later NN call of this context. */
int ficp_set_target(ficp_ctx *ctx, const double *tgt, int64_t m, int64_t ld, int32_t md);
/* The same from device columns (z may be NULL when md == 2): stream-ordered, returns
   without waiting.  It copies the columns, reduces their bbox and queues the bbox's
   report to the host, which the next run collects; queue other work (a source reset)
   after this call and the report lands while it runs. */
int ficp_set_target_device(ficp_ctx *ctx, const double *x, const double *y, const double *z,
                           int64_t m, int32_t md);

/* --- the hot-path operations (ficp.py method each replaces) -------------- */
/* find_correspondences (ficp.py:65-71): idx[i], dist[i] of the exact 1-NN of src row i. */
int ficp_nn(ficp_ctx *ctx, const double *src, int64_t n, int64_t ld, int32_t *idx, double *dist);
/* find_optimal_fraction (ficp.py:73-86): n rows of src/corr/dist, N = len(self.source). */
int ficp_optimal_fraction(ficp_ctx *ctx, const double *src, int64_t lds, const double *corr,
                          int64_t ldc, const double *dist, int64_t n, int64_t n_source,
                          int32_t md, double lambda_val, double *frac, int64_t *k);
/* frmsd (ficp.py:54-60): squared differences summed over `rows` rows, divided by
   num_elements; +inf when num_elements == 0. */
int ficp_frmsd(ficp_ctx *ctx, const double *src, int64_t lds, const double *corr, int64_t ldc,
               int64_t rows, int64_t num_elements, int32_t md, double fraction,
               double lambda_val, double *out);
/* argsort (ficp.py:63,78): stable order of d (ties by index). */
int ficp_argsort(ficp_ctx *ctx, const double *d, int64_t n, int64_t *order);
/* compute_optimal_transform_2d (ficp.py:89-110) on k pairs (XY columns). */
int ficp_fit_rigid2d(ficp_ctx *ctx, const double *src, int64_t lds, const double *tgt,
                     int64_t ldt, int64_t k, int32_t allow_reflection, double T[9]);
/* apply_transform_2d_xy_only (ficp.py:112-119): writes the new XY to out_xy (n x 2). */
int ficp_apply_xy(ficp_ctx *ctx, const double *pts, int64_t n, int64_t ld, const double T[9],
                  double *out_xy);

/* --- the whole ICP ---------------------------------------------------- */
/* _iterate (ficp.py:122-147) for `nstages` stages with lambdas[s]; run()
   (ficp.py:149-154) is nstages = 2 with {lambda_val, 0.95 if md == 3 else 1.3}.
   src (n x ld, host) columns 0,1 are updated in place; md from ficp_set_target. */
int ficp_run(ficp_ctx *ctx, double *src, int64_t n, int64_t ld, int32_t nstages,
             const double *lambdas, double threshold, int32_t max_iterations,
             int32_t allow_reflection, ficp_stats *stats);
/* ficp_run with separate input and output rows: `out` (n x ld) receives `src` with
 * columns 0, 1 moved (out may alias src: that is ficp_run).  Replaces the copy the caller
 * needs for ficp.py:114,135 (`self.source` is replaced by a new array, the constructor's
 * is never written); when `out` is page-locked the rows come back in one direct D2H. */
int ficp_run_into(ficp_ctx *ctx, const double *src, double *out, int64_t n, int64_t ld,
                  int32_t nstages, const double *lambdas, double threshold,
                  int32_t max_iterations, int32_t allow_reflection, ficp_stats *stats);
/* Same on device-resident SoA source; x, y updated in place. */
int ficp_run_device(ficp_ctx *ctx, double *x, double *y, const double *z, int64_t n,
                    int32_t nstages, const double *lambdas, double threshold,
                    int32_t max_iterations, int32_t allow_reflection, ficp_stats *stats);

/* --- many plots in one device pass (a stand's Join of every plot) ------- */
/* Result of one plot of a batch: what ficp_stats reports for a single run. */
typedef struct ficp_plot_stats {
    double T_total[9];   /* out: composite transform applied to the plot's trees  */
    double frmsd_last;   /* out: FRMSD of the plot's last fraction call           */
    int64_t k_last;      /* out: k of that call                                   */
    int32_t n_nn_calls;  /* out: NN calls of the plot (all stages)                */
    int32_t n_fits;      /* out: loop bodies of the plot                          */
    int32_t iters[2];    /* out: loop bodies in stages 1 and 2                    */
} ficp_plot_stats;

/* FractionalICP(plot trees, plot CHM).run() for `nplots` independent plots at once
   (App.join_plot, app.py:630-661, once per plot; ficp.py:122-154 per plot, each plot
   with its own convergence test).  Plot p moves source rows src_off[p]..src_off[p+1]-1
   against target rows tgt_off[p]..tgt_off[p+1]-1; src_off[0] = tgt_off[0] = 0 and both
   non-decreasing.  All plots share md, lambdas, threshold, max_iterations and
   allow_reflection; 0 < nplots <= 65535.  Source columns 0,1 are updated in place;
   per_plot (nullable) receives nplots records.  Independent of ficp_set_target. */
/* Per-call k trace of the next batch runs (no reference counterpart; the batch's analogue
   of ficp_stats::trace_k, for tests): trace_k[p * max_calls + j] = k of plot p's j-th NN /
   fraction call (ficp.py:73-86), -1 past its last call; (nullptr, 0) turns it off.  The
   host array must hold nplots * max_calls entries and outlive the runs. */
int ficp_set_batch_trace(ficp_ctx *ctx, int64_t *trace_k, int32_t max_calls);
int ficp_run_batch(ficp_ctx *ctx, int32_t nplots, const int64_t *src_off, double *src,
                   int64_t lds, const int64_t *tgt_off, const double *tgt, int64_t ldt,
                   int32_t md, int32_t nstages, const double *lambdas, double threshold,
                   int32_t max_iterations, int32_t allow_reflection, ficp_plot_stats *per_plot);
/* Same on device-resident SoA layers (offsets stay host arrays); x, y updated in place. */
int ficp_run_batch_device(ficp_ctx *ctx, int32_t nplots, const int64_t *src_off, double *x,
                          double *y, const double *z, const int64_t *tgt_off, const double *tx,
                          const double *ty, const double *tz, int32_t md, int32_t nstages,
                          const double *lambdas, double threshold, int32_t max_iterations,
                          int32_t allow_reflection, ficp_plot_stats *per_plot);

/* --- CHM stems matched by a joined plot --------------------------------- */
/* CHMPlot.remove_matches (chm_plot.py:223-285) against the CHM layer set with
   ficp_set_target (md 3: x, y, height; md 2: x, y).  For each plot tree in order, its
   nearest REMAINING stem (scipy cdist distance, first index on equal distances) is
   removed iff that distance < thresh[i] (the caller passes min_dist_percent/100 * the
   tree's height, with the reference's 10 m rule in 2-D).  Stops when no stem remains.
   removed[0 .. *n_removed) = the removed stems' row indices in removal order (capacity
   >= min(n, m)).  GPU k-nearest candidates + the reference's greedy walk on the host. */
int ficp_remove_matches(ficp_ctx *ctx, const double *plot, int64_t n, int64_t ld,
                        const double *thresh, int32_t *removed, int64_t *n_removed);

/* --- partitioned CHM layer (one large plot over several GPUs) ------------ */
/* The target is split into contiguous row ranges (shards), one per rank; the source is
   replicated.  Per NN call each rank runs ficp_nn_device against its shard, the caller
   merges the shards (all-reduce MIN of d2, then all-reduce MIN of idx where the rank's
   d2 equals the merged d2: the lowest global index wins a tie, as in ficp_nn), and every
   rank runs ficp_select_fit_device on the merged result (deterministic: identical T on
   every rank), then ficp_apply_device.  All pointers are device pointers. */
/* find_correspondences (ficp.py:65-71) against the shard set with ficp_set_target*:
   d2[i] = squared distance, idx[i] = idx_offset + shard index of the nearest stem.
   An empty shard yields d2 = +inf, idx = INT32_MAX. */
int ficp_nn_device(ficp_ctx *ctx, const double *x, const double *y, const double *z, int64_t n,
                   int64_t idx_offset, double *d2, int32_t *idx);
/* find_optimal_fraction + compute_optimal_transform_2d (ficp.py:73-110) on merged
   correspondences: tx, ty = the whole CHM layer (rows addressed by idx).  Returns k and
   its FRMSD; T = the fit on the first k pairs (identity when k == 0).  The fit's sums are
   taken relative to (pivot_x, pivot_y): pass the same pivot on every rank. */
int ficp_select_fit_device(ficp_ctx *ctx, const double *x, const double *y, int64_t n,
                           const double *d2, const int32_t *idx, const double *tx,
                           const double *ty, int64_t n_source, double lambda_val,
                           int32_t allow_reflection, double pivot_x, double pivot_y, int64_t *k,
                           double *frmsd, double T[9]);
/* apply_transform_2d_xy_only (ficp.py:112-119) in place on device-resident XY. */
int ficp_apply_device(ficp_ctx *ctx, double *x, double *y, int64_t n, const double T[9]);

/* --- distributed run of one plot, stream-ordered (C5) --------------------- */
/* The whole of ficp.py:149-154 for one plot split over ranks, with every step enqueued on
   the context's stream; the caller runs its collectives (RCCL via torch.distributed) on the
   same stream, so no step waits for the host.  Per iteration (one NN call) the host
   enqueues the steps below and then waits for the previous iteration's done flag
   (ficp_dist_wait); iterations enqueued past the end are no-ops.  Device pointers.
   mode 1, target-partitioned: every rank holds all n rows and a shard of the layer:
     fit_sums -> fit_solve(world 1; applies T) -> nn_shard per shard -> caller: MIN merge
     of (d2, idx) as for ficp_nn_device -> select_merged.
   mode 2, source-partitioned: every rank holds the whole layer and rows [row0, row0 +
   n_local) of n_total: fit_sums -> caller: all-gather (8 f64 per rank) -> fit_solve ->
   nn_local -> caller: MAX all-reduce of range2 (2 int64) -> hist -> caller: SUM
   all-reduce of hist (ficp_dist_hist_words() int64) -> candidates -> caller: all-gather
   of the packs (4 + 3 capd int64 per rank) -> final.  Every rank derives the same k,
   threshold and T from the exact integer histogram and the rank-ordered sums. */
int ficp_set_stream(ficp_ctx *ctx, void *hip_stream);  /* NULL: the context's own stream */
int ficp_dist_begin(ficp_ctx *ctx, int32_t mode, double *x, double *y, const double *z,
                    int64_t n_local, int64_t n_total, int64_t n_max, int64_t row0,
                    int32_t nstages, const double *lambdas, double threshold,
                    int32_t max_iterations, int32_t allow_reflection, double pivot_x,
                    double pivot_y, int32_t world, int32_t capd);
int ficp_dist_fit_sums(ficp_ctx *ctx, double *sums8);
int ficp_dist_fit_solve(ficp_ctx *ctx, const double *sums, int32_t world);
int ficp_dist_nn_shard(ficp_ctx *shard, ficp_ctx *ctrl, int64_t idx_offset, double *d2,
                       int32_t *idx);
int ficp_dist_select_merged(ficp_ctx *ctx, const double *d2, const int32_t *idx,
                            const double *tx, const double *ty, int64_t iteration);
int ficp_dist_nn_local(ficp_ctx *ctx, int64_t *range2);
int ficp_dist_hist_words(void);
int ficp_dist_hist(ficp_ctx *ctx, const int64_t *range2, int64_t *hist);
int ficp_dist_candidates(ficp_ctx *ctx, const int64_t *hist, int64_t *pack, int32_t capd);
int ficp_dist_final(ficp_ctx *ctx, const int64_t *packs, int32_t world, int32_t capd,
                    int64_t iteration);
int ficp_dist_wait(ficp_ctx *ctx, int64_t iteration, int32_t *done);
int ficp_dist_end(ficp_ctx *ctx, ficp_stats *stats);

/* --- device memory helpers (for callers without their own allocator) ---- */
int ficp_dev_alloc(ficp_ctx *ctx, int64_t bytes, void **ptr);
int ficp_dev_free(ficp_ctx *ctx, void *ptr);
int ficp_memcpy_h2d(ficp_ctx *ctx, void *dst, const void *src, int64_t bytes);
int ficp_memcpy_d2h(ficp_ctx *ctx, void *dst, const void *src, int64_t bytes);
int ficp_memcpy_d2d(ficp_ctx *ctx, void *dst, const void *src, int64_t bytes);
int ficp_synchronize(ficp_ctx *ctx);

/* --- host memory for the drop-in facade (no context needed) --------------------------
   Page-locked host memory (hipHostMalloc): the facade keeps its layer copies
   (ficp.py:34-35 np.array) in pooled blocks of it, so a new instance per Join
   (app.py:658) neither page-faults fresh memory nor stages its uploads.
   ficp_host_copy: memcpy split over up to 8 host threads. */
int ficp_host_alloc(int64_t bytes, void **ptr);
int ficp_host_free(void *ptr);
int ficp_host_copy(void *dst, const void *src, int64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* FICP_H */
