/*
 * ficp_oracle.c -- CPU restatement of the reference Fractional ICP (ficp.py).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (coregistrationgame_amd/,
 * include/, libficp) links, loads or calls this file.  It is imported only by
 * tests/ (as the checker), by __graft_entry__.smoke() (as the checker) and by
 * bench.py's cpu_baseline leg (as the timed CPU baseline, kind "port").
 *
 * Parity pin: tests/test_oracle_golden.py checks every function below against
 * the golden vectors generated from /root/reference/ficp.py by
 * tests/golden/make_golden.py (NN idx/dist bit-exact, k exact where the
 * reference's own FRMSD curve has a gap, T within 1e-9, apply bit-exact, run
 * traces).
 *
 * Arithmetic conventions (all IEEE fp64, compiled with -ffp-contract=off):
 *  - squared distance  d2 = ((0 + dx*dx) + dy*dy) + dz*dz, argmin over d2,
 *    dist = sqrt(d2): reproduces scipy cKDTree.query(k=1) bit-exactly
 *    (SURVEY.md §8(a) a3 probe); exact ties go to the LOWEST target index
 *    (cKDTree's own tie choice is traversal dependent, so fixtures are tie-free).
 *  - selection order: stable sort of dist by (dist, index) (ficp.py:63,78).
 *  - fraction: S_k = sequential prefix sum of r_i = sum_md (src-corr)^2 in that
 *    order, FRMSD(k) = (1.0 / ((k/N)**lambda)) * sqrt(S_k / k), first strict
 *    minimum (ficp.py:54-60, 73-86).
 *  - fit: centroids, 2x2 cross-covariance, 2x2 SVD, R = Vt^T U^T with the
 *    Kabsch flip of Vt's last row unless allow_reflection (ficp.py:89-110).
 *  - apply: x' = fma(y, T01, x*T00) + T02 (and the same for y'), which is what
 *    numpy's (N,3)@(3,3) matmul through OpenBLAS dgemm produces on this host
 *    (pinned bit-exactly by tests/golden/apply.npz) (ficp.py:112-119).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

static inline double sqd(const double *q, const double *p, int md) {
    /* ficp.py:69-70 via cKDTree: ((0 + dx^2) + dy^2) + dz^2 */
    double dx = q[0] - p[0];
    double dy = q[1] - p[1];
    double s = 0.0 + dx * dx;
    s = s + dy * dy;
    if (md == 3) {
        double dz = q[2] - p[2];
        s = s + dz * dz;
    }
    return s;
}

static inline int better(double d2, int64_t i, double best, int64_t bi) {
    return d2 < best || (d2 == best && i < bi);
}

/* ---------------------------------------------------------------- brute NN */
/* ficp.py:65-71 (find_correspondences), brute-force restatement. */
EXPORT int orc_nn_brute(const double *src, int64_t n, int64_t lds, const double *tgt, int64_t m,
                        int64_t ldt, int md, int32_t *idx, double *dist, double *d2out, int nthreads) {
    if (n <= 0 || m <= 0) return 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i) {
        const double *q = src + i * lds;
        double best = INFINITY;
        int64_t bi = 0;
        for (int64_t j = 0; j < m; ++j) {
            double d2 = sqd(q, tgt + j * ldt, md);
            if (d2 < best) { best = d2; bi = j; }   /* j ascending: strict < keeps lowest index */
        }
        idx[i] = (int32_t)bi;
        if (d2out) d2out[i] = best;
        dist[i] = sqrt(best);
    }
    return 0;
}

/* ---------------------------------------------------------------- kd-tree NN */
typedef struct {
    int32_t lo, hi;     /* point range [lo, hi) in perm order */
    int32_t left, right;/* child nodes or -1 */
    int32_t dim;
    double split;
} kdnode;

typedef struct {
    int md;
    int64_t m;
    double *pts;      /* m x 3, reordered */
    int32_t *orig;    /* original index of reordered point */
    kdnode *nodes;
    int32_t nnodes, cap;
} kdtree;

static void kd_swap(kdtree *t, int64_t a, int64_t b) {
    double tmp[3];
    memcpy(tmp, t->pts + 3 * a, sizeof tmp);
    memcpy(t->pts + 3 * a, t->pts + 3 * b, sizeof tmp);
    memcpy(t->pts + 3 * b, tmp, sizeof tmp);
    int32_t o = t->orig[a]; t->orig[a] = t->orig[b]; t->orig[b] = o;
}

/* quickselect so that element k (within [lo,hi)) is in place along dim */
static void kd_select(kdtree *t, int64_t lo, int64_t hi, int64_t k, int dim) {
    while (hi - lo > 1) {
        int64_t mid = lo + (hi - lo) / 2;
        /* median of three pivot */
        double a = t->pts[3 * lo + dim], b = t->pts[3 * mid + dim], c = t->pts[3 * (hi - 1) + dim];
        int64_t piv = (a < b) ? ((b < c) ? mid : ((a < c) ? hi - 1 : lo)) : ((a < c) ? lo : ((b < c) ? hi - 1 : mid));
        double pv = t->pts[3 * piv + dim];
        kd_swap(t, piv, hi - 1);
        int64_t st = lo;
        for (int64_t i = lo; i < hi - 1; ++i)
            if (t->pts[3 * i + dim] < pv) kd_swap(t, i, st++);
        kd_swap(t, st, hi - 1);
        if (st == k) return;
        if (k < st) hi = st; else lo = st + 1;
    }
}

static int32_t kd_build_rec(kdtree *t, int32_t lo, int32_t hi) {
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->nodes = (kdnode *)realloc(t->nodes, sizeof(kdnode) * t->cap);
    }
    int32_t id = t->nnodes++;
    kdnode nd = {lo, hi, -1, -1, 0, 0.0};
    if (hi - lo > 16) {
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int32_t i = lo; i < hi; ++i)
            for (int d = 0; d < t->md; ++d) {
                double v = t->pts[3 * i + d];
                if (v < mn[d]) mn[d] = v;
                if (v > mx[d]) mx[d] = v;
            }
        int dim = 0;
        for (int d = 1; d < t->md; ++d)
            if (mx[d] - mn[d] > mx[dim] - mn[dim]) dim = d;
        if (mx[dim] > mn[dim]) {
            int32_t mid = lo + (hi - lo) / 2;
            kd_select(t, lo, hi, mid, dim);
            nd.dim = dim;
            nd.split = t->pts[3 * mid + dim];
            /* left = [lo, mid) has coord <= split, right = [mid, hi) has coord >= split */
            int32_t l = kd_build_rec(t, lo, mid);
            int32_t r = kd_build_rec(t, mid, hi);
            nd.left = l;
            nd.right = r;
        }
    }
    t->nodes[id] = nd;
    return id;
}

EXPORT void *orc_kd_build(const double *tgt, int64_t m, int64_t ldt, int md) {
    kdtree *t = (kdtree *)calloc(1, sizeof(kdtree));
    t->md = md;
    t->m = m;
    t->pts = (double *)calloc((size_t)(m > 0 ? m : 1) * 3, sizeof(double));
    t->orig = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
    for (int64_t i = 0; i < m; ++i) {
        for (int d = 0; d < md; ++d) t->pts[3 * i + d] = tgt[i * ldt + d];
        t->orig[i] = (int32_t)i;
    }
    if (m > 0) kd_build_rec(t, 0, (int32_t)m);
    return t;
}

EXPORT void orc_kd_free(void *p) {
    kdtree *t = (kdtree *)p;
    if (!t) return;
    free(t->pts);
    free(t->orig);
    free(t->nodes);
    free(t);
}

static void kd_query1(const kdtree *t, const double *q, double *best, int64_t *bi) {
    int32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const kdnode *nd = &t->nodes[stack[--sp]];
        if (nd->left < 0) {
            for (int32_t i = nd->lo; i < nd->hi; ++i) {
                double d2 = sqd(q, t->pts + 3 * i, t->md);
                if (better(d2, t->orig[i], *best, *bi)) { *best = d2; *bi = t->orig[i]; }
            }
            continue;
        }
        double diff = q[nd->dim] - nd->split;
        int32_t nearc = diff < 0 ? nd->left : nd->right;
        int32_t farc = diff < 0 ? nd->right : nd->left;
        /* prune the far side only when its plane bound strictly exceeds best (ties may
           still hold a lower index); monotone rounding makes this exact. */
        if (diff * diff <= *best) stack[sp++] = farc;
        stack[sp++] = nearc;
    }
}

EXPORT int orc_kd_query(const void *tp, const double *src, int64_t n, int64_t lds, int32_t *idx,
                        double *dist, double *d2out, int nthreads) {
    const kdtree *t = (const kdtree *)tp;
    if (n <= 0 || t->m <= 0) return 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1024)
#endif
    for (int64_t i = 0; i < n; ++i) {
        double q[3] = {src[i * lds], src[i * lds + 1], t->md == 3 ? src[i * lds + 2] : 0.0};
        double best = INFINITY;
        int64_t bi = INT64_MAX;
        kd_query1(t, q, &best, &bi);
        idx[i] = (int32_t)bi;
        if (d2out) d2out[i] = best;
        dist[i] = sqrt(best);
    }
    return 0;
}

/* ---------------------------------------------------------------- ordering */
/* ficp.py:63,78 -- argsort(distances), ties by index (stable): the order of the
   comparison (d_i < d_j) || (d_i == d_j && i < j).  Stable LSD radix sort (4 passes of 16
   bits) over the order-preserving u64 image of each double, starting from index order,
   so equal keys keep index order.  -0.0 maps to +0.0 (they compare equal). */
static inline uint64_t ord_bits(double v) {
    if (v == 0.0) v = 0.0;
    uint64_t u;
    memcpy(&u, &v, 8);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

EXPORT void orc_sort_order(const double *d, int64_t n, int64_t *order) {
    if (n <= 0) return;
    uint64_t *key = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    uint64_t *key2 = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    size_t *cnt = (size_t *)malloc(sizeof(size_t) * 65536);
    for (int64_t i = 0; i < n; ++i) { order[i] = i; key[i] = ord_bits(d[i]); }
    int64_t *src = order, *dst = tmp;
    uint64_t *ks = key, *kd = key2;
    for (int pass = 0; pass < 4; ++pass) {
        const int sh = 16 * pass;
        memset(cnt, 0, sizeof(size_t) * 65536);
        for (int64_t i = 0; i < n; ++i) cnt[(ks[i] >> sh) & 0xffff]++;
        size_t run = 0;
        for (int b = 0; b < 65536; ++b) { size_t c = cnt[b]; cnt[b] = run; run += c; }
        for (int64_t i = 0; i < n; ++i) {
            size_t at = cnt[(ks[i] >> sh) & 0xffff]++;
            dst[at] = src[i];
            kd[at] = ks[i];
        }
        int64_t *t = src; src = dst; dst = t;
        uint64_t *tk = ks; ks = kd; kd = tk;
    }
    /* 4 passes: the result is back in `order` */
    free(key); free(key2); free(tmp); free(cnt);
}

/* ---------------------------------------------------------------- fraction */
static inline double frmsd_val(double frac, double lam, double S, int64_t k) {
    /* ficp.py:59-60 */
    return (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
}

/* ficp.py:73-86.  r_i = sum_md (src_i - corr_i)^2 (ficp.py:58-59).  N = len(self.source).
   literal != 0 recomputes every prefix sum from scratch (the O(N^2) cost model of
   ficp.py:80-85); the values are identical to the O(N) cumsum. */
static int optimal_fraction_ex(const double *src, int64_t lds, const double *corr, int64_t ldc,
                               const double *d, int64_t n, int64_t N, int md, double lam, int literal,
                               double *frac_out, int64_t *k_out, double *frmsd_out, double *gap_out,
                               int64_t *order_out) {
    *frac_out = 0.0;
    *k_out = 0;
    if (frmsd_out) *frmsd_out = INFINITY;
    if (gap_out) *gap_out = INFINITY;
    if (N == 0 || n == 0) return 0;
    int64_t *order = order_out ? order_out : (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    double *r = (double *)malloc(sizeof(double) * (size_t)n);
    orc_sort_order(d, n, order);
    for (int64_t j = 0; j < n; ++j) {
        const double *s = src + order[j] * lds, *c = corr + order[j] * ldc;
        double acc = 0.0;
        for (int t = 0; t < md; ++t) {
            double df = s[t] - c[t];
            acc = acc + df * df;
        }
        r[j] = acc;
    }
    double best = INFINITY, second = INFINITY, bfrac = 0.0, S = 0.0;
    int64_t bk = 0;
    for (int64_t k = 1; k <= N; ++k) {
        if (literal) {
            S = 0.0;
            int64_t kk = k < n ? k : n;
            for (int64_t j = 0; j < kk; ++j) S = S + r[j];
        } else if (k <= n) {
            S = S + r[k - 1];
        }
        double frac = (double)k / (double)N;
        double v = frmsd_val(frac, lam, S, k);
        if (v < best) { second = best; best = v; bfrac = frac; bk = k; }
        else if (v < second) second = v;
    }
    if (!order_out) free(order);
    free(r);
    *frac_out = bfrac;
    *k_out = bk;
    if (frmsd_out) *frmsd_out = best;
    /* relative FRMSD gap between the best k and the runner-up: where it is at rounding
       level the winning k is not pinned by any implementation (tests/conftest.py) */
    if (gap_out) *gap_out = (best > 0.0 && isfinite(second)) ? (second - best) / best : INFINITY;
    return 0;
}

EXPORT int orc_optimal_fraction(const double *src, int64_t lds, const double *corr, int64_t ldc,
                                const double *d, int64_t n, int64_t N, int md, double lam,
                                int literal, double *frac_out, int64_t *k_out, double *frmsd_out) {
    return optimal_fraction_ex(src, lds, corr, ldc, d, n, N, md, lam, literal, frac_out, k_out, frmsd_out,
                               NULL, NULL);
}

/* ficp.py:54-60 */
/* ficp.py:54-60: the squared differences of ALL `rows` rows given, divided by k
   (num_elements, which callers may pass different from the row count) */
EXPORT double orc_frmsd(double fraction, int64_t k, const double *src, int64_t lds,
                        const double *corr, int64_t ldc, int64_t rows, int md, double lam) {
    if (k == 0) return INFINITY;
    double S = 0.0;
    for (int64_t i = 0; i < rows; ++i)
        for (int t = 0; t < md; ++t) {
            double df = src[i * lds + t] - corr[i * ldc + t];
            S = S + df * df;
        }
    return frmsd_val(fraction, lam, S, k);
}

/* ---------------------------------------------------------------- fit */
/* 2x2 SVD H = U diag(s) Vt with rotation-parametrised factors. */
static void svd2x2(const double H[4], double U[4], double s[2], double Vt[4]) {
    double a = H[0], b = H[1], c = H[2], d = H[3];
    double E = (a + d) * 0.5, F = (a - d) * 0.5, G = (c + b) * 0.5, Hh = (c - b) * 0.5;
    double Q = hypot(E, Hh), R = hypot(F, G);
    double sx = Q + R, sy = Q - R;
    double a1 = atan2(G, F), a2 = atan2(Hh, E);
    double th = (a2 - a1) * 0.5, ph = (a2 + a1) * 0.5;
    double cp = cos(ph), sp = sin(ph), ct = cos(th), st = sin(th);
    U[0] = cp; U[1] = -sp; U[2] = sp; U[3] = cp;        /* Rot(phi) */
    Vt[0] = ct; Vt[1] = -st; Vt[2] = st; Vt[3] = ct;    /* Rot(theta) */
    if (sy < 0) {                                       /* make singular values >= 0 */
        sy = -sy;
        Vt[2] = -Vt[2];
        Vt[3] = -Vt[3];
    }
    s[0] = sx;
    s[1] = sy;
}

/* ficp.py:89-110 */
EXPORT void orc_fit_rigid2d(const double *src, int64_t lds, const double *tgt, int64_t ldt,
                            int64_t k, int allow_reflection, double *T) {
    double csx = 0, csy = 0, ctx = 0, cty = 0;
    for (int64_t i = 0; i < k; ++i) {
        csx += src[i * lds]; csy += src[i * lds + 1];
        ctx += tgt[i * ldt]; cty += tgt[i * ldt + 1];
    }
    csx /= (double)k; csy /= (double)k; ctx /= (double)k; cty /= (double)k;
    double H[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < k; ++i) {
        double xs = src[i * lds] - csx, ys = src[i * lds + 1] - csy;
        double xt = tgt[i * ldt] - ctx, yt = tgt[i * ldt + 1] - cty;
        H[0] += xs * xt; H[1] += xs * yt; H[2] += ys * xt; H[3] += ys * yt;
    }
    double U[4], s[2], Vt[4];
    svd2x2(H, U, s, Vt);
    /* R = Vt^T U^T */
    double R[4];
    R[0] = Vt[0] * U[0] + Vt[2] * U[1];
    R[1] = Vt[0] * U[2] + Vt[2] * U[3];
    R[2] = Vt[1] * U[0] + Vt[3] * U[1];
    R[3] = Vt[1] * U[2] + Vt[3] * U[3];
    double det = R[0] * R[3] - R[1] * R[2];
    if (!allow_reflection && det < 0) {
        Vt[2] = -Vt[2];
        Vt[3] = -Vt[3];
        R[0] = Vt[0] * U[0] + Vt[2] * U[1];
        R[1] = Vt[0] * U[2] + Vt[2] * U[3];
        R[2] = Vt[1] * U[0] + Vt[3] * U[1];
        R[3] = Vt[1] * U[2] + Vt[3] * U[3];
    }
    /* t = ct - cs @ R^T */
    double tx = ctx - (csx * R[0] + csy * R[1]);
    double ty = cty - (csx * R[2] + csy * R[3]);
    T[0] = R[0]; T[1] = R[1]; T[2] = tx;
    T[3] = R[2]; T[4] = R[3]; T[5] = ty;
    T[6] = 0.0; T[7] = 0.0; T[8] = 1.0;
}

/* ficp.py:112-119: columns 0,1 rewritten, every other column preserved. */
EXPORT void orc_apply_xy(double *pts, int64_t n, int64_t ld, const double *T) {
    for (int64_t i = 0; i < n; ++i) {
        double x = pts[i * ld], y = pts[i * ld + 1];
        pts[i * ld] = fma(y, T[1], x * T[0]) + T[2];
        pts[i * ld + 1] = fma(y, T[4], x * T[3]) + T[5];
    }
}

/* ---------------------------------------------------------------- run */
typedef struct {
    int32_t max_calls;     /* capacity of the arrays below (NN calls)            */
    int32_t n_calls;       /* out: NN calls made (= fraction calls)              */
    int32_t n_fits;        /* out: fits applied                                  */
    int32_t iters[2];      /* out: loop bodies per stage                         */
    int64_t *k;            /* [max_calls] selected k per NN call                 */
    double *frmsd;         /* [max_calls]                                        */
    double *lam;           /* [max_calls]                                        */
    double *T;             /* [max_calls * 9] fits (n_fits of them)              */
    int32_t *idx;          /* [max_calls * n] NN idx per call, nullable          */
    double *gap;           /* [max_calls] FRMSD best vs runner-up (relative), nullable */
} orc_trace;

typedef struct {
    const double *tgt;
    int64_t m, ldt;
    int md, literal, nthreads;
    void *kd;
} nnctx;

static void run_nn(nnctx *c, const double *src, int64_t n, int64_t lds, int32_t *idx, double *dist,
                   double *d2) {
    if (c->literal) {
        /* ficp.py:69: the reference rebuilds the index on every call */
        void *kd = orc_kd_build(c->tgt, c->m, c->ldt, c->md);
        orc_kd_query(kd, src, n, lds, idx, dist, d2, c->nthreads);
        orc_kd_free(kd);
    } else {
        orc_kd_query(c->kd, src, n, lds, idx, dist, d2, c->nthreads);
    }
}

static int64_t choose(nnctx *c, const double *src, int64_t n, int64_t lds, int32_t *idx, double *dist,
                      double *d2, double *corr, int64_t *order, double lam, double *fr_out, double *frac_out,
                      double *gap_out) {
    run_nn(c, src, n, lds, idx, dist, d2);
    for (int64_t i = 0; i < n; ++i)
        for (int t = 0; t < c->md; ++t) corr[i * 3 + t] = c->tgt[(int64_t)idx[i] * c->ldt + t];
    double frac, fr;
    int64_t k;
    /* the fraction's argsort is the selection's order too (ficp.py:63,78: same input) */
    optimal_fraction_ex(src, lds, corr, 3, dist, n, n, c->md, lam, c->literal, &frac, &k, &fr, gap_out, order);
    *fr_out = fr;
    *frac_out = frac;
    return k;
}

static void trace_call(orc_trace *tr, int64_t k, double fr, double lam, const int32_t *idx, int64_t n,
                       double gap) {
    if (!tr) return;
    int32_t c = tr->n_calls++;
    if (c >= tr->max_calls) return;
    if (tr->k) tr->k[c] = k;
    if (tr->frmsd) tr->frmsd[c] = fr;
    if (tr->lam) tr->lam[c] = lam;
    if (tr->gap) tr->gap[c] = gap;
    if (tr->idx) memcpy(tr->idx + (int64_t)c * n, idx, sizeof(int32_t) * (size_t)n);
}

/* ficp.py:122-147 (_iterate) for one stage. */
static int iterate(nnctx *c, double *src, int64_t n, int64_t lds, double lam, double thr,
                   int max_iter, int allow_reflection, orc_trace *tr, int stage) {
    if (n == 0 || c->m == 0) return 0;
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    double *dist = (double *)malloc(sizeof(double) * (size_t)n);
    double *d2 = (double *)malloc(sizeof(double) * (size_t)n);
    double *corr = (double *)calloc((size_t)n * 3, sizeof(double));
    int64_t *order = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    double *ss = (double *)malloc(sizeof(double) * (size_t)n * 2);
    double *cc = (double *)malloc(sizeof(double) * (size_t)n * 2);
    double cur, frac, gap;
    int64_t k = choose(c, src, n, lds, idx, dist, d2, corr, order, lam, &cur, &frac, &gap);
    trace_call(tr, k, cur, lam, idx, n, gap);
    int it = 0;
    if (k > 0) {
        while (it < max_iter) {
            for (int64_t j = 0; j < k; ++j) {
                ss[2 * j] = src[order[j] * lds];
                ss[2 * j + 1] = src[order[j] * lds + 1];
                cc[2 * j] = corr[order[j] * 3];
                cc[2 * j + 1] = corr[order[j] * 3 + 1];
            }
            double T[9];
            orc_fit_rigid2d(ss, 2, cc, 2, k, allow_reflection, T);
            if (tr) {
                if (tr->T && tr->n_fits < tr->max_calls) memcpy(tr->T + 9 * tr->n_fits, T, sizeof T);
                tr->n_fits++;
            }
            orc_apply_xy(src, n, lds, T);
            double nw;
            k = choose(c, src, n, lds, idx, dist, d2, corr, order, lam, &nw, &frac, &gap);
            trace_call(tr, k, nw, lam, idx, n, gap);
            if (cur - nw <= thr) break;
            cur = nw;
            it++;
        }
    }
    if (tr) tr->iters[stage] = it;
    free(idx); free(dist); free(d2); free(corr); free(order); free(ss); free(cc);
    return 0;
}

/* ficp.py:149-154 (run): stage 1 with lam0, stage 2 with lam1. src is (n, lds) row-major,
   modified in place (columns 0,1 only). nn_literal != 0 gives the reference's cost model
   (index rebuilt per call, O(N^2) fraction scan). */
EXPORT int orc_run(double *src, int64_t n, int64_t lds, const double *tgt, int64_t m, int64_t ldt,
                   int md, double lam0, double lam1, double thr, int max_iter, int allow_reflection,
                   int literal, int nthreads, orc_trace *tr) {
    nnctx c = {tgt, m, ldt, md, literal, nthreads, NULL};
    if (!literal && m > 0) c.kd = orc_kd_build(tgt, m, ldt, md);
    if (tr) { tr->n_calls = 0; tr->n_fits = 0; tr->iters[0] = tr->iters[1] = 0; }
    iterate(&c, src, n, lds, lam0, thr, max_iter, allow_reflection, tr, 0);
    iterate(&c, src, n, lds, lam1, thr, max_iter, allow_reflection, tr, 1);
    if (c.kd) orc_kd_free(c.kd);
    return 0;
}

EXPORT int orc_num_threads_max(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
