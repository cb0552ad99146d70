/*
 * san_driver.c -- runs one call of the CPU oracle (ficp_oracle.c) per process, for the
 * AddressSanitizer / UndefinedBehaviorSanitizer build (`make -C oracle asan`).
 *
 * TEST INFRASTRUCTURE ONLY, like ficp_oracle.c.  tests/test_oracle_sanitized.py routes
 * every oracle entry point of tests/test_oracle_golden.py through this executable
 * (ficp_oracle.py's ctypes surface, marshalled over stdin/stdout), so the golden tests
 * run unchanged on the instrumented oracle: an out-of-bounds access, a leak or UB in
 * the checker fails the CPU suite (SURVEY.md §5 "Race detection / sanitizers").
 *
 * Request (stdin, native little-endian):  i64 op; i64 ni; i64 ints[ni]; i64 nd;
 *   f64 dbls[nd]; i64 na; na x (i64 nbytes; bytes).
 * Reply (stdout): i64 rc; i64 na; na x (i64 nbytes; bytes).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ficp_oracle.c"

enum { OP_NN_BRUTE = 1, OP_NN_KD = 2, OP_SORT = 3, OP_FRAC = 4, OP_FRMSD = 5, OP_FIT = 6,
       OP_APPLY = 7, OP_RUN = 8, OP_THREADS = 9 };

typedef struct { int64_t n; void *p; } blob;

static void rd(void *dst, size_t n) {
    if (n && fread(dst, 1, n, stdin) != n) { fprintf(stderr, "san_driver: short read\n"); exit(3); }
}
static int64_t rd64(void) { int64_t v; rd(&v, 8); return v; }

static blob out_blobs[16];
static int n_out = 0;

static void *out_alloc(int64_t nbytes) {
    blob b = {nbytes, calloc(1, nbytes > 0 ? (size_t)nbytes : 1)};
    out_blobs[n_out++] = b;
    return b.p;
}
static void out_copy(const void *src, int64_t nbytes) { memcpy(out_alloc(nbytes), src, (size_t)nbytes); }

int main(void) {
    int64_t op = rd64();
    int64_t ni = rd64();
    int64_t *I = calloc((size_t)(ni > 0 ? ni : 1), 8);
    rd(I, (size_t)ni * 8);
    int64_t nd = rd64();
    double *D = calloc((size_t)(nd > 0 ? nd : 1), 8);
    rd(D, (size_t)nd * 8);
    int64_t na = rd64();
    blob A[16];
    if (na < 0 || na > 16) { fprintf(stderr, "san_driver: %lld arrays\n", (long long)na); return 3; }
    for (int64_t i = 0; i < na; ++i) {
        A[i].n = rd64();
        /* exact-size allocations: an overrun of any input is an ASan report */
        A[i].p = malloc((size_t)(A[i].n > 0 ? A[i].n : 1));
        rd(A[i].p, (size_t)A[i].n);
    }
    int64_t rc = 0;
    switch (op) {
    case OP_NN_BRUTE:
    case OP_NN_KD: {  /* ints: n, lds, m, ldt, md, nthreads; arrays: src, tgt */
        int64_t n = I[0], lds = I[1], m = I[2], ldt = I[3];
        int md = (int)I[4], nt = (int)I[5];
        int32_t *idx = out_alloc(n * 4);
        double *dist = out_alloc(n * 8), *d2 = out_alloc(n * 8);
        if (op == OP_NN_BRUTE) {
            rc = orc_nn_brute(A[0].p, n, lds, A[1].p, m, ldt, md, idx, dist, d2, nt);
        } else {
            void *kd = orc_kd_build(A[1].p, m, ldt, md);
            rc = orc_kd_query(kd, A[0].p, n, lds, idx, dist, d2, nt);
            orc_kd_free(kd);
        }
        break;
    }
    case OP_SORT: {  /* ints: n; arrays: d */
        int64_t *order = out_alloc(I[0] * 8);
        orc_sort_order(A[0].p, I[0], order);
        break;
    }
    case OP_FRAC: {  /* ints: lds, ldc, n, N, md, literal; dbls: lam; arrays: src, corr, d */
        double res[3];
        int64_t k = 0;
        rc = orc_optimal_fraction(A[0].p, I[0], A[1].p, I[1], A[2].p, I[2], I[3], (int)I[4], D[0], (int)I[5],
                                  &res[0], &k, &res[2]);
        memcpy(&res[1], &k, 8);
        out_copy(res, sizeof res);
        break;
    }
    case OP_FRMSD: {  /* ints: k, lds, ldc, rows, md; dbls: fraction, lam; arrays: src, corr */
        double v = orc_frmsd(D[0], I[0], A[0].p, I[1], A[1].p, I[2], I[3], (int)I[4], D[1]);
        out_copy(&v, 8);
        break;
    }
    case OP_FIT: {  /* ints: k, lds, ldt, allow_reflection; arrays: src, tgt */
        double *T = out_alloc(9 * 8);
        orc_fit_rigid2d(A[0].p, I[1], A[1].p, I[2], I[0], (int)I[3], T);
        break;
    }
    case OP_APPLY: {  /* ints: n, ld; arrays: pts, T */
        orc_apply_xy(A[0].p, I[0], I[1], A[1].p);
        out_copy(A[0].p, A[0].n);
        break;
    }
    case OP_RUN: {  /* ints: n, lds, m, ldt, md, max_iter, allow, literal, nthreads, max_calls, want_idx;
                       dbls: lam0, lam1, thr; arrays: src, tgt */
        int64_t n = I[0], mc = I[9];
        orc_trace tr;
        memset(&tr, 0, sizeof tr);
        tr.max_calls = (int32_t)mc;
        tr.k = out_alloc(mc * 8);
        tr.frmsd = out_alloc(mc * 8);
        tr.lam = out_alloc(mc * 8);
        tr.gap = out_alloc(mc * 8);
        tr.T = out_alloc(mc * 9 * 8);
        tr.idx = I[10] ? out_alloc(mc * n * 4) : NULL;
        rc = orc_run(A[0].p, n, I[1], A[1].p, I[2], I[3], (int)I[4], D[0], D[1], D[2], (int)I[5], (int)I[6],
                     (int)I[7], (int)I[8], &tr);
        out_copy(A[0].p, A[0].n);
        int64_t cnt[4] = {tr.n_calls, tr.n_fits, tr.iters[0], tr.iters[1]};
        out_copy(cnt, sizeof cnt);
        break;
    }
    case OP_THREADS: {
        int64_t t = orc_num_threads_max();
        out_copy(&t, 8);
        break;
    }
    default:
        fprintf(stderr, "san_driver: unknown op %lld\n", (long long)op);
        return 3;
    }
    fwrite(&rc, 8, 1, stdout);
    int64_t no = n_out;
    fwrite(&no, 8, 1, stdout);
    for (int i = 0; i < n_out; ++i) {
        fwrite(&out_blobs[i].n, 8, 1, stdout);
        fwrite(out_blobs[i].p, 1, (size_t)out_blobs[i].n, stdout);
        free(out_blobs[i].p);
    }
    for (int64_t i = 0; i < na; ++i) free(A[i].p);
    free(I);
    free(D);
    return 0;
}
