// selcheck.hip -- GPU self-check and per-kernel timing of the bucketed FRMSD selection
// (coregistrationgame_amd/csrc/k_select.hip; tools only, not shipped).
// Build: make -C coregistrationgame_amd/csrc selcheck
// Run:   ./tools/selcheck [n] [reps] [mode] [lambda]
//   mode 0: C3-like residuals (60 % inliers: 0.09 (x1^2 + x2^2) + x3^2, 40 % outliers:
//           Rayleigh(2 m) distances); 1: 30 % exact zeros + exponential; 2: all rows
//           equal; 3: 5 distinct distances; 4: exponential; 5: geometric (huge range)
// Checks k, FRMSD and the threshold pair against a CPU sort by (key, orig); prints the
// time of each of the four kernels (events around each, median over reps).
#include "../coregistrationgame_amd/csrc/k_select.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

using namespace ficp;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

static unsigned long long hkey(double v) {
    unsigned long long u;
    memcpy(&u, &v, 8);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

static double hfrmsd(long long k, long long N, double S, double lam) {
    const double frac = (double)k / (double)N;
    return (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
}

// `selcheck log2`: the bounds' fast log2 (frmsd_bounds.h fb::lg2 / fast_log2) against the
// host's long-double log2 over random doubles of every exponent (subnormals, |e| ~ 1000),
// the mantissa split point sqrt(1/2), powers of two and the extremes.  The selection's
// margin kMarg (1e-9, log2 units) assumes an absolute error far below it: the check
// fails above kMarg / 100.
__global__ void k_lg2_probe(const double *x, double *y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = fb::lg2(x[i]);
}

static int log2_check() {
    std::mt19937_64 rng(2025);
    std::vector<double> x;
    const double edge[] = {1.0, 2.0, 0.5, 0.70710678118654752, 0.7071067811865475, 0.7071067811865476,
                           1.4142135623730951, 1.4142135623730950, 1.0 + 1e-16, 1.0 - 1e-16,
                           1.7976931348623157e308, 2.2250738585072014e-308, 2.2250738585072009e-308,
                           4.9406564584124654e-324, 1e-320, 3.0, 1e300, 1e-300};
    for (double v : edge) x.push_back(v);
    for (int e = -1074; e <= 1023; ++e) x.push_back(ldexp(1.0, e));
    for (int i = 0; i < 2000000; ++i) {
        unsigned long long u = rng();
        u &= 0x7fffffffffffffffULL;                    // positive
        if ((u >> 52) == 0x7ff) u &= ~(1ULL << 62);    // finite
        double v;
        memcpy(&v, &u, 8);
        if (v > 0.0) x.push_back(v);
    }
    const int n = (int)x.size();
    double *dx, *dy;
    CK(hipMalloc(&dx, 8 * (size_t)n));
    CK(hipMalloc(&dy, 8 * (size_t)n));
    CK(hipMemcpy(dx, x.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    k_lg2_probe<<<(n + 255) / 256, 256>>>(dx, dy, n);
    CK(hipGetLastError());
    std::vector<double> y(n);
    CK(hipMemcpy(y.data(), dy, 8 * (size_t)n, hipMemcpyDeviceToHost));
    CK(hipFree(dx));
    CK(hipFree(dy));
    double worst = 0.0, worst_x = 0.0, worst_sub = 0.0;
    for (int i = 0; i < n; ++i) {
        const double err = (double)fabsl((long double)y[i] - log2l((long double)x[i]));
        if (!(err <= worst)) { worst = err; worst_x = x[i]; }
        if (x[i] < 2.2250738585072014e-308 && err > worst_sub) worst_sub = err;
    }
    const double bound = fb::kMarg / 100.0;
    printf("log2 n=%d max_abs_err=%.3e at x=%.17g (subnormal max %.3e) bound=%.1e %s\n", n, worst, worst_x,
           worst_sub, bound, worst < bound ? "ok" : "FAIL");
    return worst < bound ? 0 : 1;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "log2") == 0) return log2_check();
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const double lam = argc > 4 ? atof(argv[4]) : 3.0;
    std::mt19937_64 rng(7 + mode);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    std::exponential_distribution<double> ex(1.0);
    std::vector<unsigned long long> key(n);
    std::vector<uint32_t> orig(n);
    std::vector<double> r(n);
    for (int64_t i = 0; i < n; ++i) {
        double d2 = 0.0;
        if (mode == 0) {
            if (ud(rng) < 0.6) {
                const double a = nd(rng), b = nd(rng), c = nd(rng);
                d2 = 0.09 * (a * a + b * b) + c * c;
            } else {
                const double d = 2.0 * sqrt(-2.0 * log(1.0 - ud(rng)));
                d2 = d * d;
            }
        } else if (mode == 1) {
            d2 = ud(rng) < 0.3 ? 0.0 : ex(rng);
        } else if (mode == 2) {
            d2 = 2.25;
        } else if (mode == 3) {
            d2 = floor(ex(rng) * 1.25);
        } else if (mode == 4) {
            d2 = ex(rng);
        } else {
            d2 = pow(10.0, -8.0 + 12.0 * ud(rng));
        }
        const double d = sqrt(d2);
        key[i] = hkey(d);
        r[i] = d2;
        orig[i] = (uint32_t)i;
    }
    std::shuffle(orig.begin(), orig.end(), rng);
    // CPU reference: stable order by (key, orig), prefix sums, first minimum
    std::vector<uint32_t> ord(n);
    for (int64_t i = 0; i < n; ++i) ord[i] = (uint32_t)i;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
        return key[a] < key[b] || (key[a] == key[b] && orig[a] < orig[b]);
    });
    std::vector<double> S(n + 1, 0.0);
    for (int64_t j = 0; j < n; ++j) S[j + 1] = S[j] + r[ord[j]];
    long long bk = 0;
    double bf = INFINITY;
    for (int64_t k = 1; k <= n; ++k) {
        const double f = hfrmsd(k, n, S[k], lam);
        if (f < bf) {
            bf = f;
            bk = k;
        }
    }
    // device
    unsigned long long *dkey, *drange;
    uint32_t *dorig;
    double *dr;
    void *tmp;
    IterState *st;
    CK(hipMalloc(&dkey, n * 8));
    CK(hipMalloc(&dorig, n * 4));
    CK(hipMalloc(&dr, n * 8));
    CK(hipMalloc(&drange, 64));
    CK(hipMalloc(&tmp, sel_tmp_bytes(n)));
    CK(hipMalloc(&st, sizeof(IterState)));
    CK(hipMemset(st, 0, sizeof(IterState)));
    CK(hipMemcpy(dkey, key.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dorig, orig.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, r.data(), n * 8, hipMemcpyHostToDevice));
    unsigned long long kmn = ~0ULL, kmx = 0;
    for (int64_t i = 0; i < n; ++i) {
        kmn = std::min(kmn, key[i]);
        kmx = std::max(kmx, key[i]);
    }
    unsigned long long hr[2] = {~kmn, kmx};
    CK(hipMemcpy(drange, hr, 16, hipMemcpyHostToDevice));
    CK(launch_select_init(tmp, n, 0));
    const SelWS w = carve(tmp, n);
    const int gb = gather_blocks(n);
    hipEvent_t ev[5];
    for (auto &evx : ev) CK(hipEventCreate(&evx));
    std::vector<std::vector<float>> tk(4), tkw(4);
    int bad = 0;
    // even reps: the uniform bucket map (a stage's first call); odd reps: the windowed map
    // centred on the true threshold key moved by 0, +8, -64, +512 uniform bucket widths
    // (a later call; the last two put the threshold outside the fine window)
    const int s_uni = kmx > kmn ? std::max(0, 64 - __builtin_clzll(kmx - kmn) - NB_LOG) : 0;
    const unsigned long long tk_true = bk > 0 ? key[ord[bk - 1]] : kmn;
    unsigned cand_u = 0, cand_w[4] = {0, 0, 0, 0};
    for (int it = 0; it < reps; ++it) {
        IterState hs{};
        const int wq = (it / 2) % 4;
        if (it & 1) {
            const long long offs[4] = {0, 8, -64, 512};
            const long long d = offs[wq] * (long long)(1ULL << s_uni);
            unsigned long long c = tk_true + (unsigned long long)d;
            if (d < 0 && tk_true - kmn < (unsigned long long)(-d)) c = kmn;
            if (d > 0 && kmx - tk_true < (unsigned long long)d) c = kmx;
            hs.phase = PH_LOOP;
            hs.k = 1;
            hs.tkey = c;
            hs.tmove = 0;
        } else {
            hs.phase = PH_HEAD;
        }
        CK(hipMemcpy(st, &hs, sizeof hs, hipMemcpyHostToDevice));
        CK(hipEventRecord(ev[0], 0));
        hipLaunchKernelGGL(k_sel_hist, dim3(hist_blocks(n)), dim3(HHT), 0, 0, dkey, dr, n, drange,
                           (int64_t)0, w, (const int *)nullptr, hist_pack(n), (const IterState *)st);
        hipLaunchKernelGGL(k_sel_reduce, dim3(NB / RBPB), dim3(1024), 0, 0, w, hist_blocks(n),
                           (const int *)nullptr, hist_pack(n), (long long *)nullptr);
        CK(hipEventRecord(ev[1], 0));
        static unsigned gen = 0;
        LoopCtl lc{};
        const bool bgf = (it % 8) >= 6;  // reps 6, 7 of every 8 (both maps): the library's
                                         // default, bounds + gather + final in one launch
        if (bgf) {
            CK(hipEventRecord(ev[2], 0));
            hipLaunchKernelGGL(k_sel_bgf, dim3(gb + 1), dim3(GT), 0, 0, dkey, dorig, dr, n, w, lam,
                               (const double *)nullptr, (const int *)nullptr, hist_pack(n).fixb,
                               FitSrc{}, gen + 1, gen + 1, st, lc, 0, (int *)nullptr,
                               (int64_t)std::max<int64_t>(n, 1));
            ++gen;
        } else if (it & 2) {  // reps 2, 3 of every 4: bounds + gather in one launch
            CK(hipEventRecord(ev[2], 0));
            hipLaunchKernelGGL(k_sel_bounds_gather, dim3(gb + 1), dim3(GT), 0, 0, dkey, dorig, dr,
                               n, w, lam, (const double *)nullptr, (const int *)nullptr,
                               hist_pack(n).fixb, FitSrc{}, gen + 1, gen + 1);
            ++gen;
        } else {
            hipLaunchKernelGGL(k_sel_bounds, dim3(1), dim3(HT), 0, 0, w, n, lam,
                               (const double *)nullptr, (const int *)nullptr, hist_pack(n).fixb);
            CK(hipEventRecord(ev[2], 0));
            hipLaunchKernelGGL(k_sel_gather, dim3(gb), dim3(GT), 0, 0, dkey, dorig, dr, n, w,
                               (const int *)nullptr, FitSrc{});
        }
        CK(hipEventRecord(ev[3], 0));
        if (!bgf)
            hipLaunchKernelGGL(k_sel_final, dim3(1), dim3(HT), 0, 0, w, gb, n, lam,
                               (const double *)nullptr, st, (const int *)nullptr, lc, 0, (int *)nullptr,
                               FitSrc{}, (int64_t)std::max<int64_t>(n, 1));
        CK(hipEventRecord(ev[4], 0));
        CK(hipEventSynchronize(ev[4]));
        for (int q = 0; q < 4; ++q) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[q], ev[q + 1]));
            ((it & 1) ? tkw : tk)[q].push_back(ms * 1000.f);
        }
        {
            SelCtl cc;
            CK(hipMemcpy(&cc, w.ctl, sizeof cc, hipMemcpyDeviceToHost));
            if (it & 1) cand_w[wq] = cc.ccount;
            else cand_u = cc.ccount;
        }
        IterState h;
        CK(hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost));
        bool ok = h.k == bk;
        if (!ok && h.k > 0 && h.k <= n) {  // a rounding-level tie of the FRMSD curve
            const double fg = hfrmsd(h.k, n, S[h.k], lam);
            ok = fabs(fg - bf) <= 1e-12 * bf;
        }
        if (ok && h.k > 0) {
            const uint32_t tp = ord[h.k - 1];
            ok = h.tkey == key[tp] && (uint32_t)h.torig == orig[tp] &&
                 fabs(h.frmsd - hfrmsd(h.k, n, S[h.k], lam)) <= 1e-12 * h.frmsd;
        }
        if (!ok) {
            ++bad;
            if (bad < 4)
                printf("MISMATCH rep %d: gpu k=%lld f=%.17g tkey=%llx torig=%lld | cpu k=%lld "
                       "f=%.17g\n",
                       it, h.k, h.frmsd, h.tkey, h.torig, bk, bf);
        }
    }
    SelCtl ctl;
    CK(hipMemcpy(&ctl, w.ctl, sizeof ctl, hipMemcpyDeviceToHost));
    const unsigned stats[3] = {ctl.err, ctl.levels, ctl.radix};  // the report's three words
    const char *names[4] = {"hist+red", "bounds", "gather", "final"};
    printf("n=%lld mode=%d lam=%g k=%lld cand=%u window cand (+0,+8,-64,+512)=%u,%u,%u,%u "
           "buckets=[%d,%d] levels=%u chunked=%u radix=%u err=%u bad=%d/%d\n",
           (long long)n, mode, lam, bk, cand_u, cand_w[0], cand_w[1], cand_w[2], cand_w[3], ctl.b0,
           ctl.b1, stats[1] & 0xffffu, stats[1] >> 16, stats[2], stats[0], bad, reps);
    for (int wv = 0; wv < 2; ++wv) {
        auto &tt = wv ? tkw : tk;
        if (tt[0].empty()) continue;
        float tot = 0.f;
        printf("  %s map:", wv ? "window " : "uniform");
        for (int q = 0; q < 4; ++q) {
            std::sort(tt[q].begin(), tt[q].end());
            const float med = tt[q][tt[q].size() / 2];
            tot += med;
            printf(" %s %.2f", names[q], med);
        }
        printf(" total %.2f us (median)\n", tot);
    }
#ifdef SEL_PROF
    unsigned long long ts[32];
    CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_selprof), sizeof ts));
    printf("  final phases (us, last rep):");
    for (int q = 1; q <= 6; ++q) printf(" %d:%.2f", q, (double)(ts[q] - ts[q - 1]) / 100.0);
    printf("\n  final_lds: minmax %.2f count %.2f scan %.2f scatter %.2f rank %.2f vscan %.2f frmsd %.2f\n",
           (ts[16] - ts[2]) / 100.0, (ts[17] - ts[16]) / 100.0, (ts[18] - ts[17]) / 100.0,
           (ts[19] - ts[18]) / 100.0, (ts[3] - ts[19]) / 100.0, (ts[20] - ts[3]) / 100.0,
           (ts[4] - ts[20]) / 100.0);
    unsigned long long tc[32];
    CK(hipMemcpyFromSymbol(tc, HIP_SYMBOL(g_selclk), sizeof tc));
    printf("  clock: bounds %llu cycles in %.2f us (%.0f MHz); final %llu cycles in %.2f us (%.0f MHz)\n",
           tc[14] - tc[8], (ts[14] - ts[8]) / 100.0, (double)(tc[14] - tc[8]) / ((ts[14] - ts[8]) / 100.0),
           tc[6] - tc[0], (ts[6] - ts[0]) / 100.0, (double)(tc[6] - tc[0]) / ((ts[6] - ts[0]) / 100.0));
    printf("  bounds: loads %.2f sums+scans %.2f U1 %.2f U %.2f lb %.2f tail %.2f\n",
           (ts[9] - ts[8]) / 100.0, (ts[10] - ts[9]) / 100.0, (ts[11] - ts[10]) / 100.0,
           (ts[12] - ts[11]) / 100.0, (ts[13] - ts[12]) / 100.0, (ts[14] - ts[13]) / 100.0);
#endif
    return bad ? 1 : 0;
}
