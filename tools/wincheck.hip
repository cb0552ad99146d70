// wincheck.hip -- adversarial self-check of the window selection path (k_select.hip
// k_sel_win) against a CPU stable sort + scan, and against the full
// bucketed path (launch_select) on the same state (tools only, not shipped).
// Build: make -C coregistrationgame_amd/csrc wincheck
// Run:   ./tools/wincheck [n] [mode] [lambda]
//   mode 0: C3-like residuals; 1: 30 % exact zeros + exponential; 2: all rows equal;
//        3: 5 distinct distances; 4: exponential; 5: 20 decades; 6: C3-like with 0.2 %
//        inf and 0.1 % NaN rows; 7: C3-like, the rows of the first quarter sorted by r
//        (hundreds of window rows in one workgroup); 8: C3-like on a 1e-3 grid (exact
//        ties everywhere, the threshold's included)
// For every window size (the floor at its start, 3 doublings below and above, one past
// the limit) and every placement of the previous threshold key c relative to the true
// threshold key tk (at it, just inside / just outside either window edge, 512 window
// widths away on either side), one k_sel_win launch from a loop-body state must either
//   * decide: k, FRMSD, the threshold pair (key, caller index) equal to the CPU's (k may
//     differ only inside a rounding-level tie of the curve, 1e-12 relative) and to the
//     full path's, the fused fit's T equal to the CPU fit of the selected rows; or
//   * fall back (kFlagRetry): the state unchanged but win_fail / nn_reuse, and the full
//     selection run after it bit-identical (whole IterState) to the full path run alone.
// Prints one line per case; exit status 1 on any mismatch.
#include "../coregistrationgame_amd/csrc/k_select.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

using namespace ficp;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

__global__ void k_keys_of_r(const double *r, int64_t n, unsigned long long *key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = key_of_r(r[i]);  // the selection's own key derivation
}

static double hfrmsd(long long k, long long N, double S, double lam) {
    const double frac = (double)k / (double)N;
    return (1.0 / pow(frac, lam)) * sqrt(S / (double)k);
}

// the CPU fit of the selected rows (ficp.py:89-110 in the closed form of fit_solve_T, long
// double sums of the pivot-shifted pairs, pivot 0)
static void cpu_fit(const std::vector<uint32_t> &ord, long long k, const std::vector<double> &xs,
                    const std::vector<double> &ys, const std::vector<double> &xt,
                    const std::vector<double> &yt, double T[6]) {
    long double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (long long j = 0; j < k; ++j) {
        const uint32_t i = ord[j];
        c[0] += xs[i], c[1] += ys[i], c[2] += xt[i], c[3] += yt[i];
        c[4] += (long double)xs[i] * xt[i], c[5] += (long double)xs[i] * yt[i];
        c[6] += (long double)ys[i] * xt[i], c[7] += (long double)ys[i] * yt[i];
    }
    const long double kk = (long double)k;
    const long double ctx = c[2] / kk, cty = c[3] / kk, csx = c[0] / kk, csy = c[1] / kk;
    const long double H0 = c[4] - c[0] * ctx, H1 = c[5] - c[0] * cty, H2 = c[6] - c[1] * ctx,
                      H3 = c[7] - c[1] * cty;
    const long double A = H0 + H3, B = H1 - H2, nrm = sqrtl(A * A + B * B);
    const long double cc = nrm > 0 ? A / nrm : 1.0L, ss = nrm > 0 ? B / nrm : 0.0L;
    T[0] = (double)cc, T[1] = (double)-ss, T[3] = (double)ss, T[4] = (double)cc;
    T[2] = (double)(ctx - (csx * cc - csy * ss));
    T[5] = (double)(cty - (csx * ss + csy * cc));
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    const double lam = argc > 3 ? atof(argv[3]) : 3.0;
    std::mt19937_64 rng(11 + 7 * mode);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    std::exponential_distribution<double> ex(1.0);
    std::vector<double> r(n + 1, 0.0), xs(n + 1), ys(n + 1), xt(n + 1), yt(n + 1);
    auto c3 = [&]() {
        if (ud(rng) < 0.6) {
            const double a = nd(rng), b = nd(rng), c = nd(rng);
            return 0.09 * (a * a + b * b) + c * c;
        }
        const double d = 2.0 * sqrt(-2.0 * log(1.0 - ud(rng)));
        return d * d;
    };
    for (int64_t i = 0; i < n; ++i) {
        double d2;
        switch (mode) {
            case 1: d2 = ud(rng) < 0.3 ? 0.0 : ex(rng); break;
            case 2: d2 = 2.25; break;
            case 3: d2 = floor(ex(rng) * 1.25); break;
            case 4: d2 = ex(rng); break;
            case 5: d2 = pow(10.0, -8.0 + 12.0 * ud(rng)); break;
            case 6: {
                const double u = ud(rng);
                d2 = u < 0.002 ? INFINITY : (u < 0.003 ? NAN : c3());
                break;
            }
            case 8: d2 = std::round(c3() * 1000.0) / 1000.0; break;
            default: d2 = c3();
        }
        r[i] = d2;
        // correspondences: a rotated, shifted copy + noise (the fused fit's inputs)
        xs[i] = -50.0 + 100.0 * ud(rng);
        ys[i] = -50.0 + 100.0 * ud(rng);
        xt[i] = 0.999 * xs[i] - 0.0447 * ys[i] + 0.3 + 0.05 * nd(rng);
        yt[i] = 0.0447 * xs[i] + 0.999 * ys[i] - 0.2 + 0.05 * nd(rng);
    }
    if (mode == 7) std::sort(r.begin(), r.begin() + n / 4);
    std::vector<uint32_t> orig(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) orig[i] = (uint32_t)i;
    std::shuffle(orig.begin(), orig.begin() + n, rng);

    double *dr, *dxs, *dys, *dxt, *dyt;
    uint32_t *dorig;
    unsigned long long *dkey, *drange;
    double *dlams;
    void *tmp;
    IterState *st;
    int *dflag;
    CK(hipMalloc(&dr, (n + 1) * 8));
    CK(hipMalloc(&dxs, (n + 1) * 8));
    CK(hipMalloc(&dys, (n + 1) * 8));
    CK(hipMalloc(&dxt, (n + 1) * 8));
    CK(hipMalloc(&dyt, (n + 1) * 8));
    CK(hipMalloc(&dorig, (n + 1) * 4));
    CK(hipMalloc(&dkey, (n + 1) * 8));
    CK(hipMalloc(&drange, 64));
    CK(hipMalloc(&dlams, 16));
    CK(hipMalloc(&tmp, sel_tmp_bytes(n)));
    CK(hipMalloc(&st, sizeof(IterState)));
    CK(hipMalloc(&dflag, 4));
    CK(hipMemcpy(dr, r.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxs, xs.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dys, ys.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxt, xt.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyt, yt.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dorig, orig.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    const double lams[2] = {lam, lam};
    CK(hipMemcpy(dlams, lams, 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_keys_of_r, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dr, n, dkey);
    std::vector<unsigned long long> key(n);
    CK(hipMemcpy(key.data(), dkey, n * 8, hipMemcpyDeviceToHost));
    // the NN's key range of the call (every row)
    unsigned long long kmn = ~0ULL, kmx = 0;
    for (int64_t i = 0; i < n; ++i) kmn = std::min(kmn, key[i]), kmx = std::max(kmx, key[i]);
    const unsigned long long hr[2] = {~kmn, kmx};
    CK(hipMemcpy(drange, hr, 16, hipMemcpyHostToDevice));

    // CPU reference: stable order by (key, orig), prefix sums, first minimum (strict <)
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
        if (f < bf) bf = f, bk = k;
    }
    if (bk == 0) {
        printf("n=%lld mode=%d: no finite FRMSD, nothing to check\n", (long long)n, mode);
        return 0;
    }
    const unsigned long long tk = key[ord[bk - 1]];
    auto cpu_ok = [&](const IterState &h, const char *who, char *why) -> bool {
        bool ok = h.k == bk;
        if (!ok && h.k > 0 && h.k <= n)  // a rounding-level tie of the curve
            ok = fabs(hfrmsd(h.k, n, S[h.k], lam) - bf) <= 1e-12 * bf;
        if (!ok) {
            sprintf(why, "%s k=%lld cpu k=%lld", who, h.k, bk);
            return false;
        }
        const uint32_t tp = ord[h.k - 1];
        if (h.tkey != key[tp] || (uint32_t)h.torig != orig[tp]) {
            sprintf(why, "%s threshold (%llx,%lld) cpu (%llx,%u)", who, h.tkey, h.torig, key[tp], orig[tp]);
            return false;
        }
        if (!(fabs(h.frmsd - hfrmsd(h.k, n, S[h.k], lam)) <= 1e-12 * h.frmsd)) {
            sprintf(why, "%s frmsd %.17g cpu %.17g", who, h.frmsd, hfrmsd(h.k, n, S[h.k], lam));
            return false;
        }
        double T[6];
        cpu_fit(ord, h.k, xs, ys, xt, yt, T);
        const int el[6] = {0, 1, 2, 3, 4, 5};
        for (int e : el) {
            const double tol = (e == 2 || e == 5) ? 1e-9 : 1e-12;
            if (!(fabs(h.T[e] - T[e]) <= tol)) {
                sprintf(why, "%s T[%d] %.17g cpu %.17g", who, e, h.T[e], T[e]);
                return false;
            }
        }
        return true;
    };

    CK(launch_select_init(tmp, n, 0));
    LoopCtl lc{};
    lc.lams = dlams;
    lc.lam_in[0] = lc.lam_in[1] = lam;
    lc.nstages = 2;
    lc.max_iter = 1000;
    lc.threshold = 1e-6;
    const FitSrc fs{dxs, dys, dxt, dyt, 0.0, 0.0, 1, 0};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    const int wstart = win_start_log(n), whmax = win_hmax_log(n);
    // floors: lh = floor + 1 (tmove 0); the last one is past the limit (lh > hmax: the
    // launch must refuse at once)
    const int floors[5] = {std::max(kWinHMinLog, wstart - 3), wstart, wstart + 2, whmax - 1, whmax};
    int bad = 0, n_win = 0, n_fb = 0;
    float t_win = 0.f;
    int n_t = 0;
    for (int fl : floors) {
        const int lh = fl + 1;
        const unsigned long long H = 1ULL << lh;
        auto sat_add = [](unsigned long long a, unsigned long long b) { return a > ~0ULL - b ? ~0ULL : a + b; };
        auto sat_sub = [](unsigned long long a, unsigned long long b) { return a < b ? 0ULL : a - b; };
        const struct {
            const char *name;
            unsigned long long c;
        } places[7] = {
            {"at", tk},
            {"in_lo_edge", sat_add(tk, H)},       // wlo = tk: the threshold is the window's lowest key
            {"out_lo_edge", sat_add(tk, H + 1)},  // wlo = tk + 1: just below the window
            {"in_hi_edge", sat_sub(tk, H - 1)},   // whi = tk + 1: the window's highest key
            {"out_hi_edge", sat_sub(tk, H)},      // whi = tk: just above the window
            {"far_above", sat_add(tk, 512 * H)},
            {"far_below", sat_sub(tk, 512 * H)},
        };
        for (const auto &pl : places) {
            IterState s0{};
            s0.phase = PH_LOOP;
            s0.stage = 0;
            s0.it = 1;
            s0.k = bk;
            s0.n_src = n;
            s0.lam_cur = lam;
            s0.tkey = pl.c;
            s0.torig = 0;
            s0.tmove = 0;
            s0.wfloor = fl;
            s0.cur = 1e300;  // the loop goes on: the fused fit is solved
            s0.n_nn = 3;
            s0.n_fit = 2;
            s0.apply = 1;
            for (int e = 0; e < 9; ++e) s0.T[e] = s0.Ttot[e] = (e % 4 == 0) ? 1.0 : 0.0;
            const unsigned long long wlo = pl.c > H ? pl.c - H : 0ULL;
            const unsigned long long whi = pl.c < ~0ULL - H ? pl.c + H : ~0ULL;
            long long wrows = 0;
            for (int64_t i = 0; i < n; ++i) wrows += (key[i] >= wlo && key[i] < whi) ? 1 : 0;
            // (1) the full path alone from s0
            IterState full{};
            CK(hipMemcpy(st, &s0, sizeof s0, hipMemcpyHostToDevice));
            CK(launch_select(nullptr, dorig, dr, n, 0.0, &st->lam_cur, drange, 0, tmp, st, &st->done, &lc,
                             dflag, 0, &fs, 0));
            CK(hipMemcpy(&full, st, sizeof full, hipMemcpyDeviceToHost));
          {
            // (2) the window path from s0 (k_sel_win)
            IterState win{};
            int flag = -1;
            CK(hipMemcpy(st, &s0, sizeof s0, hipMemcpyHostToDevice));
            CK(hipMemcpy(dflag, &flag, 4, hipMemcpyHostToDevice));
            CK(hipEventRecord(e0, 0));
            CK(launch_select_win(dr, dorig, n, drange, 0, tmp, st, lc, dflag, 0, fs, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipMemcpy(&win, st, sizeof win, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&flag, dflag, 4, hipMemcpyDeviceToHost));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            char why[256] = "";
            bool ok = cpu_ok(full, "full", why);
            const char *path;
            if (flag == kFlagRetry) {
                path = "fallback";
                ++n_fb;
                IterState want = s0;
                want.win_fail = 1;
                want.nn_reuse = 1;
                if (ok && memcmp(&want, &win, sizeof want) != 0) {
                    ok = false;
                    sprintf(why, "fallback changed the state beyond win_fail / nn_reuse");
                }
                // the host's retry: the full selection of the same call on that state
                IterState again{};
                CK(launch_select(nullptr, dorig, dr, n, 0.0, &st->lam_cur, drange, 0, tmp, st, &st->done,
                                 &lc, dflag, 0, &fs, 0));
                CK(hipMemcpy(&again, st, sizeof again, hipMemcpyDeviceToHost));
                if (ok && memcmp(&again, &full, sizeof again) != 0) {
                    ok = false;
                    sprintf(why, "retry's full path differs from the full path alone (k %lld vs %lld)",
                            again.k, full.k);
                }
            } else {
                path = "window";
                ++n_win;
                t_win += ms * 1000.f;
                ++n_t;
                if (ok) ok = cpu_ok(win, "window", why);
                if (ok && (win.k != full.k || win.tkey != full.tkey || win.torig != full.torig ||
                           win.phase != full.phase || win.it != full.it || win.n_nn != full.n_nn ||
                           win.win_fail != 0 || win.nn_reuse != full.nn_reuse)) {
                    ok = false;
                    sprintf(why, "window vs full: k %lld/%lld phase %d/%d", win.k, full.k, win.phase, full.phase);
                }
                if (ok && !(flag == (win.done | kFlagWinNext) || flag == win.done)) {
                    ok = false;
                    sprintf(why, "host flag %d", flag);
                }
            }
            if (!ok) ++bad;
            printf("n=%lld mode=%d lam=%g floor=2^%d window=2^%d place=%-11s rows_in_window=%-7lld "
                   "form=%s path=%-8s k=%lld %s%s\n",
                   (long long)n, mode, lam, fl, lh, pl.name, wrows, "sel_win ", path,
                   (long long)(flag == kFlagRetry ? full.k : win.k), ok ? "ok" : "MISMATCH: ", ok ? "" : why);
          }
        }
    }
    printf("summary n=%lld mode=%d lam=%g cpu_k=%lld launches=%d window=%d fallback=%d bad=%d "
           "window_launch_us(mean)=%.1f\n",
           (long long)n, mode, lam, bk, n_win + n_fb, n_win, n_fb, bad, n_t ? t_win / n_t : 0.f);
    return bad ? 1 : 0;
}
