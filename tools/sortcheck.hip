// sortcheck.hip -- GPU self-check of the residual sort (tools only, not shipped).
// Build: make -C coregistrationgame_amd/csrc sortcheck
// Run:   ./tools/sortcheck [n] [reps] [use_orig] [mode] [with_r]
//   mode 0: exponential distances; 1: work-order cell keys (cell << 32 | i), random
//   cells; 2: cell keys, monotone cells; 3: all keys equal; 4: 5 distinct distances
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../coregistrationgame_amd/csrc/ficp_internal.h"

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

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int use_orig = argc > 3 ? atoi(argv[3]) : 1;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    const int with_r = argc > 5 ? atoi(argv[5]) : 1;
    std::mt19937_64 rng(42);
    std::exponential_distribution<double> ex(1.0);
    std::vector<unsigned long long> key(n);
    std::vector<uint32_t> orig(n);
    std::vector<double> r(n);
    for (int64_t i = 0; i < n; ++i) {
        double d = ex(rng);
        if (mode == 4) d = floor(d * 1.25);
        key[i] = hkey(d);
        if (mode == 1) key[i] = ((unsigned long long)(rng() % 4000000ULL) << 32) | (uint64_t)i;
        if (mode == 2) key[i] = ((unsigned long long)(i / 2) << 32) | (uint64_t)i;
        if (mode == 3) key[i] = hkey(1.5);
        r[i] = d * d;
        orig[i] = (uint32_t)i;
    }
    if (use_orig) std::shuffle(orig.begin(), orig.end(), rng);
    // expected order: positions sorted by (key, orig)
    std::vector<uint32_t> exp(n);
    for (int64_t i = 0; i < n; ++i) exp[i] = (uint32_t)i;
    std::stable_sort(exp.begin(), exp.end(), [&](uint32_t a, uint32_t b) {
        if (key[a] != key[b]) return key[a] < key[b];
        return orig[a] < orig[b];
    });
    unsigned long long *dk, *drange;
    uint32_t *dorig, *dorder;
    double *dr, *drs;
    void *tmp;
    CK(hipMalloc(&dk, n * 8));
    CK(hipMalloc(&drange, 64));
    CK(hipMalloc(&dorig, n * 4));
    CK(hipMalloc(&dorder, n * 4));
    CK(hipMalloc(&dr, n * 8));
    CK(hipMalloc(&drs, n * 8));
    CK(hipMalloc(&tmp, sort_tmp_bytes(n)));
    CK(hipMemcpy(dk, key.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dorig, orig.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, r.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemset(sort_timeout_flag(tmp, n), 0, 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint32_t> got(n);
    std::vector<double> grs(n);
    int bad = 0;
    for (int rep = 0; rep < reps; ++rep) {
        CK(launch_key_range(dk, n, drange, s));
        CK(launch_sort(dk, use_orig ? dorig : nullptr, n, drange, dorder, with_r ? dr : nullptr,
                              with_r ? drs : nullptr, tmp, nullptr, s));
        CK(hipStreamSynchronize(s));
        uint32_t flag = 0;
        CK(hipMemcpy(&flag, sort_timeout_flag(tmp, n), 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(got.data(), dorder, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(grs.data(), drs, n * 8, hipMemcpyDeviceToHost));
        int64_t mism = 0, rsm = 0, first = -1;
        for (int64_t j = 0; j < n; ++j) {
            if (got[j] != exp[j]) {
                if (first < 0) first = j;
                ++mism;
            }
            if (with_r && got[j] < n && grs[j] != r[got[j]]) ++rsm;
        }
        printf("rep %d: flag=%u mismatches=%lld rs_mism=%lld first=%lld\n", rep, flag,
               (long long)mism, (long long)rsm, (long long)first);
        if (mism || flag || rsm) ++bad;
        fflush(stdout);
    }
    printf("%s\n", bad ? "SORTCHECK FAIL" : "SORTCHECK OK");
    return bad ? 1 : 0;
}
