// win_pass.h -- the window selection's per-workgroup pass over rows an NN workgroup has
// just written (k_grid_nn.hip k_nn_grid_q; tools/wincheck.hip drives it alone).  The
// decision is k_select.hip's win_tail (k_sel_win_tail).
#pragma once
#include "ficp_internal.h"
#include "frmsd_bounds.h"

namespace ficp {

// ---- the window selection's pass, fused into the certified NN kernel (round 4)
// k_select.hip k_sel_win reads every row's r, moved XY, match XY and caller index back
// (44 B per row, ~12 us of pass at C3 plus its launch); here the NN workgroup that has just
// written its kWinNNRows rows classifies them against the key window of the loop state
// (the same win_map the tail rebuilds) and stores k_sel_win's per-workgroup outputs: the
// record (count, sum of r and the 8 fit sums of the rows below the window, the window
// rows' count and sum, the key range), the window rows (at most kWinSlot, in (row slot,
// wave, lane) order) and the coarse buckets (LDS, then agent-scope atomics).  The tail
// (k_sel_win_tail, one workgroup) then decides exactly as k_sel_win's last workgroup does.
constexpr int kWinNCB = 2 * fb::kWinNCS;
static_assert(kWinNCB == 256, "one coarse bucket per thread of the NN workgroup");

template <int Q>
__device__ __forceinline__ void nn_win_pass(const NNArgs &a, int64_t i0, int64_t tile) {
    using fb::u64;
    const NNWin &W = *a.win;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    constexpr int NCS = fb::kWinNCS, WREP = 2, WRS = kWinNCB + 1;
    __shared__ unsigned s_cc[WREP * WRS];
    __shared__ u64 s_cf[WREP * WRS];
    __shared__ int s_ce[kWinNCB];
    __shared__ double s_red[4][11];
    __shared__ unsigned s_wc[Q][4];
    __shared__ u64 s_kr[4][2];
    const fb::WMap m0 = fb::win_map(W.st->tkey, W.st->tmove, W.st->wfloor, a.n);
    for (int b = t; b < WREP * WRS; b += 256) {
        s_cc[b] = 0u;
        s_cf[b] = 0ULL;
    }
    s_ce[t] = fb::win_bucket_exp(m0, t);
    // (also orders this workgroup's NN stores before the loads below: one CU, one L1)
    __syncthreads();
    double rr[Q], xs[Q], ys[Q], xt[Q], yt[Q];
    uint32_t oo[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t i = i0 + (int64_t)q * 256 + t;
        const int64_t j = i < a.n ? i : 0;  // unconditional loads of a clamped row
        rr[q] = a.r[j];
        xs[q] = a.sx[j];
        ys[q] = a.sy[j];
        xt[q] = a.cx[j];
        yt[q] = a.cy[j];
        oo[q] = W.orig[j];
    }
    unsigned nbel = 0, nbad = 0, inw = 0;
    u64 kmn = ~0ULL, kmx = 0ULL;
    double sb = 0.0, swn = 0.0;
    double c8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u64 kk[Q];
    unsigned *my_cc = s_cc + (lane % WREP) * WRS;
    u64 *my_cf = s_cf + (lane % WREP) * WRS;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t i = i0 + (int64_t)q * 256 + t;
        kk[q] = 0ULL;
        if (i >= a.n) continue;
        const double v = rr[q];
        if (!(v < INFINITY)) {  // inf / NaN: the full selection's special cases
            ++nbad;
            continue;
        }
        const u64 k = key_of_r(v);
        kk[q] = k;
        kmn = min(kmn, k);
        kmx = max(kmx, k);
        int b = -1;
        if (k < m0.wlo) {
            ++nbel;
            sb = sb + v;
            fit_add(c8, xs[q], ys[q], xt[q], yt[q], W.px, W.py);
            b = NCS - 1 - fb::win_cq((m0.wlo - 1ULL - k) >> m0.su);
        } else if (k < m0.whi) {
            inw |= 1u << q;
            swn = swn + v;
        } else {
            b = NCS + fb::win_cq((k - m0.whi) >> m0.su);
        }
        if (b >= 0) {
            const int e = s_ce[b];
            atomicAdd(&my_cc[b], 1u);
            atomicAdd(&my_cf[b], e < 1024 ? (u64)ldexp(v, m0.fxb - e) : 0ULL);
        }
    }
    u64 masks[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        masks[q] = __ballot((inw >> q) & 1u);
        if (lane == 0) s_wc[q][wave] = (unsigned)__popcll(masks[q]);
    }
    sb = wave_sum63(sb);
    swn = wave_sum63(swn);
#pragma unroll
    for (int e = 0; e < 8; ++e) c8[e] = wave_sum63(c8[e]);
    const u64 cnt = wave_sum63_u64((u64)nbel | ((u64)nbad << 32));
    u64 pka = ~kmn, pkb = kmx;
    wave_range_reduce(pka, pkb);
    if (lane == 63) {
        s_kr[wave][0] = pka;
        s_kr[wave][1] = pkb;
        s_red[wave][0] = sb;
#pragma unroll
        for (int e = 0; e < 8; ++e) s_red[wave][1 + e] = c8[e];
        s_red[wave][9] = __longlong_as_double((long long)cnt);
        s_red[wave][10] = swn;
    }
    __syncthreads();
    {  // the coarse buckets (one per thread)
        unsigned c = 0;
        u64 f = 0;
#pragma unroll
        for (int q = 0; q < WREP; ++q) {
            c += s_cc[q * WRS + t];
            f += s_cf[q * WRS + t];
        }
        if (c) {
            const int cp = (int)(blockIdx.x % kWinCopies) * kWinNCB + t;  // (the XCD's copy)
            __hip_atomic_fetch_add(&W.o.gcc[cp], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&W.o.gcf[cp], f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the window rows: slot of (row slot q, wave, lane) in that order
    unsigned wall = 0, wpos = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const unsigned c = s_wc[q][w];
            wall += c;
        }
    if (wall && wall <= (unsigned)kWinSlot) {
        const u64 lt = (1ULL << lane) - 1ULL;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            unsigned base = wpos;
            for (int w = 0; w < wave; ++w) base += s_wc[q][w];
            if ((inw >> q) & 1u) {
                const int64_t slot = tile * kWinSlot + base + (unsigned)__popcll(masks[q] & lt);
                W.o.wsk[slot] = kk[q];
                W.o.wsr[slot] = rr[q];
                W.o.wso[slot] = oo[q];
                W.o.wsp[slot] = (uint32_t)(i0 + (int64_t)q * 256 + t);
            }
            for (int w = 0; w < 4; ++w) wpos += s_wc[q][w];
        }
    }
    u64 *rec = W.o.wrec + tile * kWinRec;
    if (t == 255 - 11) {  // the key range words: max(~key), max(key)
        u64 x = s_kr[0][0], y = s_kr[0][1];
        for (int w = 1; w < 4; ++w) {
            x = max(x, s_kr[w][0]);
            y = max(y, s_kr[w][1]);
        }
        rec[13] = x;
        rec[14] = y;
    }
    if (t >= 256 - 11) {  // count below, window rows, bad rows, sum of r below, fit sums, window r
        const int f = t - (256 - 11);
        double v = s_red[0][f];
        u64 cv = (u64)__double_as_longlong(s_red[0][9]);
        for (int w = 1; w < 4; ++w) {
            v = v + s_red[w][f];
            cv += (u64)__double_as_longlong(s_red[w][9]);
        }
        if (f == 9) {
            rec[0] = cv & 0xffffffffULL;
            rec[1] = (u64)wall;
            rec[2] = (cv >> 32) + (wall > (unsigned)kWinSlot ? 1ULL : 0ULL);
        } else {
            rec[f < 9 ? 3 + f : 12] = (u64)__double_as_longlong(v);
        }
    }
}

}  // namespace ficp
