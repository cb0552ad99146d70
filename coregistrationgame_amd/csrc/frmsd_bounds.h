// frmsd_bounds.h -- bound arithmetic of the bucketed FRMSD-optimal-fraction selection,
// shared by the single-plot selection (k_select.hip) and the per-plot batch selection
// (k_batch.hip).  ficp.py:73-86 picks the first k minimising
//   FRMSD(k) = (1 / (k/N)^lambda) * sqrt(S_k / k),  S_k = sum of the k smallest r,
// which is monotone in h(k, S) = log2 S - p log2 k with p = 2 lambda + 1.  Inside a run
// of sorted positions whose rows are all >= lo, S_{C0+j} >= S_C0 + j lo makes h
// quasi-concave in j (p >= 1): the run's lower bound is the smaller of its end values.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace ficp {
namespace fb {

__device__ __forceinline__ int bits_of(unsigned long long v) {
    return v ? 64 - __clzll((long long)v) : 0;
}

// smallest r = d^2 of any row whose key (ordkey(d)) is >= klo (d = sqrt(d2) correctly
// rounded, so d >= d_lo implies d2 >= d_lo^2 up to the rounding the factor covers)
__device__ __forceinline__ double lo_r(unsigned long long klo) {
    if (!(klo >> 63)) return 0.0;
    const double d = __longlong_as_double((long long)(klo & 0x7fffffffffffffffULL));
    return d * d * (1.0 - 1e-15);
}

// lg2 is the fp64 log2 (ocml, ~1 ulp).  kMarg (log2 units) covers its rounding, the
// rounding of p log2 k and that of the fp64 prefix sums of the bucket sums the bounds are
// built from (relative ~1e-12 at 2^13 buckets or 16k rows): 1e-9 leaves a factor ~100.
// (The float log of round 1 forced 1e-5, which kept every position within ~3.5e-6 of the
// minimum FRMSD a candidate: 700-2200 rows at C3 whatever the bucket width.)
constexpr double kMarg = 1e-9;

__device__ __forceinline__ double lg2(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -INFINITY : NAN;
    if (!(x < INFINITY)) return INFINITY;
    return log2(x);
}

__device__ __forceinline__ double h_of(long long k, double S, double p) {
    return lg2(S) - p * lg2((double)k);
}

// lower bound of h over k in (C0, C0 + c] when the c rows there are all >= lo: the
// smaller end value, minus the margin
__device__ __forceinline__ double block_lb(long long C0, long long c, double P0, double lo,
                                           double p) {
    const double a = h_of(C0 + 1, P0 + lo, p);
    const double b = h_of(C0 + c, P0 + (double)c * lo, p);
    return fmin(a, b) - kMarg;
}

}  // namespace fb
}  // namespace ficp
