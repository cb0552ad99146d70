"""ctypes wrapper of the CPU oracle (oracle/ficp_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  The product (coregistrationgame_amd)
never imports this module.

`OracleFICP` mirrors the reference `FractionalICP` surface (ficp.py:5-154) on
top of the C restatement so that tests can compare it with the golden vectors
of the reference and with the HIP path on identical inputs.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "libficp_oracle.so"

_i64 = C.c_int64
_dp = C.POINTER(C.c_double)
_ip32 = C.POINTER(C.c_int32)
_ip64 = C.POINTER(C.c_int64)


class OrcTrace(C.Structure):
    _fields_ = [
        ("max_calls", C.c_int32), ("n_calls", C.c_int32), ("n_fits", C.c_int32),
        ("iters", C.c_int32 * 2),
        ("k", _ip64), ("frmsd", _dp), ("lam", _dp), ("T", _dp), ("idx", _ip32), ("gap", _dp),
    ]


def build(force: bool = False) -> Path:
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "ficp_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.orc_nn_brute.argtypes = [_dp, _i64, _i64, _dp, _i64, _i64, C.c_int, _ip32, _dp, _dp, C.c_int]
        L.orc_kd_build.argtypes = [_dp, _i64, _i64, C.c_int]
        L.orc_kd_build.restype = C.c_void_p
        L.orc_kd_free.argtypes = [C.c_void_p]
        L.orc_kd_query.argtypes = [C.c_void_p, _dp, _i64, _i64, _ip32, _dp, _dp, C.c_int]
        L.orc_sort_order.argtypes = [_dp, _i64, _ip64]
        L.orc_optimal_fraction.argtypes = [_dp, _i64, _dp, _i64, _dp, _i64, _i64, C.c_int, C.c_double,
                                           C.c_int, _dp, _ip64, _dp]
        L.orc_frmsd.argtypes = [C.c_double, _i64, _dp, _i64, _dp, _i64, _i64, C.c_int, C.c_double]
        L.orc_frmsd.restype = C.c_double
        L.orc_fit_rigid2d.argtypes = [_dp, _i64, _dp, _i64, _i64, C.c_int, _dp]
        L.orc_apply_xy.argtypes = [_dp, _i64, _i64, _dp]
        L.orc_run.argtypes = [_dp, _i64, _i64, _dp, _i64, _i64, C.c_int, C.c_double, C.c_double,
                              C.c_double, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(OrcTrace)]
        L.orc_num_threads_max.restype = C.c_int
        _lib = L
    return _lib


def _p(a, t=_dp):
    return a.ctypes.data_as(t)


def _c64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    return a


def match_dims(src, tgt):
    return 3 if (src.shape[1] >= 3 and tgt.shape[1] >= 3) else 2


def nn(src, tgt, md, method="kdtree", nthreads=1):
    """Exact 1-NN (ficp.py:65-71) -> (idx int32, dist, d2)."""
    src, tgt = _c64(src), _c64(tgt)
    n, m = len(src), len(tgt)
    idx = np.zeros(n, np.int32)
    dist = np.zeros(n)
    d2 = np.zeros(n)
    if n == 0 or m == 0:
        return idx, dist, d2
    L = lib()
    if method == "brute":
        L.orc_nn_brute(_p(src), n, src.shape[1], _p(tgt), m, tgt.shape[1], md, _p(idx, _ip32), _p(dist), _p(d2), nthreads)
    else:
        kd = L.orc_kd_build(_p(tgt), m, tgt.shape[1], md)
        try:
            L.orc_kd_query(kd, _p(src), n, src.shape[1], _p(idx, _ip32), _p(dist), _p(d2), nthreads)
        finally:
            L.orc_kd_free(kd)
    return idx, dist, d2


class KDIndex:
    """A static kd-tree over the target (reused across calls: the 'fair' CPU mode)."""

    def __init__(self, tgt, md):
        self.tgt = _c64(tgt)
        self.md = md
        self.h = lib().orc_kd_build(_p(self.tgt), len(self.tgt), self.tgt.shape[1], md)

    def query(self, src, nthreads=1):
        src = _c64(src)
        n = len(src)
        idx = np.zeros(n, np.int32)
        dist = np.zeros(n)
        d2 = np.zeros(n)
        if n and len(self.tgt):
            lib().orc_kd_query(self.h, _p(src), n, src.shape[1], _p(idx, _ip32), _p(dist), _p(d2), nthreads)
        return idx, dist, d2

    def __del__(self):
        try:
            lib().orc_kd_free(self.h)
        except Exception:
            pass


def sort_order(d):
    d = np.ascontiguousarray(d, dtype=np.float64)
    order = np.zeros(len(d), np.int64)
    if len(d):
        lib().orc_sort_order(_p(d), len(d), _p(order, _ip64))
    return order


def optimal_fraction(src, corr, d, N, md, lam, literal=False):
    """ficp.py:73-86 -> (frac, k, frmsd_at_k)."""
    src, corr = _c64(src), _c64(corr)
    d = np.ascontiguousarray(d, dtype=np.float64)
    frac = C.c_double()
    k = C.c_int64()
    fr = C.c_double()
    lib().orc_optimal_fraction(_p(src), src.shape[1], _p(corr), corr.shape[1], _p(d), len(d), N, md,
                               lam, int(literal), C.byref(frac), C.byref(k), C.byref(fr))
    return frac.value, k.value, fr.value


def frmsd(fraction, k, src, corr, md, lam):
    src, corr = _c64(src), _c64(corr)
    if len(src) != len(corr):
        raise ValueError("operands could not be broadcast together")
    return lib().orc_frmsd(fraction, k, _p(src), src.shape[1], _p(corr), corr.shape[1], len(src), md, lam)


def fit_rigid2d(src, tgt, allow_reflection=False):
    src, tgt = _c64(src), _c64(tgt)
    T = np.zeros(9)
    lib().orc_fit_rigid2d(_p(src), src.shape[1], _p(tgt), tgt.shape[1], len(src), int(allow_reflection), _p(T))
    return T.reshape(3, 3)


def apply_xy(pts, T):
    out = np.array(pts, dtype=np.float64, copy=True, order="C")
    T = np.ascontiguousarray(T, dtype=np.float64)
    if len(out):
        lib().orc_apply_xy(_p(out), len(out), out.shape[1], _p(T))
    return out


def run(src, tgt, lam0=3.0, lam1=None, threshold=1e-6, max_iterations=1000, allow_reflection=False,
        literal=False, nthreads=1, trace=True, trace_idx=False, max_calls=4096):
    """ficp.py:149-154 on the oracle.  Returns (final_source, trace dict)."""
    src = np.array(src, dtype=np.float64, copy=True, order="C")
    tgt = _c64(tgt)
    md = match_dims(src, tgt)
    if lam1 is None:
        lam1 = 0.95 if md == 3 else 1.3
    n = len(src)
    tr = OrcTrace()
    karr = np.zeros(max_calls, np.int64)
    farr = np.zeros(max_calls)
    larr = np.zeros(max_calls)
    garr = np.zeros(max_calls)
    Tarr = np.zeros(max_calls * 9)
    iarr = np.zeros((max_calls, n), np.int32) if trace_idx else None
    tr.max_calls = max_calls
    tr.k, tr.frmsd, tr.lam, tr.T, tr.gap = _p(karr, _ip64), _p(farr), _p(larr), _p(Tarr), _p(garr)
    tr.idx = _p(iarr, _ip32) if iarr is not None else None
    lib().orc_run(_p(src), n, src.shape[1], _p(tgt), len(tgt), tgt.shape[1], md, lam0, lam1, threshold,
                  max_iterations, int(allow_reflection), int(literal), nthreads, C.byref(tr))
    nc, nf = min(tr.n_calls, max_calls), min(tr.n_fits, max_calls)
    out = dict(k=karr[:nc].copy(), frmsd=farr[:nc].copy(), lam=larr[:nc].copy(), gap=garr[:nc].copy(),
               T=Tarr[:nf * 9].reshape(nf, 3, 3).copy(), iters=(tr.iters[0], tr.iters[1]),
               n_calls=tr.n_calls, n_fits=tr.n_fits)
    if iarr is not None:
        out["idx"] = iarr[:nc].copy()
    return src, out


class OracleFICP:
    """The reference FractionalICP surface (ficp.py:5-154) over the C oracle."""

    def __init__(self, source, target, lambda_val=3.0, threshold=1e-6, max_iterations=1000,
                 allow_reflection=False):
        self.source = np.array(source, dtype=float)
        self.target = np.array(target, dtype=float)
        if self.source.ndim != 2 or self.target.ndim != 2:
            raise ValueError("source and target must be 2D arrays (N, D).")
        self.match_dims = match_dims(self.source, self.target)
        self.lambda_val = lambda_val
        self.threshold = threshold
        self.max_iterations = max_iterations
        self.allow_reflection = allow_reflection

    def find_correspondences(self, source, target):
        if len(target) == 0 or len(source) == 0:
            return np.empty((0, target.shape[1])), np.array([])
        idx, dist, _ = nn(source, target, self.match_dims)
        return target[idx], dist

    def find_optimal_fraction(self, corresponding_targets, distances):
        N = len(self.source)
        if N == 0 or len(distances) == 0:
            return 0.0, 0
        frac, k, _ = optimal_fraction(self.source, corresponding_targets, distances, N, self.match_dims,
                                      self.lambda_val)
        return frac, k

    def compute_optimal_transform_2d(self, source_subset, target_subset):
        return fit_rigid2d(source_subset, target_subset, self.allow_reflection)

    def apply_transform_2d_xy_only(self, points, T):
        return apply_xy(points, T)

    def run(self):
        lam1 = 0.95 if self.match_dims == 3 else 1.3
        self.source, self.trace = run(self.source, self.target, self.lambda_val, lam1, self.threshold,
                                      self.max_iterations, self.allow_reflection)
        self.lambda_val = lam1
        return self.source


# ----------------------------------------------------------------- remove_matches
def remove_matches(plot, chm, min_dist_percent=15.0):
    """CHMPlot.remove_matches (chm_plot.py:223-285) restated on arrays: plot and chm are
    (n, 3) / (m, 3) [x, y, height] (height NaN = missing).  Returns the removal order as
    indices into chm.  Pure-Python sequential loop: test infrastructure for small cases.

    * 3-D when every height of both layers is present (chm_plot.py:238-250), else 2-D
      (chm_plot.py:263-283) with the plot tree's height or 10 m as the threshold base;
    * distance as scipy's cdist: sqrt(((dx*dx) + dy*dy) + dz*dz);
    * argmin over the remaining stems in their original order (first index on ties);
    * removal iff distance < min_dist_percent / 100 * height; stop when none remain.
    """
    plot = np.asarray(plot, dtype=np.float64)
    chm = np.asarray(chm, dtype=np.float64)
    use3d = bool(not np.isnan(plot[:, 2]).any() and not np.isnan(chm[:, 2]).any())  # np.isnan only
    remaining = list(range(len(chm)))
    removed = []
    for i in range(len(plot)):
        if not remaining:
            break
        t = chm[remaining]
        dx = t[:, 0] - plot[i, 0]
        dy = t[:, 1] - plot[i, 1]
        d2 = dx * dx
        d2 = d2 + dy * dy
        if use3d:
            dz = t[:, 2] - plot[i, 2]
            d2 = d2 + dz * dz
        d = np.sqrt(d2)
        j = int(np.argmin(d))
        h = plot[i, 2]
        if not use3d and np.isnan(h):
            h = 10.0
        if d[j] < (min_dist_percent / 100.0) * h:
            removed.append(remaining.pop(j))
    return np.array(removed, dtype=np.int64)
