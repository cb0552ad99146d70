"""Generate the golden fixtures under tests/golden/ from the REFERENCE ficp.py.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden.py

The reference module is imported from /root/reference/ficp.py (numpy + scipy
cKDTree) purely to produce input/expected-output vectors; nothing of the
reference is copied into the repository, and nothing under tests/ imports the
reference at test time.  The fixtures are small .npz files (data only).

Fixture families:
  nn.npz      find_correspondences (ficp.py:65-71): idx (cKDTree) + dists + corr,
              tie-free by construction (2nd-NN gap checked)
  frac.npz    find_optimal_fraction (ficp.py:73-86) for lambda in {3.0, 0.95, 1.3},
              with the best-vs-second FRMSD relative gap of the reference's own curve
  fit.npz     compute_optimal_transform_2d (ficp.py:89-110), incl. k=1, collinear,
              reflected inputs, allow_reflection False/True, geo offsets
  apply.npz   apply_transform_2d_xy_only (ficp.py:112-119), D = 2, 3, 5
  run_*.npz   FractionalICP.run() (ficp.py:149-154) per-NN-call traces: lambda, k,
              frac, FRMSD-curve gap, NN idx, T of every fit, final source
              (run_refl_*: allow_reflection=True, reflected fits included)
  empty.npz   the empty-input contracts (ficp.py:56-57, 66-68, 75-77, 125-126)
"""
from __future__ import annotations

import importlib.util
import os
import sys
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path(os.environ.get("FICP_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REPO))

from coregistrationgame_amd import synth  # noqa: E402


def load_reference():
    spec = importlib.util.spec_from_file_location("reference_ficp", REF / "ficp.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ref = load_reference()
RefFICP = ref.FractionalICP


def md_of(src, tgt):
    return 3 if (src.shape[1] >= 3 and tgt.shape[1] >= 3) else 2


def nn_idx(src, tgt, md):
    tree = cKDTree(np.ascontiguousarray(tgt[:, :md]))
    d2, i2 = tree.query(np.ascontiguousarray(src[:, :md]), k=2) if len(tgt) > 1 else (None, None)
    d, i = tree.query(np.ascontiguousarray(src[:, :md]), k=1)
    gap = np.inf
    if d2 is not None:
        gap = float(np.min((d2[:, 1] - d2[:, 0]) / np.maximum(d2[:, 0], 1e-300)))
    return i.astype(np.int64), d, gap


def frmsd_curve(icp, corr, d):
    """The reference's own FRMSD values for every k (same calls as ficp.py:80-85)."""
    N = len(icp.source)
    order = np.argsort(d)
    vals = np.empty(N)
    for k in range(1, N + 1):
        sel = order[:k]
        vals[k - 1] = icp.frmsd(k / N, k, icp.source[sel], corr[sel])
    return vals


def curve_gap(vals):
    """Relative gap between the best and second-best FRMSD values of the curve."""
    if len(vals) < 2:
        return np.inf
    s = np.sort(vals)
    return float((s[1] - s[0]) / max(abs(s[0]), 1e-300))


# ------------------------------------------------------------------ nn
def make_nn():
    out = {}
    cases = [
        ("d2_unit", 2000, 1500, 2, False, 11),
        ("d3_unit", 2000, 1500, 3, False, 12),
        ("d2_geo", 1200, 1000, 2, True, 13),
        ("d3_geo", 1200, 1000, 3, True, 14),
        ("d4_unit", 700, 600, 4, False, 15),   # extra column: corr keeps all Dt columns
        ("d3_vs_d2", 500, 400, 0, False, 16),  # source D=3, target D=2 -> match_dims = 2
    ]
    names = []
    for name, n, m, D, geo, seed in cases:
        rng = np.random.default_rng(seed)
        if name == "d3_vs_d2":
            src = rng.uniform(0, 40, size=(n, 3))
            tgt = rng.uniform(0, 40, size=(m, 2))
        else:
            src = rng.uniform(0, 60, size=(n, D))
            tgt = rng.uniform(0, 60, size=(m, D))
            if D >= 3:
                src[:, 2] = rng.uniform(5, 30, n)
                tgt[:, 2] = rng.uniform(5, 30, m)
        if geo:
            src[:, :2] += synth.GEO_OFFSET
            tgt[:, :2] += synth.GEO_OFFSET
        icp = RefFICP(src.copy(), tgt)
        corr, dist = icp.find_correspondences(icp.source, icp.target)
        idx, d_chk, gap = nn_idx(src, tgt, icp.match_dims)
        assert np.array_equal(corr, tgt[idx]), name
        assert np.array_equal(dist, d_chk), name
        assert gap > 1e-9, (name, gap)
        out[f"{name}/src"] = src
        out[f"{name}/tgt"] = tgt
        out[f"{name}/idx"] = idx
        out[f"{name}/dist"] = dist
        out[f"{name}/md"] = np.int64(icp.match_dims)
        names.append(name)
        print(f"nn {name}: n={n} m={m} md={icp.match_dims} min 2nd-NN gap {gap:.2e}")
    out["names"] = np.array(names)
    np.savez_compressed(HERE / "nn.npz", **out)


# ------------------------------------------------------------------ frac
def make_frac():
    out = {}
    names = []
    specs = [
        ("synth3_f08", dict(n=1200, m=1200, f=0.8, seed=21, md=3)),
        ("synth3_f06", dict(n=1500, m=1500, f=0.6, seed=22, md=3)),
        ("synth2_f07", dict(n=1000, m=1100, f=0.7, seed=23, md=2)),
        ("synth3_small", dict(n=60, m=80, f=0.5, seed=24, md=3)),
    ]
    for name, kw in specs:
        p = synth.make_plot(geo=True, **kw)
        for lam in (3.0, 0.95, 1.3):
            icp = RefFICP(p.source.copy(), p.target, lambda_val=lam)
            corr, d = icp.find_correspondences(icp.source, icp.target)
            frac, k = icp.find_optimal_fraction(corr, d)
            vals = frmsd_curve(icp, corr, d)
            assert int(np.argmin(vals)) + 1 == k
            key = f"{name}_l{lam}"
            out[f"{key}/src"] = p.source
            out[f"{key}/corr"] = corr
            out[f"{key}/dist"] = d
            out[f"{key}/lambda"] = np.float64(lam)
            out[f"{key}/k"] = np.int64(k)
            out[f"{key}/frac"] = np.float64(frac)
            out[f"{key}/frmsd"] = np.float64(vals[k - 1])
            out[f"{key}/gap"] = np.float64(curve_gap(vals))
            out[f"{key}/md"] = np.int64(icp.match_dims)
            names.append(key)
            print(f"frac {key}: k={k} frac={frac:.4f} gap={curve_gap(vals):.2e}")
    out["names"] = np.array(names)
    np.savez_compressed(HERE / "frac.npz", **out)


# ------------------------------------------------------------------ fit
def make_fit():
    out = {}
    names = []
    rng = np.random.default_rng(31)
    cases = []
    for i in range(12):
        k = int(rng.integers(3, 400))
        X = rng.uniform(-50, 50, size=(k, 3))
        th = rng.uniform(-np.pi, np.pi)
        R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        Y = X.copy()
        Y[:, :2] = X[:, :2] @ R.T + rng.uniform(-5, 5, 2) + rng.normal(0, 0.3, (k, 2))
        if i % 3 == 0:
            X[:, :2] += synth.GEO_OFFSET
            Y[:, :2] += synth.GEO_OFFSET
        cases.append((f"rand{i}", X, Y, False))
    # k = 1: H = 0, SVD path gives R = I (ficp.py:99-103)
    X = np.array([[1.0, 2.0, 3.0]]); Y = np.array([[4.0, -1.0, 7.0]])
    cases.append(("k1", X, Y, False))
    X1 = X + [[*synth.GEO_OFFSET, 0.0]]; Y1 = Y + [[*synth.GEO_OFFSET, 0.0]]
    cases.append(("k1_geo", X1, Y1, False))
    # k = 2 and collinear sets (rank-1 H)
    X = np.array([[0.0, 0.0, 1.0], [3.0, 1.0, 2.0]]); Y = np.array([[1.0, 1.0, 0.0], [0.5, 4.0, 0.0]])
    cases.append(("k2", X, Y, False))
    s = np.linspace(0, 10, 25)
    X = np.column_stack([s, 0.5 * s, s]); Y = np.column_stack([2 - 0.5 * s, 1 + s, s])
    cases.append(("collinear", X, Y, False))
    # reflected input: det(R_svd) < 0 -> Kabsch flip when allow_reflection=False
    X = rng.uniform(-10, 10, size=(40, 3)); Y = X.copy(); Y[:, 0] = -Y[:, 0] + 3.0
    cases.append(("reflected_noflip", X, Y, False))
    cases.append(("reflected_allow", X, Y, True))
    X = rng.uniform(-10, 10, size=(40, 3)); Y = X.copy()
    th = 0.7; R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    Y[:, :2] = X[:, :2] @ R.T + [1.0, 2.0]
    cases.append(("rotation_allow", X, Y, True))
    # 2-column inputs (the XY fallback, app.py:654-656)
    X = rng.uniform(0, 30, size=(90, 2)); th = -0.2
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    Y = X @ R.T + [0.3, -0.4] + rng.normal(0, 0.05, (90, 2))
    cases.append(("d2", X, Y, False))
    for name, X, Y, allow in cases:
        icp = RefFICP(X.copy(), Y.copy(), allow_reflection=allow)
        T = icp.compute_optimal_transform_2d(X, Y)
        out[f"{name}/src"] = X
        out[f"{name}/tgt"] = Y
        out[f"{name}/allow_reflection"] = np.int64(allow)
        out[f"{name}/T"] = T
        names.append(name)
    out["names"] = np.array(names)
    np.savez_compressed(HERE / "fit.npz", **out)
    print(f"fit: {len(names)} cases")


# ------------------------------------------------------------------ apply
def make_apply():
    out = {}
    names = []
    rng = np.random.default_rng(41)
    for D, geo in ((2, False), (3, True), (5, False), (3, False)):
        n = 3000
        P = rng.uniform(-100, 100, size=(n, D))
        if geo:
            P[:, :2] += synth.GEO_OFFSET
        th = rng.uniform(-0.5, 0.5)
        T = np.eye(3)
        T[:2, :2] = [[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]]
        T[:2, 2] = rng.uniform(-3, 3, 2)
        icp = RefFICP(P.copy(), P.copy())
        O = icp.apply_transform_2d_xy_only(P, T)
        name = f"D{D}{'_geo' if geo else ''}"
        out[f"{name}/pts"] = P
        out[f"{name}/T"] = T
        out[f"{name}/out"] = O
        names.append(name)
    out["names"] = np.array(names)
    np.savez_compressed(HERE / "apply.npz", **out)
    print(f"apply: {names}")


# ------------------------------------------------------------------ run traces
class TracedFICP(RefFICP):
    """Records every NN call, fraction choice and fit of a reference run()."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.tr_idx, self.tr_lambda, self.tr_k, self.tr_frac, self.tr_gap, self.tr_T = [], [], [], [], [], []
        self.tr_frmsd = []
        self._last = None

    def find_correspondences(self, source, target):
        corr, d = super().find_correspondences(source, target)
        if len(target) and len(source):
            i, d_chk, _ = nn_idx(source, target, self.match_dims)
            assert np.array_equal(d, d_chk)
            self.tr_idx.append(i.astype(np.int32))
        self._last = (corr, d)
        return corr, d

    def find_optimal_fraction(self, corresponding_targets, distances):
        frac, k = super().find_optimal_fraction(corresponding_targets, distances)
        if k > 0:
            vals = frmsd_curve(self, corresponding_targets, distances)
            self.tr_gap.append(curve_gap(vals))
            self.tr_frmsd.append(vals[k - 1])
        else:
            self.tr_gap.append(np.inf)
            self.tr_frmsd.append(np.inf)
        self.tr_lambda.append(self.lambda_val)
        self.tr_k.append(k)
        self.tr_frac.append(frac)
        return frac, k

    def compute_optimal_transform_2d(self, source_subset, target_subset):
        T = super().compute_optimal_transform_2d(source_subset, target_subset)
        self.tr_T.append(T)
        return T


def trace_run(src, tgt, **kw):
    icp = TracedFICP(src.copy(), tgt, **kw)
    icp.run()
    return icp


def save_run(name, src, tgt, **kw):
    icp = trace_run(src, tgt, **kw)
    n_calls = len(icp.tr_k)
    # reference semantics: a 'fraction' call follows every NN call inside _iterate
    d = dict(
        src=src, tgt=tgt, final=icp.source,
        lam=np.array(icp.tr_lambda, dtype=np.float64),
        k=np.array(icp.tr_k, dtype=np.int64),
        frac=np.array(icp.tr_frac, dtype=np.float64),
        gap=np.array(icp.tr_gap, dtype=np.float64),
        frmsd=np.array(icp.tr_frmsd, dtype=np.float64),
        T=np.array(icp.tr_T, dtype=np.float64).reshape(-1, 3, 3),
        idx=(np.stack(icp.tr_idx) if icp.tr_idx else np.zeros((0, len(src)), np.int32)),
        md=np.int64(icp.match_dims),
        lambda_final=np.float64(icp.lambda_val),
        kwargs_threshold=np.float64(kw.get("threshold", 1e-6)),
        kwargs_max_iterations=np.int64(kw.get("max_iterations", 1000)),
        kwargs_allow_reflection=np.int64(bool(kw.get("allow_reflection", False))),
    )
    np.savez_compressed(HERE / f"run_{name}.npz", **d)
    print(f"run {name}: n={len(src)} m={len(tgt)} md={icp.match_dims} calls={n_calls} "
          f"k={list(icp.tr_k)} min gap={min(icp.tr_gap) if icp.tr_gap else None:.2e}")


def real_plots():
    """Data/2014 field plots (XY only -> 2D fallback, app.py:654-656) vs the
    Data/2019 stems as the CHM layer, as the Join button would pair them."""
    import pandas as pd
    trees = pd.read_csv(REF / "Data/2014/Stand_10_trees.csv")
    chm = pd.read_csv(REF / "Data/2019/Stand_10_trees.csv")
    tgt = chm[["CurrentX", "CurrentY"]].to_numpy(dtype=float)
    plots = []
    for pid, g in trees.groupby("PlotID", sort=True):
        plots.append((int(pid), g[["CurrentX", "CurrentY"]].to_numpy(dtype=float)))
    return plots, tgt


def make_runs():
    for name, src, tgt in synth.reference_scenarios():
        save_run(name, src, tgt)
    specs = [
        ("synth3_geo_500", dict(n=500, m=600, f=0.8, seed=51, md=3)),
        ("synth3_geo_2000_f06", dict(n=2000, m=2000, f=0.6, seed=52, md=3)),
        ("synth2_geo_1500", dict(n=1500, m=1500, f=0.8, seed=53, md=2)),
    ]
    for name, kw in specs:
        p = synth.make_plot(geo=True, **kw)
        save_run(name, p.source, p.target)
    p = synth.make_plot(n=800, m=800, f=0.8, seed=54, md=3)
    save_run("synth3_fixed25_nothresh", p.source, p.target, threshold=-np.inf, max_iterations=5)
    plots, tgt = real_plots()
    out = {}
    for pid, src in plots:
        icp = trace_run(src, tgt)
        out[f"{pid}/src"] = src
        out[f"{pid}/final"] = icp.source
        out[f"{pid}/k"] = np.array(icp.tr_k, dtype=np.int64)
        out[f"{pid}/gap"] = np.array(icp.tr_gap, dtype=np.float64)
        out[f"{pid}/T"] = np.array(icp.tr_T, dtype=np.float64).reshape(-1, 3, 3)
        out[f"{pid}/idx"] = np.stack(icp.tr_idx)
    out["tgt"] = tgt
    out["plot_ids"] = np.array([pid for pid, _ in plots], dtype=np.int64)
    np.savez_compressed(HERE / "run_real_stand10.npz", **out)
    print(f"real plots: {len(plots)} plots vs {len(tgt)} CHM stems")


def mirrored_strip(n, md, seed, geo):
    """CHM stems along a narrow strip (x within +-0.6 m, y over 400 m) and a tree layer
    that is their mirror image in x, slightly rotated and shifted: the trees' nearest
    stems are mostly their own originals, so the SVD of the cross-covariance returns a
    reflection (det(Vt^T U^T) < 0, ficp.py:99-103)."""
    rng = np.random.default_rng(seed)
    tgt = np.column_stack([rng.uniform(-0.6, 0.6, n), np.sort(rng.uniform(0, 400, n)),
                           rng.uniform(5, 30, n)])[:, :md]
    src = tgt.copy()
    src[:, 0] = -src[:, 0]
    th = 0.004
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    c = np.array([0.0, 200.0])
    src[:, :2] = (src[:, :2] - c) @ R.T + c + [0.15, -0.1] + rng.normal(0, 0.03, (n, 2))
    if geo:
        src[:, :2] += synth.GEO_OFFSET
        tgt[:, :2] += synth.GEO_OFFSET
    return src, tgt


def make_refl_runs():
    """run() with allow_reflection=True (ficp.py:13, 101-103): two mirrored strips whose
    fits are reflections, and a regular plot (rotations) under the same flag."""
    cases = []
    s, t = mirrored_strip(160, 3, 61, geo=False)
    cases.append(("refl_strip3", s, t))
    s, t = mirrored_strip(220, 2, 62, geo=True)
    cases.append(("refl_strip2_geo", s, t))
    p = synth.make_plot(n=500, m=600, f=0.8, seed=63, md=3, geo=True)
    cases.append(("refl_allow_plot3", p.source, p.target))
    for name, s, t in cases:
        icp = trace_run(s, t, allow_reflection=True)
        dets = [float(np.linalg.det(T[:2, :2])) for T in icp.tr_T]
        print(f"  {name}: fits with det < 0: {sum(d < 0 for d in dets)} of {len(dets)}")
        save_run(name, s, t, allow_reflection=True)


def make_empty():
    out = {}
    src = synth.make_cloud(n=5, seed=42)
    icp = RefFICP(np.empty((0, 3)), src)
    a = icp.run()
    out["empty_source/shape"] = np.array(a.shape)
    icp = RefFICP(synth.make_cloud(n=4, seed=24), np.empty((0, 3)))
    corr, d = icp.find_correspondences(icp.source, icp.target)
    frac, k = icp.find_optimal_fraction(corr, d)
    out["empty_target/corr_shape"] = np.array(corr.shape)
    out["empty_target/dist_size"] = np.int64(d.size)
    out["empty_target/frac"] = np.float64(frac)
    out["empty_target/k"] = np.int64(k)
    b = icp.run()
    out["empty_target/run_equal"] = np.int64(np.array_equal(b, icp.source))
    np.savez_compressed(HERE / "empty.npz", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["nn", "frac", "fit", "apply", "runs", "refl", "empty"]
    for w in which:
        {"nn": make_nn, "frac": make_frac, "fit": make_fit, "apply": make_apply,
         "runs": make_runs, "refl": make_refl_runs, "empty": make_empty}[w]()
