"""Synthetic tree-layer / CHM-layer plots for parity tests and the benchmark.

The generator is the one SURVEY.md §8(d) specifies.  It imitates a field plot
(Layer 1, the moving "tree layer") that was surveyed with a small rigid
misregistration against a canopy-height-model stem map (Layer 2, the static
"CHM layer"), at the stem density of the reference's own sample stand
(`Data/2019/Stand_10_trees.csv`, ~0.05 stems / m^2) and in its geo-referenced
coordinate frame (x ~ 4.2e5, y ~ 6.48e6; first data row of that file).

* CHM layer: M stems, (x, y) ~ U[0, L]^2 with L = sqrt(M / rho), height ~ U(5, 30) m.
* Tree layer: round(f * N) distinct CHM stems with N(0, 0.3 m) XY and N(0, 1 m)
  height jitter, plus (1 - f) * N uniformly placed outlier trees; shuffled.
* Misregistration: rotation theta ~ U(-theta_max, theta_max) about the tree-layer
  centroid, theta_max = min(5 deg, 5 m / (L / 2)) (<= ~5 m at the plot edge),
  then a translation t ~ U(-2, 2)^2 m.
* Both layers are shifted by the geo offset (420000, 6483000).

`f` is the generator's inlier fraction; FRMSD picks its own k (ficp.py:73-86).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

GEO_OFFSET = (420000.0, 6483000.0)
DENSITY = 0.05  # stems per m^2


@dataclass
class SynthPlot:
    source: np.ndarray  # (N, D) tree layer, moving
    target: np.ndarray  # (M, D) CHM layer, static
    theta: float  # applied rotation (rad) -- the misregistration
    t: np.ndarray  # applied translation (2,)
    pivot: np.ndarray  # rotation centre (2,)
    inlier_of: np.ndarray  # (N,) target index an inlier was drawn from, -1 for outliers


def make_plot(n: int, m: int, f: float, seed: int, md: int = 3, geo: bool = True,
              density: float = DENSITY) -> SynthPlot:
    """Draw one synthetic plot.  ``md`` = 3 gives (x, y, height)
    columns like `app.py:638-652`; ``md`` = 2 gives the XY fallback of `app.py:654-656`."""
    if md not in (2, 3):
        raise ValueError("md must be 2 or 3")
    rng = np.random.default_rng(seed)
    L = math.sqrt(max(m, 1) / density)
    txy = rng.uniform(0.0, L, size=(m, 2))
    tz = rng.uniform(5.0, 30.0, size=m)

    n_in = min(int(round(f * n)), m)
    n_out = n - n_in
    pick = rng.choice(m, size=n_in, replace=False) if n_in > 0 else np.empty(0, dtype=np.int64)
    sxy_in = txy[pick] + rng.normal(0.0, 0.3, size=(n_in, 2))
    sz_in = tz[pick] + rng.normal(0.0, 1.0, size=n_in)
    sxy_out = rng.uniform(0.0, L, size=(n_out, 2))
    sz_out = rng.uniform(5.0, 30.0, size=n_out)
    sxy = np.vstack([sxy_in, sxy_out])
    sz = np.concatenate([sz_in, sz_out])
    owner = np.concatenate([pick.astype(np.int64), np.full(n_out, -1, dtype=np.int64)])
    perm = rng.permutation(n)
    sxy, sz, owner = sxy[perm], sz[perm], owner[perm]

    theta_max = min(math.radians(5.0), 5.0 / (L / 2.0))
    theta = float(rng.uniform(-theta_max, theta_max))
    t = rng.uniform(-2.0, 2.0, size=2)
    pivot = sxy.mean(axis=0) if n > 0 else np.zeros(2)
    c, s = math.cos(theta), math.sin(theta)
    R = np.array([[c, -s], [s, c]])
    sxy = (sxy - pivot) @ R.T + pivot + t

    off = np.array(GEO_OFFSET) if geo else np.zeros(2)
    sxy = sxy + off
    txy = txy + off
    if md == 3:
        src = np.column_stack([sxy, sz])
        tgt = np.column_stack([txy, tz])
    else:
        src = np.ascontiguousarray(sxy)
        tgt = np.ascontiguousarray(txy)
    return SynthPlot(src, tgt, theta, t, pivot + off, owner)


def make_cloud(n: int = 200, seed: int = 9) -> np.ndarray:
    """The point cloud of the reference's FICP tests (`tests/test_ficp.py:12-16`)."""
    rng = np.random.default_rng(seed)
    xy = rng.normal(size=(n, 2)) @ np.array([[1.0, 0.3], [0.0, 0.6]]).T
    z = np.linspace(0.0, 20.0, n).reshape(-1, 1) + rng.normal(scale=0.02, size=(n, 1))
    return np.hstack([xy, z])


def apply_rigid(src: np.ndarray, angle_deg: float, t_xy) -> np.ndarray:
    """Rigid XY motion of the reference's FICP tests (`tests/test_ficp.py:19-24`)."""
    th = np.deg2rad(angle_deg)
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    xy = src[:, :2] @ R.T + np.asarray(t_xy)
    return np.hstack([xy, src[:, 2][:, None]])


def reference_scenarios():
    """The three recovery scenarios of `tests/test_ficp.py:39-101` as (name, src, tgt)."""
    out = []
    src = make_cloud(n=150, seed=1)
    out.append(("basic_rigid_exact", src, apply_rigid(src, 27.0, [1.6, -2.2])))

    src = make_cloud(n=200, seed=2)
    full = apply_rigid(src, 31.0, [2.5, -1.8])
    rng = np.random.default_rng(123)
    keep = rng.choice(full.shape[0], size=full.shape[0] // 2, replace=False)
    out.append(("missing_points", src, full[keep]))

    src = make_cloud(n=200, seed=3)
    clean = apply_rigid(src, -22.0, [-1.2, 2.0])
    rng = np.random.default_rng(7)
    keep = rng.choice(clean.shape[0], size=clean.shape[0] // 2, replace=False)
    tgt = clean[keep]
    num_out = int(0.3 * tgt.shape[0])
    out_xy = rng.uniform(low=-20, high=20, size=(num_out, 2))
    out_z = rng.uniform(low=-5, high=25, size=(num_out, 1))
    out.append(("missing_plus_outliers", src, np.vstack([tgt, np.hstack([out_xy, out_z])])))
    return out


def make_batch(n_plots: int, n: int, m: int, f: float, seed0: int, md: int = 3):
    """C4 batch: plot p drawn with seed ``seed0 + p``."""
    return [make_plot(n, m, f, seed0 + p, md=md) for p in range(n_plots)]
