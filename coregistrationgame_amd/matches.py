"""`remove_matches` -- CHMPlot.remove_matches (chm_plot.py:223-285) on the MI355X engine.

After a plot is joined, `App` removes from the CHM layer the stems that the plot's trees
claim (`app.py:745,762`). For each plot tree in order, the nearest remaining CHM stem is
removed when it lies closer than `min_dist_percent` % of the tree's height. The search
is 3-D (x, y, height) when every height of both layers is present, and 2-D otherwise,
where a missing plot-tree height counts as 10 m. The walk is greedy: an earlier tree's
removal changes a later tree's nearest stem.

The engine computes every tree's 8 nearest stems at once on the GPU (grid k-NN in
scipy-cdist order: rounded distance, then stem index). It then walks the trees in the
reference's order, and re-queries with the removed stems masked only when all 8 of a
tree's candidates are gone. The result is the reference's removal sequence exactly
(`tests/golden/matches.npz`).

Two entry points:
  `remove_matches_arrays(plot, chm)` on (n, 3)/(m, 3) [x, y, height] arrays (height
  NaN = missing): the removal order as row indices of `chm`.
  `remove_matches(chm_plot, plot)` on the reference's CHMPlot/Plot objects: the same
  edit of `chm_plot.trees` and `chm_plot.removed_stems` as the method it replaces.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def thresholds(plot_h, use_3d: bool, min_dist_percent=15) -> np.ndarray:
    """The per-tree distance limits of chm_plot.py:249 (3-D) and 273-282 (2-D)."""
    h = np.asarray(plot_h, dtype=np.float64)
    if not use_3d:
        h = np.where(np.isnan(h), 10.0, h)  # chm_plot.py:276-281: 10 m when NaN (inf stays)
    return (min_dist_percent / 100.0) * h


def remove_matches_arrays(plot, chm, min_dist_percent=15, *, device=None) -> np.ndarray:
    plot = np.asarray(plot, dtype=np.float64)
    chm = np.asarray(chm, dtype=np.float64)
    if plot.ndim != 2 or chm.ndim != 2 or plot.shape[1] < 3 or chm.shape[1] < 3:
        raise ValueError("plot and chm must be (N, 3) arrays of x, y, height.")
    if len(plot) == 0 or len(chm) == 0:
        return np.zeros(0, np.int64)
    # chm_plot.py:236-244 tests np.isnan only: an infinite height keeps the 3-D search
    use_3d = bool(not np.isnan(plot[:, 2]).any() and not np.isnan(chm[:, 2]).any())
    md = 3 if use_3d else 2
    with _lib.borrowed(device, _lib.NN_GRID) as ctx:
        ctx.set_target(np.ascontiguousarray(chm[:, :md]), md)
        return ctx.remove_matches(np.ascontiguousarray(plot[:, :md]),
                                  thresholds(plot[:, 2], use_3d, min_dist_percent))


def _height(t) -> float:
    """A tree's height as chm_plot.py:238-245 tests it: NaN when missing or unreadable."""
    try:
        if t.height is None:
            return np.nan
        return float(t.height)
    except (TypeError, ValueError):
        return np.nan


def remove_matches(chm_plot, plot, min_dist_percent=15, *, device=None):
    """Drop-in for `chm_plot.remove_matches(plot, min_dist_percent)` (reference objects)."""
    ptrees, ctrees = list(plot.trees), list(chm_plot.trees)
    P = np.array([[float(t.currentx), float(t.currenty), _height(t)] for t in ptrees]).reshape(-1, 3)
    M = np.array([[float(t.currentx), float(t.currenty), _height(t)] for t in ctrees]).reshape(-1, 3)
    order = remove_matches_arrays(P, M, min_dist_percent, device=device)
    removed = [ctrees[i] for i in order]
    for t in removed:  # list.remove by identity, as the reference does
        chm_plot.trees.remove(t)
    chm_plot.removed_stems.append(removed)
    return removed
