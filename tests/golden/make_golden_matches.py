"""Golden fixtures for CHMPlot.remove_matches (chm_plot.py:223-285) from the REFERENCE.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_matches.py

The reference classes (chm_plot.CHMPlot, trees.Tree, trees.Plot) are imported from
/root/reference purely to produce input/expected-output vectors. The reference's own
remove_matches runs on reference Tree objects. Nothing of the reference is copied into
the repository, and nothing under tests/ imports it at test time.

Writes matches.npz: per case, the plot layer (x, y, h; h NaN = no height), the CHM
layer (x, y, h), min_dist_percent, and the expected removal order as indices into the
CHM layer (a sequence of calls on one shrinking CHM layer where `calls` > 1).
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("FICP_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REF))

import chm_plot  # noqa: E402  (reference, build container only)
import trees as ref_trees  # noqa: E402


def mk_trees(arr):
    out = []
    for i, (x, y, h) in enumerate(arr):
        t = ref_trees.Tree(i, float(x), float(y))
        t.height = None if np.isnan(h) else float(h)
        out.append(t)
    return out


def run_reference(plots, chm, pct):
    """Sequential remove_matches calls on one CHM layer; returns per-call removal indices."""
    c = chm_plot.CHMPlot.__new__(chm_plot.CHMPlot)
    c.trees = mk_trees(chm)
    c.removed_stems = []
    where = {id(t): i for i, t in enumerate(c.trees)}
    res = []
    for k, pa in enumerate(plots):
        p = ref_trees.Plot(k)
        p.trees = mk_trees(pa)
        c.remove_matches(p, min_dist_percent=pct)
        res.append(np.array([where[id(t)] for t in c.removed_stems[-1]], dtype=np.int64))
    return res


def case_random(rng, n, m, frac_near, nan_plot=False, nan_chm=False, geo=False):
    chm = np.column_stack([rng.uniform(-40, 40, m), rng.uniform(-40, 40, m), rng.uniform(5, 30, m)])
    pick = rng.integers(0, m, n)
    plot = chm[pick] + np.column_stack([rng.normal(0, 0.8, n), rng.normal(0, 0.8, n), rng.normal(0, 1.0, n)])
    far = rng.random(n) > frac_near
    plot[far, :2] = rng.uniform(-40, 40, (far.sum(), 2))
    if nan_plot:
        plot[rng.random(n) < 0.2, 2] = np.nan
    if nan_chm:
        chm[rng.random(m) < 0.1, 2] = np.nan
    if geo:
        plot[:, :2] += (420000.0, 6483000.0)
        chm[:, :2] += (420000.0, 6483000.0)
    return plot, chm


def case_ties():
    # CHM stems on a ring around each plot tree: equal 2-D/3-D distances, lowest index wins
    chm, plot = [], []
    for c in range(6):
        cx, cy = 10.0 * c, 0.0
        for a in range(4):
            ang = a * np.pi / 2
            chm.append((cx + np.cos(ang) * 0.5, cy + np.sin(ang) * 0.5, 20.0))
        plot.append((cx, cy, 20.0))
        plot.append((cx, cy, 20.0))  # a twin: must take the next tied stem
    chm = np.array(chm)
    perm = np.random.default_rng(5).permutation(len(chm))
    return np.array(plot), chm[perm]


def main():
    rng = np.random.default_rng(20240)
    out = {}
    cases = {}
    p, c = case_random(rng, 60, 300, 0.7)
    cases["rand3d"] = ([p], c)
    p, c = case_random(rng, 200, 120, 0.9)  # more plot trees than stems near them: conflicts
    cases["conflicts"] = ([p], c)
    p, c = case_random(rng, 80, 200, 0.8, nan_plot=True)  # missing plot heights: 2-D, 10 m rule
    cases["plot2d"] = ([p], c)
    p, c = case_random(rng, 80, 200, 0.8, nan_chm=True)  # missing CHM heights: 2-D
    cases["chm2d"] = ([p], c)
    p, c = case_random(rng, 100, 40, 1.0)  # the CHM layer runs out: the loop stops
    cases["exhaust"] = ([p], c)
    p, c = case_random(rng, 60, 300, 0.7, geo=True)
    cases["geo3d"] = ([p], c)
    p, c = case_ties()
    cases["ties"] = ([p], c)
    # one CHM layer, several plots in a row (App: remove_matches after each Join)
    c = np.column_stack([rng.uniform(-80, 80, 900), rng.uniform(-80, 80, 900), rng.uniform(5, 30, 900)])
    plots = []
    for k in range(5):
        pick = rng.integers(0, 900, 70)
        plots.append(c[pick] + np.column_stack([rng.normal(0, 0.6, 70), rng.normal(0, 0.6, 70),
                                                rng.normal(0, 1.0, 70)]))
    cases["sequence"] = (plots, c)
    # infinite heights: chm_plot.py:236-244 tests np.isnan only, so inf keeps the 3-D
    # search (and an infinite distance limit); in 2-D an infinite plot height is kept
    p, c = case_random(rng, 60, 200, 0.8)
    p[[3, 17, 40], 2] = np.inf
    c[[5, 50], 2] = np.inf
    cases["inf3d"] = ([p], c)
    p, c = case_random(rng, 80, 200, 0.8, nan_plot=True)
    p[[1, 2, 30], 2] = np.inf
    cases["inf2d"] = ([p], c)
    for name, (plots, chm) in cases.items():
        exp = run_reference(plots, chm, 15)
        out[f"{name}/chm"] = chm
        out[f"{name}/calls"] = np.array(len(plots))
        for k, (pa, e) in enumerate(zip(plots, exp)):
            out[f"{name}/plot{k}"] = pa
            out[f"{name}/removed{k}"] = e
        print(name, [len(e) for e in exp])
    np.savez_compressed(HERE / "matches.npz", **out)


if __name__ == "__main__":
    main()
