"""The callers on either side of the FICP path, headless.

* `join_plot(plot, chm_stand)`: App.join_plot (app.py:630-661). It builds the (x, y,
  height) arrays, or (x, y) when any height is missing. It runs FractionalICP on the
  GPU and writes the moved XY back with `plot.update_tree_positions`.
* `get_transform(plot)`: Plot.get_transform (trees.py:248-280). It returns the
  Procrustes R, t from the loaded to the current tree positions, with a reflection
  allowed iff the plot was flipped. The fit is the engine's `ficp_fit_rigid2d`.
* `transformation_record(plot)`, `save_transformations(records, stand_id, directory)`:
  App.store_transformations (app.py:884-925) and the Transformations CSV of
  App.save_files (app.py:774-786).
* `join_stand(stand, chm_stand)`: the Join loop of app.py:735-762 over every plot of a
  stand. For each plot it runs join, stores the transformation, then removes the matched
  CHM stems (`matches.remove_matches`), so each plot sees the stems its predecessors
  left, as in the app.
* `join_plots_batched(...)`: the same joins for array plots against one fixed CHM layer
  in a single device pass (`FractionalICPBatch`). This is C4's driver. It ignores the
  stem removals between plots.

The objects are the reference's own (trees.Plot, trees.Stand, chm_plot.CHMPlot) or any
objects with the same attributes; nothing here imports the reference.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib
from .batch import FractionalICPBatch
from .ficp import FractionalICP
from .matches import remove_matches

TRANSFORM_COLUMNS = ["PlotID", "original_center", "final_center", "tx", "ty", "r00", "r01", "r10",
                     "r11", "flip"]


def _object_rows(rows):
    """np.array of mixed per-tree rows, as Plot.get_tree_current_array builds them
    (trees.py:240-244: a string tree id makes every field a string; astype(float) then
    parses the shortest round-trip repr back to the same double)."""
    return np.array(rows) if rows else np.empty((0, 4))


def join_plot(plot, chm_stand, *, device=None) -> bool:
    """App.join_plot without the UI: False where the app flashes a message and returns."""
    if plot is None or not plot.trees:
        return False  # app.py:631-633 "No trees in current plot"
    if not chm_stand.trees:
        return False  # app.py:634-636 "No CHM trees to match against"
    cur = _object_rows([[t.tree_id, t.currentx, t.currenty, t.height] for t in plot.trees])
    src_3d = cur[:, -3:]
    tgt_3d = np.array([[t.x, t.y, t.height] for t in chm_stand.trees], dtype=object)
    use_3d = True
    try:  # app.py:641-648: 2-D as soon as any height is missing
        src_h = src_3d[:, 2].astype(float)
        tgt_h = tgt_3d[:, 2].astype(float)
        if np.isnan(src_h).any() or np.isnan(tgt_h).any():
            use_3d = False
    except Exception:
        use_3d = False
    if use_3d:
        source_array = src_3d.astype(float)
        target_array = tgt_3d.astype(float)
    else:
        source_array = cur[:, 1:3].astype(float)
        target_array = np.array([[t.x, t.y] for t in chm_stand.trees], dtype=float)
    icp = FractionalICP(source_array, target_array, device=device)
    icp.run()
    new_coords = icp.source[:, :2]
    if hasattr(plot, "update_tree_positions"):
        plot.update_tree_positions(new_coords)
    else:
        for t, (x, y) in zip(plot.trees, new_coords):
            t.currentx, t.currenty = x, y
    return True


def get_transform(plot, *, device=None):
    """Plot.get_transform on the GPU: (R (2, 2), t (2,), flipped), current ~ R @ source + t."""
    if not plot.trees:
        raise ValueError("No trees available to compute transform.")
    src = _object_rows([[t.tree_id, t.x, t.y, t.height] for t in plot.trees])[:, 1:3].astype(float)
    tgt = _object_rows([[t.tree_id, t.currentx, t.currenty, t.height] for t in plot.trees])[:, 1:3].astype(float)
    flipped = bool(getattr(plot, "flipped", False))
    with _lib.borrowed(device) as ctx:  # trees.py:267-278: reflection kept only for a flipped plot
        T = ctx.fit_rigid2d(src, tgt, allow_reflection=flipped)
    return T[:2, :2].copy(), T[:2, 2].copy(), getattr(plot, "flipped", False)


def transformation_record(plot, fail=False, *, device=None) -> dict:
    """App.store_transformations (app.py:884-925) for one plot: the row of the CSV."""
    na = {k: None for k in TRANSFORM_COLUMNS[2:]}
    if not plot.trees or fail:
        return {"original_center": tuple(map(float, plot.center)), **na}
    R, t, flip = get_transform(plot, device=device)
    return {
        "original_center": tuple(map(float, plot.center)),
        "final_center": tuple(map(float, plot.current_center)),
        "tx": float(t[0]), "ty": float(t[1]),
        "r00": float(R[0, 0]), "r01": float(R[0, 1]), "r10": float(R[1, 0]), "r11": float(R[1, 1]),
        "flip": bool(flip),
    }


def save_transformations(records: dict, stand_id, directory="./Transformations") -> str:
    """The Transformations CSV of App.save_files (app.py:776-786); returns its path."""
    import pandas as pd
    df = pd.DataFrame.from_dict(records, orient="index")
    df.index.name = "PlotID"
    df = df.reset_index()
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"Stand_{stand_id}_transformation.csv")
    df.to_csv(path, index=False)
    return path


def join_stand(stand, chm_stand, *, remove=True, min_dist_percent=15, device=None) -> dict:
    """Join every plot of `stand` in order, like repeated Join + confirm in the app
    (app.py:735-762).  Returns {plot_id: transformation record}."""
    records = {}
    for plot in stand.plots:
        join_plot(plot, chm_stand, device=device)
        records[plot.plotid] = transformation_record(plot, device=device)
        if remove:
            remove_matches(chm_stand, plot, min_dist_percent, device=device)
    return records


def join_plots_batched(plots, chm, *, device=None, **kw):
    """FractionalICP(plot_p, chm).run() for array plots against one CHM layer, one
    device pass (C4).  Returns (moved plots, per-plot stats records)."""
    b = FractionalICPBatch(list(plots), [chm] * len(plots), device=device, **kw)
    out = b.run()
    return out, b.stats
