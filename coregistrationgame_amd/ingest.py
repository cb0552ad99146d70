"""Array-level CSV ingest for the FICP path.

The reference builds one Python object per tree and finds each row's plot with a linear
scan over the plots already seen (`trees.py:444`, O(rows x plots)). At 1M-tree scale
that loader, not FICP, is the wall clock. These loaders read the same CSV files and give
the arrays the engine consumes, in the same order and with the same parsing rules. Rows
become per-plot slices of SoA arrays. Plots keep their first-appearance order.

* `load_stand(ID, path, mapping, sep, impute_dbh, impute_h, naslund_params)`: trees.Stand
  (`trees.py:333-451`): the StandID filter, the column mapping, heights in metres via
  decimetres, the Näslund height imputation from DBH and the DBH imputation from height.
* `load_saved_stand(ID, path)`: trees.SavedStand (`trees.py:478-520`), the format the
  app writes.
* `load_chm(path, x, y, dist, height_unit, mapping, sep, impute_h)`: CHMPlot
  (`chm_plot.py:102-219`): the radial crop, the height unit, the 45 m cap, and skipping
  rows with neither height nor DBH.

DBH imputation is Tree.get_diameter (`trees.py:84-97`, `110-116`): the inverse Näslund
height by the same bounded `scipy.optimize.minimize_scalar` call on (0, 100) m, capped at
1.5 m, for a tree whose DBH is missing (None: no DBH column, an empty or unparseable
field) and whose height is not None.  `StandArrays.stemdiam_m` is Tree.stemdiam (metres,
imputed where the reference imputes), so `stemdiam_m * 100` is `Stand.write_out`'s
Diameter_cm (`trees.py:465-483`); `dbh_cm` keeps the centimetres as read.  No part of the
FICP path reads DBH.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

NASLUND_DEFAULT = (1.74105089, 0.35979281, 3.56879791)  # trees.py:28


@dataclass
class StandArrays:
    stand_id: object
    plot_ids: list                    # first-appearance order
    offsets: np.ndarray               # plot p = rows offsets[p]:offsets[p+1]
    tree_id: np.ndarray               # object
    x: np.ndarray
    y: np.ndarray
    height: np.ndarray                # metres, NaN = missing
    dbh_cm: np.ndarray                # centimetres as read, NaN = missing
    plot_center: np.ndarray           # (P, 2): XC/YC of the plot's first row (Stand), centroid (SavedStand)
    center: tuple = field(default=None)  # the stand centre: mean of the plot centroids
    stemdiam_m: np.ndarray = field(default=None)  # Tree.stemdiam (m, imputed), NaN = None

    def write_out_diameter_cm(self):
        """Stand.write_out's Diameter_cm column (trees.py:466-481), in load order."""
        return self.stemdiam_m * 100.0

    def plot(self, p):
        s = slice(self.offsets[p], self.offsets[p + 1])
        return np.column_stack([self.x[s], self.y[s], self.height[s]])


@dataclass
class ChmArrays:
    tree_id: np.ndarray
    x: np.ndarray
    y: np.ndarray
    height: np.ndarray                # metres, NaN = missing
    center: np.ndarray

    def xyh(self):
        return np.column_stack([self.x, self.y, self.height])


def _mapping_value(mapping, key, default, allow_none=False):
    """trees._resolve_mapping_value / chm_plot._resolve_mapping_value."""
    if not mapping:
        return default
    v = mapping.get(key, default)
    if v is None:
        return None if allow_none else default
    if isinstance(v, str):
        v = v.strip()
        if not v:
            return None if allow_none else default
    return v


def _opt_float(v):
    """`float(v) if v not in (None, "") else None` with failures -> None (trees.py:406-418).
    A NaN read from an empty CSV field stays NaN (it is neither None nor "")."""
    if v is None:
        return None
    if isinstance(v, str) and v == "":
        return None
    try:
        return float(v)
    except (ValueError, TypeError):
        return None


def naslund_height(stemdiam_m, params=NASLUND_DEFAULT):
    """Tree.naslund_1936 (trees.py:70-81): height (m) from DBH stored in metres."""
    a, b, c = params
    d_cm = stemdiam_m * 100.0
    return 1.3 + (d_cm / (a + b * d_cm)) ** c


def naslund_diameter(height_m, params=NASLUND_DEFAULT):
    """Tree.get_diameter (trees.py:84-97): DBH (m) whose Näslund height is height_m, by the
    reference's bounded 1-D minimisation on (0, 100), capped at 1.5 m."""
    from scipy.optimize import minimize_scalar

    def objective(x):
        return (height_m - naslund_height(x, params)) ** 2

    return min(minimize_scalar(objective, bounds=(0, 100), method="bounded").x, 1.5)


def _centroids(x, y, offsets):
    """Plot._update_centroid (trees.py:149-153): np.mean of the (n, 2) C-ordered array."""
    out = np.zeros((len(offsets) - 1, 2))
    for p in range(len(offsets) - 1):
        s = slice(offsets[p], offsets[p + 1])
        out[p] = np.mean(np.column_stack([x[s], y[s]]), axis=0)
    return out


def _stand_center(cen):
    """Stand._update_center (trees.py:453-460): plain Python sums over the plots."""
    return (sum(float(c[0]) for c in cen) / len(cen), sum(float(c[1]) for c in cen) / len(cen))


def _group(plot_vals):
    """Stable grouping by plot id in first-appearance order: (order, plot ids, offsets)."""
    first, ids = {}, []
    for i, v in enumerate(plot_vals):
        if v not in first:
            first[v] = len(ids)
            ids.append(v)
    g = np.fromiter((first[v] for v in plot_vals), dtype=np.int64, count=len(plot_vals))
    order = np.argsort(g, kind="stable")
    offsets = np.zeros(len(ids) + 1, np.int64)
    offsets[1:] = np.cumsum(np.bincount(g, minlength=len(ids)))
    return order, ids, offsets


def load_stand(ID, path, mapping=None, sep="\t", impute_h=True, naslund_params=None,
               impute_dbh=True) -> StandArrays:
    import pandas as pd
    recs = pd.read_csv(path, sep=sep)
    cols = set(recs.columns)
    if mapping:
        stand_col = _mapping_value(mapping, "StandID", "", allow_none=True)
        plot_col = _mapping_value(mapping, "PlotID", "PLOT")
        tree_col = _mapping_value(mapping, "TreeID", "TreeID")
        x_col = _mapping_value(mapping, "X", "X_GROUND")
        y_col = _mapping_value(mapping, "Y", "Y_GROUND")
        dbh_col = _mapping_value(mapping, "DBH", "STEMDIAM")
        h_col = _mapping_value(mapping, "H", "H", allow_none=True)
        xc_col = _mapping_value(mapping, "XC", x_col)
        yc_col = _mapping_value(mapping, "YC", y_col)
    else:
        stand_col, plot_col, tree_col = "Stand", "PLOT", "TreeID"
        x_col, y_col, dbh_col, h_col, xc_col, yc_col = "X_GROUND", "Y_GROUND", "STEMDIAM", "H", "XC", "YC"
    cache = {}

    def get(c):  # one Python list per column, built once
        if c not in cache:
            cache[c] = recs[c].tolist() if c in cols else [None] * len(recs)
        return cache[c]

    keep = np.ones(len(recs), bool)
    if stand_col:  # trees.py:382-398: rows of this stand only
        for i, v in enumerate(get(stand_col)):
            try:
                keep[i] = v is not None and int(v) == int(ID)
            except (ValueError, TypeError):
                keep[i] = False
    rows = np.flatnonzero(keep)
    if len(rows) == 0:
        raise ValueError(f"No data found for Stand ID: {ID}")
    PV = get(plot_col)
    pv = [PV[i] for i in rows]
    order, ids, offsets = _group(pv)
    rows = rows[order]
    X, Y, TID = get(x_col), get(y_col), get(tree_col)
    DBH = get(dbh_col) if dbh_col in cols else [None] * len(recs)
    H = get(h_col) if (h_col and h_col in cols) else [None] * len(recs)
    XC = get(xc_col) if xc_col in cols else X
    YC = get(yc_col) if yc_col in cols else Y
    n = len(rows)
    x = np.array([X[i] for i in rows], dtype=float)
    y = np.array([Y[i] for i in rows], dtype=float)
    dbh = np.full(n, np.nan)
    sd = np.full(n, np.nan)
    h = np.full(n, np.nan)
    params = tuple(naslund_params) if naslund_params is not None else NASLUND_DEFAULT
    for j, i in enumerate(rows):
        dcm = _opt_float(DBH[i])
        hdm = None
        hv = _opt_float(H[i])
        if hv is not None:
            hdm = hv * 10.0
        dbh[j] = np.nan if dcm is None else dcm
        height = None if hdm is None else hdm / 10  # Tree stores metres (trees.py:67)
        if height is None and impute_h and dcm is not None:  # Tree.impute_height
            height = naslund_height(dcm / 100, params)
        stem = None if dcm is None else dcm / 100  # Tree stores metres (trees.py:66)
        if stem is None and impute_dbh and height is not None:  # Tree.impute_dbh
            stem = naslund_diameter(height, params)
        sd[j] = np.nan if stem is None else stem
        h[j] = np.nan if height is None else height
    centers = np.array([[XC[rows[offsets[p]]], YC[rows[offsets[p]]]] for p in range(len(ids))], dtype=float)
    cen = _centroids(x, y, offsets)
    return StandArrays(ID, ids, offsets, np.array([TID[i] for i in rows], dtype=object), x, y, h, dbh,
                       centers, _stand_center(cen), sd)


def load_saved_stand(ID, path, naslund_params=None) -> StandArrays:
    import pandas as pd
    recs = pd.read_csv(path)
    cols = set(recs.columns)
    order, ids, offsets = _group(recs["PlotID"].tolist())
    x = recs["CurrentX"].to_numpy(dtype=float)[order]
    y = recs["CurrentY"].to_numpy(dtype=float)[order]
    H = recs["Height_m"].tolist() if "Height_m" in cols else [None] * len(recs)
    D = recs["Diameter_cm"].tolist() if "Diameter_cm" in cols else [None] * len(recs)
    h = np.full(len(recs), np.nan)
    dbh = np.full(len(recs), np.nan)
    for j, i in enumerate(order):
        hv = _opt_float(H[i])
        h[j] = np.nan if hv is None else (hv * 10.0) / 10  # trees.py:486-491 via decimetres
        dv = _opt_float(D[i])
        dbh[j] = np.nan if dv is None else dv
    cen = _centroids(x, y, offsets)
    return StandArrays(ID, ids, offsets, recs["TreeID"].to_numpy(dtype=object)[order], x, y, h, dbh,
                       cen.copy(), _stand_center(cen), dbh / 100)


def load_chm(path, x=None, y=None, dist=40, height_unit="m", mapping=None, sep="\t", impute_h=False,
             naslund_params=None) -> ChmArrays:
    import pandas as pd
    df = pd.read_csv(path, sep=sep)
    x_col = _mapping_value(mapping, "X", "X")
    y_col = _mapping_value(mapping, "Y", "Y")
    h_col = _mapping_value(mapping, "H", "H")
    id_col = _mapping_value(mapping, "TreeID", "IDALS")
    dbh_col = _mapping_value(mapping, "DBH", "DBH")
    missing_height = h_col not in df.columns
    if x is not None and y is not None and dist is not None and dist > 0:  # chm_plot.py:144-149
        c = df[[x_col, y_col]].to_numpy(dtype=float)
        dx = c[:, 0] - x
        dy = c[:, 1] - y
        d = np.sqrt(dx * dx + dy * dy)
        df = df[d <= dist]
    if height_unit not in ("m", "dm", "cm"):
        raise ValueError(f"Unsupported height_unit '{height_unit}'. Use one of: ['cm', 'dm', 'm'].")
    params = tuple(naslund_params) if naslund_params is not None else NASLUND_DEFAULT
    ids, xs, ys, hs = [], [], [], []
    for row in df.to_dict(orient="records"):
        if not missing_height:
            try:
                v = row[h_col]
                height = v * 10 if height_unit == "m" else (v if height_unit == "dm" else v / 10)
            except Exception:
                continue
            dcm = None
        else:
            try:
                dcm = float(row[dbh_col]) if (dbh_col in row and row[dbh_col] not in [None, ""]) else None
            except Exception:
                dcm = None
            height = None
        if height is not None and height > 450:  # chm_plot.py:186-187
            continue
        if ((height is None or (isinstance(height, float) and math.isnan(height)))
                and (dcm is None or (isinstance(dcm, float) and math.isnan(dcm)))):
            continue
        hm = None if height is None else height / 10
        if hm is None and impute_h and dcm is not None:
            hm = naslund_height(dcm / 100, params)
        ids.append(row[id_col])
        xs.append(row[x_col])
        ys.append(row[y_col])
        hs.append(np.nan if hm is None else hm)
    x_a, y_a = np.array(xs, dtype=float), np.array(ys, dtype=float)
    center = np.mean(np.column_stack([x_a, y_a]), axis=0) if len(x_a) else np.array([0.0, 0.0])
    return ChmArrays(np.array(ids, dtype=object), x_a, y_a, np.array(hs, dtype=float), center)
