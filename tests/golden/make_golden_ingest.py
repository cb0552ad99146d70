"""Golden fixtures for the CSV ingest (trees.Stand, trees.SavedStand, chm_plot.CHMPlot)
from the REFERENCE loaders.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_ingest.py

Inputs are the reference's own data files (Data/2014, Data/2019) and small synthetic
CSVs with the corner cases the loaders handle. They are stored as CSV text in the
fixture. The expected outputs are what the reference loaders build: per tree id, x, y
and height in load order, plot order, and centres.
"""
from __future__ import annotations

import io
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import pandas as pd

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("FICP_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REF))

import chm_plot  # noqa: E402  (reference, build container only)
import trees as ref_trees  # noqa: E402


def stand_record(st):
    tid, x, y, h, sd, pid, cen = [], [], [], [], [], [], []
    for p in st.plots:
        pid.append(str(p.plotid))
        cen.append([float(p.center[0]), float(p.center[1])])
        for t in p.trees:
            tid.append(str(t.tree_id))
            x.append(float(t.x))
            y.append(float(t.y))
            h.append(np.nan if t.height is None else float(t.height))
            sd.append(np.nan if t.stemdiam is None else float(t.stemdiam))
    # Stand.write_out's Diameter_cm column (trees.py:465-483), in the same tree order
    wo = st.write_out()["Diameter_cm"].to_numpy(dtype=float)
    return dict(tree_id=np.array(tid), x=np.array(x), y=np.array(y), height=np.array(h),
                stemdiam=np.array(sd), diameter_cm_out=wo,
                plot_ids=np.array(pid), sizes=np.array([len(p.trees) for p in st.plots]),
                plot_center=np.array(cen), center=np.array(st.center, dtype=float))


def chm_record(c):
    return dict(tree_id=np.array([str(t.tree_id) for t in c.trees]),
                x=np.array([float(t.x) for t in c.trees]), y=np.array([float(t.y) for t in c.trees]),
                height=np.array([np.nan if t.height is None else float(t.height) for t in c.trees]),
                center=np.array(c.center, dtype=float))


def main():
    out = {}
    tmp = Path(tempfile.mkdtemp())

    def put(name, text, kind, kwargs, rec):
        out[f"{name}/csv"] = np.array(text)
        out[f"{name}/kind"] = np.array(kind)
        out[f"{name}/kwargs"] = np.array(repr(kwargs))
        for k, v in rec.items():
            out[f"{name}/{k}"] = v

    def run(name, text, kind, kwargs):
        f = tmp / f"{name}.csv"
        f.write_text(text)
        if kind == "saved":
            obj = ref_trees.SavedStand(file_path=f, **kwargs)
            put(name, text, kind, kwargs, stand_record(obj))
        elif kind == "stand":
            obj = ref_trees.Stand(file_path=f, **kwargs)
            put(name, text, kind, kwargs, stand_record(obj))
        else:
            obj = chm_plot.CHMPlot(f, **kwargs)
            put(name, text, kind, kwargs, chm_record(obj))
        return obj

    t14 = (REF / "Data/2014/Stand_10_trees.csv").read_text()
    t19 = (REF / "Data/2019/Stand_10_trees.csv").read_text()
    s14 = run("saved2014", t14, "saved", dict(ID=10))
    run("saved2019", t19, "saved", dict(ID=10))
    cmap = {"X": "CurrentX", "Y": "CurrentY", "H": "Height_m", "TreeID": "TreeID", "DBH": "Diameter_cm"}
    run("chm2019_crop70", t19, "chm", dict(x=float(s14.center[0]), y=float(s14.center[1]), dist=70, mapping=cmap,
                                            sep=","))
    run("chm2019_all", t19, "chm", dict(mapping=cmap, sep=",", dist=0))
    # field-data stand: two stands, bad numbers, missing heights -> Näslund imputation
    rng = np.random.default_rng(4)
    rows = []
    for i in range(60):
        rows.append({"Stand": 1 if i % 5 else 2, "PLOT": int(rng.integers(1, 5)), "TreeID": f"t{i}",
                     "X_GROUND": float(rng.uniform(0, 50)), "Y_GROUND": float(rng.uniform(0, 50)),
                     "STEMDIAM": "bad" if i % 11 == 3 else float(rng.uniform(8, 45)),
                     "H": "bad" if i % 7 == 2 else ("" if i % 13 == 5 else float(rng.uniform(5, 30))),
                     "Species": 1, "XC": 25.0 + (i % 3), "YC": 26.0})
    buf = io.StringIO()
    pd.DataFrame(rows).to_csv(buf, index=False)
    run("stand_field", buf.getvalue(), "stand", dict(ID=1, sep=",", impute_dbh=False, impute_h=True))
    mapping = {"StandID": "Stand", "PlotID": "PLOT", "TreeID": "TreeID", "X": "X_GROUND",
               "Y": "Y_GROUND", "DBH": "STEMDIAM", "H": "H"}
    run("stand_mapped", buf.getvalue(), "stand", dict(ID=2, mapping=mapping, sep=",", impute_dbh=False,
                                                       impute_h=True))
    run("stand_noimpute", buf.getvalue(), "stand", dict(ID=1, sep=",", impute_dbh=False, impute_h=False))
    # DBH imputation (Tree.impute_dbh, trees.py:84-97, 110-116): unparseable DBH fields
    # with a height, and a file without a DBH column at all
    run("stand_impute_dbh", buf.getvalue(), "stand", dict(ID=1, sep=",", impute_dbh=True, impute_h=True))
    buf2 = io.StringIO()
    pd.DataFrame([{k: v for k, v in r.items() if k != "STEMDIAM"} for r in rows]).to_csv(buf2, index=False)
    run("stand_no_dbh_column", buf2.getvalue(), "stand", dict(ID=2, sep=",", impute_dbh=True,
                                                               impute_h=True))
    # CHM detections: units, the 45 m cap, the DBH-only fallback
    crow = [{"X": float(a), "Y": float(b), "IDALS": f"c{i}", "H": float(h), "DBH": float(d)}
            for i, (a, b, h, d) in enumerate(zip(rng.uniform(0, 60, 40), rng.uniform(0, 60, 40),
                                                 rng.uniform(5, 50, 40), rng.uniform(8, 45, 40)))]
    buf = io.StringIO()
    pd.DataFrame(crow).to_csv(buf, index=False, sep="\t")
    run("chm_m", buf.getvalue(), "chm", dict(height_unit="m"))
    run("chm_dm_crop", buf.getvalue(), "chm", dict(x=30.0, y=30.0, dist=25, height_unit="dm"))
    run("chm_cm", buf.getvalue(), "chm", dict(height_unit="cm"))
    buf = io.StringIO()
    pd.DataFrame([{k: v for k, v in r.items() if k != "H"} for r in crow]).to_csv(buf, index=False, sep="\t")
    run("chm_dbh_only", buf.getvalue(), "chm", dict(impute_h=True))
    np.savez_compressed(HERE / "ingest.npz", **out)
    print(sorted({k.split("/")[0] for k in out}))


if __name__ == "__main__":
    main()
