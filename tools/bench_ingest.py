"""Ingest throughput: rows/s of coregistrationgame_amd.ingest vs the
reference's object loaders (trees.Stand / chm_plot.CHMPlot), on synthetic CSVs of the
field-data and CHM formats.  The reference loaders are importable only in the build
container (/root/reference); elsewhere only our side is timed."""
import io
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import pandas as pd

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from coregistrationgame_amd import ingest  # noqa: E402


def main(rows=50_000, plots=500):
    rng = np.random.default_rng(0)
    tmp = Path(tempfile.mkdtemp())
    df = pd.DataFrame({"Stand": 1, "PLOT": rng.integers(0, plots, rows), "TreeID": np.arange(rows),
                       "X_GROUND": rng.uniform(0, 5000, rows), "Y_GROUND": rng.uniform(0, 5000, rows),
                       "STEMDIAM": rng.uniform(8, 45, rows), "H": rng.uniform(5, 30, rows), "Species": 1})
    fs = tmp / "stand.csv"
    df.to_csv(fs, index=False)
    cd = pd.DataFrame({"X": rng.uniform(0, 5000, rows), "Y": rng.uniform(0, 5000, rows),
                       "IDALS": np.arange(rows), "H": rng.uniform(5, 30, rows), "DBH": rng.uniform(8, 45, rows)})
    fc = tmp / "chm.csv"
    cd.to_csv(fc, index=False, sep="\t")
    out = {"rows": rows, "plots": plots}
    t = time.perf_counter()
    ingest.load_stand(1, fs, sep=",", impute_h=True)
    out["ours_stand_rows_per_s"] = rows / (time.perf_counter() - t)
    t = time.perf_counter()
    ingest.load_chm(fc)
    out["ours_chm_rows_per_s"] = rows / (time.perf_counter() - t)
    ref = Path(os.environ.get("FICP_REFERENCE", "/root/reference"))
    if ref.exists():
        sys.path.insert(0, str(ref))
        import chm_plot
        import trees
        t = time.perf_counter()
        trees.Stand(1, fs, sep=",", impute_dbh=False, impute_h=True)
        out["reference_stand_rows_per_s"] = rows / (time.perf_counter() - t)
        t = time.perf_counter()
        chm_plot.CHMPlot(fc)
        out["reference_chm_rows_per_s"] = rows / (time.perf_counter() - t)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
