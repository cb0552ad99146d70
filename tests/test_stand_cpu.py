"""CPU tests of the headless callers: the Transformations CSV
of App.save_files (app.py:774-786) and the empty-plot record of
App.store_transformations (app.py:886-898). Neither touches the GPU."""
from types import SimpleNamespace as NS

import numpy as np
import pandas as pd

from coregistrationgame_amd.stand import TRANSFORM_COLUMNS, save_transformations, transformation_record


def test_empty_plot_record_and_csv(tmp_path):
    rec = transformation_record(NS(trees=[], center=(1.5, 2.0)))
    assert rec["original_center"] == (1.5, 2.0)
    assert all(rec[k] is None for k in TRANSFORM_COLUMNS[2:])
    full = {"original_center": (0.0, 0.0), "final_center": (1.0, 2.0), "tx": 1.0, "ty": 2.0,
            "r00": 1.0, "r01": 0.0, "r10": 0.0, "r11": 1.0, "flip": False}
    path = save_transformations({7: rec, 8: full}, 10, directory=str(tmp_path))
    assert path.endswith("Stand_10_transformation.csv")
    df = pd.read_csv(path)
    assert list(df.columns) == TRANSFORM_COLUMNS
    assert list(df["PlotID"]) == [7, 8]
    assert np.isnan(df.loc[0, "tx"]) and df.loc[1, "tx"] == 1.0
    assert df.loc[1, "final_center"] == "(1.0, 2.0)"
