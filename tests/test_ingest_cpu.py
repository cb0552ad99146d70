"""CPU tests of the array-level CSV ingest against the reference
loaders' own output (tests/golden/ingest.npz, from trees.Stand, trees.SavedStand and
chm_plot.CHMPlot on the reference's Data files and on corner-case CSVs)."""
import ast

import numpy as np
import pytest

import conftest
from coregistrationgame_amd import ingest

Z = np.load(conftest.GOLDEN / "ingest.npz")
CASES = sorted({k.split("/")[0] for k in Z.files})


@pytest.mark.parametrize("name", CASES)
def test_loader_matches_reference(name, tmp_path):
    f = tmp_path / f"{name}.csv"
    f.write_text(str(Z[f"{name}/csv"]))
    kind = str(Z[f"{name}/kind"])
    kw = ast.literal_eval(str(Z[f"{name}/kwargs"]))
    if kind == "chm":
        kw.pop("impute_dbh", None)
        got = ingest.load_chm(f, **kw)
    else:
        ID = kw.pop("ID")
        if kind == "saved":
            kw.pop("impute_dbh", None)
        got = (ingest.load_saved_stand if kind == "saved" else ingest.load_stand)(ID, f, **kw)
        if f"{name}/stemdiam" in Z.files:  # Tree.stemdiam, DBH imputation included
            np.testing.assert_array_equal(got.stemdiam_m, Z[f"{name}/stemdiam"])
            np.testing.assert_array_equal(got.write_out_diameter_cm(), Z[f"{name}/diameter_cm_out"])
        assert [str(p) for p in got.plot_ids] == list(Z[f"{name}/plot_ids"])
        np.testing.assert_array_equal(np.diff(got.offsets), Z[f"{name}/sizes"])
        np.testing.assert_array_equal(got.plot_center, Z[f"{name}/plot_center"])
    assert [str(t) for t in got.tree_id] == list(Z[f"{name}/tree_id"])
    np.testing.assert_array_equal(got.x, Z[f"{name}/x"])
    np.testing.assert_array_equal(got.y, Z[f"{name}/y"])
    np.testing.assert_array_equal(got.height, Z[f"{name}/height"])  # NaN == NaN here
    np.testing.assert_array_equal(np.asarray(got.center, dtype=float), Z[f"{name}/center"])


def test_no_rows_for_stand(tmp_path):
    f = tmp_path / "s.csv"
    f.write_text("Stand,PLOT,TreeID,X_GROUND,Y_GROUND\n1,1,a,0,0\n")
    with pytest.raises(ValueError, match="No data found for Stand ID: 7"):
        ingest.load_stand(7, f, sep=",")
