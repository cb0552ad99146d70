"""frmsd (ficp.py:54-60) and equal distances at the cut (ficp.py:63, 78) against fixtures
made by the reference itself (tests/golden/make_golden_ties.py).

Ties: the reference orders the distances with np.argsort's default (unstable) quicksort;
the build orders equal distances by row index.  The selected SET can differ only when the
cut at k splits a block of equal distances:
  * with lambda >= 0 FRMSD is quasi-concave over a block of equal r (k_select.hip
    header), so the first minimum is never strictly inside one unless the block's r are
    0 (S_k = 0 for every k in it, FRMSD = 0, the first minimum k = 1).  The 90 "curves"
    place tie blocks all over the curve: the reference never splits one, and the build's
    k and selected set are the reference's;
  * "zeros" is the d = 0 block: the reference's cut at k = 1 takes one of 40 tied rows
    (argsort's choice, recorded) and the build takes the lowest index; every tied row
    gives the same fit (T = I), so T, k and the final source are pinned;
  * "dups": duplicated trees (bit-identical rows): any cut through them fits the same.
A cut through tied rows of DIFFERENT geometry at a rounding-level tie of the curve is the
remaining case; no fixture can pin it (the reference's pick depends on argsort's
platform-specific order), and none of these fixtures has one.
"""
import numpy as np
import pytest

from conftest import GOLDEN, K_GAP_PIN, assert_T_close


def _z(name):
    return np.load(GOLDEN / f"{name}.npz", allow_pickle=False)


def _frmsd_cases():
    z = _z("frmsd")
    return z, [str(n) for n in z["names"]]


# ------------------------------------------------------------------ CPU: the oracle
def test_oracle_frmsd_golden(oracle):
    z, names = _frmsd_cases()
    for n in names:
        v = oracle.frmsd(float(z[f"{n}/frac"]), int(z[f"{n}/k"]), z[f"{n}/src"], z[f"{n}/corr"],
                         int(z[f"{n}/md"]), float(z[f"{n}/lambda"]))
        # the reference sums np.sum(diff**2) pairwise, the oracle in row order
        np.testing.assert_allclose(v, float(z[f"{n}/value"]), rtol=1e-13, err_msg=n)
    assert float(z["zero_k/value"]) == float("inf")


def test_oracle_tie_curves(oracle):
    z = _z("ties")
    names = [str(n) for n in z["curve_names"]]
    assert len(names) == 90
    assert sum(int(z[f"{n}/split"]) for n in names) == 0  # the reference never splits a block
    for n in names:
        src, corr, d = z[f"{n}/src"], z[f"{n}/corr"], z[f"{n}/dist"]
        frac, k, _ = oracle.optimal_fraction(src, corr, d, len(src), 3, float(z[f"{n}/lambda"]))
        assert k == int(z[f"{n}/k"]), n
        assert frac == float(z[f"{n}/frac"]), n
        sel = np.sort(oracle.sort_order(d)[:k])
        np.testing.assert_array_equal(sel, z[f"{n}/ref_sel"], err_msg=n)


@pytest.mark.parametrize("case", ["zeros_md3", "zeros_md2", "dups"])
def test_oracle_tie_runs(oracle, case):
    z = _z("ties")
    src, tgt = z[f"{case}/src"], z[f"{case}/tgt"]
    final, tr = oracle.run(src, tgt)
    _check_run(case, z, tr["k"], tr["T"], final, src)


def _check_run(case, z, k, T, final, src):
    kref, Tref = z[f"{case}/k"], z[f"{case}/T"]
    if case.startswith("zeros"):
        assert int(z[f"{case}/first_split"]) == 1 and int(z[f"{case}/n_zero"]) == 40
        np.testing.assert_array_equal(k, kref)
        for a in T:  # every tied row gives T = I: the reference's pick and ours agree
            np.testing.assert_array_equal(a, np.eye(3))
        np.testing.assert_array_equal(final, z[f"{case}/final"])
        return
    gap = z[f"{case}/gap"]
    pin = len(gap) if (gap > K_GAP_PIN).all() else int(np.argmin(gap > K_GAP_PIN))
    np.testing.assert_array_equal(np.asarray(k)[:pin], kref[:pin])
    for i in range(min(pin, len(Tref), len(T))):
        assert_T_close(T[i], Tref[i], src, msg=f"{case} fit {i}")
    assert float(np.max(np.abs(final[:, :2] - z[f"{case}/final"][:, :2]))) < 1e-6
    np.testing.assert_array_equal(final[:, 2], src[:, 2])


# ------------------------------------------------------------------ GPU: the HIP path
@pytest.mark.gpu
def test_frmsd_golden():
    from coregistrationgame_amd import FractionalICP
    z, names = _frmsd_cases()
    for n in names:
        src, corr = z[f"{n}/src"], z[f"{n}/corr"]
        md = int(z[f"{n}/md"])
        icp = FractionalICP(np.zeros((3, src.shape[1])), np.zeros((3, corr.shape[1])),
                            lambda_val=float(z[f"{n}/lambda"]), device=0)
        assert icp.match_dims == md
        v = icp.frmsd(float(z[f"{n}/frac"]), int(z[f"{n}/k"]), src, corr)
        # device reduction tree vs numpy's pairwise np.sum: rounding-level, written here
        np.testing.assert_allclose(v, float(z[f"{n}/value"]), rtol=1e-13, err_msg=n)
    icp = FractionalICP(np.zeros((3, 3)), np.zeros((3, 3)), device=0)
    assert icp.frmsd(0.5, 0, np.zeros((0, 3)), np.zeros((0, 3))) == float(z["zero_k/value"])


@pytest.mark.gpu
def test_tie_curves_k_and_selected_set():
    from coregistrationgame_amd import FractionalICP
    z = _z("ties")
    for n in [str(x) for x in z["curve_names"]]:
        src, corr, d = z[f"{n}/src"], z[f"{n}/corr"], z[f"{n}/dist"]
        icp = FractionalICP(src, corr, lambda_val=float(z[f"{n}/lambda"]), device=0)
        frac, k = icp.find_optimal_fraction(corr, d)
        assert k == int(z[f"{n}/k"]), n
        assert frac == float(z[f"{n}/frac"]), n
        np.testing.assert_array_equal(np.sort(icp.get_n_first_elements(k, d)), z[f"{n}/ref_sel"], err_msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["zeros_md3", "zeros_md2", "dups"])
def test_tie_runs(case):
    from coregistrationgame_amd import FractionalICP
    z = _z("ties")
    src, tgt = z[f"{case}/src"], z[f"{case}/tgt"]
    icp = FractionalICP(src, tgt, device=0)
    final = icp.run(trace=True)
    st = icp.last_stats
    _check_run(case, z, st["k"], st["T"], final, src)
