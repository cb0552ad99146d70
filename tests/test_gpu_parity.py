"""Parity of the HIP path (libficp.so through the C ABI) with the reference.

Golden vectors come from the reference ficp.py (tests/golden/make_golden.py); at sizes
the reference cannot reach, the pinned CPU oracle (oracle/) is the checker, and at the
full benchmark size the tests use size-independent properties.
Bars: NN idx and dist bit-exact; k exact where pinned (conftest.pinned_prefix); T and
final XY within 1e-6 abs (north star); Z and extra columns bit-identical.
"""
import numpy as np
import pytest

from conftest import (K_GAP_PIN, RUN_FIXTURES, allow_refl, assert_T_close, load_cases, load_run,
                      pinned_prefix)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from coregistrationgame_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


# ------------------------------------------------------------------ NN
@pytest.mark.parametrize("mode", ["brute", "grid"])
def test_nn_golden_bit_exact(ctx, mode):
    from coregistrationgame_amd import _lib
    ctx.set_nn_mode({"brute": _lib.NN_BRUTE, "grid": _lib.NN_GRID}[mode])
    cases, _ = load_cases("nn")
    try:
        for name, c in cases.items():
            md = int(c["md"])
            ctx.set_target(c["tgt"][:, :md], md)
            idx, dist = ctx.nn(c["src"][:, :md])
            np.testing.assert_array_equal(idx, c["idx"], err_msg=f"{mode} {name}")
            np.testing.assert_array_equal(bits(dist), bits(c["dist"]), err_msg=f"{mode} {name}")
    finally:
        ctx.set_nn_mode(_lib.NN_AUTO)


def test_facade_find_correspondences_all_columns():
    from coregistrationgame_amd import FractionalICP
    cases, _ = load_cases("nn")
    for name in ("d4_unit", "d3_vs_d2", "d3_geo"):
        c = cases[name]
        icp = FractionalICP(c["src"], c["tgt"])
        corr, dist = icp.find_correspondences(icp.source, icp.target)
        assert corr.shape == (len(c["src"]), c["tgt"].shape[1])
        np.testing.assert_array_equal(corr, c["tgt"][c["idx"]])
        np.testing.assert_array_equal(bits(dist), bits(c["dist"]))


@pytest.mark.parametrize("md", [2, 3])
def test_grid_equals_brute_100k(ctx, md):
    """Two independent exact searches agree bit-for-bit on a geo-referenced 100k plot."""
    from coregistrationgame_amd import _lib, synth
    p = synth.make_plot(100_000, 100_000, 0.8, seed=100_000 + md, md=md)
    ctx.set_target(p.target, md)
    try:
        ctx.set_nn_mode(_lib.NN_GRID)
        ig, dg = ctx.nn(p.source)
        ctx.set_nn_mode(_lib.NN_BRUTE)
        ib, db = ctx.nn(p.source)
    finally:
        ctx.set_nn_mode(_lib.NN_AUTO)
    np.testing.assert_array_equal(ig, ib)
    np.testing.assert_array_equal(bits(dg), bits(db))


def test_grid_vs_oracle_1M(ctx, oracle):
    """BASELINE full size (1M x 1M, md=3): grid NN == oracle kd-tree, bit-exact."""
    from coregistrationgame_amd import _lib, synth
    p = synth.make_plot(1_000_000, 1_000_000, 0.6, seed=1_000_000, md=3)
    ctx.set_nn_mode(_lib.NN_GRID)
    try:
        ctx.set_target(p.target, 3)
        idx, dist = ctx.nn(p.source)
    finally:
        ctx.set_nn_mode(_lib.NN_AUTO)
    oi, od, _ = oracle.nn(p.source, p.target, 3, "kdtree", nthreads=16)
    np.testing.assert_array_equal(idx, oi)
    np.testing.assert_array_equal(bits(dist), bits(od))


def test_grid_edge_layouts(ctx, oracle):
    """Degenerate CHM layers: duplicates (exact ties -> lowest index), collinear, single
    stem, queries far outside the grid."""
    from coregistrationgame_amd import _lib
    rng = np.random.default_rng(7)
    cases = []
    t = rng.uniform(0, 50, (300, 3)); t = np.vstack([t, t[:100]])      # exact duplicates
    cases.append((t, rng.uniform(0, 50, (500, 3))))
    s = np.linspace(0, 100, 400); cases.append((np.column_stack([s, 2 * s + 1]), rng.uniform(0, 100, (300, 2))))
    cases.append((np.array([[3.0, 4.0, 5.0]]), rng.uniform(-10, 10, (50, 3))))
    t = rng.uniform(0, 10, (1000, 2)); cases.append((t, rng.uniform(-500, 500, (400, 2))))
    t = np.zeros((64, 2)); cases.append((t, rng.uniform(-1, 1, (100, 2))))   # all stems identical
    for mode in (_lib.NN_BRUTE, _lib.NN_GRID):
        ctx.set_nn_mode(mode)
        for ci, (tgt, src) in enumerate(cases):
            md = tgt.shape[1]
            ctx.set_target(tgt, md)
            idx, dist = ctx.nn(src)
            oi, od, _ = oracle.nn(src, tgt, md, "brute")
            np.testing.assert_array_equal(idx, oi, err_msg=f"mode {mode} case {ci}")
            np.testing.assert_array_equal(bits(dist), bits(od), err_msg=f"mode {mode} case {ci}")
    ctx.set_nn_mode(_lib.NN_AUTO)


def test_grid_clustered_layers(ctx, oracle):
    """Clustered layers: thousands of stems (and trees) in one grid cell, so the grid
    build's and the work order's bucket sort take their oversized-bucket path (global
    scratch, k_bsort.hip); NN bit-exact vs brute force, and a whole run vs the oracle."""
    from coregistrationgame_amd import FractionalICP, _lib
    rng = np.random.default_rng(11)
    clump = rng.normal(0.0, 0.2, (4000, 2)) + np.array([300.0, 300.0])
    spread = rng.uniform(0, 1000, (3000, 2))
    tgt = np.column_stack([np.vstack([clump, spread]), rng.uniform(5, 30, 7000)])
    src = tgt[rng.permutation(7000)[:5000]].copy()
    src[:, :2] += rng.normal(0.0, 0.05, (5000, 2))
    ctx.set_nn_mode(_lib.NN_GRID)
    ctx.set_target(tgt, 3)
    idx, dist = ctx.nn(src)
    oi, od, _ = oracle.nn(src, tgt, 3, "brute")
    np.testing.assert_array_equal(idx, oi)
    np.testing.assert_array_equal(bits(dist), bits(od))
    ctx.set_nn_mode(_lib.NN_AUTO)
    icp = FractionalICP(src, tgt, nn_mode="grid")
    final = icp.run()
    ofinal, otr = oracle.run(src, tgt, nthreads=16)
    assert icp.last_stats["n_nn_calls"] == len(otr["k"])
    np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)


def test_selection_selfcheck():
    """tools/selcheck: the bucketed FRMSD selection (k_select.hip) against a CPU sort on
    residual distributions that exercise its refinement and radix paths (zeros, all
    equal, five distinct values, 20 decades), the 4097-8192-candidate LDS path (flat
    FRMSD curves at 1M rows, lambda 0.95 and 1.3) and the chunked scan (8M rows)."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "tools" / "selcheck"
    if not exe.exists():
        pytest.skip("tools/selcheck not built (make -C coregistrationgame_amd/csrc selcheck)")
    for args in (["200000", "3", "0", "3.0"], ["200000", "3", "0", "0.95"], ["100000", "3", "1", "3.0"],
                 ["50000", "2", "2", "3.0"], ["100000", "2", "3", "0.95"], ["200000", "3", "5", "1.3"],
                 ["3000", "3", "4", "3.0"], ["1000000", "2", "0", "0.95"], ["1000000", "2", "0", "1.3"],
                 ["8000000", "2", "0", "3.0"]):
        r = subprocess.run([str(exe)] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr


def test_fast_log2_error_bound():
    """The selection bounds' fast fp64 log2 (frmsd_bounds.h fast_log2: frexp, rcp + one
    Newton step, atanh series) against long-double log2 on the host over 2M random
    positive doubles of every exponent, all 2098 powers of two (subnormals included) and
    the mantissa split point: max |error| below kMarg / 100."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "tools" / "selcheck"
    if not exe.exists():
        pytest.skip("tools/selcheck not built (make -C coregistrationgame_amd/csrc selcheck)")
    r = subprocess.run([str(exe), "log2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and " ok" in r.stdout, r.stdout + r.stderr


WINCHECK_CASES = [("1000000", "0", "3.0"), ("1000000", "0", "0.95"), ("1000000", "0", "1.3"),
                  ("100000", "1", "3.0"), ("200000", "2", "3.0"), ("300000", "3", "0.95"),
                  ("1000000", "4", "3.0"), ("1000000", "5", "3.0"), ("3000", "0", "3.0"),
                  ("8000000", "0", "3.0"), ("1000000", "6", "3.0"), ("1000000", "7", "3.0"),
                  ("1000000", "8", "0.95")]


def test_window_selection_selfcheck():
    """tools/wincheck: the one-launch window selection (k_select.hip k_sel_win) on the ten
    residual distributions of tools/selcheck plus non-finite rows, hundreds of window rows
    in one workgroup and exact ties on a grid, for 5 window sizes x 7 placements of the
    previous threshold (at the true one, just inside / outside both window edges, 512
    widths away): every launch either decides k, FRMSD, the threshold pair and the fused
    fit equal to a CPU stable sort + scan and to the full path, or falls back leaving the
    state untouched, after which the full path's result is bit-identical (ficp.py:73-86)."""
    import re
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "tools" / "wincheck"
    if not exe.exists():
        pytest.skip("tools/wincheck not built (make -C coregistrationgame_amd/csrc wincheck)")
    decided = 0
    for args in WINCHECK_CASES:
        r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-4000:] + r.stderr
        m = re.search(r"window=(\d+) fallback=(\d+) bad=0", r.stdout)
        assert m, r.stdout[-2000:]
        decided += int(m.group(1))
        if args[1] == "0" and args[0] == "1000000":
            assert int(m.group(1)) >= 3, r.stdout  # the checker reaches the window's proof
    assert decided >= 20


# ------------------------------------------------------------------ sort / fraction
def test_argsort_stable(ctx):
    rng = np.random.default_rng(3)
    cases = [
        rng.uniform(0, 10, 1000),
        np.round(rng.uniform(0, 5, 5000), 1),                       # many exact ties
        1.0 + rng.uniform(0, 1e-9, 20000),                          # equal top-32 bits: fix-up runs
        np.concatenate([np.zeros(3000), rng.exponential(1.0, 3000)]),
        rng.normal(0, 1, 7000),                                     # negatives
        rng.exponential(1.0, 1_000_003),
    ]
    for i, d in enumerate(cases):
        o = ctx.argsort(d)
        np.testing.assert_array_equal(o, np.argsort(d, kind="stable"), err_msg=f"case {i}")


def test_fraction_golden(ctx):
    cases, _ = load_cases("frac")
    for name, c in cases.items():
        md = int(c["md"])
        frac, k = ctx.optimal_fraction(c["src"][:, :md], c["corr"][:, :md], c["dist"], len(c["src"]), md,
                                       float(c["lambda"]))
        if float(c["gap"]) > K_GAP_PIN:
            assert k == int(c["k"]), (name, k, int(c["k"]))
            assert frac == float(c["frac"]), name


def test_fraction_vs_oracle_large(ctx, oracle):
    from coregistrationgame_amd import synth
    for seed, (n, f, md) in enumerate([(300_000, 0.8, 3), (200_000, 0.6, 2), (50_001, 0.5, 3)]):
        p = synth.make_plot(n, n, f, seed=700 + seed, md=md)
        idx, dist, _ = oracle.nn(p.source, p.target, md, "kdtree", nthreads=16)
        corr = p.target[idx]
        for lam in (3.0, 0.95, 1.3):
            of, ok, ofr = oracle.optimal_fraction(p.source, corr, dist, n, md, lam)
            frac, k = ctx.optimal_fraction(p.source[:, :md], corr[:, :md], dist, n, md, lam)
            assert k == ok, (n, f, md, lam, k, ok)
            assert frac == of


def test_frmsd_and_get_n_first(ctx):
    from coregistrationgame_amd import FractionalICP
    rng = np.random.default_rng(5)
    src = rng.uniform(0, 10, (500, 3))
    corr = src + rng.normal(0, 0.1, (500, 3))
    icp = FractionalICP(src, corr)
    v = icp.frmsd(0.7, 350, src[:350], corr[:350])
    ref = (1.0 / (0.7 ** 3.0)) * np.sqrt(np.sum((src[:350] - corr[:350]) ** 2) / 350)
    np.testing.assert_allclose(v, ref, rtol=1e-13)
    assert icp.frmsd(0.5, 0, src[:0], corr[:0]) == float("inf")
    d = np.linalg.norm(src - corr, axis=1)
    np.testing.assert_array_equal(icp.get_n_first_elements(100, d), np.argsort(d, kind="stable")[:100])


# ------------------------------------------------------------------ fit / apply
def test_fit_golden(ctx):
    cases, _ = load_cases("fit")
    for name, c in cases.items():
        T = ctx.fit_rigid2d(c["src"][:, :2], c["tgt"][:, :2], bool(c["allow_reflection"]))
        assert_T_close(T, c["T"], c["src"], atol_R=1e-12, atol_xy=1e-7, msg=name)
        np.testing.assert_array_equal(T[2], [0.0, 0.0, 1.0])


def test_fit_arrival_many_grid_sizes(ctx, oracle):
    """k_fit_sums' two-level arrival (8 group counters + a top counter, the last workgroup
    solves) over 120 fits back to back whose sizes give 1 to ~100 workgroups (groups of
    uneven size, fewer workgroups than groups) against the oracle's SVD fit."""
    rng = np.random.default_rng(2024)
    sizes = np.unique(np.r_[1, 2, 3, 4095, 4096, 4097, 8191, 8193, 3 * 4096 + 1,
                            rng.integers(1, 400_000, 111)])
    for k in sizes:
        k = int(k)
        src = rng.normal(0, 50, (k, 2)) + [6.4e5, 6.48e6]
        th = rng.uniform(-0.1, 0.1)
        R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        tgt = src @ R.T + rng.uniform(-3, 3, 2) + rng.normal(0, 0.3, (k, 2))
        T = ctx.fit_rigid2d(src, tgt, False)
        Tref = oracle.fit_rigid2d(src, tgt, False)
        assert_T_close(T, Tref, src, msg=f"k={k}")


def test_apply_golden_bit_exact():
    from coregistrationgame_amd import FractionalICP
    cases, _ = load_cases("apply")
    for name, c in cases.items():
        icp = FractionalICP(c["pts"], c["pts"])
        out = icp.apply_transform_2d_xy_only(c["pts"], c["T"])
        np.testing.assert_array_equal(bits(out), bits(c["out"]), err_msg=name)


# ------------------------------------------------------------------ whole runs
@pytest.mark.parametrize("nn_mode", ["auto", "grid", "auto_loop"])
@pytest.mark.parametrize("name", RUN_FIXTURES)
def test_run_trace(name, nn_mode, monkeypatch):
    """Every golden run trace: "auto" takes the one-workgroup path (k_small.hip) where the
    plot fits it, "auto_loop" the multi-kernel loop at the same size (FICP_SMALL=0),
    "grid" the grid NN."""
    from coregistrationgame_amd import FractionalICP, _lib
    r = load_run(name)
    if nn_mode == "auto_loop":
        monkeypatch.setenv("FICP_SMALL", "0")
    icp = FractionalICP(r["src"], r["tgt"], threshold=float(r["kwargs_threshold"]),
                        max_iterations=int(r["kwargs_max_iterations"]), nn_mode=nn_mode.split("_")[0],
                        allow_reflection=allow_refl(r))
    final = icp.run(trace=True, trace_idx=True)
    tr = icp.last_stats
    fits = len(r["src"]) <= 1024 and len(r["tgt"]) <= 4096 and len(r["src"]) * len(r["tgt"]) <= 1 << 18
    assert tr["path"] == ("small" if nn_mode == "auto" and fits else "loop")
    np.testing.assert_allclose(final[:, :2], r["final"][:, :2], atol=1e-6, rtol=0)
    np.testing.assert_array_equal(bits(final[:, 2:]), bits(r["final"][:, 2:]))
    assert icp.lambda_val == float(r["lambda_final"])
    scale = 1.0 + np.abs(r["src"][:, :2]).max()
    first = pinned_prefix(r["gap"], r["frmsd"], scale)
    np.testing.assert_array_equal(tr["k"][:first], r["k"][:first])
    np.testing.assert_array_equal(tr["lam"][:first], r["lam"][:first])
    np.testing.assert_array_equal(tr["idx"][:first], r["idx"][:first])
    if first == len(r["k"]):
        assert tr["n_nn_calls"] == len(r["k"])
        assert_T_close(tr["T"], r["T"], r["src"], msg=name)
    else:
        nf = min(first, len(r["T"]))
        assert_T_close(tr["T"][:nf], r["T"][:nf], r["src"], msg=name)


def test_small_run_vs_oracle(oracle):
    """The one-workgroup run (k_small.hip) on plots of every size it takes -- 1 tree, 1
    stem, the Join button's 5-44 trees vs ~260 stems, 1024 trees, 4096 stems, md 2 and 3,
    geo-referenced, fixed iteration counts -- against the oracle run: k and NN index of
    every pinned call, XY within 1e-6, Z untouched."""
    from coregistrationgame_amd import FractionalICP, synth
    rng = np.random.default_rng(404)
    # (a plot whose selection maps onto one CHM stem has a zero cross-covariance: its rotation
    # is rounding noise in the reference, unpinnable -- test_batch_vs_oracle_mixed)
    shapes = [(1, 1), (1, 50), (7, 20), (5, 259), (44, 259), (20, 259), (300, 800), (1024, 256),
              (64, 4096), (500, 500), (1000, 200), (130, 2000)]
    for q, (n, m) in enumerate(shapes):
        md = 3 if q % 3 else 2
        p = synth.make_plot(n, m, float(rng.uniform(0.5, 0.9)), seed=4000 + q, md=md)
        kw = dict(threshold=float("-inf"), max_iterations=7) if q % 4 == 1 else {}
        icp = FractionalICP(p.source, p.target, **kw)
        final = icp.run(trace=True, trace_idx=True)
        st = icp.last_stats
        assert st["path"] == "small", (n, m)
        ofinal, otr = oracle.run(p.source, p.target, trace_idx=True,
                                 threshold=kw.get("threshold", 1e-6), max_iterations=kw.get("max_iterations", 1000))
        scale = 1.0 + np.abs(p.source[:, :2]).max()
        first = pinned_prefix(otr["gap"], otr["frmsd"], scale)
        np.testing.assert_array_equal(st["k"][:first], otr["k"][:first], err_msg=str((n, m)))
        np.testing.assert_array_equal(st["idx"][:first], otr["idx"][:first], err_msg=str((n, m)))
        if first == len(otr["k"]):
            assert st["n_nn_calls"] == otr["n_calls"], (n, m)
        np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str((n, m)))
        np.testing.assert_array_equal(bits(final[:, 2:]), bits(p.source[:, 2:]))


def test_real_stand10():
    from coregistrationgame_amd import FractionalICP
    import conftest
    z = np.load(conftest.GOLDEN / "run_real_stand10.npz")
    tgt = z["tgt"]
    for pid in z["plot_ids"]:
        src = z[f"{pid}/src"]
        icp = FractionalICP(src, tgt)
        final = icp.run(trace=True, trace_idx=True)
        np.testing.assert_allclose(final, z[f"{pid}/final"], atol=1e-6, rtol=0, err_msg=str(pid))
        gap = z[f"{pid}/gap"]
        if np.all(gap > K_GAP_PIN):
            np.testing.assert_array_equal(icp.last_stats["k"], z[f"{pid}/k"])
            np.testing.assert_array_equal(icp.last_stats["idx"], z[f"{pid}/idx"])


def test_run_vs_oracle_100k(oracle):
    """C2 scale (100k x 100k, f=0.8): whole run vs the pinned oracle."""
    from coregistrationgame_amd import FractionalICP, synth
    p = synth.make_plot(100_000, 100_000, 0.8, seed=100_000, md=3)
    icp = FractionalICP(p.source, p.target)
    final = icp.run(trace=True)
    ofinal, otr = oracle.run(p.source, p.target, nthreads=16)
    np.testing.assert_array_equal(icp.last_stats["k"], otr["k"])
    np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)
    np.testing.assert_array_equal(bits(final[:, 2]), bits(p.source[:, 2]))


# the switches DESIGN.md names as fallbacks: the separate fit pass (FICP_FUSE_FIT=0), the
# sorts the grid build and the work order fall back to for layers the bucket sort cannot
# plan (global-atomic grid build, 64-bit radix work order), and the two launch forms that
# avoid the selection's in-launch hand-offs (FICP_SEL_SPLIT=1: bounds and gather as two
# kernels; FICP_SEL_BGF=0: the final as its own launch) -- DESIGN §4.2, §4.3, §4.5
KNOBS = [{}, {"FICP_FUSE_FIT": "0"},
         {"FICP_GRID_ATOMIC": "1", "FICP_WORK_RADIX": "1", "FICP_FUSE_FIT": "0"},
         {"FICP_SEL_SPLIT": "1"}, {"FICP_SEL_BGF": "0"}]


@pytest.mark.parametrize("knobs,md", [(k, 3) for k in KNOBS] + [({}, 2), ({"FICP_GRID_ATOMIC": "1"}, 2)],
                         ids=lambda v: ",".join(f"{a}={b}" for a, b in v.items()) or "default"
                         if isinstance(v, dict) else f"md{v}")
def test_run_untraced_vs_oracle_100k(oracle, knobs, md, monkeypatch):
    """The production loop (no traces: the selection's last kernel runs the loop step; with
    by default it also runs the rigid fit, FICP_FUSE_FIT=0 a separate pass; half-step
    lookahead, certified NN reuse; the sort keys derived from r unless FICP_NN_KEYS=1)
    against the pinned oracle at 100k, 3-D and 2-D matching, under every kernel switch."""
    from coregistrationgame_amd import FractionalICP, synth
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    p = synth.make_plot(100_000, 100_000, 0.8, seed=100_000, md=md)
    icp = FractionalICP(p.source, p.target)
    final = icp.run()
    ofinal, otr = oracle.run(p.source, p.target, nthreads=16)
    assert icp.last_stats["n_nn_calls"] == len(otr["k"])
    assert icp.last_stats["k_last"] == otr["k"][-1]
    np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)
    if md == 3:
        np.testing.assert_array_equal(bits(final[:, 2]), bits(p.source[:, 2]))


@pytest.mark.parametrize("md", [2, 3])
def test_run_certified_reuse_near_ties(oracle, md):
    """Certified match reuse (k_grid_nn.hip cert_try / cert_scan_group) on a layout built
    for near-ties: stems on a 2 m lattice (a tenth of them duplicated), sources at lattice
    midpoints and points +-1 mm from them, under a small rigid misregistration.  Every NN
    call's idx must equal the oracle's, call by call."""
    from coregistrationgame_amd import FractionalICP
    rng = np.random.default_rng(77 + md)
    gx, gy = np.meshgrid(np.arange(160) * 2.0, np.arange(160) * 2.0)
    stems = np.c_[gx.ravel() + 5.0e5, gy.ravel() + 6.5e6]
    stems = np.r_[stems, stems[rng.choice(len(stems), len(stems) // 10, replace=False)]]
    tgt = np.c_[stems, rng.uniform(10, 30, len(stems)).round(1)]
    pick = rng.choice(len(gx.ravel()), 20_000, replace=False)
    src = tgt[pick].copy()
    src[:5000, :2] += 1.0                                   # midpoints of four stems
    src[5000:10000, 0] += 1.0 + rng.choice([-1e-3, 1e-3], 5000)   # near-midpoint of two
    src[10000:, :2] += rng.normal(0, 0.2, (10000, 2))
    th = 0.004
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    c0 = src[:, :2].mean(0)
    src[:, :2] = (src[:, :2] - c0) @ R.T + c0 + [0.7, -0.4]
    if md == 2:
        src, tgt = src[:, :2].copy(), tgt[:, :2].copy()
    icp = FractionalICP(src, tgt, nn_mode="grid")
    final = icp.run(trace=True, trace_idx=True)
    tr = icp.last_stats
    ofinal, otr = oracle.run(src, tgt, nthreads=16, trace_idx=True)
    ncall = min(len(tr["k"]), len(otr["k"]))
    same = np.flatnonzero(tr["k"][:ncall] != otr["k"][:ncall])
    upto = int(same[0]) + 1 if len(same) else ncall  # trajectories agree through here
    assert upto >= 3
    np.testing.assert_array_equal(tr["idx"][:upto], otr["idx"][:upto])
    if not len(same):
        np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)


@pytest.mark.parametrize("md", [2, 3])
def test_device_resident_path_matches_host_path(md):
    """The bench's path (ficp_set_target_device: one kernel copies the target and reduces
    its bbox; ficp_run_device on device columns) gives the host path's bits, twice in a
    row on one context (the second target set replaces the first)."""
    from coregistrationgame_amd import _lib, synth
    C = _lib.C
    lib = _lib.lib()
    ctx = _lib.Context(0)
    bufs = []

    def dev(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        p = C.c_void_p()
        _lib._check(lib.ficp_dev_alloc(ctx.h, a.nbytes, C.byref(p)))
        _lib._check(lib.ficp_memcpy_h2d(ctx.h, p, a.ctypes.data_as(C.c_void_p), a.nbytes))
        bufs.append(p)
        return p.value

    def back(ptr, n):
        out = np.empty(n)
        _lib._check(lib.ficp_memcpy_d2h(ctx.h, out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), 8 * n))
        return out

    try:
        lam = [3.0, 0.95 if md == 3 else 1.3]
        for seed in (5, 6):
            p = synth.make_plot(50_000, 60_000, 0.7, seed=seed, md=md)
            ref = _lib.Context(0)
            want = p.source.copy()
            ref.set_target(p.target, md)
            ref.run(want, lam, 1e-6, 1000, False)
            ref.close()
            sx, sy = dev(p.source[:, 0]), dev(p.source[:, 1])
            sz = dev(p.source[:, 2]) if md == 3 else 0
            tx, ty = dev(p.target[:, 0]), dev(p.target[:, 1])
            tz = dev(p.target[:, 2]) if md == 3 else 0
            ctx.set_target_device(tx, ty, tz, len(p.target), md)
            ctx.run_device(sx, sy, sz, len(p.source), lam, 1e-6, 1000)
            np.testing.assert_array_equal(bits(back(sx, len(p.source))), bits(want[:, 0]))
            np.testing.assert_array_equal(bits(back(sy, len(p.source))), bits(want[:, 1]))
    finally:
        for b in bufs:
            lib.ficp_dev_free(ctx.h, b)
        ctx.close()


@pytest.mark.gpu
def test_target_replaced_while_bbox_report_pending():
    """ficp_set_target_device queues its bbox report at once (capi.hip bbox_collect).  A
    second target set before any run -- device or host -- must collect that report first,
    so the run plans its grid on the second target's bbox: the bits of a fresh context
    given only the second target."""
    from coregistrationgame_amd import _lib, synth
    C = _lib.C
    lib = _lib.lib()
    md = 3
    lam = [3.0, 0.95]
    p = synth.make_plot(40_000, 50_000, 0.7, seed=11, md=md)
    decoy = p.target.copy()
    decoy[:, :2] = decoy[:, :2] * 3.0 + 5000.0  # another bbox entirely
    ref = _lib.Context(0)
    want = p.source.copy()
    ref.set_target(p.target, md)
    ref.run(want, lam, 1e-6, 1000, False)
    ref.close()
    ctx = _lib.Context(0)
    bufs = []

    def dev(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        q = C.c_void_p()
        _lib._check(lib.ficp_dev_alloc(ctx.h, a.nbytes, C.byref(q)))
        _lib._check(lib.ficp_memcpy_h2d(ctx.h, q, a.ctypes.data_as(C.c_void_p), a.nbytes))
        bufs.append(q)
        return q.value

    try:
        cols = [dev(decoy[:, j]) for j in range(3)]
        real = [dev(p.target[:, j]) for j in range(3)]
        # device then device
        ctx.set_target_device(cols[0], cols[1], cols[2], len(decoy), md)
        ctx.set_target_device(real[0], real[1], real[2], len(p.target), md)
        sx, sy, sz = (dev(p.source[:, j]) for j in range(3))
        ctx.run_device(sx, sy, sz, len(p.source), lam, 1e-6, 1000)
        for j, s in ((0, sx), (1, sy)):
            out = np.empty(len(p.source))
            _lib._check(lib.ficp_memcpy_d2h(ctx.h, out.ctypes.data_as(C.c_void_p), C.c_void_p(s), out.nbytes))
            np.testing.assert_array_equal(bits(out), bits(want[:, j]))
        # device then host
        ctx.set_target_device(cols[0], cols[1], cols[2], len(decoy), md)
        ctx.set_target(p.target, md)
        got = p.source.copy()
        ctx.run(got, lam, 1e-6, 1000, False)
        np.testing.assert_array_equal(bits(got[:, :2]), bits(want[:, :2]))
    finally:
        for b in bufs:
            lib.ficp_dev_free(ctx.h, b)
        ctx.close()


def test_run_many_stages_matches_split_runs():
    """Six stages in one ficp_run (lambdas past the fourth come from the device array, the
    first four from the kernel arguments) equal the same stages run as two calls."""
    from coregistrationgame_amd import _lib, synth
    p = synth.make_plot(80_000, 90_000, 0.7, seed=31, md=3)
    lams = [3.0, 0.95, 1.3, 2.0, 0.95, 3.0]
    one = p.source.copy()
    c1 = _lib.Context(0)
    c1.set_target(p.target, 3)
    s1 = c1.run(one, lams, 1e-6, 1000, False)
    c1.close()
    two = p.source.copy()
    c2 = _lib.Context(0)
    c2.set_target(p.target, 3)
    a = c2.run(two, lams[:2], 1e-6, 1000, False)
    b = c2.run(two, lams[2:], 1e-6, 1000, False)
    c2.close()
    # the second call rebuilds the work order from moved positions, so the fit's sums
    # run in another order: XY agree to the north-star bar, not bit for bit
    assert s1["n_nn_calls"] == a["n_nn_calls"] + b["n_nn_calls"]
    np.testing.assert_allclose(one[:, :2], two[:, :2], atol=1e-6, rtol=0)
    np.testing.assert_array_equal(bits(one[:, 2]), bits(p.source[:, 2]))


def test_run_1M_properties():
    """C3 (1M x 1M, f=0.6, to convergence): the run undoes the synthetic misregistration
    (size-independent property) and a second run from its output is a fixed point."""
    from coregistrationgame_amd import FractionalICP, synth
    p = synth.make_plot(1_000_000, 1_000_000, 0.6, seed=1_000_000, md=3)
    icp = FractionalICP(p.source, p.target)
    final = icp.run()
    st = icp.last_stats
    assert st["n_nn_calls"] >= 3
    inl = p.inlier_of >= 0
    resid = np.linalg.norm(final[inl, :2] - p.target[p.inlier_of[inl], :2], axis=1)
    # inliers carry N(0, 0.3 m) jitter per axis: the median 2-D error is ~0.35 m when aligned
    assert np.median(resid) < 0.45, np.median(resid)
    np.testing.assert_array_equal(bits(final[:, 2]), bits(p.source[:, 2]))
    icp2 = FractionalICP(final, p.target)
    again = icp2.run()
    assert np.max(np.abs(again[:, :2] - final[:, :2])) < 1e-3


# ------------------------------------------------------------------ reference tests, re-stated
def _nn_rmsd(A, B, oracle):
    md = 3 if (A.shape[1] >= 3 and B.shape[1] >= 3) else 2
    _, d, _ = oracle.nn(A, B, md, "brute")
    return np.sqrt(np.mean(d ** 2))


def _inlier_fraction_xy(aligned, target, oracle, tol=0.10):
    _, d, _ = oracle.nn(aligned[:, :2], target[:, :2], 2, "brute")
    return np.mean(d < tol)


def test_ref_basic_rigid_exact(oracle):
    """tests/test_ficp.py:39-58"""
    from coregistrationgame_amd import FractionalICP, synth
    src = synth.make_cloud(n=150, seed=1)
    angle, t = 27.0, np.array([1.6, -2.2])
    tgt = synth.apply_rigid(src, angle, t)
    aligned = FractionalICP(src.copy(), tgt).run()
    X, Y = src[:, :2], aligned[:, :2]
    Xc, Yc = X - X.mean(0), Y - Y.mean(0)
    A = np.linalg.lstsq(Xc, Yc, rcond=None)[0].T
    ang_est = np.rad2deg(np.arctan2(A[1, 0], A[0, 0]))
    assert np.allclose(aligned[:, 2], src[:, 2])
    assert abs(np.linalg.det(A) - 1.0) < 1e-2
    assert abs(((ang_est - angle + 180) % 360) - 180) < 0.2
    assert _nn_rmsd(aligned, tgt, oracle) < 2e-3


def test_ref_missing_points_frmsd(oracle):
    """tests/test_ficp.py:61-76"""
    from coregistrationgame_amd import FractionalICP, synth
    _, src, tgt = synth.reference_scenarios()[1]
    aligned = FractionalICP(src.copy(), tgt).run()
    assert np.allclose(aligned[:, 2], src[:, 2])
    assert _nn_rmsd(aligned, tgt, oracle) < _nn_rmsd(src, tgt, oracle) * 0.4
    assert _inlier_fraction_xy(aligned, tgt, oracle, tol=0.12) > 0.55


def test_ref_missing_plus_outliers_frmsd(oracle):
    """tests/test_ficp.py:79-101"""
    from coregistrationgame_amd import FractionalICP, synth
    src = synth.make_cloud(n=200, seed=3)
    clean = synth.apply_rigid(src, -22.0, [-1.2, 2.0])
    _, _, tgt_noisy = synth.reference_scenarios()[2]
    aligned = FractionalICP(src.copy(), tgt_noisy).run()
    assert np.allclose(aligned[:, 2], src[:, 2])
    assert _nn_rmsd(aligned, tgt_noisy, oracle) < _nn_rmsd(src, tgt_noisy, oracle) * 0.5
    assert _inlier_fraction_xy(aligned, clean, oracle, tol=0.12) > 0.90


def test_ref_transform_is_planar_and_preserves_z():
    """tests/test_rigid_2d_operations.py:59-75"""
    from coregistrationgame_amd import FractionalICP
    src = np.array([[0.0, 0.0, 1.0], [1.0, 0.0, 2.0], [0.0, 1.0, 3.0]])
    theta = np.deg2rad(15.0)
    rot = np.array([[np.cos(theta), -np.sin(theta)], [np.sin(theta), np.cos(theta)]])
    tgt = np.hstack([src[:, :2] @ rot.T + np.array([0.3, -0.4]), src[:, 2:]])
    icp = FractionalICP(src.copy(), tgt)
    T = icp.compute_optimal_transform_2d(src, tgt)
    transformed = icp.apply_transform_2d_xy_only(src, T)
    R = T[:2, :2]
    np.testing.assert_allclose(R.T @ R, np.eye(2), atol=1e-7)
    np.testing.assert_allclose(np.linalg.det(R), 1.0, atol=1e-7)
    np.testing.assert_array_equal(transformed[:, 2], src[:, 2])


def test_drop_in_module_import():
    """`from ficp import FractionalICP` resolves to the engine (app.py:20)."""
    import ficp
    from coregistrationgame_amd.ficp import FractionalICP
    assert ficp.FractionalICP is FractionalICP


# ------------------------------------------------------------ remove_matches (§8 f1)
def test_remove_matches_golden():
    """CHMPlot.remove_matches on the GPU: the reference's removal sequence, every case
    (3-D, 2-D by missing heights, conflicts, exhaustion, geo coordinates, exact ties, a
    sequence of plots on one shrinking layer)."""
    import conftest
    from coregistrationgame_amd.matches import remove_matches_arrays
    from test_oracle_golden import _matches_sequence
    z = np.load(conftest.GOLDEN / "matches.npz")
    for name in sorted({k.split("/")[0] for k in z.files}):
        got = _matches_sequence(remove_matches_arrays, z, name)
        for k, g in enumerate(got):
            np.testing.assert_array_equal(g, z[f"{name}/removed{k}"], err_msg=f"{name} call {k}")


def test_remove_matches_crowded_vs_oracle(oracle):
    """Many plot trees fighting over few stems: most trees lose all 8 GPU candidates and
    the walk re-queries with the removed stems masked."""
    from coregistrationgame_amd.matches import remove_matches_arrays
    rng = np.random.default_rng(11)
    chm = np.column_stack([rng.uniform(0, 60, 400), rng.uniform(0, 60, 400), rng.uniform(5, 30, 400)])
    centre = chm[rng.integers(0, 400, 30)]
    plot = centre[rng.integers(0, 30, 600)] + np.column_stack(
        [rng.normal(0, 1.5, 600), rng.normal(0, 1.5, 600), rng.normal(0, 2, 600)])
    np.testing.assert_array_equal(remove_matches_arrays(plot, chm), oracle.remove_matches(plot, chm))
    plot[::3, 2] = np.nan  # 2-D with the 10 m rule
    np.testing.assert_array_equal(remove_matches_arrays(plot, chm), oracle.remove_matches(plot, chm))


def test_remove_matches_objects():
    """The object-level drop-in edits chm.trees / chm.removed_stems like the reference."""
    from types import SimpleNamespace as NS
    from coregistrationgame_amd.matches import remove_matches
    rng = np.random.default_rng(2)
    stems = [NS(currentx=float(x), currenty=float(y), height=float(h))
             for x, y, h in zip(rng.uniform(0, 30, 50), rng.uniform(0, 30, 50), rng.uniform(5, 30, 50))]
    trees = [NS(currentx=s.currentx + 0.1, currenty=s.currenty, height=s.height) for s in stems[:10]]
    trees.append(NS(currentx=100.0, currenty=100.0, height=None))  # far, no height -> 2-D
    chm = NS(trees=list(stems), removed_stems=[])
    removed = remove_matches(chm, NS(trees=trees))
    assert [id(t) for t in removed] == [id(s) for s in stems[:10]]
    assert len(chm.trees) == 40 and chm.removed_stems == [removed]


# ------------------------------------------------------------ callers (§8 f2, f3)
def _ns_plot(xy, cur, flipped=False, heights=None):
    from types import SimpleNamespace as NS
    trees = [NS(tree_id=f"t{i}", x=float(a), y=float(b), currentx=float(c), currenty=float(d),
                height=None if heights is None else float(heights[i]))
             for i, ((a, b), (c, d)) in enumerate(zip(xy, cur))]
    return NS(trees=trees, flipped=flipped, center=tuple(np.mean(xy, axis=0)),
              current_center=tuple(np.mean(cur, axis=0)), plotid=0)


def test_get_transform_golden():
    """Plot.get_transform (trees.py:248-280) on the GPU vs the reference's SVD result:
    1..120 trees, flipped or not, unit and geo-referenced coordinates."""
    import conftest
    from coregistrationgame_amd.stand import get_transform
    z = np.load(conftest.GOLDEN / "transforms.npz")
    for case in sorted({k.split("/")[0] for k in z.files}):
        xy, cur = z[f"{case}/xy"], z[f"{case}/cur"]
        R, t, fl = get_transform(_ns_plot(xy, cur, bool(z[f"{case}/flipped"])))
        assert fl == bool(z[f"{case}/flipped"])
        # With collinear trees (n <= 2) H has rank 1: a rotation and a reflection fit the
        # trees equally well, and a flipped plot keeps whichever LAPACK's singular vectors
        # give -- parity unpinned for R there, pinned for its action on the trees.
        if len(xy) > 2 or not fl:
            np.testing.assert_allclose(R, z[f"{case}/R"], atol=1e-9, rtol=0, err_msg=case)
        np.testing.assert_allclose(xy @ R.T + t, xy @ z[f"{case}/R"].T + z[f"{case}/t"], atol=1e-6,
                                   rtol=0, err_msg=case)


def test_join_stand_real_vs_oracle(oracle):
    """The app's Join loop over stand 10 (16 real plots, one shrinking 259-stem CHM layer):
    join (2-D: no plot heights), transformation record, remove_matches -- vs the oracle's
    run + remove_matches composed the same way."""
    import conftest
    from types import SimpleNamespace as NS
    from coregistrationgame_amd.stand import join_stand
    z = np.load(conftest.GOLDEN / "run_real_stand10.npz")
    tgt = z["tgt"]
    stems = [NS(tree_id=i, x=float(a), y=float(b), currentx=float(a), currenty=float(b), height=None)
             for i, (a, b) in enumerate(tgt)]
    chm = NS(trees=list(stems), removed_stems=[])
    plots = [_ns_plot(z[f"{pid}/src"], z[f"{pid}/src"]) for pid in z["plot_ids"]]
    for pid, p in zip(z["plot_ids"], plots):
        p.plotid = int(pid)
    records = join_stand(NS(plots=plots), chm)
    alive = list(range(len(tgt)))
    for pid, p in zip(z["plot_ids"], plots):
        src = z[f"{pid}/src"]
        final, _ = oracle.run(src, tgt[alive], nthreads=4)
        got = np.array([[t.currentx, t.currenty] for t in p.trees])
        np.testing.assert_allclose(got, final[:, :2], atol=1e-6, rtol=0, err_msg=str(pid))
        plot_xyh = np.column_stack([final[:, :2], np.full(len(final), np.nan)])
        chm_xyh = np.column_stack([tgt[alive], np.full(len(alive), np.nan)])
        rem = [alive[i] for i in oracle.remove_matches(plot_xyh, chm_xyh)]
        for r in rem:
            alive.remove(r)
        assert records[int(pid)]["flip"] is False
    assert sorted(t.tree_id for t in chm.trees) == alive


# ------------------------------------------------------------------ allow_reflection=True
REFL_FIXTURES = [n for n in RUN_FIXTURES if n.startswith("refl_")]


@pytest.mark.parametrize("knobs", [{}, {"FICP_SMALL": "0"}, {"FICP_SMALL": "0", "FICP_FUSE_FIT": "0"},
                                   {"FICP_SMALL": "0", "FICP_SEL_WIN": "0"}],
                         ids=["small", "loop", "loop_fit_pass", "loop_no_window"])
@pytest.mark.parametrize("name", REFL_FIXTURES)
def test_run_allow_reflection_golden(name, knobs, monkeypatch):
    """run(allow_reflection=True) (ficp.py:13, 101-103) against the reference's own runs:
    mirrored strips whose first fit is a reflection (det R = -1) and a regular plot under
    the flag.  One-workgroup kernel, multi-kernel loop (fused fit, separate fit pass,
    window selection off).  Per pinned call k and NN idx exact, T within 1e-6 in action,
    final XY within 1e-6."""
    from coregistrationgame_amd import FractionalICP
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    r = load_run(name)
    assert allow_refl(r)
    icp = FractionalICP(r["src"], r["tgt"], allow_reflection=True)
    final = icp.run(trace=True, trace_idx=True)
    tr = icp.last_stats
    fits = len(r["src"]) <= 1024 and len(r["tgt"]) <= 4096 and len(r["src"]) * len(r["tgt"]) <= 1 << 18
    assert tr["path"] == ("small" if fits and not knobs else "loop")
    np.testing.assert_allclose(final[:, :2], r["final"][:, :2], atol=1e-6, rtol=0)
    np.testing.assert_array_equal(bits(final[:, 2:]), bits(r["final"][:, 2:]))
    scale = 1.0 + np.abs(r["src"][:, :2]).max()
    first = pinned_prefix(r["gap"], r["frmsd"], scale)
    np.testing.assert_array_equal(tr["k"][:first], r["k"][:first])
    np.testing.assert_array_equal(tr["idx"][:first], r["idx"][:first])
    nf = min(first, len(r["T"]))
    assert_T_close(tr["T"][:nf], r["T"][:nf], r["src"], msg=name)
    ref_dets = np.linalg.det(r["T"][:nf, :2, :2])
    np.testing.assert_array_equal(np.sign(np.linalg.det(np.asarray(tr["T"]).reshape(-1, 3, 3)[:nf, :2, :2])), np.sign(ref_dets))
    if name.startswith("refl_strip"):
        assert ref_dets[0] < 0  # the fixture really exercises the reflection branch


def _mirrored_strip(n, seed, th, noise, fout, md=3):
    """n CHM stems on a 1.2 m-wide strip (4 m apart on average along it) and a tree layer
    that is their mirror image in x, rotated by th about the strip's centre, shifted, with
    noise and a fraction fout of outliers pushed sideways: the first fit is a reflection."""
    rng = np.random.default_rng(seed)
    L = 4.0 * n
    tgt = np.column_stack([rng.uniform(-0.6, 0.6, n), rng.uniform(0, L, n), rng.uniform(5, 30, n)])[:, :md]
    src = tgt.copy()
    src[:, 0] = -src[:, 0]
    c = np.array([0.0, L / 2])
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    src[:, :2] = (src[:, :2] - c) @ R.T + c + [0.15, -0.1] + rng.normal(0, noise, (n, 2))
    k = int(fout * n)
    src[:k, 0] += rng.uniform(-20, 20, k)
    src[:, :2] += [5.0e5, 6.5e6]
    tgt[:, :2] += [5.0e5, 6.5e6]
    return src, tgt


@pytest.mark.parametrize("case", ["strip3_200k", "strip2_200k", "plot3_300k"])
def test_run_allow_reflection_large_vs_oracle(case, oracle, monkeypatch):
    """run(allow_reflection=True) on the production loop at sizes where the half-step
    lookahead and the window selection run (>= 64k rows), vs the pinned oracle (whose
    reflection branch the run_refl_* fixtures pin): the NN-call count, k of every call the
    oracle's curve separates (conftest.K_GAP_PIN_LARGE), the sign of det R of every fit,
    final XY within 1e-6.  The fused fit and the separate fit pass both."""
    from conftest import K_GAP_PIN_LARGE
    from coregistrationgame_amd import FractionalICP, _lib, synth
    if case == "plot3_300k":
        p = synth.make_plot(300_000, 300_000, 0.7, seed=300_001, md=3)
        src, tgt = p.source, p.target
    else:
        src, tgt = _mirrored_strip(200_000, 5, 2e-7, 0.05, 0.2, md=3 if case[5] == "3" else 2)
    ofinal, otr = oracle.run(src, tgt, allow_reflection=True, nthreads=16)
    odet = np.sign(np.linalg.det(np.asarray(otr["T"]).reshape(-1, 3, 3)[:, :2, :2]))
    if case != "plot3_300k":
        assert odet[0] < 0
    pinned = otr["gap"] > K_GAP_PIN_LARGE
    for knobs in ({}, {"FICP_FUSE_FIT": "0"}):
        monkeypatch.delenv("FICP_FUSE_FIT", raising=False)
        for k, v in knobs.items():
            monkeypatch.setenv(k, v)
        icp = FractionalICP(src, tgt, allow_reflection=True)
        final = icp.run(trace=True)
        st = icp.last_stats
        assert st["n_nn_calls"] == otr["n_calls"], knobs
        np.testing.assert_array_equal(np.asarray(st["k"])[pinned], otr["k"][pinned])
        np.testing.assert_array_equal(np.sign(np.linalg.det(np.asarray(st["T"]).reshape(-1, 3, 3)[:, :2, :2])), odet)
        np.testing.assert_allclose(final[:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str(knobs))
    # the untraced production loop (fused selection, window path where eligible)
    monkeypatch.delenv("FICP_FUSE_FIT", raising=False)
    ctx = _lib.Context(0, _lib.NN_GRID)
    try:
        md = 3 if src.shape[1] >= 3 and tgt.shape[1] >= 3 else 2
        ctx.set_target(tgt, md)
        out = np.array(src)
        st = ctx.run(out, [3.0, 0.95 if md == 3 else 1.3], 1e-6, 1000, True)
        ps = ctx.path_stats()
    finally:
        ctx.close()
    assert st["n_nn_calls"] == otr["n_calls"]
    assert st["k_last"] == otr["k"][-1]
    np.testing.assert_allclose(out[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)
    print(f"{case}: window calls {ps['win_calls']}, retries {ps['win_retries']}")
    if case == "plot3_300k":
        assert ps["win_calls"] >= 1, ps
