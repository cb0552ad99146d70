"""GPU parity of the multi-plot path (ficp_run_batch, C4) against the golden traces and
the pinned oracle, plot by plot.  Each plot of a batch must end exactly where its own
FractionalICP(source, target).run() ends (ficp.py:122-154)."""
import numpy as np
import pytest

from conftest import GOLDEN, K_GAP_PIN, RUN_FIXTURES, allow_refl, load_run, pinned_prefix

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def test_batch_golden_runs():
    """Every golden run fixture (md 2 and 3, unit and geo coordinates, threshold -inf)
    in one batch call per (threshold, max_iterations) group."""
    from coregistrationgame_amd import FractionalICPBatch
    runs = {name: load_run(name) for name in RUN_FIXTURES}
    groups = {}
    for name, r in runs.items():
        key = (float(r["kwargs_threshold"]), int(r["kwargs_max_iterations"]), allow_refl(r))
        groups.setdefault(key, []).append(name)
    for (thr, mx, refl), names in groups.items():
        b = FractionalICPBatch([runs[n]["src"] for n in names], [runs[n]["tgt"] for n in names],
                               threshold=thr, max_iterations=mx, allow_reflection=refl)
        finals = b.run()
        for j, name in enumerate(names):
            r = runs[name]
            np.testing.assert_allclose(finals[j][:, :2], r["final"][:, :2], atol=1e-6, rtol=0, err_msg=name)
            np.testing.assert_array_equal(bits(finals[j][:, 2:]), bits(r["final"][:, 2:]))
            scale = 1.0 + np.abs(r["src"][:, :2]).max()
            if pinned_prefix(r["gap"], r["frmsd"], scale) == len(r["k"]):
                st = b.stats[j]
                assert st["n_nn_calls"] == len(r["k"]), name
                assert st["n_fits"] == len(r["T"]), name
                assert st["k_last"] == r["k"][-1], name


def test_batch_real_stand10():
    """The 16 real plots of Data/2014 against the whole Data/2019 stem layer, as a batch."""
    from coregistrationgame_amd import FractionalICPBatch
    z = np.load(GOLDEN / "run_real_stand10.npz")
    tgt = z["tgt"]
    pids = list(z["plot_ids"])
    b = FractionalICPBatch([z[f"{pid}/src"] for pid in pids], [tgt] * len(pids))
    finals = b.run()
    for j, pid in enumerate(pids):
        np.testing.assert_allclose(finals[j], z[f"{pid}/final"], atol=1e-6, rtol=0, err_msg=str(pid))
        if np.all(z[f"{pid}/gap"] > K_GAP_PIN):
            assert b.stats[j]["n_nn_calls"] == len(z[f"{pid}/k"]), pid
            assert b.stats[j]["k_last"] == z[f"{pid}/k"][-1], pid


@pytest.mark.parametrize("knobs", [{}, {"FICP_GRID_ATOMIC": "1"}, {"FICP_BATCH_STREAMS": "1"},
                                   {"FICP_BATCH_STREAMS": "4"}, {"FICP_BATCH_FUSE": "0"}],
                         ids=["bsort_grid_2streams", "atomic_grid", "one_stream", "four_streams",
                              "fit_update_launches"])
def test_batch_vs_oracle_mixed(oracle, knobs, monkeypatch):
    """64 synthetic plots of mixed sizes (incl. 1-tree plots, empty layers, md=2 plots)
    vs the oracle run of each plot alone, with the batch grid built by the bucket sort
    (default) and by the global-atomic fallback, as two sub-batches on two streams (the
    default at 64-384 plots) and as one, with the loop step and the fit inside the
    selection (default) and as their own launches.  (A plot whose selection can map onto a single
    CHM stem has a zero cross-covariance: its rotation is rounding noise in the reference
    and unpinnable, so the CHM layers here have >= 60 stems.)"""
    from coregistrationgame_amd import FractionalICPBatch, synth
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(7)
    srcs, tgts = [], []
    for p in range(64):
        n = int(rng.choice([1, 2, 50, 400, 3000]))
        m = int(rng.choice([60, 500, 4000]))
        pl = synth.make_plot(n, m, 0.8, seed=20_000 + p, md=3)
        s, t = pl.source, pl.target
        if p % 7 == 3:
            s, t = s[:, :2], t[:, :2]  # 2-D plot: lambda 1.3 in stage 2
        srcs.append(s)
        tgts.append(t)
    srcs[5] = srcs[5][:0]            # empty tree layer
    tgts[9] = tgts[9][:0]            # empty CHM layer
    b = FractionalICPBatch(srcs, tgts)
    finals = b.run(trace=True)
    for p in range(64):
        if len(srcs[p]) == 0 or len(tgts[p]) == 0:
            np.testing.assert_array_equal(finals[p], srcs[p])
            assert b.stats[p]["n_nn_calls"] == 0
            assert len(b.k_trace[p]) == 0
            continue
        ofinal, otr = oracle.run(srcs[p], tgts[p], nthreads=8)
        np.testing.assert_allclose(finals[p][:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str(p))
        np.testing.assert_array_equal(bits(finals[p][:, 2:]), bits(srcs[p][:, 2:]))
        assert b.stats[p]["n_nn_calls"] == len(otr["k"]), p
        assert b.stats[p]["k_last"] == otr["k"][-1], p
        # k of every call the oracle's curve pins (per call, not only the last)
        first = pinned_prefix(otr["gap"], otr["frmsd"], 1.0 + np.abs(srcs[p][:, :2]).max())
        assert len(b.k_trace[p]) == len(otr["k"]), p
        np.testing.assert_array_equal(b.k_trace[p][:first], otr["k"][:first], err_msg=str(p))


def _far_apart_batch(n_plots=80):
    """Plots at distinct geo offsets ~km apart (each plot's own CHM bbox centre is its fit
    pivot), with empty CHM layers in the first sub-batch (pivot (0, 0))."""
    from coregistrationgame_amd import synth
    srcs, tgts = [], []
    for p in range(n_plots):
        pl = synth.make_plot(600, 900, 0.8, seed=40_000 + p, md=3)
        shift = np.array([3_000.0 * (p % 9), 7_000.0 * (p // 9)])
        s, t = pl.source.copy(), pl.target.copy()
        s[:, :2] += shift
        t[:, :2] += shift
        srcs.append(s)
        tgts.append(t)
    for p in (2, 11):  # empty CHM layers in the first half
        tgts[p] = tgts[p][:0]
    return srcs, tgts


def test_batch_sub_batches_far_apart_bit_identical(oracle, monkeypatch):
    """with two sub-batches, the fused selection's fit must use the
    pivot of its own plot, not of the plot at the same position in the first sub-batch.
    One stream vs two streams must be bit-identical; the fused step and the separate
    fit/update launches (FICP_BATCH_FUSE=0) must take the same NN calls and k; a sample
    of plots in the second sub-batch equals the oracle."""
    from coregistrationgame_amd import FractionalICPBatch
    srcs, tgts = _far_apart_batch()
    outs = {}
    for name, knobs in (("two", {"FICP_BATCH_STREAMS": "2"}), ("one", {"FICP_BATCH_STREAMS": "1"}),
                        ("unfused", {"FICP_BATCH_STREAMS": "2", "FICP_BATCH_FUSE": "0"})):
        for k, v in knobs.items():
            monkeypatch.setenv(k, v)
        b = FractionalICPBatch(srcs, tgts)
        outs[name] = (b.run(trace=True), b.stats, b.k_trace)
        monkeypatch.delenv("FICP_BATCH_FUSE", raising=False)
    (f2, s2, k2), (f1, s1, k1), (fu, su, ku) = outs["two"], outs["one"], outs["unfused"]
    for p in range(len(srcs)):
        np.testing.assert_array_equal(bits(f2[p]), bits(f1[p]), err_msg=str(p))
        np.testing.assert_array_equal(k2[p], k1[p], err_msg=str(p))
        np.testing.assert_array_equal(k2[p], ku[p], err_msg=str(p))
        assert s2[p]["n_nn_calls"] == su[p]["n_nn_calls"], p
        assert s2[p]["k_last"] == su[p]["k_last"], p
        np.testing.assert_allclose(f2[p][:, :2], fu[p][:, :2], atol=1e-6, rtol=0, err_msg=str(p))
    for p in (40, 42, 51, 79):
        ofinal, otr = oracle.run(srcs[p], tgts[p], nthreads=8)
        np.testing.assert_allclose(f2[p][:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str(p))
        assert s2[p]["n_nn_calls"] == len(otr["k"]), p


def test_batch_matches_single_runs():
    """Batch == one FractionalICP per plot on the GPU (same NN calls, same k, same XY)."""
    from coregistrationgame_amd import FractionalICP, FractionalICPBatch, synth
    plots = synth.make_batch(24, 10_000, 10_000, 0.8, 10_000_000, md=3)
    b = FractionalICPBatch([p.source for p in plots], [p.target for p in plots])
    finals = b.run()
    for j, p in enumerate(plots):
        icp = FractionalICP(p.source, p.target, nn_mode="grid")
        single = icp.run()
        np.testing.assert_allclose(finals[j][:, :2], single[:, :2], atol=1e-6, rtol=0)
        assert b.stats[j]["n_nn_calls"] == icp.last_stats["n_nn_calls"]
        assert b.stats[j]["n_fits"] == icp.last_stats["n_fits"]
        assert b.stats[j]["k_last"] == icp.last_stats["k_last"]


def test_batch_c4_size_plots_vs_oracle(oracle, monkeypatch):
    """plots of C4's own size (10k trees x 10k stems) inside a batch, against the
    oracle run of each plot alone: NN-call count, k of every call the oracle's curve pins,
    XY within 1e-6, Z bit-identical -- in the batch work order (default) and in caller
    order (FICP_BATCH_WORK=0), which must take the same calls and k.  Plot 5 has duplicated
    trees (exact equal distances: ties at k are broken by the caller's row in both orders)."""
    from coregistrationgame_amd import FractionalICPBatch, synth
    plots = synth.make_batch(64, 10_000, 10_000, 0.8, 10_000_000, md=3)
    srcs = [p.source for p in plots]
    tgts = [p.target for p in plots]
    dup = srcs[5].copy()
    dup[1::2] = dup[0::2][: len(dup[1::2])]  # every odd tree repeats its even neighbour
    srcs[5] = dup
    runs = {}
    for name, env in (("work", "1"), ("caller", "0")):
        monkeypatch.setenv("FICP_BATCH_WORK", env)
        b = FractionalICPBatch(srcs, tgts)
        runs[name] = (b.run(trace=True), b.stats, b.k_trace)
    (fw, sw, kw), (fc, sc, kc) = runs["work"], runs["caller"]
    for j in range(64):
        np.testing.assert_array_equal(kw[j], kc[j], err_msg=str(j))
        np.testing.assert_allclose(fw[j][:, :2], fc[j][:, :2], atol=1e-6, rtol=0, err_msg=str(j))
    for j in (0, 5, 31, 40, 63):  # both sub-batches
        ofinal, otr = oracle.run(srcs[j], tgts[j], nthreads=8)
        assert sw[j]["n_nn_calls"] == len(otr["k"]), j
        first = pinned_prefix(otr["gap"], otr["frmsd"], 1.0 + np.abs(srcs[j][:, :2]).max())
        assert first >= 3, (j, first)
        np.testing.assert_array_equal(kw[j][:first], otr["k"][:first], err_msg=str(j))
        assert sw[j]["k_last"] == otr["k"][-1], j
        np.testing.assert_allclose(fw[j][:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str(j))
        np.testing.assert_array_equal(bits(fw[j][:, 2]), bits(srcs[j][:, 2]))


@pytest.mark.parametrize("work", ["1", "0"])
def test_plot_sort_equals_bucket_sort(work, monkeypatch):
    """The per-plot LDS sort (k_plot_sort: the batch grid and the batch work order, one
    workgroup per plot) orders by (key, row) as the two-level bucket sort does, so whole
    batch runs are bit-identical with either (mixed plot sizes, an empty CHM layer, 2-D
    plots, duplicated stems sharing cells)."""
    from coregistrationgame_amd import FractionalICPBatch, synth
    monkeypatch.setenv("FICP_BATCH_WORK", work)
    rng = np.random.default_rng(17)
    srcs, tgts = [], []
    for p in range(70):
        n = int(rng.choice([1, 40, 900, 6000, 12000]))
        m = int(rng.choice([60, 700, 5000, 9000]))  # (grids within one plot-sort workgroup)
        pl = synth.make_plot(n, m, 0.8, seed=60_000 + p, md=3)
        s, t = pl.source, pl.target
        if p % 9 == 4:
            s, t = s[:, :2], t[:, :2]
        if p % 11 == 6 and len(t) <= 5000:
            t = np.concatenate([t, t[: len(t) // 3]])  # duplicated stems: equal keys, rows decide
        srcs.append(s)
        tgts.append(t)
    tgts[3] = tgts[3][:0]
    out = {}
    for name, env in (("plot", "1"), ("bucket", "0")):
        monkeypatch.setenv("FICP_PLOT_SORT", env)
        b = FractionalICPBatch(srcs, tgts)
        out[name] = (b.run(trace=True), b.stats, b.k_trace)
    (fp, sp, kp), (fb, sb, kb) = out["plot"], out["bucket"]
    for j in range(len(srcs)):
        np.testing.assert_array_equal(bits(fp[j]), bits(fb[j]), err_msg=str(j))
        np.testing.assert_array_equal(kp[j], kb[j], err_msg=str(j))
        assert sp[j]["n_nn_calls"] == sb[j]["n_nn_calls"], j


def test_batch_c4_properties():
    """C4 at full size (1024 plots x 10k/10k): every plot undoes its misregistration, the
    per-plot transforms reproduce the moved XY, and stage counters are consistent."""
    from coregistrationgame_amd import FractionalICPBatch, synth
    plots = synth.make_batch(1024, 10_000, 10_000, 0.8, 10_000_000, md=3)
    b = FractionalICPBatch([p.source for p in plots], [p.target for p in plots])
    finals = b.run()
    st = b.stats
    # a stage that ends by the convergence test (ficp.py:142) counts its last body as a
    # fit but not as a completed iteration
    extra = st["n_fits"] - st["iters"].sum(axis=1)
    assert np.all((extra >= 0) & (extra <= 2))
    assert np.all(st["n_nn_calls"] == st["n_fits"] + 2)
    for j in range(0, 1024, 37):
        p = plots[j]
        inl = p.inlier_of >= 0
        resid = np.linalg.norm(finals[j][inl, :2] - p.target[p.inlier_of[inl], :2], axis=1)
        assert np.median(resid) < 0.45, (j, np.median(resid))
        T = st["T_total"][j].reshape(3, 3)
        xy = p.source[:, :2] @ T[:2, :2].T + T[:2, 2]
        np.testing.assert_allclose(xy, finals[j][:, :2], atol=1e-6, rtol=0)


# ------------------------------------------------------------ partitioned CHM layer (C5)
@pytest.mark.parametrize("mode", ["target", "source"])
@pytest.mark.parametrize("shards", [1, 3, 8])
def test_partitioned_matches_single(shards, mode, oracle):
    """One plot split over shards -- the CHM layer (target mode: merged by the min /
    lowest-index rule) or the tree rows (source mode: summed integer histogram, gathered
    candidates and fit sums) -- gives the run of the unsplit plot: same NN calls and k per
    call, XY within 1e-6, vs the oracle.  Stream-ordered (ficp_dist_*): the host only
    reads the done flags."""
    from coregistrationgame_amd import FractionalICP, synth
    from coregistrationgame_amd.partitioned import PartitionedFICP
    p = synth.make_plot(20_000, 20_000, 0.8, seed=77, md=3)
    part = PartitionedFICP(p.source, p.target, local_shards=shards, mode=mode)
    out = part.run()
    icp = FractionalICP(p.source, p.target)
    single = icp.run(trace=True)
    ofinal, otr = oracle.run(p.source, p.target, nthreads=8)
    np.testing.assert_allclose(out[:, :2], single[:, :2], atol=1e-6, rtol=0)
    np.testing.assert_allclose(out[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)
    np.testing.assert_array_equal(bits(out[:, 2]), bits(p.source[:, 2]))
    np.testing.assert_array_equal(np.array(part.last_stats["k"]), otr["k"])
    assert part.lambda_val == 0.95


def test_source_mode_pack_overflow_is_exact(oracle):
    """Source mode when a rank's candidates overflow its pack (ERR_CAP in round 2): packs
    of one candidate overflow as soon as a rank holds two (flat FRMSD curves near lambda =
    1 hold many); the run restarts with full packs and gives the unsplit run (k per call,
    XY within 1e-6) and the oracle's."""
    from coregistrationgame_amd import FractionalICP, synth
    from coregistrationgame_amd.partitioned import PartitionedFICP
    p = synth.make_plot(30_000, 30_000, 0.6, seed=91, md=3)
    restarts = 0
    for lam in (3.0, 0.95, 1.3):
        part = PartitionedFICP(p.source, p.target, lambda_val=lam, local_shards=8, mode="source")
        part.CAPD, part.CAPD_FRAC = 1, 1 << 30  # packs of one candidate
        out = part.run()
        restarts += getattr(part, "n_cap_restarts", 0)
        icp = FractionalICP(p.source, p.target, lambda_val=lam)
        single = icp.run(trace=True)
        np.testing.assert_allclose(out[:, :2], single[:, :2], atol=1e-6, rtol=0)
        np.testing.assert_array_equal(np.array(part.last_stats["k"]), icp.last_stats["k"])
        ofinal, otr = oracle.run(p.source, p.target, lam0=lam, nthreads=8)
        np.testing.assert_allclose(out[:, :2], ofinal[:, :2], atol=1e-6, rtol=0)
    assert restarts >= 2, restarts


@pytest.mark.parametrize("mode", ["target", "source"])
def test_partitioned_2d_and_tiny_shards(mode):
    """2-D layers and more shards than stems (target: empty shards) or a few rows per
    shard (source) still give the single run."""
    from coregistrationgame_amd import FractionalICP
    from coregistrationgame_amd.partitioned import PartitionedFICP
    rng = np.random.default_rng(3)
    tgt = rng.uniform(0, 30, (6, 2))
    src = tgt[rng.integers(0, 6, 40)] + rng.normal(0, 0.2, (40, 2))
    out = PartitionedFICP(src, tgt, local_shards=9, mode=mode).run()
    single = FractionalICP(src, tgt).run()
    np.testing.assert_allclose(out, single, atol=1e-6, rtol=0)


@pytest.mark.parametrize("sizes", [(20_000, 17_000), (14_000, 10_500), (10_000, 9_000)],
                         ids=["uncached", "cached32", "cached20"])
def test_batch_large_and_degenerate_plots(oracle, sizes):
    """The selection kernel's three forms, picked by the batch's largest plot: above its
    register-cached size (> 16384 trees: every pass re-reads the rows), 32 cached rows per
    thread (<= 16384) and 20 (<= 10240, C4's plots); with a plot whose trees sit exactly on
    stems (all distances 0: one bucket holds the whole plot) and one with many exactly
    equal distances (a lattice shifted by a fixed offset), vs the oracle run of each plot
    alone."""
    from coregistrationgame_amd import FractionalICPBatch, synth
    srcs, tgts = [], []
    for n, seed in zip(sizes, (501, 502)):
        pl = synth.make_plot(n, n, 0.7, seed=seed, md=3)
        srcs.append(pl.source)
        tgts.append(pl.target)
    rng = np.random.default_rng(5)
    t = np.c_[rng.uniform(0, 200, (3000, 2)), rng.uniform(5, 30, 3000)]
    srcs.append(t[:2000].copy())          # exact: every distance 0
    tgts.append(t)
    gx, gy = np.meshgrid(np.arange(60) * 3.0, np.arange(60) * 3.0)
    lat = np.c_[gx.ravel(), gy.ravel(), np.full(gx.size, 20.0)]
    s = lat.copy()
    s[:, :2] += [0.5, 0.25]               # equal distances everywhere
    s[::7, :2] += rng.normal(0, 0.3, (len(s[::7]), 2))
    srcs.append(s)
    tgts.append(lat)
    b = FractionalICPBatch(srcs, tgts)
    finals = b.run()
    for p in range(len(srcs)):
        ofinal, otr = oracle.run(srcs[p], tgts[p], nthreads=8)
        np.testing.assert_allclose(finals[p][:, :2], ofinal[:, :2], atol=1e-6, rtol=0, err_msg=str(p))
        np.testing.assert_array_equal(bits(finals[p][:, 2:]), bits(srcs[p][:, 2:]))
        assert b.stats[p]["n_nn_calls"] == len(otr["k"]), p
        assert b.stats[p]["k_last"] == otr["k"][-1], p
