"""Sticky device error paths and the pooled host path.

* ERR_SPIN: the test-only fault injection (ficp_set_fault) makes the in-launch hand-off
  publish a wrong token (block 0 of k_sel_bounds_gather), so every waiting workgroup's
  bounded wait runs out.  The run must end (no hang), append nothing out of bounds, and raise FicpError
  naming the flag; the same context must run clean afterwards (the flag is per run).
* The facade borrows pooled contexts: a second FractionalICP reuses the first one's
  context, and results do not depend on which pooled context ran them.
"""
import time

import numpy as np
import pytest

from coregistrationgame_amd import _lib, synth
from coregistrationgame_amd.ficp import FractionalICP

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [3000, 120_000])  # below / above the half-step lookahead (64k rows)
def test_err_spin_reaches_python(n, oracle):
    p = synth.make_plot(n, n, 0.8, seed=77, md=3)
    ctx = _lib.Context(0, _lib.NN_GRID)
    try:
        ctx.set_target(p.target, 3)
        ctx.set_fault(1)
        src = np.array(p.source)
        t0 = time.perf_counter()
        with pytest.raises(_lib.FicpError, match="ERR_SPIN"):
            ctx.run(src, [3.0, 0.95], 1e-6, 1000, False)
        assert time.perf_counter() - t0 < 60.0
        # the flag is per run: the same context, fault off, gives the oracle's answer
        ctx.set_fault(0)
        src = np.array(p.source)
        st = ctx.run(src, [3.0, 0.95], 1e-6, 1000, False)
        ref, tr = oracle.run(p.source, p.target)
        assert st["n_nn_calls"] == tr["n_calls"]
        assert float(np.max(np.abs(src[:, :2] - ref[:, :2]))) < 1e-6
    finally:
        ctx.close()


def test_pool_reuses_contexts_and_matches_fresh():
    _lib.drain_pool()
    p = synth.make_plot(20_000, 20_000, 0.8, seed=78, md=3)
    a = FractionalICP(p.source, p.target, device=0).run()
    assert _lib.pool_size() == 1  # the borrowed context came back
    b = FractionalICP(p.source, p.target, device=0).run()
    assert _lib.pool_size() == 1  # ... and was reused, not a second one made
    np.testing.assert_array_equal(a, b)
    # a smaller plot on the same (larger) pooled buffers, then the big one again
    q = synth.make_plot(3000, 2500, 0.6, seed=79, md=2)
    fresh = _lib.Context(0)
    try:
        fresh.set_target(q.target, 2)
        s1 = np.array(q.source)
        fresh.run(s1, [3.0, 1.3], 1e-6, 1000, False)
    finally:
        fresh.close()
    s2 = FractionalICP(q.source, q.target, device=0).run()
    np.testing.assert_array_equal(s1, s2)
    c = FractionalICP(p.source, p.target, device=0).run()
    np.testing.assert_array_equal(a, c)
    assert np.array_equal(c[:, 2], p.source[:, 2])


def test_host_ms_tiles_the_call():
    p = synth.make_plot(200_000, 200_000, 0.6, seed=80, md=3)
    FractionalICP(p.source, p.target, device=0).run()  # pool warm-up
    t0 = time.perf_counter()
    icp = FractionalICP(p.source, p.target, device=0)
    icp.run()
    total = 1e3 * (time.perf_counter() - t0)
    h = icp.last_stats["host_ms"]
    tiled = sum(h.values())
    assert tiled <= total * 1.001 + 0.05
    assert tiled >= 0.8 * total, (h, total)
    lib = icp.last_stats["lib_host_ms"]
    assert lib["upload"] + lib["loop"] + lib["result"] <= h["run"] * 1.001 + 0.05
    assert icp.last_stats["gpu_ms"] <= lib["loop"] * 1.001 + 0.05


def test_pooled_host_arrays_are_private_copies():
    """The facade's layer copies live in pooled pinned blocks (_lib.copy_array): each is a
    private copy (ficp.py:34-35 np.array semantics), a block is not recycled while any view
    of it is alive, and the run's result is the same as from plain numpy memory."""
    p = synth.make_plot(60_000, 60_000, 0.7, seed=5, md=3)  # 1.4 MB per layer: pooled
    src_in = np.array(p.source)
    icp = FractionalICP(src_in, p.target, device=0)
    assert _lib.is_pooled(icp.source) and _lib.is_pooled(icp.target)
    src_in[:, 0] += 1000.0  # the caller's later writes do not reach the instance
    assert np.array_equal(icp.source, p.source)
    out = icp.run()
    assert _lib.is_pooled(out)
    keep = out[:, :2]  # a view: its block stays out of the pool
    kept = keep.copy()
    del icp, out
    for _ in range(3):  # new instances take other blocks, never the viewed one
        FractionalICP(p.source, p.target, device=0).run()
    assert np.array_equal(keep, kept)
    # same answer as an instance whose layers are plain (small-path threshold aside)
    ctx = _lib.Context(0, _lib.NN_AUTO)
    try:
        ctx.set_target(np.array(p.target), 3)
        ref = np.array(p.source)
        ctx.run(ref, [3.0, 0.95], 1e-6, 1000, False)
    finally:
        ctx.close()
    assert np.array_equal(kept, ref[:, :2])
