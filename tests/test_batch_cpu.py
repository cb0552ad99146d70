"""CPU tests of the multi-plot host logic: the balanced deal of plots over ranks, the
end-of-run all-gather of per-plot records (gloo, world_size 2), the record layout and
the batch facade's argument contract (ficp.py:37-38 per plot)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def test_plot_stats_layout():
    from coregistrationgame_amd import _lib
    d = _lib.PLOT_STATS_DTYPE
    assert d.itemsize == 104
    assert [d.fields[k][1] for k in ("T_total", "frmsd_last", "k_last", "n_nn_calls", "n_fits", "iters")] == \
        [0, 72, 80, 88, 92, 96]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_deal_covers_and_balances(world):
    from coregistrationgame_amd import shard
    rng = np.random.default_rng(world)
    work = rng.integers(1, 10_000, 1024).astype(float) ** 2
    deal = shard.deal_plots(work, world)
    allp = np.sort(np.concatenate(deal))
    np.testing.assert_array_equal(allp, np.arange(1024))
    sizes = [len(d) for d in deal]
    assert max(sizes) - min(sizes) <= 1
    loads = np.array([work[d].sum() for d in deal])
    assert loads.max() <= loads.mean() * 1.05 + work.max()
    for d in deal:
        assert np.all(np.diff(d) > 0)


def test_deal_equal_plots_round_robin():
    from coregistrationgame_amd import shard
    deal = shard.deal_plots(np.ones(1024), 8)
    assert all(len(d) == 128 for d in deal)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gather_worker(rank, world, port, nplots, q):
    import torch.distributed as dist
    from coregistrationgame_amd import _lib, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        deal = shard.deal_plots(np.arange(nplots, dtype=float) % 7 + 1, world)
        mine = deal[rank]
        rec = np.zeros(len(mine), _lib.PLOT_STATS_DTYPE)
        rec["k_last"] = mine * 10
        rec["n_nn_calls"] = mine + 2
        rec["T_total"] = np.eye(3).ravel()
        rec["T_total"][:, 2] = mine + 0.5
        rec["frmsd_last"] = mine * 0.25
        out = shard.gather_plot_stats(deal, rec, rank)
        q.put((rank, out.tobytes()))
    finally:
        dist.destroy_process_group()


def test_gather_plot_stats_gloo():
    from coregistrationgame_amd import _lib
    world, nplots = 2, 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, nplots, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs = [np.frombuffer(got[r], _lib.PLOT_STATS_DTYPE) for r in range(world)]
    assert outs[0].tobytes() == outs[1].tobytes()
    o = outs[0]
    ids = np.arange(nplots)
    np.testing.assert_array_equal(o["k_last"], ids * 10)
    np.testing.assert_array_equal(o["n_nn_calls"], ids + 2)
    np.testing.assert_array_equal(o["T_total"][:, 2], ids + 0.5)
    np.testing.assert_array_equal(o["frmsd_last"], ids * 0.25)


def test_batch_facade_contract():
    from coregistrationgame_amd import FractionalICPBatch
    with pytest.raises(ValueError, match=r"source and target must be 2D arrays \(N, D\)\."):
        FractionalICPBatch([np.zeros(3)], [np.zeros((3, 3))])
    with pytest.raises(ValueError):
        FractionalICPBatch([np.zeros((3, 3))], [])
    b = FractionalICPBatch([np.zeros((4, 3)), np.zeros((4, 2)), np.zeros((0, 3))],
                           [np.zeros((5, 3)), np.zeros((5, 3)), np.zeros((5, 3))])
    assert b.match_dims == [3, 2, 3]


def test_batch_facade_all_empty_needs_no_gpu():
    """Plots with an empty layer never reach the device: nothing moves (ficp.py:125-126)."""
    from coregistrationgame_amd import FractionalICPBatch
    s = np.arange(12.0).reshape(4, 3)
    b = FractionalICPBatch([s, np.zeros((0, 3))], [np.zeros((0, 3)), s])
    out = b.run()
    np.testing.assert_array_equal(out[0], s)
    assert out[1].shape == (0, 3)
    assert np.all(b.stats["n_nn_calls"] == 0)
    np.testing.assert_array_equal(b.stats["T_total"][0], np.eye(3).ravel())


def test_run_batch_rejects_bad_arguments_without_gpu():
    """The C ABI validates before it touches a device: a null context is EINVAL."""
    from coregistrationgame_amd import _lib
    L = _lib.lib()
    so = np.array([0, 2], np.int64)
    src = np.zeros((2, 3))
    lam = np.array([3.0, 0.95])
    rc = L.ficp_run_batch(None, 1, so.ctypes.data_as(C.POINTER(C.c_int64)), src.ctypes.data_as(C.POINTER(C.c_double)),
                          3, so.ctypes.data_as(C.POINTER(C.c_int64)), src.ctypes.data_as(C.POINTER(C.c_double)), 3,
                          3, 2, lam.ctypes.data_as(C.POINTER(C.c_double)), 1e-6, 1000, 0, None)
    assert rc == _lib.FICP_EINVAL
    assert b"null context" in L.ficp_last_error()
