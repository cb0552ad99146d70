"""CPU tests of the partitioned-CHM-layer host logic: shard ranges and
the two-collective merge of per-shard nearest neighbours -- the minimum squared distance,
the lowest global index among equal distances (the single-GPU tie rule, ficp_nn), empty
shards and NaN queries -- in-process and over gloo with world_size 2."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from coregistrationgame_amd.partitioned import INT32_MAX, merge_local, merge_shards, shard_bounds


@pytest.mark.parametrize("m,world", [(0, 1), (5, 8), (1_000_000, 8), (17, 3), (8, 8)])
def test_shard_bounds(m, world):
    b = shard_bounds(m, world)
    assert len(b) == world
    assert b[0][0] == 0
    for (o0, c0), (o1, _) in zip(b, b[1:]):
        assert o1 == o0 + c0
    assert sum(c for _, c in b) == m
    assert max(c for _, c in b) - min(c for _, c in b) <= 1


def _case(n, shards, seed):
    """Per-shard (d2, global idx) with cross-shard exact ties, an empty shard and a NaN query."""
    rng = np.random.default_rng(seed)
    sizes = [int(s) for s in rng.integers(0, 50, shards)]
    sizes[1] = 0
    offs = np.concatenate([[0], np.cumsum(sizes)])[:-1]
    d2s, idxs = [], []
    for s in range(shards):
        if sizes[s] == 0:
            d2s.append(np.full(n, np.inf))
            idxs.append(np.full(n, INT32_MAX, np.int32))
            continue
        d = rng.integers(1, 6, n).astype(float)  # small integers: many exact ties
        d2s.append(d)
        idxs.append((offs[s] + rng.integers(0, sizes[s], n)).astype(np.int32))
    for d in d2s:
        d[0] = np.nan  # query 0 is NaN on every shard
    D = np.stack(d2s)
    I = np.stack(idxs)
    dmin = np.min(D, axis=0)
    exp_i = np.where(D == dmin, I, INT32_MAX).min(axis=0)
    exp_i[0] = I[:, 0].min()
    return d2s, idxs, dmin, exp_i


def test_merge_local_rule():
    d2s, idxs, dmin, exp_i = _case(500, 5, 1)
    dm, im = merge_local([torch.from_numpy(d) for d in d2s], [torch.from_numpy(i) for i in idxs])
    np.testing.assert_array_equal(dm.numpy()[1:], dmin[1:])
    assert np.isnan(dm.numpy()[0])
    np.testing.assert_array_equal(im.numpy(), exp_i)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _merge_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d2s, idxs, _, _ = _case(300, 2 * world, 7)
        # this rank holds shards 2r and 2r+1: merge locally, then across ranks
        dl, il = merge_local([torch.from_numpy(d2s[2 * rank + j]) for j in range(2)],
                             [torch.from_numpy(idxs[2 * rank + j]) for j in range(2)])
        dm, im = merge_shards(dl, il)
        q.put((rank, dm.numpy().tobytes(), im.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def test_merge_shards_gloo():
    world = 2
    _, _, dmin, exp_i = _case(300, 2 * world, 7)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (d, i)) for r, d, i in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        dm = np.frombuffer(got[r][0], np.float64)
        im = np.frombuffer(got[r][1], np.int32)
        np.testing.assert_array_equal(dm[1:], dmin[1:])
        np.testing.assert_array_equal(im, exp_i)


# ------------------------------------------------ source-partitioned exchanges (mode "source")
def _src_case(ranks, seed):
    """Per-rank exchange records: key range words (int64, flipped top bit), integer
    histogram totals, 8 fit sums and a candidate pack."""
    rng = np.random.default_rng(seed)
    ranges = [rng.integers(-2**62, 2**62, 2) for _ in range(ranks)]
    hists = [rng.integers(0, 2**40, 16) for _ in range(ranks)]
    sums = [rng.normal(0, 1e3, 8) for _ in range(ranks)]
    packs = [rng.integers(-2**60, 2**60, 10) for _ in range(ranks)]
    return ranges, hists, sums, packs


def test_source_merges_local():
    from coregistrationgame_amd.partitioned import gather_ranked, merge_hist, merge_range
    ranges, hists, sums, packs = _src_case(5, 3)
    T = torch.from_numpy
    np.testing.assert_array_equal(merge_range([T(r) for r in ranges]).numpy(), np.max(ranges, axis=0))
    np.testing.assert_array_equal(merge_hist([T(h) for h in hists]).numpy(), np.sum(hists, axis=0))
    np.testing.assert_array_equal(gather_ranked([T(s) for s in sums]).numpy(), np.stack(sums))
    np.testing.assert_array_equal(gather_ranked([T(p) for p in packs]).numpy(), np.stack(packs))


def _source_worker(rank, world, port, q):
    import torch.distributed as dist
    from coregistrationgame_amd.partitioned import gather_ranked, merge_hist, merge_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ranges, hists, sums, packs = _src_case(2 * world, 11)
        mine = slice(2 * rank, 2 * rank + 2)  # this process holds ranks 2r and 2r+1
        T = torch.from_numpy
        r = merge_range([T(x) for x in ranges[mine]], world=world)
        h = merge_hist([T(x) for x in hists[mine]], world=world)
        s = gather_ranked([T(x) for x in sums[mine]], world=world)
        p = gather_ranked([T(x) for x in packs[mine]], world=world)
        q.put((rank, r.numpy().tobytes(), h.numpy().tobytes(), s.numpy().tobytes(), p.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def test_source_merges_gloo():
    """The source mode's exchanges over gloo, world size 2 with two ranks per process: the
    range MAX, the exact integer histogram SUM, and the rank-ordered gathers of the fit
    sums and candidate packs are identical on every process."""
    world = 2
    ranges, hists, sums, packs = _src_case(2 * world, 11)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_source_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {g[0]: g[1:] for g in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        rb, hb, sb, pb = got[r]
        np.testing.assert_array_equal(np.frombuffer(rb, np.int64), np.max(ranges, axis=0))
        np.testing.assert_array_equal(np.frombuffer(hb, np.int64), np.sum(hists, axis=0))
        np.testing.assert_array_equal(np.frombuffer(sb, np.float64).reshape(-1, 8), np.stack(sums))
        np.testing.assert_array_equal(np.frombuffer(pb, np.int64).reshape(-1, 10), np.stack(packs))
