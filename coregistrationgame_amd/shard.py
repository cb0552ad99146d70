"""Multi-GPU batch: independent plots dealt over ranks, one process per GPU.

SURVEY.md §8(e): a batch of plots (C4) shards with no exchange on the data path. Each
rank runs `ficp_run_batch` on its own plots. The per-plot result records (104 B each)
are gathered once at the end with one all-gather, over RCCL on GPUs or gloo on CPU.

Balance: plots are sorted by their NN work (N·M) in decreasing order and dealt in a
serpentine (0..R-1, R-1..0, ...). The deal depends only on the plot sizes, so every rank
computes the same deal without communicating.
"""
from __future__ import annotations

import numpy as np

from . import _lib

_WORDS = _lib.PLOT_STATS_DTYPE.itemsize // 8  # 13 int64 words per record


def deal_plots(work, world_size: int) -> list[np.ndarray]:
    """Plot ids of every rank; the ids of each rank are in ascending order."""
    work = np.asarray(work, dtype=np.float64)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    order = np.argsort(-work, kind="stable")
    lanes = np.arange(len(order)) % (2 * world_size)
    rank_of = np.where(lanes < world_size, lanes, 2 * world_size - 1 - lanes)
    owner = np.empty(len(order), np.int64)
    owner[order] = rank_of
    return [np.flatnonzero(owner == r) for r in range(world_size)]


def gather_plot_stats(deal: list[np.ndarray], local_stats: np.ndarray, rank: int, group=None,
                      device=None) -> np.ndarray:
    """All-gather of per-plot records into one array in plot order (same on every rank).

    ``local_stats`` holds the records of ``deal[rank]`` in that order. ``device`` is
    the torch device of the collective ("cuda:<local>" for RCCL, None/"cpu" for gloo).
    """
    import torch
    import torch.distributed as dist

    world = len(deal)
    nplots = int(sum(len(d) for d in deal))
    if len(local_stats) != len(deal[rank]):
        raise ValueError("local_stats must hold one record per plot of this rank")
    width = max(len(d) for d in deal)
    buf = np.zeros((width, _WORDS), np.int64)
    if len(local_stats):
        buf[:len(local_stats)] = np.ascontiguousarray(local_stats).view(np.int64).reshape(-1, _WORDS)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    mine = torch.from_numpy(buf).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    out = np.zeros(nplots, _lib.PLOT_STATS_DTYPE)
    for r in range(world):
        rows = parts[r].cpu().numpy()[:len(deal[r])]
        out[deal[r]] = np.ascontiguousarray(rows).view(_lib.PLOT_STATS_DTYPE).reshape(-1)
    return out
