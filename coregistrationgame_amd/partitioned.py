"""Fractional ICP against a CHM layer partitioned across GPUs.

One process per GPU. The CHM layer (target) is split into contiguous row ranges, one
shard per rank, so a stem's global index is its shard offset plus its shard index. The
tree layer (source) is replicated. Every NN call of the reference's `_iterate`
(ficp.py:122-147) becomes:

1. `ficp_nn_device` on every rank, against its own shard only;
2. the one exchange of the path: an all-reduce MIN of the squared distances, then an
   all-reduce MIN of the indices where a rank's distance equals the merged one. The
   lowest global index wins a tie, which is the single-GPU rule (`ficp_nn`). Both
   collectives run over RCCL (torch.distributed "nccl" backend);
3. `ficp_select_fit_device` on every rank with identical inputs, so every rank derives
   the same k, FRMSD and transform (find_optimal_fraction + compute_optimal_transform_2d);
4. `ficp_apply_device` on the replicated source.

With one process, `local_shards` splits the layer inside the process and merges with
the same rule. This is the single-GPU rehearsal of the multi-GPU path.

PyTorch only provides device buffers and the collectives; all arithmetic runs in
libficp.so. There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib

INT32_MAX = 2**31 - 1


def shard_bounds(m: int, world: int) -> list[tuple[int, int]]:
    """Contiguous (offset, count) row ranges of an m-row layer over `world` shards."""
    if world < 1:
        raise ValueError("world must be >= 1")
    base, extra = divmod(int(m), world)
    out, off = [], 0
    for r in range(world):
        cnt = base + (1 if r < extra else 0)
        out.append((off, cnt))
        off += cnt
    return out


def _offer(d2, dmin, idx):
    import torch
    # a NaN query has no nearest stem on any shard: every shard offers its index
    return torch.where((d2 == dmin) | torch.isnan(dmin), idx, torch.full_like(idx, INT32_MAX))


def merge_shards(d2, idx, group=None):
    """All-reduce merge of per-rank (d2, global idx): min d2, then lowest idx among ties."""
    import torch.distributed as dist
    dmin = d2.clone()
    dist.all_reduce(dmin, op=dist.ReduceOp.MIN, group=group)
    cand = _offer(d2, dmin, idx)
    dist.all_reduce(cand, op=dist.ReduceOp.MIN, group=group)
    return dmin, cand


def merge_local(d2s, idxs):
    """The same merge for shards held by one process."""
    import torch
    dmin = d2s[0].clone()
    for d in d2s[1:]:
        dmin = torch.minimum(dmin, d)  # propagates NaN like the MIN collective's inputs
    cand = _offer(d2s[0], dmin, idxs[0])
    for d, i in zip(d2s[1:], idxs[1:]):
        cand = torch.minimum(cand, _offer(d, dmin, i))
    return dmin, cand


class PartitionedFICP:
    def __init__(self, source, target, lambda_val=3.0, threshold=1e-6, max_iterations=1000,
                 allow_reflection=False, *, group=None, device=None, local_shards=1):
        self.source = np.array(source, dtype=float)
        self.target = np.array(target, dtype=float)
        if self.source.ndim != 2 or self.target.ndim != 2:  # ficp.py:37-38
            raise ValueError("source and target must be 2D arrays (N, D).")
        self.match_dims = 3 if (self.source.shape[1] >= 3 and self.target.shape[1] >= 3) else 2
        self.lambda_val = lambda_val
        self.threshold = threshold
        self.max_iterations = max_iterations
        self.allow_reflection = allow_reflection
        self.group = group
        self.device = device
        self.local_shards = int(local_shards)
        self.last_stats = None

    def _topology(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(self.group), dist.get_world_size(self.group)
        return 0, 1

    def _setup(self):
        """Resident device state: layers, shard contexts (grids built on first use), merge
        buffers.  Reused by every run of this object."""
        if getattr(self, "_res", None) is not None:
            return self._res
        import torch
        n, m, md = len(self.source), len(self.target), self.match_dims
        rank, world = self._topology()
        dev_id = _lib.default_device() if self.device is None else int(self.device)
        dev = torch.device("cuda", dev_id)
        torch.cuda.set_device(dev)
        shards = shard_bounds(m, world * self.local_shards)
        mine = shards[rank * self.local_shards:(rank + 1) * self.local_shards]
        tgt = [torch.as_tensor(np.ascontiguousarray(self.target[:, j]), device=dev) for j in range(md)]
        src0 = [torch.as_tensor(np.ascontiguousarray(self.source[:, j]), device=dev) for j in range(md)]
        ctxs = []
        for off, cnt in mine:
            c = _lib.Context(dev_id)
            c.set_target_device(tgt[0].data_ptr() + 8 * off, tgt[1].data_ptr() + 8 * off,
                                tgt[2].data_ptr() + 8 * off if md == 3 else 0, cnt, md)
            ctxs.append(c)
        x0, x1 = self.target[:, 0].min(), self.target[:, 0].max()
        y0, y1 = self.target[:, 1].min(), self.target[:, 1].max()
        self._res = dict(
            dev=dev, world=world, mine=mine, tgt=tgt, src0=src0, src=[t.clone() for t in src0],
            ctxs=ctxs, d2s=[torch.empty(n, dtype=torch.float64, device=dev) for _ in mine],
            idxs=[torch.empty(n, dtype=torch.int32, device=dev) for _ in mine],
            pivot=(x0 + 0.5 * (x1 - x0), y0 + 0.5 * (y1 - y0)))  # the single-GPU pivot
        return self._res

    def close(self):
        res = getattr(self, "_res", None)
        if res is not None:
            for c in res["ctxs"]:
                c.close()
            self._res = None

    def run(self):
        """Both stages of ficp.py:149-154 over the partitioned layer; returns the source."""
        n, m = len(self.source), len(self.target)
        lam2 = 0.95 if self.match_dims == 3 else 1.3
        if n == 0 or m == 0:  # ficp.py:66-68, 125-126: nothing moves
            self.lambda_val = lam2
            self.last_stats = dict(k=[], frmsd=[], lam=[], T=[], n_nn_calls=0, n_fits=0, iters=[0, 0])
            return self.source
        res = self._setup()
        self.run_resident()
        out = self.source.copy()
        out[:, 0] = res["src"][0].cpu().numpy()
        out[:, 1] = res["src"][1].cpu().numpy()
        self.close()
        self.source = out
        return self.source

    def run_resident(self, lambda0=None):
        """One run from the pristine resident source; the result stays on the device."""
        import torch
        res = self._setup()
        n, md = len(self.source), self.match_dims
        dev, world, mine, ctxs = res["dev"], res["world"], res["mine"], res["ctxs"]
        src, tgt, d2s, idxs = res["src"], res["tgt"], res["d2s"], res["idxs"]
        for a, b in zip(src, res["src0"]):
            a.copy_(b)
        lam1 = self.lambda_val if lambda0 is None else lambda0
        lam2 = 0.95 if md == 3 else 1.3
        stats = dict(k=[], frmsd=[], lam=[], T=[], n_nn_calls=0, n_fits=0, iters=[0, 0])
        zp = src[2].data_ptr() if md == 3 else 0

        def nn_select(lam):
            torch.cuda.current_stream(dev).synchronize()
            for c, (off, _), d2, ix in zip(ctxs, mine, d2s, idxs):
                c.nn_device(src[0].data_ptr(), src[1].data_ptr(), zp, n, off, d2.data_ptr(), ix.data_ptr())
            dmin, imin = merge_local(d2s, idxs) if len(ctxs) > 1 else (d2s[0], idxs[0])
            if world > 1:
                dmin, imin = merge_shards(dmin, imin, self.group)
            torch.cuda.current_stream(dev).synchronize()
            k, f, T = ctxs[0].select_fit_device(src[0].data_ptr(), src[1].data_ptr(), n, dmin.data_ptr(),
                                                imin.data_ptr(), tgt[0].data_ptr(), tgt[1].data_ptr(), n,
                                                lam, self.allow_reflection, res["pivot"])
            stats["n_nn_calls"] += 1
            stats["k"].append(k)
            stats["frmsd"].append(f)
            stats["lam"].append(lam)
            return k, f, T

        for s, lam in enumerate((lam1, lam2)):
            k, cur, T = nn_select(lam)  # ficp.py:123-129
            if k == 0:
                continue
            it = 0
            while it < self.max_iterations:  # ficp.py:132-145
                ctxs[0].apply_device(src[0].data_ptr(), src[1].data_ptr(), n, T)
                stats["T"].append(T)
                stats["n_fits"] += 1
                k, new, T = nn_select(lam)
                if cur - new <= self.threshold:
                    break
                cur = new
                it += 1
            stats["iters"][s] = it
        self.lambda_val = lam2  # ficp.py:152
        torch.cuda.current_stream(dev).synchronize()
        self.last_stats = stats
        return stats
