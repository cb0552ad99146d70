"""One large plot over several GPUs, in two modes.

One process per GPU.  Each NN call of the reference's `_iterate` (ficp.py:122-147) is a
fixed sequence of libficp steps (include/ficp.h ficp_dist_*) and collectives, all
enqueued on the torch stream the contexts run on (`ficp_set_stream`): nothing waits for
the host except one done flag per iteration, read one iteration behind.

* mode "target" (the CHM layer split into contiguous row shards, one per rank; the tree
  rows replicated): every rank runs the NN of all rows against its shard
  (`ficp_dist_nn_shard`), then the one exchange of this mode -- an all-reduce MIN of the
  squared distances, then an all-reduce MIN of the indices where a rank's distance equals
  the merged one (the lowest global index wins a tie: the single-GPU rule, `ficp_nn`) --
  and the same selection, loop step, fit and apply on every rank.  Exchange per NN call:
  12 B per tree.
* mode "source" (the tree rows split into contiguous ranges; the layer replicated): every
  rank runs the NN, histogram and candidate gather of its own rows against the whole
  layer; the exchanges are a MAX all-reduce of the key range (16 B), a SUM all-reduce of
  the selection histogram's exact integer totals (128 KB), an all-gather of the ranks'
  candidates (a few hundred rows) and an all-gather of the 8 fit sums.  Every rank then
  derives the same k, threshold and transform.  Exchange per NN call: ~130 KB whatever
  the plot size.

The collectives run over RCCL (torch.distributed "nccl").  With one process,
`local_shards` splits the layer (target) or the rows (source) inside the process and
merges with the same rules: the single-GPU rehearsal of the multi-GPU path.  PyTorch only
provides device buffers, the stream and the collectives; all arithmetic runs in
libficp.so.  There is no CPU fallback.
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


def merge_range(parts, group=None, world=1):
    """Source mode: the key range words of the local ranks' rows (int64[2] each, top bit
    flipped: signed order = unsigned order), MAX over them and over the process group."""
    import torch
    r = parts[0].clone()
    for p in parts[1:]:
        r = torch.maximum(r, p)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(r, op=dist.ReduceOp.MAX, group=group)
    return r


def merge_hist(parts, group=None, world=1):
    """Source mode: the ranks' integer histogram totals (int64), summed: exact and
    independent of the order."""
    import torch
    h = parts[0].clone()
    for p in parts[1:]:
        h = h + p
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    return h


def gather_ranked(parts, group=None, world=1):
    """Source mode: every rank's record (fit sums, candidate pack), stacked in rank order
    (process rank, then local rank) on every process."""
    import torch
    mine = torch.stack(parts)
    if world <= 1:
        return mine.contiguous()
    import torch.distributed as dist
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return torch.cat(out).contiguous()


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
    # source mode: candidates one rank may contribute per NN call: at least CAPD, and 1/64
    # of the rank's largest row range (a stage's first call, on the uniform bucket map, can
    # leave ~1e-3 of the rows as candidates: 8M rows on one rank overflowed 8192).  A call
    # whose candidates exceed that on any rank (flat FRMSD curves near lambda = 1, tied
    # distances) is not an error: every rank sees the same merged overflow bit, the device
    # loop stops at that call on every rank, and the run starts over with packs that hold
    # every row of a rank (capd = the largest row range), where the final selection's
    # refinement levels / chunked scan take any candidate count (exact, as one GPU).
    CAPD = 8192
    CAPD_FRAC = 64

    def __init__(self, source, target, lambda_val=3.0, threshold=1e-6, max_iterations=1000,
                 allow_reflection=False, *, mode="target", group=None, device=None, local_shards=1):
        self.source = np.array(source, dtype=float)
        self.target = np.array(target, dtype=float)
        if self.source.ndim != 2 or self.target.ndim != 2:  # ficp.py:37-38
            raise ValueError("source and target must be 2D arrays (N, D).")
        if mode not in ("target", "source"):
            raise ValueError("mode must be 'target' or 'source'")
        self.match_dims = 3 if (self.source.shape[1] >= 3 and self.target.shape[1] >= 3) else 2
        self.lambda_val = lambda_val
        self.threshold = threshold
        self.max_iterations = max_iterations
        self.allow_reflection = allow_reflection
        self.mode = mode
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
        """Resident device state: layers, contexts on the torch stream (grids built once),
        exchange buffers.  Reused by every run of this object."""
        if getattr(self, "_res", None) is not None:
            return self._res
        import torch
        n, m, md = len(self.source), len(self.target), self.match_dims
        rank, world = self._topology()
        dev_id = _lib.default_device() if self.device is None else int(self.device)
        dev = torch.device("cuda", dev_id)
        torch.cuda.set_device(dev)
        # one torch stream for the library steps and the collectives (the default stream
        # has handle 0, which ficp_set_stream reads as "the context's own stream")
        self._stream = torch.cuda.Stream(dev)
        self._stream.wait_stream(torch.cuda.current_stream(dev))
        stream = self._stream.cuda_stream
        ls = self.local_shards
        parts = shard_bounds(m if self.mode == "target" else n, world * ls)
        mine = parts[rank * ls:(rank + 1) * ls]
        tgt = [torch.as_tensor(np.ascontiguousarray(self.target[:, j]), device=dev) for j in range(md)]
        src0 = [torch.as_tensor(np.ascontiguousarray(self.source[:, j]), device=dev) for j in range(md)]
        ctxs = []
        for off, cnt in mine:
            c = _lib.Context(dev_id)
            c.set_stream(stream)
            if self.mode == "target":  # this shard of the layer
                c.set_target_device(tgt[0].data_ptr() + 8 * off, tgt[1].data_ptr() + 8 * off,
                                    tgt[2].data_ptr() + 8 * off if md == 3 else 0, cnt, md)
            else:  # the whole layer
                c.set_target_device(tgt[0].data_ptr(), tgt[1].data_ptr(), tgt[2].data_ptr() if md == 3 else 0,
                                    m, md)
            ctxs.append(c)
        x0, x1 = self.target[:, 0].min(), self.target[:, 0].max()
        y0, y1 = self.target[:, 1].min(), self.target[:, 1].max()
        W = world * ls
        res = dict(dev=dev, world=world, W=W, mine=mine, parts=parts, tgt=tgt, src0=src0,
                   src=[t.clone() for t in src0], ctxs=ctxs,
                   pivot=(x0 + 0.5 * (x1 - x0), y0 + 0.5 * (y1 - y0)))  # the single-GPU pivot
        i64, f64 = torch.int64, torch.float64
        if self.mode == "target":
            res.update(d2s=[torch.empty(n, dtype=f64, device=dev) for _ in mine],
                       idxs=[torch.empty(n, dtype=torch.int32, device=dev) for _ in mine],
                       sums=torch.zeros(8, dtype=f64, device=dev))
        else:
            hw = _lib.dist_hist_words()
            n_max = max(c for _, c in parts)
            self.capd = min(n_max, max(self.CAPD, -(-n_max // self.CAPD_FRAC)))
            res.update(sums=[torch.zeros(8, dtype=f64, device=dev) for _ in mine],
                       range2=[torch.zeros(2, dtype=i64, device=dev) for _ in mine],
                       hist=[torch.zeros(hw, dtype=i64, device=dev) for _ in mine],
                       pack=[torch.zeros(4 + 3 * self.capd, dtype=i64, device=dev) for _ in mine],
                       n_max=n_max)
        self._res = res
        return res

    def close(self):
        res = getattr(self, "_res", None)
        if res is not None:
            for c in res["ctxs"]:
                c.close()
            self._res = None

    def run(self):
        """Both stages of ficp.py:149-154 over the partitioned plot; returns the source."""
        n, m = len(self.source), len(self.target)
        lam2 = 0.95 if self.match_dims == 3 else 1.3
        if n == 0 or m == 0:  # ficp.py:66-68, 125-126: nothing moves
            self.lambda_val = lam2
            self.last_stats = dict(k=[], n_nn_calls=0, n_fits=0, iters=(0, 0))
            return self.source
        res = self._setup()
        self.run_resident()
        xy = self._gather_xy(res)
        out = self.source.copy()
        out[:, 0] = xy[0]
        out[:, 1] = xy[1]
        self.close()
        self.source = out
        return self.source

    def _gather_xy(self, res):
        """The moved XY of every row on this process (source mode: each rank moved its
        own rows; they are exchanged once, after the run)."""
        import torch
        x, y = res["src"][0], res["src"][1]
        torch.cuda.current_stream(res["dev"]).wait_stream(self._stream)
        if self.mode == "target" or res["W"] == 1:
            return x.cpu().numpy(), y.cpu().numpy()
        nm = res["n_max"]
        loc = []
        for off, cnt in res["mine"]:
            t = torch.zeros(2, nm, dtype=torch.float64, device=res["dev"])
            t[0, :cnt] = x[off:off + cnt]
            t[1, :cnt] = y[off:off + cnt]
            loc.append(t)
        allp = gather_ranked(loc, self.group, res["world"])
        ox, oy = np.empty(len(self.source)), np.empty(len(self.source))
        a = allp.cpu().numpy()
        for v, (off, cnt) in enumerate(res["parts"]):
            ox[off:off + cnt] = a[v, 0, :cnt]
            oy[off:off + cnt] = a[v, 1, :cnt]
        return ox, oy

    def run_resident(self, lambda0=None):
        """One run from the pristine resident source, stream-ordered; the result stays on
        the device (source mode: each rank's own rows)."""
        import torch
        res = self._setup()
        self._stream.wait_stream(torch.cuda.current_stream(res["dev"]))
        with torch.cuda.stream(self._stream):
            out = self._run_on_stream(res, lambda0)
        torch.cuda.current_stream(res["dev"]).wait_stream(self._stream)
        return out

    def _run_on_stream(self, res, lambda0):
        try:
            return self._run_once(res, lambda0)
        except _lib.FicpError as e:
            if self.mode != "source" or "ERR_CAP" not in str(e) or self.capd >= res["n_max"]:
                raise
        # a rank's candidates overflowed its pack: every rank stopped at the same call (the
        # overflow bit is merged); start over with packs that can hold every row
        import torch
        self.capd = res["n_max"]
        res["pack"] = [torch.zeros(4 + 3 * self.capd, dtype=torch.int64, device=res["dev"]) for _ in res["mine"]]
        self.n_cap_restarts = getattr(self, "n_cap_restarts", 0) + 1
        return self._run_once(res, lambda0)

    def _run_once(self, res, lambda0):
        n, md = len(self.source), self.match_dims
        world, W, ctxs, mine = res["world"], res["W"], res["ctxs"], res["mine"]
        src, tgt = res["src"], res["tgt"]
        for a, b in zip(src, res["src0"]):
            a.copy_(b)
        lam1 = self.lambda_val if lambda0 is None else lambda0
        lam2 = 0.95 if md == 3 else 1.3
        lams = [lam1, lam2]
        zp = src[2].data_ptr() if md == 3 else 0
        if self.mode == "target":
            ctrl = ctxs[0]
            ctrl.dist_begin(1, src[0].data_ptr(), src[1].data_ptr(), zp, n, n, n, 0, lams, self.threshold,
                            self.max_iterations, self.allow_reflection, res["pivot"], 1, 1)
            step, last = self._step_target, ctrl
        else:
            for c, (off, cnt) in zip(ctxs, mine):
                c.dist_begin(2, src[0].data_ptr() + 8 * off, src[1].data_ptr() + 8 * off,
                             zp + 8 * off if md == 3 else 0, cnt, n, res["n_max"], off, lams, self.threshold,
                             self.max_iterations, self.allow_reflection, res["pivot"], W, self.capd)
            step, last = self._step_source, ctxs[-1]
        cap = 2 * (max(int(self.max_iterations), 0) + 1)
        done, j = False, 0
        while j < cap and not done:
            step(res, j)
            if j >= 1:
                done = last.dist_wait(j - 1)  # one iteration behind: the device never idles
            j += 1
        if not done:
            last.dist_wait(j - 1)
        stats = None
        for c in ctxs if self.mode == "source" else ctxs[:1]:
            stats = c.dist_end()
        self.lambda_val = lam2  # ficp.py:152
        self.last_stats = stats
        return stats

    def _step_target(self, res, j):
        """One NN call (and the fit + apply before it) of the target-partitioned mode."""
        ctxs, mine, tgt = res["ctxs"], res["mine"], res["tgt"]
        ctrl = ctxs[0]
        ctrl.dist_fit_sums(res["sums"].data_ptr())
        ctrl.dist_fit_solve(res["sums"].data_ptr(), 1)
        for c, (off, _), d2, ix in zip(ctxs, mine, res["d2s"], res["idxs"]):
            c.dist_nn_shard(ctrl, off, d2.data_ptr(), ix.data_ptr())
        dmin, imin = merge_local(res["d2s"], res["idxs"]) if len(ctxs) > 1 else (res["d2s"][0], res["idxs"][0])
        if res["world"] > 1:
            dmin, imin = merge_shards(dmin, imin, self.group)
        res["_keep"] = (dmin, imin)  # alive until the stream has consumed them
        ctrl.dist_select_merged(dmin.data_ptr(), imin.data_ptr(), tgt[0].data_ptr(), tgt[1].data_ptr(), j)

    def _step_source(self, res, j):
        """One NN call (and the fit before it) of the source-partitioned mode."""
        ctxs, world, W = res["ctxs"], res["world"], res["W"]
        for c, s8 in zip(ctxs, res["sums"]):
            c.dist_fit_sums(s8.data_ptr())
        sums = gather_ranked(res["sums"], self.group, world)
        for c in ctxs:
            c.dist_fit_solve(sums.data_ptr(), W)
        for c, r2 in zip(ctxs, res["range2"]):
            c.dist_nn_local(r2.data_ptr())
        rg = merge_range(res["range2"], self.group, world)
        for c, h in zip(ctxs, res["hist"]):
            c.dist_hist(rg.data_ptr(), h.data_ptr())
        hg = merge_hist(res["hist"], self.group, world)
        for c, pk in zip(ctxs, res["pack"]):
            c.dist_candidates(hg.data_ptr(), pk.data_ptr(), self.capd)
        packs = gather_ranked(res["pack"], self.group, world)
        for c in ctxs:
            c.dist_final(packs.data_ptr(), W, self.capd, j)
        res["_keep"] = (sums, rg, hg, packs)
