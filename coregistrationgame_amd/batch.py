"""`FractionalICPBatch` -- `FractionalICP(source_p, target_p).run()` for many plots at once.

The reference joins one plot at a time: `App.join_plot` (app.py:630-661) builds a
`FractionalICP` from the plot's trees and its CHM stems and calls `run()`
(ficp.py:149-154). A stand holds many plots (`Stand.plots`, trees.py:333-451), and each
plot's co-registration is independent of the others. This class runs them all in one
device pass through `ficp_run_batch` (include/ficp.h). Every plot follows its own
two-stage loop with its own convergence test, exactly as it would alone. Plots with
different match dims (ficp.py:40) go to separate device passes.

There is no CPU fallback. Without libficp.so or a GPU, `run()` raises.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def stage_lambdas(lambda_val: float, match_dims: int) -> list[float]:
    """The two stages of run(): lambda_val, then 0.95 (3D) or 1.3 (2D) (ficp.py:151-153)."""
    return [float(lambda_val), 0.95 if match_dims == 3 else 1.3]


class FractionalICPBatch:
    def __init__(self, sources, targets, lambda_val=3.0, threshold=1e-6, max_iterations=1000,
                 allow_reflection=False, *, device=None):
        if len(sources) != len(targets):
            raise ValueError("sources and targets must have the same number of plots.")
        self.sources = [np.array(s, dtype=float) for s in sources]
        self.targets = [np.array(t, dtype=float) for t in targets]
        for s, t in zip(self.sources, self.targets):
            if s.ndim != 2 or t.ndim != 2:  # ficp.py:37-38, per plot
                raise ValueError("source and target must be 2D arrays (N, D).")
        self.match_dims = [3 if (s.shape[1] >= 3 and t.shape[1] >= 3) else 2
                           for s, t in zip(self.sources, self.targets)]
        self.lambda_val = lambda_val
        self.threshold = threshold
        self.max_iterations = max_iterations
        self.allow_reflection = allow_reflection
        self.device = device
        self.stats = None  # PLOT_STATS_DTYPE records, one per plot, after run()
        self._ctx = None

    def _context(self) -> _lib.Context:
        if self._ctx is None:
            self._ctx = _lib.Context(self.device)
        return self._ctx

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def run(self, trace: bool = False, max_trace: int = 256) -> list[np.ndarray]:
        """Runs every plot; returns (and stores in .sources) the moved source arrays.
        trace=True also records every plot's k per NN / fraction call in .k_trace (a list of
        int64 arrays, up to max_trace calls each)."""
        nplots = len(self.sources)
        self._trace = max_trace if trace else 0
        self.k_trace = [np.zeros(0, np.int64) for _ in range(nplots)] if trace else None
        stats = np.zeros(nplots, _lib.PLOT_STATS_DTYPE)
        ident = np.eye(3).ravel()
        stats["T_total"] = ident
        stats["frmsd_last"] = np.inf
        for md in (3, 2):
            plots = [p for p in range(nplots) if self.match_dims[p] == md]
            # an empty layer moves nothing (ficp.py:66-68, 125-126)
            plots = [p for p in plots if len(self.sources[p]) and len(self.targets[p])]
            for lo in range(0, len(plots), 65535):
                self._run_group(plots[lo:lo + 65535], md, stats)
        self.stats = stats
        return self.sources

    def _run_group(self, plots, md, stats):
        if not plots:
            return
        src = np.ascontiguousarray(np.concatenate([self.sources[p][:, :md] for p in plots]))
        tgt = np.ascontiguousarray(np.concatenate([self.targets[p][:, :md] for p in plots]))
        so = np.zeros(len(plots) + 1, np.int64)
        to = np.zeros(len(plots) + 1, np.int64)
        so[1:] = np.cumsum([len(self.sources[p]) for p in plots])
        to[1:] = np.cumsum([len(self.targets[p]) for p in plots])
        ctx = self._context()
        tr = np.full((len(plots), self._trace), -1, np.int64) if self._trace else None
        ctx.set_batch_trace(tr)
        try:
            out = ctx.run_batch(so, src, to, tgt, md, stage_lambdas(self.lambda_val, md),
                                self.threshold, self.max_iterations, self.allow_reflection)
        finally:
            if tr is not None:
                ctx.set_batch_trace(None)
        for j, p in enumerate(plots):
            if tr is not None:
                row = tr[j]
                self.k_trace[p] = row[row >= 0].copy()
            moved = self.sources[p].copy()  # columns 0,1 move; the rest stay bit-identical
            moved[:, :2] = src[so[j]:so[j + 1], :2]
            self.sources[p] = moved
            stats[p] = out[j]
