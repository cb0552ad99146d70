#!/usr/bin/env python3
"""Where the drop-in call's time goes: times every host-side piece of
`FractionalICP(src, tgt).run()` at C3 separately, plus the raw H2D/D2H rates from pageable
and pinned memory.  Prints one JSON object.  GPU box only."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from coregistrationgame_amd import _lib, synth  # noqa: E402
from coregistrationgame_amd.ficp import FractionalICP  # noqa: E402


def ms(f, reps=5):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        out.append(1e3 * (time.perf_counter() - t0))
    return float(np.median(out)), [round(x, 3) for x in out]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    plot = synth.make_plot(n, n, 0.6, 1_000_000, md=3)
    src, tgt = plot.source, plot.target
    res = {"n": n}
    res["np_array_copy_src"] = ms(lambda: np.array(src, dtype=float))
    res["np_empty_like_touch"] = ms(lambda: np.empty_like(src).fill(0.0))
    import torch
    a = torch.from_numpy(np.ascontiguousarray(src))
    pin = torch.empty(a.shape, dtype=a.dtype, pin_memory=True)
    pin.copy_(a)
    d = torch.empty(a.shape, dtype=a.dtype, device="cuda")
    torch.cuda.synchronize()

    def h2d(x):
        d.copy_(x, non_blocking=False)
        torch.cuda.synchronize()

    res["h2d_pageable_24MB"] = ms(lambda: h2d(a))
    res["h2d_pinned_24MB"] = ms(lambda: h2d(pin))
    res["memcpy_to_pinned_24MB"] = ms(lambda: pin.copy_(a))
    out_pg = np.empty_like(src)

    def d2h_pg():
        out_pg[...] = d.cpu().numpy()

    res["d2h_pageable_24MB_via_torch"] = ms(d2h_pg)
    res["pin_alloc_24MB"] = ms(lambda: torch.empty(a.shape, dtype=a.dtype, pin_memory=True))
    del d
    torch.cuda.empty_cache()
    # context life cycle
    res["ctx_create_destroy"] = ms(lambda: _lib.Context(0).close())
    ctx = _lib.Context(0)
    res["set_target_reused_ctx"] = ms(lambda: (ctx.set_target(tgt, 3), ctx.synchronize()))
    s = np.array(src)

    def run_reused():
        s[...] = src
        return ctx.run(s, [3.0, 0.95], 1e-6, 1000, False)

    res["run_reused_ctx"] = ms(run_reused)
    res["gpu_loop_ms"] = run_reused()["gpu_ms"]
    ctx.close()
    # the whole drop-in call, fresh instance each time (app.py:658-660)

    def full():
        icp = FractionalICP(src, tgt, device=0)
        icp.run()
        icp.close()

    res["full_call"] = ms(full)

    def full_noclose():
        icp = FractionalICP(src, tgt, device=0)
        icp.run()
        return icp

    res["full_call_no_close"] = ms(full_noclose)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
