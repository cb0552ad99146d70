"""Window-path probe (tools only): C3 runs with the window path off (twice), forced to fall
back, and on; prints bit differences, per-call k and the path counters."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from coregistrationgame_amd import _lib, synth  # noqa: E402


def run(p, md, lams, win, fault=0):
    os.environ["FICP_SEL_WIN"] = "1" if win else "0"
    ctx = _lib.Context(0, _lib.NN_GRID)
    try:
        ctx.set_target(p.target, md)
        ctx.set_fault(fault)
        src = np.array(p.source)
        st = ctx.run(src, lams, 1e-6, 1000, False, trace=True)
        return src, st, ctx.path_stats()
    finally:
        ctx.close()


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
p = synth.make_plot(n, n, 0.6, seed=1_000_000, md=3)
lams = [3.0, 0.95]
res = {"off1": run(p, 3, lams, False), "off2": run(p, 3, lams, False), "fault": run(p, 3, lams, True, 2),
       "on1": run(p, 3, lams, True), "on2": run(p, 3, lams, True)}
for k, (src, st, ps) in res.items():
    print(k, ps, "k:", list(st["k"]), "T0:", st["T"][0].ravel()[:3] if len(st["T"]) else None)
b = res["off1"][0]
for k, (src, st, ps) in res.items():
    d = np.max(np.abs(src[:, :2] - b[:, :2]))
    nd = int(np.count_nonzero(src[:, :2] != b[:, :2]))
    Td = [float(np.max(np.abs(st["T"][i] - res["off1"][1]["T"][i]))) for i in range(min(len(st["T"]), len(res["off1"][1]["T"])))]
    print(k, "max|dXY| vs off1", d, "entries differing", nd, "T diffs per fit", Td)
