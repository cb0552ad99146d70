"""Probe: run-to-run determinism of the 100k untraced/traced runs (2-D by default) and the
per-call k against the oracle, under the current environment.  tools only."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from coregistrationgame_amd import FractionalICP, synth  # noqa: E402
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import ficp_oracle  # noqa: E402

md = int(sys.argv[1]) if len(sys.argv) > 1 else 2
p = synth.make_plot(100_000, 100_000, 0.8, seed=100_000, md=md)
ofinal, otr = ficp_oracle.run(p.source, p.target, nthreads=16)
runs = []
for rep in range(4):
    icp = FractionalICP(p.source, p.target)
    icp.run(trace=True)
    st = icp.last_stats
    runs.append((np.array(st["k"]), np.array(st["T"]), icp.source.copy()))
k0, T0, s0 = runs[0]
for q, (k, T, s) in enumerate(runs):
    n = min(len(T), len(T0))
    dT = [i for i in range(n) if not np.array_equal(T[i], T0[i])]
    print(f"run {q}: k {list(k)}\n   first T diff vs run0 at call {dT[:1]}, xy equal {np.array_equal(s, s0)}")
print("oracle k", list(otr["k"]))
oT = otr.get("T")
if oT is not None:
    for i in range(min(len(oT), len(T0))):
        d = np.max(np.abs(np.asarray(T0[i]) - np.asarray(oT[i])))
        print(f"  call {i}: |T_gpu - T_oracle| = {d:.3e}")
