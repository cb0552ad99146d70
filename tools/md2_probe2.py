"""Probe: which part of a run differs between repeated runs (per-call NN idx with
trace_idx, k, T).  tools only."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from coregistrationgame_amd import FractionalICP, synth  # noqa: E402

md = int(sys.argv[1]) if len(sys.argv) > 1 else 2
tidx = len(sys.argv) > 2 and sys.argv[2] == "idx"
mode = sys.argv[3] if len(sys.argv) > 3 else "auto"
p = synth.make_plot(100_000, 100_000, 0.8, seed=100_000, md=md)
runs = []
for rep in range(4):
    icp = FractionalICP(p.source, p.target, nn_mode=mode)
    icp.run(trace=True, trace_idx=tidx)
    st = icp.last_stats
    runs.append(st)
s0 = runs[0]
for q, st in enumerate(runs[1:], 1):
    n = min(len(st["T"]), len(s0["T"]))
    dT = [i for i in range(n) if not np.array_equal(st["T"][i], s0["T"][i])]
    dk = [i for i in range(n) if st["k"][i] != s0["k"][i]]
    di = []
    if tidx:
        di = [i for i in range(min(len(st["idx"]), len(s0["idx"]))) if not np.array_equal(st["idx"][i], s0["idx"][i])]
    print(f"run {q} vs 0: T diff calls {dT[:3]} k diff {dk[:3]} idx diff {di[:3]} path {st.get('path')}")
print("k0", list(s0["k"]))
