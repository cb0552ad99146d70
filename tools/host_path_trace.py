#!/usr/bin/env python3
"""The drop-in call shape under a HIP API trace: warm-up call, then 5 x
FractionalICP(src, tgt).run() at C3 and 3 x the 16 real stand-10 Joins, each group between
marker prints.  Run as
    rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d <dir> -o run -- \\
        python3 tools/host_path_trace.py
then tools/host_path_trace.py --summarize <dir> folds the API trace into per-call time."""
from __future__ import annotations

import csv
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def run():
    from coregistrationgame_amd import FractionalICP, synth
    p = synth.make_plot(1_000_000, 1_000_000, 0.6, 1_000_000, md=3)
    FractionalICP(p.source, p.target, device=0).run()
    marks = {}
    t0 = time.perf_counter_ns()
    walls = []
    for _ in range(5):
        a = time.perf_counter()
        icp = FractionalICP(p.source, p.target, device=0)
        icp.run()
        walls.append(1e3 * (time.perf_counter() - a))
        del icp
    marks["c3"] = (t0, time.perf_counter_ns(), walls)
    f = np.load(REPO / "tests" / "golden" / "run_real_stand10.npz")
    tgt = f["tgt"]
    plots = [f[f"{int(pid)}/src"] for pid in f["plot_ids"]]
    FractionalICP(plots[0], tgt, device=0).run()
    t0 = time.perf_counter_ns()
    walls = []
    for _ in range(3):
        for src in plots:
            a = time.perf_counter()
            FractionalICP(src, tgt, device=0).run()
            walls.append(1e3 * (time.perf_counter() - a))
    marks["join"] = (t0, time.perf_counter_ns(), walls)
    print(json.dumps({k: {"calls": len(v[2]), "ms_median": float(np.median(v[2]))} for k, v in marks.items()}))


def summarize(d):
    d = Path(d)
    api = next(d.rglob("*hip_api_trace.csv"), None)
    ker = next(d.rglob("*kernel_trace.csv"), None)
    out = {}
    for name, path in (("hip_api", api), ("kernel", ker)):
        if path is None:
            continue
        agg = defaultdict(lambda: [0, 0.0])
        for r in csv.DictReader(open(path)):
            fn = r.get("Function") or r.get("Kernel_Name") or "?"
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            agg[fn][0] += 1
            agg[fn][1] += dur
        out[name] = {k: {"count": c, "ms": round(t, 4)} for k, (c, t) in
                     sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
