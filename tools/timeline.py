"""Per-run kernel timeline from a rocprofv3 kernel trace (CSV): durations and the idle
gaps between consecutive kernels of the last complete run().  usage:
python tools/timeline.py <run_kernel_trace.csv> [marker-kernel-substring]"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_minmax2_partial"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
# the run to show: FICP_TL_RUN (default -1, the last complete one; the default bench
# command ends with the drop-in host-path runs, whose first NN calls are cold)
ri = int(__import__("os").environ.get("FICP_TL_RUN", "-1"))
a, b = starts[ri - 1], starts[ri]
run = rows[a:b]
t0 = int(run[0]["Start_Timestamp"])
prev_end = t0
agg = defaultdict(lambda: [0, 0.0])
gap_tot = 0.0
for r in run:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("ficp::(anonymous namespace)::", "").replace("void ", ""))
    gap = (s - prev_end) / 1e3
    gap_tot += max(gap, 0.0)
    agg[name][0] += 1
    agg[name][1] += (e - s) / 1e3
    if "-v" in sys.argv:
        print(f"{(s - t0) / 1e3:9.2f} +{gap:6.2f} {(e - s) / 1e3:8.2f}  {name}")
    prev_end = e
span = (int(run[-1]["End_Timestamp"]) - t0) / 1e3
print(f"run span {span:.1f} us, {len(run)} kernels, idle gaps {gap_tot:.1f} us")
for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:9.1f} us {c:4d}x  {t / c:7.2f}  {name}")
