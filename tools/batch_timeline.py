"""Per-run kernel table of a batch run from a rocprofv3 kernel trace (CSV): every launch of
the last complete run (k_batch_init to k_batch_init) with its start, duration and queue,
then per kernel the summed time and the union of its launch intervals over the queues.
usage: python tools/batch_timeline.py <run_kernel_trace.csv> [-v]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_batch_init" in r["Kernel_Name"]]
ri = int(__import__("os").environ.get("FICP_TL_RUN", "-1"))
a, b = (starts[ri - 1], starts[ri]) if len(starts) > 1 else (starts[0], len(rows))
run = rows[a:b]
t0 = int(run[0]["Start_Timestamp"])
qcol = "Queue_Id" if "Queue_Id" in run[0] else ("Stream_Id" if "Stream_Id" in run[0] else None)


def name_of(r):
    return re.sub(r"\(.*", "", r["Kernel_Name"].replace("ficp::(anonymous namespace)::", "").replace("void ", ""))


iv = defaultdict(list)
for r in run:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = name_of(r)
    iv[n].append((s, e))
    if "-v" in sys.argv:
        print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q{r[qcol] if qcol else '?'}  {n}")


def union(v):
    v = sorted(v)
    tot, cs, ce = 0, None, None
    for s, e in v:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot / 1e3


span = (max(int(r["End_Timestamp"]) for r in run) - t0) / 1e3
print(f"run span {span:.1f} us, {len(run)} kernels, busy (union) {union([(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in run]):.1f} us")
for n, v in sorted(iv.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
    d = [(e - s) / 1e3 for s, e in v]
    print(f"{sum(d):9.1f} us {len(d):4d}x  mean {sum(d) / len(d):7.2f}  first {d[0]:7.2f}  union {union(v):8.1f}  {n}")
