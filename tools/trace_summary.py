"""Per-kernel dispatch durations from a rocprofv3 kernel_trace.csv.

`all_avg_us` matches rocprofv3 --stats (every dispatch); `active_avg_us` leaves out the
early-exit launches the device-resident ICP loop enqueues past the end of a run (shorter
than 10 % of the kernel's median), which is what bench.py's `avg_launch_us` measures with
HIP events over the real NN calls.  usage: trace_summary.py <kernel_trace.csv> [prefix...]"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(path, prefixes):
    dur = defaultdict(list)
    for r in csv.DictReader(open(path)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, v in sorted(dur.items()):
        if prefixes and not any(k.startswith(p) for p in prefixes):
            continue
        med = sorted(v)[len(v) // 2]
        act = [x for x in v if x >= 0.1 * med]
        out[k] = {"dispatches": len(v), "all_avg_us": sum(v) / len(v), "active_dispatches": len(act),
                  "active_avg_us": sum(act) / len(act), "median_us": med}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
