"""Per-kernel totals per step from a rocprofv3 kernel_stats.csv: tools/kstats.py <csv> <steps>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
agg, cnt = {}, {}
for r in rows:
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?\(", r["Name"])
    n = (m.group(1) + (m.group(2) or "")) if m else r["Name"][:40]
    agg[n] = agg.get(n, 0.0) + float(r["TotalDurationNs"])
    cnt[n] = cnt.get(n, 0) + int(r["Calls"])
tot = sum(agg.values())
print(f"total kernel time per step: {tot / 1e3 / steps:.1f} us")
for n, v in sorted(agg.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print(f"  {n:34s} {v / 1e3 / steps:9.1f} us/step  {v / cnt[n] / 1e3:8.2f} us/call  x{cnt[n] / steps:.1f}")
