"""Per-kernel medians of the PMC passes written by tools/pmc.sh (counter_collection.csv).

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KB per dispatch.  On gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md,
HBM section): `fetch_bytes_corrected` doubles it; other access widths are uncalibrated,
so both values are kept."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # the C3 NN runs as two kernels (k_nn_grid for the first calls of a run, k_nn_grid_q
    # for the rest): their dispatches together are the bench's NN launches
    for md in ("3", "2"):
        for apply in ("true", "false"):
            parts = [acc[k] for k in (f"k_nn_grid<{md}, {apply}>", f"k_nn_grid_q<{md}, {apply}>") if k in acc]
            if len(parts) == 2:
                merged = defaultdict(list)
                for ctrs in parts:
                    for c, v in ctrs.items():
                        merged[c].extend(v)
                acc[f"k_nn_grid+q<{md}, {apply}>"] = merged
    out = {}
    for k, ctrs in acc.items():
        # median over dispatches: the device loop's few no-op launches past the end of a
        # run (early exit, ~0 bytes) would pull a mean down
        d = {c: float(sorted(v)[len(v) // 2]) for c, v in ctrs.items()}
        d["dispatches"] = max(len(v) for v in ctrs.values())
        # and the mean over the dispatches that did work (non-zero), the basis of the
        # bench's average launch duration (cold first call included)
        mean = {}
        for c, v in ctrs.items():
            nz = [x for x in v if x > 0]
            if nz:
                mean[c] = sum(nz) / len(nz)
        if "FETCH_SIZE" in mean:
            mean["fetch_bytes_raw"] = mean["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in mean:
            mean["write_bytes"] = mean["WRITE_SIZE"] * 1024.0
        d["mean_active"] = mean
        if "FETCH_SIZE" in d:
            d["fetch_bytes_raw"] = d["FETCH_SIZE"] * 1024.0
            d["fetch_bytes_corrected"] = 2.0 * d["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024.0
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out[k] = d
    json.dump(dict(sorted(out.items())), sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
