"""Turn a tools/round_profile.sh run (gpurun_out/<tag>/) into the committed profiles:
profiles/r1_c3_bench.json, r1_c3_kernel_stats.csv, r1_c3_trace_summary.json,
r1_c3_timeline.txt, r1_pmc_c3_summary.json and r1_pmc_c3_nn.json (the NN kernel's HBM
bytes per launch that bench.py reports as roofline.traffic).
usage: python tools/make_profiles.py <tag> [prefix=r1]"""
import csv
import json
import re
import shutil
import statistics
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def short(name):
    name = name.replace("ficp::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def main(tag, prefix="r1"):
    src = REPO / "gpurun_out" / tag
    dst = REPO / "profiles"
    shutil.copy(src / "bench.json", dst / f"{prefix}_c3_bench.json")
    shutil.copy(src / "kernel_stats.csv", dst / f"{prefix}_c3_kernel_stats.csv")
    trace = next((src / "prof").rglob("*kernel_trace.csv"))
    rows = list(csv.DictReader(open(trace)))
    per = {}
    for r in rows:
        per.setdefault(short(r["Kernel_Name"]), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    summ = {}
    for k, v in sorted(per.items()):
        # the device loop ends with <= 2 no-op iterations: their early-exit launches are
        # a few us; "active" drops launches under 20 % of the median
        med = statistics.median(v)
        act = [x for x in v if x >= 0.2 * med]
        summ[k] = {"dispatches": len(v), "all_avg_us": sum(v) / len(v),
                   "active_dispatches": len(act), "active_avg_us": sum(act) / len(act),
                   "median_us": med}
    (dst / f"{prefix}_c3_trace_summary.json").write_text(json.dumps(summ, indent=1))
    tl = subprocess.run([sys.executable, str(REPO / "tools" / "timeline.py"), str(trace)],  # FICP_TL_RUN picks the run
                        capture_output=True, text=True, check=True).stdout
    (dst / f"{prefix}_c3_timeline.txt").write_text(tl)
    pmc = json.loads((REPO / "gpurun_out" / tag / "pmc" / "summary.json").read_text())
    (dst / f"{prefix}_pmc_c3_summary.json").write_text(json.dumps(pmc, indent=1))
    nn = next(k for k in pmc if k.startswith("k_nn_grid<3"))
    d = pmc[nn]
    nn_json = {
        "source": "rocprofv3 --pmc, one pass per counter group (FETCH_SIZE / WRITE_SIZE / "
                  "TCC_HIT_sum TCC_MISS_sum / SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES "
                  "SQ_BUSY_CYCLES), tools/pmc.sh: python3 bench.py --no-cpu-baseline "
                  "--steps 2 --warmup 1 (C3); medians over dispatches",
        "kernel": nn,
        "per_launch_median": d,
        "hbm_bytes_per_launch": d["fetch_bytes_corrected"] + d["write_bytes"],
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half of wide "
                "reads); the kernel's reads are 8-16 B per lane, so the corrected fetch is "
                "an estimate: raw fetch + write is the lower bound",
    }
    (dst / f"{prefix}_pmc_c3_nn.json").write_text(json.dumps(nn_json, indent=1))
    # the bench line read the previous traffic file: carry this run's PMC bytes into it
    bj = json.loads((dst / f"{prefix}_c3_bench.json").read_text())
    bj["roofline"]["traffic"] = nn_json["hbm_bytes_per_launch"]
    (dst / f"{prefix}_c3_bench.json").write_text(json.dumps(bj) + "\n")
    print(json.dumps({k: summ[k]["active_avg_us"] for k in summ if k.startswith("k_nn")}))
    print("hbm bytes per NN launch", nn_json["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main(*sys.argv[1:])
