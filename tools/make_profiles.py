"""Turn a tools/round_profile.sh run (gpurun_out/<tag>/) into the committed profiles:
profiles/r1_c3_bench.json, r1_c3_kernel_stats.csv, r1_c3_trace_summary.json,
r1_c3_timeline.txt, r1_pmc_c3_summary.json and r1_pmc_c3_nn.json (the NN kernel's HBM
bytes per launch that bench.py reports as roofline.traffic).
usage: python tools/make_profiles.py <tag> [prefix=r1]
(<tag>/pmc/summary.json from tools/pmc.sh; an optional <tag>/cal_summary.json from
tools/pmc_calib.py passes is recorded beside the NN bytes)"""
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
    tl = subprocess.run([sys.executable, str(REPO / "tools" / "timeline.py"), str(trace), "k_run_start", "-v"],
                        capture_output=True, text=True, check=True).stdout  # FICP_TL_RUN picks the run
    (dst / f"{prefix}_c3_timeline.txt").write_text(tl)
    pmc = json.loads((REPO / "gpurun_out" / tag / "pmc" / "summary.json").read_text())
    (dst / f"{prefix}_pmc_c3_summary.json").write_text(json.dumps(pmc, indent=1))
    nn = next((k for k in pmc if k.startswith("k_nn_grid+q<3")), None) or \
        next(k for k in pmc if k.startswith("k_nn_grid<3"))
    d = pmc[nn]
    groups = sorted({c for k in pmc for c in pmc[k] if re.match(r"^[A-Z][A-Z0-9_]*(_sum|_avr|_max|_min)?$", c)})
    mean = d.get("mean_active")
    if mean and "fetch_bytes_raw" in mean and "write_bytes" in mean:
        # per launch as the bench's average launch duration: the mean over the dispatches
        # that did work (the cold call included); FETCH_SIZE x 2 as calibrated for 8-B
        # lane reads (tools/pmc_calib.py: k_apply_inplace, 268,435,456 B read -> 134.2 MB)
        hbm = 2.0 * mean["fetch_bytes_raw"] + mean["write_bytes"]
        basis = "mean over active dispatches; FETCH_SIZE doubled (calibrated, tools/pmc_calib.py)"
    else:
        hbm = d["fetch_bytes_corrected"] + d["write_bytes"]
        basis = "median over dispatches; FETCH_SIZE doubled per MI355X_MICROARCH.md"
    cal = REPO / "gpurun_out" / tag / "cal_summary.json"
    nn_json = {
        "source": "rocprofv3 --pmc, one pass per counter group (" + " ".join(groups) + "), "
                  "python3 bench.py --no-extra --no-cpu-baseline --steps 2 --warmup 1 (C3)",
        "kernel": nn,
        "per_launch_median": {k: v for k, v in d.items() if k != "mean_active"},
        "per_launch_mean_active": mean,
        "hbm_bytes_per_launch": hbm,
        "basis": basis,
        "calibration": json.loads(cal.read_text()) if cal.exists() else None,
    }
    (dst / f"{prefix}_pmc_c3_nn.json").write_text(json.dumps(nn_json, indent=1))
    # the bench line read the previous traffic file: carry this run's PMC bytes into it
    bj = json.loads((dst / f"{prefix}_c3_bench.json").read_text())
    bj["roofline"]["traffic"] = nn_json["hbm_bytes_per_launch"]
    bj["roofline"]["traffic_source"] = f"{prefix}_pmc_c3_nn.json"
    (dst / f"{prefix}_c3_bench.json").write_text(json.dumps(bj) + "\n")
    hp = src / "host_path_summary.json"
    if hp.exists():
        shutil.copy(hp, dst / f"{prefix}_host_path_trace.json")
    print(json.dumps({k: summ[k]["active_avg_us"] for k in summ if k.startswith("k_nn")}))
    print("hbm bytes per NN launch", nn_json["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main(*sys.argv[1:])
