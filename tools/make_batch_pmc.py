"""profiles/<prefix>_pmc_batch_nn.json from a tools/pmc.sh run of the batch workload:
    PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum" \
        bash tools/pmc.sh <tag> --workload batch --no-extra
    python3 tools/make_batch_pmc.py gpurun_out/<tag> <prefix>
The k_nn_grid_batch HBM bytes per launch that bench.py's batch line reports as
roofline.traffic (the mean over the dispatches that did work, as the bench's average launch
duration; FETCH_SIZE doubled as calibrated, tools/pmc_calib.py)."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def main(src, prefix):
    pmc = json.loads((Path(src) / "summary.json").read_text())
    k = next(k for k in pmc if k.startswith("k_nn_grid_batch"))
    d = pmc[k]
    mean = d["mean_active"]
    hbm = 2.0 * mean["fetch_bytes_raw"] + mean["write_bytes"]
    med = {c: v for c, v in d.items() if c != "mean_active"}
    if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
        med["l2_hit_rate"] = med["TCC_HIT_sum"] / max(med["TCC_HIT_sum"] + med["TCC_MISS_sum"], 1.0)
    out = {
        "source": "rocprofv3 --pmc, one pass per counter group, tools/pmc.sh --workload batch --no-extra: "
                  "python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload batch "
                  "(C4, 1024 plots x 10k)",
        "kernel": k,
        "per_launch_median": med,
        "per_launch_mean_active": mean,
        "hbm_bytes_per_launch": hbm,
        "basis": "mean over active dispatches; FETCH_SIZE doubled (calibrated, tools/pmc_calib.py)",
        "algorithmic_bytes_per_launch_all_plots_live": 1024 * 760000,
        "note": "a launch's algorithmic bytes are (live plots) x 760 KB (bench.nn_bytes_per_launch at "
                "10k x 10k); converged plots drop out of later launches",
    }
    (REPO / "profiles" / f"{prefix}_pmc_batch_nn.json").write_text(json.dumps(out, indent=1))
    print(json.dumps({"kernel": k, "hbm_bytes_per_launch": hbm}))


if __name__ == "__main__":
    main(*sys.argv[1:])
