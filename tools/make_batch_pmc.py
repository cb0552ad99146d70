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
    # the batch NN runs as k_nn_grid_batch (cold calls, and warm launches below 2M trees) and
    # k_nn_grid_batch_q (warm launches from 2M trees): every dispatch is one of the bench's
    # NN launches, so the per-launch mean weights each kernel by its dispatches
    ks = [k for k in pmc if k.startswith("k_nn_grid_batch")]
    k = " + ".join(ks)
    disp = {q: pmc[q]["dispatches"] for q in ks}
    tot = sum(disp.values())
    mean = {}
    for c in ("fetch_bytes_raw", "write_bytes", "FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
        if all(c in pmc[q]["mean_active"] for q in ks):
            mean[c] = sum(pmc[q]["mean_active"][c] * disp[q] for q in ks) / tot
    hbm = 2.0 * mean["fetch_bytes_raw"] + mean["write_bytes"]
    med = {q: {c: v for c, v in pmc[q].items() if c != "mean_active"} for q in ks}
    for q in ks:
        m = med[q]
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            m["l2_hit_rate"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1.0)
    out = {
        "source": "rocprofv3 --pmc, one pass per counter group, tools/pmc.sh --workload batch --no-extra: "
                  "python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload batch "
                  "(C4, 1024 plots x 10k)",
        "kernel": k,
        "per_kernel_median": med,
        "dispatches": disp,
        "per_launch_mean_active": mean,
        "hbm_bytes_per_launch": hbm,
        "basis": "mean over active dispatches; FETCH_SIZE doubled (calibrated, tools/pmc_calib.py)",
        "algorithmic_bytes_per_launch_all_plots_live": 512 * 760000,  # (a sub-batch: 512 plots at C4)
        "note": "a launch's algorithmic bytes are (live plots) x 760 KB (bench.nn_bytes_per_launch at "
                "10k x 10k); converged plots drop out of later launches",
    }
    (REPO / "profiles" / f"{prefix}_pmc_batch_nn.json").write_text(json.dumps(out, indent=1))
    print(json.dumps({"kernel": k, "hbm_bytes_per_launch": hbm}))


if __name__ == "__main__":
    main(*sys.argv[1:])
