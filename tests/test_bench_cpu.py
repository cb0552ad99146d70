"""CPU tests of bench.py's multi-GPU contract: `--gpus N` starts N rank processes by
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set for each), rank 0 prints one
JSON line with the world size the process group actually formed, a failing rank fails
the job, and a --gpus / WORLD_SIZE mismatch is an error (not a silent 1-rank run).
--dry-run does no GPU work, so gloo carries the process group here."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd="/tmp")


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_launcher_spawns_two_ranks_one_line():
    r = _run(["--gpus", "2", "--workload", "batch", "--dry-run", "--steps", "2", "--warmup", "0",
              "--plots", "37"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == d["ranks_seen"] == 2
    assert d["dry_run"] is True
    assert d["scaling"] == "strong"
    assert d["config"]["plots_dealt"] == 37   # every plot dealt to exactly one rank


def test_eight_rank_rehearsal_1024_plots():
    """The driver's N=8 launch of the C4 line, rehearsed with gloo: 8 ranks form the
    process group, the 1024 plots are dealt once each in the serpentine (128 per rank),
    and the end-of-run all-gather returns all 1024 records in batch order."""
    r = _run(["--gpus", "8", "--dry-run", "--workload", "batch", "--plots", "1024", "--steps", "2",
              "--warmup", "0"], timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == d["ranks_seen"] == 8
    assert d["config"]["plots_dealt"] == 1024
    assert d["config"]["plots_per_rank"] == [128] * 8
    assert d["config"]["gather_in_order"] is True


def test_serpentine_deal_balances_ragged_plots():
    """shard.deal_plots on ragged N*M: every plot once, each rank's work within the
    largest plot of the mean, ids ascending per rank."""
    import numpy as np
    from coregistrationgame_amd import shard
    rng = np.random.default_rng(0)
    work = rng.integers(1, 10_000, 1024).astype(float) * rng.integers(1, 10_000, 1024)
    deal = shard.deal_plots(work, 8)
    ids = np.sort(np.concatenate(deal))
    assert np.array_equal(ids, np.arange(1024))
    loads = np.array([work[d].sum() for d in deal])
    assert loads.max() - loads.min() <= work.max()
    assert all(np.all(np.diff(d) > 0) for d in deal)
    assert sorted(len(d) for d in deal) == [128] * 8


def test_default_workload_is_the_same_at_every_n():
    """One headline workload at every N: `value` is C3 (BASELINE.json's
    metric config, one plot per GPU) at N=1 and N=8, and the C4 strong-scaling batch
    rides along as the same `batch` key at both, dealt over the N ranks."""
    lines = {}
    for n in (1, 8):
        r = _run(["--gpus", str(n), "--dry-run", "--steps", "1", "--warmup", "0", "--plots", "1024"],
                 timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        d = _json_lines(r.stdout)
        assert len(d) == 1, r.stdout
        lines[n] = d[0]
    for n, d in lines.items():
        assert d["ranks_seen"] == n
        assert d["config"]["workload"] == "c3" and d["scaling"] == "weak"
        assert d["batch"]["scaling"] == "strong"
        assert d["batch"]["config"]["workload"] == "batch"
        assert d["batch"]["config"]["plots_dealt"] == 1024
    assert lines[1]["batch"]["config"]["plots_per_rank"] == [1024]
    assert lines[8]["batch"]["config"]["plots_per_rank"] == [128] * 8
    assert set(lines[1]) - {"batch_shares"} == set(lines[8]) - {"batch_shares"}


def test_gpus_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
    assert not _json_lines(r.stdout)


def test_failing_rank_fails_the_job():
    # no GPU here: the ranks' RCCL process group cannot form, so every rank exits non-zero
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--backend", "nccl", "--plots", "4"])
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
