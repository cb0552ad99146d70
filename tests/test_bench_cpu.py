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


def test_default_workload_is_batch_above_one_gpu():
    r = _run(["--gpus", "3", "--dry-run", "--steps", "1", "--warmup", "0", "--plots", "10"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_lines(r.stdout)[0]
    assert d["config"]["workload"] == "batch" and d["ranks_seen"] == 3


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
