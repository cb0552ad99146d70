#!/usr/bin/env python3
"""Benchmark: FICP iterations/s (BASELINE.json metric) on MI355X.

Workloads (`--workload`, default by GPU count):
  c3     (default at every N) one 1M-tree vs 1M-stem plot per GPU, f=0.6, md=3, run()
         to convergence.  A step = one complete FractionalICP.run() (ficp.py:149-154) on
         layers already resident in HBM: grid build, copy of the pristine source, the
         device-resident two-stage loop.  value = loop bodies (ficp.py:132-145) per second
         over all ranks ("scaling": "weak", one independent plot per GPU).
  batch  C4: 1024 plots of 10k x 10k dealt over the ranks (shard.deal_plots), each rank
         runs its share in one ficp_run_batch_device per step; value = plot loop bodies
         per second of the whole job ("scaling": "strong": the 1024 plots are fixed as N
         grows).  The north star's 1/2/4/8-GPU batch line.
  c2     100k x 100k, f=0.8, exactly 2 x 25 loop bodies.
  c5     one 8M x 8M plot whose CHM layer is split over the GPUs (RCCL merge per NN call).

The default line is the same workload at every N: `value` is C3 (BASELINE.json's metric
config, one plot per GPU), and the C4 strong-scaling batch rides along as the `batch` key
at every N (1024 plots dealt over the N ranks), so a 1/2/4/8 series holds two consistent
curves: `value` (C3, weak) and `batch.value` (C4, strong).  At N=1 `batch_shares` adds
the per-rank shares of N=2/4/8 timed on the one GPU.

Launch: `python bench.py --gpus N` starts N rank processes itself (before anything in
the parent touches a GPU) and exits with the first failing rank's code; under
torch.distributed.run (RANK / WORLD_SIZE set) it is one rank.  Rank 0 prints ONE JSON
line.  `--dry-run` exercises the launcher, the process group and the report with no
GPU work (CPU tests, gloo).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from coregistrationgame_amd import _lib, synth  # noqa: E402  (no GPU work at import)

METRIC = "FICP iterations/sec (and correspondences/sec) at 1M×1M points, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

WORKLOADS = {
    # name: (n, m, f, seed0, md, threshold, max_iterations, description)
    "c3": (1_000_000, 1_000_000, 0.6, 1_000_000, 3, 1e-6, 1000,
           "C3: 1M trees vs 1M CHM stems, f=0.6, md=3, run() to convergence (threshold 1e-6)"),
    "c2": (100_000, 100_000, 0.8, 100_000, 3, float("-inf"), 25,
           "C2: 100k trees vs 100k CHM stems, f=0.8, md=3, exactly 2x25 loop bodies"),
    "c5": (8_000_000, 8_000_000, 0.8, 8_000_000, 3, float("-inf"), 10,
           "C5: one 8M-tree plot vs an 8M-stem CHM layer partitioned over the GPUs, f=0.8, md=3, 2x10 loop bodies"),
    "batch": (10_000, 10_000, 0.8, 10_000_000, 3, 1e-6, 1000,
              "C4: 1024 plots of 10k trees vs 10k CHM stems, f=0.8, md=3, per-plot run() to convergence"),
}
BATCH_PLOTS = 1024


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # rehearsal of N ranks on fewer GPUs (gloo only: RCCL refuses two ranks on one GPU):
    # FICP_BENCH_SHARE_GPU=<gpus> maps rank r to GPU r % gpus
    share = int(os.environ.get("FICP_BENCH_SHARE_GPU", "0") or 0)
    if share > 0:
        local %= share
    return rank, world, local


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, argv: list[str]) -> int:
    """Start one rank process per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), wait for
    all of them; the first rank that fails stops the others.  The parent never touches
    a GPU (no HIP call, no torch.cuda), so this is not an exec from a GPU process."""
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0["MASTER_PORT"] = str(_free_port())
    env0["WORLD_SIZE"] = str(n)
    env0["LOCAL_WORLD_SIZE"] = str(n)
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        time.sleep(0.05)
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench: rank pid {p.pid} exited with {code}; stopping the others", file=sys.stderr)
                for q in alive:
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


# ----------------------------------------------------------------------------- helpers
class DevArray:
    """A device buffer owned through libficp (no torch types at the boundary): one column,
    or k columns of n rows stored one after another (host shape (k, n))."""

    def __init__(self, ctx: _lib.Context, host: np.ndarray):
        host = np.ascontiguousarray(host, dtype=np.float64)
        self.ctx = ctx
        self.n = host.shape[-1]
        self.k = host.size // max(self.n, 1)
        p = _lib.C.c_void_p()
        _lib._check(_lib.lib().ficp_dev_alloc(ctx.h, max(host.nbytes, 8), _lib.C.byref(p)))
        self.ptr = p.value
        _lib._check(_lib.lib().ficp_memcpy_h2d(ctx.h, _lib.C.c_void_p(self.ptr), host.ctypes.data_as(_lib.C.c_void_p),
                                               host.nbytes))

    def col(self, j: int) -> int:
        return self.ptr + 8 * self.n * j

    def copy_from(self, other: "DevArray", cols: int | None = None):
        """The first `cols` columns (all by default) of other, in one device copy."""
        c = self.k if cols is None else cols
        _lib._check(_lib.lib().ficp_memcpy_d2d(self.ctx.h, _lib.C.c_void_p(self.ptr), _lib.C.c_void_p(other.ptr),
                                               8 * self.n * c))

    def free(self):
        _lib.lib().ficp_dev_free(self.ctx.h, _lib.C.c_void_p(self.ptr))


def nn_bytes_per_launch(n, m, md):
    """Algorithmic HBM bytes of one fused apply+NN pass: per tree read md
    coordinates, write the moved XY (16 B), write idx (4) + dist (8); read the CHM layer
    once (8*md per stem) -- SURVEY.md §8(d)'s NN + apply terms."""
    return n * (8 * md + 16 + 12) + m * 8 * md


def iteration_bytes(n, m, md, k):
    """SURVEY.md §8(d)'s algorithmic HBM bytes of one ICP loop body (reference algorithm:
    apply, NN, sort, prefix scan, fit gather): N (32 + 8 md + 12 + 24 + 16 + 32 k/N) + 8 md M."""
    return n * (32 + 8 * md + 12 + 24 + 16) + 32 * k + 8 * md * m


def pmc_traffic(kernel_prefix, tag):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC profile
    (profiles/*_pmc_<tag>_nn.json, written from tools/pmc.sh output), or None."""
    best = None
    for f in sorted((REPO / "profiles").glob(f"*_pmc_{tag}_nn.json")):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if str(d.get("kernel", "")).startswith(kernel_prefix):  # str or tuple of prefixes
            best = (d["hbm_bytes_per_launch"], f.name)
    return best


def roofline(achieved_gbs, traffic, extra):
    out = {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic[0] if traffic else None,
           "traffic_source": traffic[1] if traffic else None}
    out.update(extra)
    return out


class Dist:
    """torch.distributed for the barrier, the max-over-ranks time and the sums (RCCL
    "nccl" on GPUs, gloo for --dry-run)."""

    def __init__(self, world, local, backend):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.gpu = backend == "nccl"
        if self.gpu:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            self.dev = torch.device("cuda", local)
        else:
            dist.init_process_group("gloo")
            self.dev = torch.device("cpu")
        self.world = dist.get_world_size()

    def barrier(self):
        self.dist.barrier()
        if self.gpu:
            self.torch.cuda.synchronize()

    def reduce(self, vals, op):
        t = self.torch.tensor([float(v) for v in vals], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=op)
        return [float(x) for x in t.cpu().numpy()]

    def max(self, vals):
        return self.reduce(vals, self.dist.ReduceOp.MAX)

    def sum(self, vals):
        return self.reduce(vals, self.dist.ReduceOp.SUM)

    def close(self):
        self.dist.destroy_process_group()


# ----------------------------------------------------------------------------- CPU baseline
def cpu_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return model, os.cpu_count() or 1, affinity


def cgroup_cpus():
    """CPUs the job's cgroup quota allows (cpu.max 'quota period'), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _oracle():
    sys.path.insert(0, str(REPO / "oracle"))
    import ficp_oracle
    ficp_oracle.build()
    return ficp_oracle


def cpu_baseline(plot, threads):
    """The pinned C oracle (oracle/ficp_oracle.c, kind "port") on the same C3 plot, timed
    on this host: bounded samples, not the target.
    * value: fair mode (kd-tree built once, O(N) FRMSD scan), 2 stages x 2 loop bodies,
      `threads` OpenMP threads (the job's CPU share);
    * value_1thread: the same, 1 thread, 2 stages x 1 loop body;
    * literal mode (ficp.py:69-85's cost model: the index rebuilt every NN call and the
      O(N^2) prefix scan) measured at N = 2k..16k on plots of C3's density, fitted with
      a*N + b*N^2 per loop body and extrapolated to 1M (labelled "extrapolated")."""
    orc = _oracle()
    model, logical, affinity = cpu_info()
    t0 = time.perf_counter()
    _, tr = orc.run(plot.source, plot.target, threshold=float("-inf"), max_iterations=2, nthreads=threads)
    dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, tr1 = orc.run(plot.source, plot.target, threshold=float("-inf"), max_iterations=1, nthreads=1)
    dt1 = time.perf_counter() - t0
    # every CPU this process may run on (os.sched_getaffinity; SURVEY.md §8(d) "Threads: 1
    # and os.cpu_count()"), same sample as `value`
    t0 = time.perf_counter()
    _, tra = orc.run(plot.source, plot.target, threshold=float("-inf"), max_iterations=2, nthreads=affinity)
    dta = time.perf_counter() - t0
    ns, per = [], []
    for n in (2000, 4000, 8000, 16000):
        p = synth.make_plot(n, n, 0.6, 1_000_000 + n, md=3)
        t0 = time.perf_counter()
        _, trl = orc.run(p.source, p.target, threshold=float("-inf"), max_iterations=1, literal=True, nthreads=1)
        ns.append(n)
        per.append((time.perf_counter() - t0) / trl["n_fits"])
    A = np.column_stack([np.array(ns, float), np.array(ns, float) ** 2])
    (a, b), *_ = np.linalg.lstsq(A, np.array(per), rcond=None)
    n_full = len(plot.source)
    return {"value": tr["n_fits"] / dt, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"C3 plot (1M x 1M, md=3): 2 stages x 2 loop bodies ({tr['n_calls']} NN calls, "
                      f"{tr['n_fits']} fits) in {dt:.2f} s; kd-tree built once, O(N) FRMSD scan, "
                      f"{threads} OpenMP threads (the job's CPU share, $OMP_NUM_THREADS)",
            "cpu_model": model, "host_logical_cpus": logical, "affinity_cpus": affinity,
            "threads_job_share": threads, "cgroup_cpu_quota": cgroup_cpus(),
            "threads_all": affinity,
            "value_threads_all": tra["n_fits"] / dta,
            "sample_threads_all": f"same sample as value ({tra['n_fits']} loop bodies) in {dta:.2f} s, "
                                  f"{affinity} OpenMP threads (every CPU in this process's affinity mask)",
            "value_1thread": tr1["n_fits"] / dt1,
            "sample_1thread": f"same plot, 2 stages x 1 loop body ({tr1['n_calls']} NN calls) in {dt1:.2f} s, 1 thread",
            "literal_samples": {"n": ns, "s_per_iteration": per},
            "literal_fit": {"a_s_per_row": float(a), "b_s_per_row2": float(b)},
            "literal_extrapolated_s_per_iter": float(a * n_full + b * n_full ** 2),
            "literal_note": "extrapolated: kd-tree rebuilt per NN call + O(N^2) FRMSD prefix scan "
                            "(ficp.py:69-85 cost model) measured at N=2k-16k, 1 thread, fitted a*N+b*N^2"}


def cpu_baseline_batch(plots, threads, budget_s=10.0):
    """The C oracle on the first plots of this rank's share, one run() each, until the
    time budget is spent (bounded sample); iterations/s = its loop bodies / time."""
    orc = _oracle()
    model, logical, affinity = cpu_info()
    fits = done = 0
    t0 = time.perf_counter()
    for pl in plots:
        _, tr = orc.run(pl.source, pl.target, nthreads=threads, trace=True)
        fits += tr["n_fits"]
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": fits / dt, "unit": "iterations/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_logical_cpus": logical,
            "sample": f"{done} C4 plots (10k x 10k, md=3), full run() each: {fits} loop bodies in "
                      f"{dt:.2f} s; kd-tree built once per plot, O(N) FRMSD scan, {threads} OpenMP threads"}


def host_path_cost(plot, device, reps=5):
    """The drop-in call shape of app.py:658-660: FractionalICP(src, tgt).run() from numpy
    arrays, a new instance per call, result back in numpy.  The instances borrow pooled
    library contexts (_lib.borrowed), so the first call of a process also pays the pool's
    context creation and device allocations (ms_first_run) and later calls do not
    (ms_per_run = median of the later calls).  The breakdown is the facade's own phase
    stamps of the same calls (FractionalICP.last_stats["host_ms"], the library's
    "lib_host_ms"): they tile the call, and `unaccounted_ms` is what they miss."""
    from coregistrationgame_amd import FractionalICP
    tot, phases = [], []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        icp = FractionalICP(plot.source, plot.target, device=device)
        icp.run()
        tot.append(1e3 * (time.perf_counter() - t0))
        st = icp.last_stats
        ph = dict(st["host_ms"])
        lib = st["lib_host_ms"]
        ph["run.upload_ms"] = lib["upload"]
        ph["run.loop_ms"] = lib["loop"]
        ph["run.gpu_loop_ms"] = st["gpu_ms"]
        ph["run.result_ms"] = lib["result"]
        ph["run.other_ms"] = ph["run"] - lib["upload"] - lib["loop"] - lib["result"]
        phases.append(ph)
        del icp
    warm = tot[1:]
    med = {k: float(np.median([p[k] for p in phases[1:]])) for k in phases[1]}
    top = ("ctor_copies", "copy_source", "borrow", "set_target", "run", "release")
    tiled = sum(med[k] for k in top)
    out = {"ms_per_run": float(np.median(warm)), "ms_first_run": tot[0], "runs": len(warm),
           "breakdown_median_ms": {k.replace("ctor_copies", "ctor_copies_ms").replace("copy_source", "copy_source_ms")
                                   .replace("borrow", "borrow_ms").replace("set_target", "set_target_ms")
                                   .replace("release", "release_ms") if not k.startswith("run") else
                                   (k if k != "run" else "run_ms"): v for k, v in med.items()},
           "tiled_ms": tiled, "unaccounted_ms": float(np.median(warm)) - tiled,
           "note": ("numpy in/out per call (app.py:658-660), pooled library context; run_ms = the library's "
                    "ficp_run (run.upload + run.loop + run.result + run.other; run.gpu_loop is the device "
                    "loop inside run.loop)")}
    return out


def app_scale_join(device, with_cpu=True):
    """The production caller's size: one Join per field plot of stand 10 (Data/2014 plots vs
    the Data/2019 stems, 2-D fallback, app.py:630-661), the 16 real plots kept as data in
    tests/golden/run_real_stand10.npz.  GPU path: FractionalICP(src, tgt).run() per plot (a
    new instance each, as join_plot does); CPU path beside it: the pinned C oracle, one
    thread, same plots.  The reference itself took 2.6-5.7 ms per plot in the build
    container (it cannot run on the GPU box)."""
    from coregistrationgame_amd import FractionalICP
    f = np.load(REPO / "tests" / "golden" / "run_real_stand10.npz")
    tgt = f["tgt"]
    plots = [f[f"{int(pid)}/src"] for pid in f["plot_ids"]]
    FractionalICP(plots[0], tgt, device=device).run()  # pool warm-up (not timed)
    per = []
    for rep in range(3):
        for src in plots:
            t0 = time.perf_counter()
            FractionalICP(src, tgt, device=device).run()
            per.append(1e3 * (time.perf_counter() - t0))
    out = {"plots": len(plots), "n_trees": [int(len(p)) for p in plots], "n_chm": int(len(tgt)), "match_dims": 2,
           "gpu_ms_per_join_median": float(np.median(per)), "gpu_ms_per_join_max": float(np.max(per)),
           "gpu_ms_per_join_min": float(np.min(per))}
    if with_cpu:
        orc = _oracle()
        cpu = []
        for rep in range(3):
            for src in plots:
                t0 = time.perf_counter()
                orc.run(src, tgt, nthreads=1)
                cpu.append(1e3 * (time.perf_counter() - t0))
        out.update({"cpu_oracle_ms_per_join_median": float(np.median(cpu)),
                    "cpu_oracle_ms_per_join_max": float(np.max(cpu)), "cpu_threads": 1,
                    "reference_ms_per_join_container": [2.6, 5.7]})
    return out


# ----------------------------------------------------------------------------- workloads
def bench_single(args, wl, rank, world, local, D, steps, warmup, with_cpu):
    """C3 / C2: one plot per rank (seed + rank), device-resident layers."""
    n, m, f, seed0, md, thr, max_it, desc = WORKLOADS[wl]
    plot = synth.make_plot(n, m, f, seed0 + rank, md=md)
    ctx = _lib.Context(local, {"auto": 0, "brute": 1, "grid": 2}[args.nn_mode])
    src0 = DevArray(ctx, plot.source.T)   # pristine source columns, resident
    src = DevArray(ctx, plot.source.T)    # working copy (x, y move)
    tgt = DevArray(ctx, plot.target.T)
    lam = [3.0, 0.95 if md == 3 else 1.3]

    def step():
        # the target first: its bbox report lands while the source's reset copy is queued
        ctx.set_target_device(tgt.col(0), tgt.col(1), tgt.col(2) if md == 3 else 0, m, md)
        src.copy_from(src0, cols=2)  # x, y restored in one copy
        return ctx.run_device(src.col(0), src.col(1), src.col(2) if md == 3 else 0, n, lam, thr, max_it)

    def barrier():
        ctx.synchronize()
        if D is not None:
            D.barrier()

    for _ in range(warmup):
        step()
    ctx.profile_report()  # drop warmup records
    # NN launch timing: HIP events carried by the NN dispatches themselves on the library
    # stream, inside the timed region.  Each timed dispatch leaves ~5 us of idle queue
    # around it, so by default only the first timed step carries them.
    ctx.profile_enable(_lib.PROF_NN if args.nn_timing != "none" else 0)
    ps0 = ctx.path_stats()
    barrier()
    t0 = time.perf_counter()
    fits = calls = timed_calls = reused = 0
    for s_i in range(steps):
        st = step()
        fits += st["n_fits"]
        calls += st["n_nn_calls"]
        reused += st.get("n_nn_reused", 0)
        if args.nn_timing == "all" or (args.nn_timing == "first" and s_i == 0):
            # NN launches that searched: a later stage's head reuses the previous call's
            # outputs (its launch is a no-op, kept in nn["ms"]: conservative)
            timed_calls += st["n_nn_calls"] - st.get("n_nn_reused", 0)
        if s_i == 0 and args.nn_timing == "first":
            ctx.profile_enable(0)
    barrier()
    dt = time.perf_counter() - t0
    ps1 = ctx.path_stats()
    ctx.profile_enable(0)
    prof = json.loads(ctx.profile_report())
    # sustained: the same step back to back for --sustain-s seconds after the timed region
    # (not part of `value`): its rate beside the K-step one, and seconds of busy GPU that a
    # sampling utilisation monitor can see (the K timed steps last ~1.2 ms each)
    sus = None
    if args.sustain_s > 0 and wl == "c3":
        barrier()
        t1 = time.perf_counter()
        k_s = f_s = 0
        while True:
            f_s += step()["n_fits"]
            k_s += 1
            if k_s % 64 == 0:
                ctx.synchronize()
                if time.perf_counter() - t1 >= args.sustain_s:
                    break
        barrier()
        ds = time.perf_counter() - t1
        sus = {"value": f_s / ds, "unit": "iterations/s", "seconds": ds, "steps": k_s,
               "note": "rank-local: the timed step back to back after the timed region, not part of value"}
    dt_max, fits_all, calls_all, reused_all = dt, fits, calls, reused
    if D is not None:
        dt_max = D.max([dt])[0]
        fits_all, calls_all, reused_all = D.sum([fits, calls, reused])
    out = None
    if rank == 0:
        nn = prof.get("nn_grid") or prof.get("nn_brute") or {"count": 0, "ms": 0.0}
        # per real NN call: the device loop also enqueues a few no-op iterations past the
        # end of each run (their early-exit launches are in nn["ms"]: conservative)
        avg_ms = nn["ms"] / max(timed_calls, 1)
        bytes_launch = nn_bytes_per_launch(n, m, md)
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        # the C3 NN's two kernels together (k_nn_grid + k_nn_grid_q, tools/pmc_summary.py)
        traffic = (pmc_traffic(("k_nn_grid+q<3", "k_nn_grid<3") if md == 3 else ("k_nn_grid+q<2", "k_nn_grid<2"), "c3")
                   if wl == "c3" else None)
        ib = iteration_bytes(n, m, md, n)
        out = {
            "metric": METRIC, "value": fits_all / dt_max, "unit": "iterations/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": 1e3 * dt_max / steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic (SURVEY.md §8(d) generator, seed {seed0}+rank, geo-referenced)",
            "config": {"workload": desc, "n_trees": n, "n_chm": m, "inlier_fraction": f, "match_dims": md,
                       "plots_per_rank": 1, "parallelism": f"{world} independent plots (1 per GPU)",
                       "nn": args.nn_mode},
            "iterations_per_step": fits_all / steps / world,
            "nn_calls_per_step": calls_all / steps / world,
            # correspondences searched per second: a later stage's head answers its NN call
            # from the previous call's outputs (the source has not moved, ficp.py:151-153),
            # so that call is not counted; the count of every call, reused included, beside it
            "correspondences_per_s": (calls_all - reused_all) * n / dt_max,
            "correspondences_per_s_incl_reused": calls_all * n / dt_max,
            "nn_calls_reused_per_step": reused_all / steps / world,
            # fraction calls per run decided by the one-launch window path
            # and those that fell back to the full selection
            "selection_paths": {"fraction_calls_per_run": calls / steps,
                                "window_calls_per_run": (ps1["win_calls"] - ps0["win_calls"]) / steps,
                                "window_fallbacks_per_run": (ps1["win_retries"] - ps0["win_retries"]) / steps},
            "roofline": roofline(achieved, traffic, {
                "kernel": "k_nn_grid (fused apply + exact 1-NN)", "avg_launch_us": avg_ms * 1e3,
                "launches": timed_calls, "timed_launches_incl_noop": nn["count"],
                "algorithmic_bytes_per_launch": bytes_launch}),
            "kernel_ms": prof,
            "sustained": sus,
            # the whole loop body against SURVEY.md §8(d)'s per-iteration bytes (k = n: the
            # upper bound of the fit term), beside the dominant kernel's line
            "iteration_roofline": {"bytes_per_iteration": ib, "achieved": ib * fits_all / dt_max / 1e9,
                                   "unit": "GB/s", "peak": HBM_PEAK_GBS,
                                   "frac": ib * fits_all / dt_max / 1e9 / HBM_PEAK_GBS},
        }
    for a in (src0, src, tgt):
        a.free()
    ctx.close()
    if rank == 0 and world == 1 and with_cpu:
        # the host-side measurements first: the CPU baseline's OpenMP threads keep spinning
        # after their regions and, under the job's CPU quota, slowed the host path ~2x
        if wl == "c3":
            out["host_path"] = host_path_cost(plot, local)
            out["app_scale_join"] = app_scale_join(local)
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(plot, threads)
    elif out is not None:
        out["cpu_baseline"] = None
    return out


def bench_batch(args, rank, world, local, D, steps, warmup, with_cpu, share_of=0):
    """C4: the batch is dealt over ranks (shard.deal_plots); each rank runs its plots in
    one ficp_run_batch_device per step; no collective on the data path.  share_of = N > 0
    (one process): run only the plots rank 0 gets when the batch is dealt over N ranks."""
    from coregistrationgame_amd import shard
    n, m, f, seed0, md, thr, max_it, desc = WORKLOADS["batch"]
    nplots = args.plots or BATCH_PLOTS
    deal = shard.deal_plots(np.full(nplots, float(n) * m), share_of or world)
    mine = deal[0 if share_of else rank]
    plots = [_batch_plot(n, m, f, seed0 + int(p), md) for p in mine]
    ctx = _lib.Context(local)
    so = np.zeros(len(plots) + 1, np.int64)
    to = np.zeros(len(plots) + 1, np.int64)
    so[1:] = np.cumsum([len(pl.source) for pl in plots])
    to[1:] = np.cumsum([len(pl.target) for pl in plots])
    S = np.concatenate([pl.source for pl in plots])
    T = np.concatenate([pl.target for pl in plots])
    src0 = DevArray(ctx, S.T)
    src = DevArray(ctx, S.T)
    tgt = DevArray(ctx, T.T)
    lam = [3.0, 0.95 if md == 3 else 1.3]

    def step():
        src.copy_from(src0, cols=2)
        return ctx.run_batch_device(so, src.col(0), src.col(1), src.col(2) if md == 3 else 0, to,
                                    tgt.col(0), tgt.col(1), tgt.col(2) if md == 3 else 0, md, lam, thr, max_it)

    def barrier():
        ctx.synchronize()
        if D is not None:
            D.barrier()

    for _ in range(warmup):
        step()
    ctx.profile_report()
    # kernel timing: HIP events around the batch kernels of the first timed step only
    # (each event record leaves a few us of idle queue)
    ctx.profile_enable(_lib.PROF_NN | _lib.PROF_FRAC | _lib.PROF_FIT)
    barrier()
    t0 = time.perf_counter()
    fits = calls = calls0 = 0
    last = None
    dt0 = 0.0
    for s_i in range(steps):
        last = step()
        fits += int(last["n_fits"].sum())
        calls += int(last["n_nn_calls"].sum())
        if s_i == 0:
            ctx.profile_enable(0)
            calls0 = calls
            dt0 = time.perf_counter() - t0
    barrier()
    dt = time.perf_counter() - t0
    ctx.profile_enable(0)
    prof = json.loads(ctx.profile_report())
    dt_max, fits_all, calls_all = dt, fits, calls
    if D is not None:
        dt_max = D.max([dt])[0]
        fits_all, calls_all = D.sum([fits, calls])
        # one all-gather of the per-plot records, outside the timed region
        shard.gather_plot_stats(deal, last, rank, device=D.dev)
    out = None
    if rank == 0:
        nn = prof.get("nn_grid_batch") or {"count": 0, "ms": 0.0, "wall_ms": 0.0}
        # algorithmic bytes of every plot-NN call this rank made in the first timed step
        # over the wall-clock time the NN kernels held the GPU in it: the union of the NN
        # launches' intervals (the two sub-batch streams run concurrently, so their summed
        # launch times overstate it); converged plots drop out of later launches
        nn_bytes = calls0 * nn_bytes_per_launch(n, m, md)
        nn_wall = nn.get("wall_ms", nn["ms"])
        achieved = nn_bytes / (nn_wall * 1e-3) / 1e9 if nn_wall > 0 else 0.0
        ib = iteration_bytes(n, m, md, n)
        out = {
            "metric": METRIC, "value": fits_all / dt_max, "unit": "iterations/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": 1e3 * dt_max / steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic (SURVEY.md §8(d) generator, seeds {seed0}+plot, geo-referenced)",
            "config": {"workload": desc, "plots": nplots, "plots_per_rank": len(mine), "n_trees": n,
                       "n_chm": m, "inlier_fraction": f, "match_dims": md,
                       "parallelism": f"plots dealt over {world} GPU(s), no data-path collective"},
            "iterations_per_step": fits_all / steps,
            "nn_calls_per_step": calls_all / steps,
            "correspondences_per_s": calls_all * n / dt_max,
            "roofline": roofline(achieved, pmc_traffic("k_nn_grid_batch", "batch"), {
                "kernel": "k_nn_grid_batch (fused apply + exact 1-NN, all live plots)",
                "avg_launch_us": 1e3 * nn["ms"] / max(nn["count"], 1), "launches": nn["count"],
                "nn_wall_ms": nn_wall, "nn_summed_launch_ms": nn["ms"],
                "step_ms_first": 1e3 * dt0,
                "algorithmic_bytes_per_plot_call": nn_bytes_per_launch(n, m, md),
                "note": "rank 0, first timed step: algorithmic bytes of its plot-NN calls / the union "
                        "of the NN launches' intervals on both sub-batch streams (no-op launches past "
                        "convergence included)"}),
            "kernel_ms": prof,
            "iteration_roofline": {"bytes_per_iteration": ib, "achieved": ib * fits_all / dt_max / 1e9,
                                   "unit": "GB/s", "peak": HBM_PEAK_GBS,
                                   "frac": ib * fits_all / dt_max / 1e9 / HBM_PEAK_GBS,
                                   "note": "per plot-iteration, SURVEY.md §8(d) bytes at 10k x 10k"},
        }
    for a in (src0, src, tgt):
        a.free()
    ctx.close()
    if out is not None:
        if world == 1 and with_cpu:
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline_batch(plots, threads)
        else:
            out["cpu_baseline"] = None
    return out


_PLOTS = {}


def _batch_plot(n, m, f, seed, md):
    """C4 plots are generated once per process (the shares reuse the full batch's)."""
    key = (n, m, f, seed, md)
    if key not in _PLOTS:
        _PLOTS[key] = synth.make_plot(n, m, f, seed, md=md)
    return _PLOTS[key]


def batch_shares(args, local, full):
    """The per-rank shares of the north star's 1/2/4/8-GPU batch line, on this one GPU: the
    plots rank 0 gets when the 1024 plots are dealt over N = 2, 4, 8 ranks (512, 256, 128
    plots), each timed alone.  A rank of an N-GPU job runs exactly that share with no
    data-path collective, so share rate x N is the job's rate before the one all-gather of
    the per-plot records (shard.gather_plot_stats) and any host-side contention."""
    out = {"1024": {"plots": full["config"]["plots_per_rank"], "plot_iterations_per_s": full["value"],
                    "ms_per_step": full["ms_per_step"], "kernel_ms": full["kernel_ms"]}}
    per_gpu_full = full["value"]
    for N in (2, 4, 8):
        b = bench_batch(args, 0, 1, local, None, max(5, args.steps), 2, False, share_of=N)
        out[str(BATCH_PLOTS // N)] = {
            "share_of_n_gpus": N, "plots": b["config"]["plots_per_rank"],
            "plot_iterations_per_s": b["value"], "ms_per_step": b["ms_per_step"],
            "kernel_ms": b["kernel_ms"], "vs_1024_per_gpu": b["value"] / per_gpu_full,
            "implied_job_rate": b["value"] * N}
    return out


def bench_c5(args, rank, world, local, D, steps, warmup):
    """C5: the CHM layer is split in contiguous row shards over the ranks;
    every NN call merges the shards with two all-reduces over RCCL.  One plot for the whole
    job: value = its loop bodies per second ("scaling": "strong")."""
    from coregistrationgame_amd.partitioned import PartitionedFICP
    n, m, f, seed0, md, thr, max_it, desc = WORKLOADS["c5"]
    if args.c5_size:
        n = m = args.c5_size
    plot = synth.make_plot(n, m, f, seed0, md=md)  # same plot on every rank (replicated source)
    part = PartitionedFICP(plot.source, plot.target, threshold=thr, max_iterations=max_it,
                           device=local, local_shards=args.local_shards, mode=args.c5_mode)
    for _ in range(warmup):
        part.run_resident(lambda0=3.0)

    def barrier():
        import torch
        torch.cuda.synchronize()
        if D is not None:
            D.barrier()

    barrier()
    t0 = time.perf_counter()
    fits = calls = 0
    for _ in range(steps):
        st = part.run_resident(lambda0=3.0)
        fits += st["n_fits"]
        calls += st["n_nn_calls"]
    barrier()
    dt = time.perf_counter() - t0
    if D is not None:
        dt = D.max([dt])[0]
    part.close()
    if rank != 0:
        return None
    return {
        "metric": METRIC, "value": fits / dt, "unit": "iterations/s", "n_gpus": world,
        "steps": steps, "warmup": warmup, "ms_per_step": 1e3 * dt / steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (SURVEY.md §8(d) generator, seed {seed0}, geo-referenced)",
        "config": {"workload": desc, "n_trees": n, "n_chm": m, "inlier_fraction": f, "match_dims": md,
                   "shards": world * args.local_shards, "mode": args.c5_mode,
                   "parallelism": (f"CHM layer in {world * args.local_shards} row shards over {world} GPU(s); "
                                   "2 all-reduces (d2 MIN, idx MIN, 12 B per tree) per NN call"
                                   if args.c5_mode == "target" else
                                   f"tree rows in {world * args.local_shards} ranges over {world} GPU(s), layer "
                                   "replicated; per NN call: range MAX (16 B), histogram SUM (128 KB), "
                                   "candidate and fit-sum all-gathers")},
        "iterations_per_step": fits / steps, "nn_calls_per_step": calls / steps,
        "correspondences_per_s": calls * n / dt, "roofline": None, "cpu_baseline": None,
    }


def _dry_deal(args, rank, world, D):
    """The batch's plot deal, checked: every plot dealt once, the end-of-run all-gather
    of the per-plot records back in batch order.  Returns rank 0's config fields."""
    from coregistrationgame_amd import shard
    nplots = args.plots or BATCH_PLOTS
    deal = shard.deal_plots(np.full(nplots, 1.0), world)
    mine = deal[rank]
    counts = D.sum([len(mine)]) if D is not None else [len(mine)]
    per_rank = [len(mine)]
    gather_ok = True
    if D is not None:
        # every rank's plot count, and its plot ids' sum, as one SUM of one-hot vectors
        oh = [0.0] * (2 * world)
        oh[rank], oh[world + rank] = float(len(mine)), float(np.sum(mine))
        red = D.sum(oh)
        per_rank = [int(v) for v in red[:world]]
        id_sums = [int(v) for v in red[world:]]
        assert sum(id_sums) == nplots * (nplots - 1) // 2  # every plot id dealt exactly once
        # the end-of-run all-gather of the per-plot records, back in batch order
        rec = np.zeros(len(mine), _lib.PLOT_STATS_DTYPE)
        rec["k_last"] = mine
        rec["n_nn_calls"] = rank
        allrec = shard.gather_plot_stats(deal, rec, rank, device=D.dev)
        owner = np.empty(nplots, np.int64)
        for r_, ids in enumerate(deal):
            owner[ids] = r_
        gather_ok = bool(np.array_equal(allrec["k_last"], np.arange(nplots))
                         and np.array_equal(allrec["n_nn_calls"], owner))
        assert gather_ok
    return {"workload": "batch", "plots": nplots, "plots_dealt": int(counts[0]),
            "plots_per_rank": per_rank, "gather_in_order": gather_ok}


def bench_dry(args, wl, rank, world, D, steps, warmup):
    """No GPU work: the launcher, the process group, the plot deal, the timed-region
    bracket with max-over-ranks, the end-of-run all-gather and the report -- with the
    same keys as the real line (c3: `value` + the `batch` key at every N)."""
    if D is not None:
        D.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        pass
    if D is not None:
        D.barrier()
    dt = max(time.perf_counter() - t0, 1e-9)
    dt_max = D.max([dt])[0] if D is not None else dt
    deal = _dry_deal(args, rank, world, D) if wl in ("batch", "c3") else None
    if rank != 0:
        return None
    base = {"metric": METRIC, "value": 0.0, "unit": "iterations/s", "n_gpus": world, "steps": steps,
            "warmup": warmup, "ms_per_step": 1e3 * dt_max / max(steps, 1), "higher_is_better": True,
            "vs_baseline": None, "dtype": "f64", "data": "none (dry run)", "dry_run": True,
            "roofline": None, "cpu_baseline": None}
    if wl == "batch":
        return dict(base, scaling="strong", config=deal)
    out = dict(base, scaling="weak",
               config={"workload": wl, "plots_per_rank": 1,
                       "parallelism": f"{world} independent plots (1 per GPU)"})
    if deal is not None and not args.no_extra:
        out["batch"] = dict(base, scaling="strong", config=deal)
    return out


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)  # (C3: ~1.2 ms per step; 10 were noisy)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sustain-s", type=float, default=4.0,
                    help="C3: seconds of back-to-back steps after the timed region (`sustained`; 0: none)")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS),
                    help="default: c3 at every N (the C4 batch rides along as the `batch` key)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the extra figures (`batch`/`batch_shares` on the c3 line, "
                         "`c3_replicas` on the batch line)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = $OMP_NUM_THREADS or min(16, host cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nn-timing", default="first", choices=["first", "all", "none"],
                    help="timed steps whose NN dispatches carry HIP events")
    ap.add_argument("--nn-mode", default="grid", choices=["auto", "brute", "grid"])
    ap.add_argument("--plots", type=int, default=0, help="batch workload: number of plots (default 1024)")
    ap.add_argument("--c5-size", type=int, default=0, help="c5 workload: trees = stems (default 8M)")
    ap.add_argument("--local-shards", type=int, default=1, help="c5 workload: shards per GPU")
    ap.add_argument("--c5-mode", default="source", choices=["source", "target"],
                    help="c5 workload: split the tree rows (source) or the CHM layer (target)")
    ap.add_argument("--dry-run", action="store_true", help="no GPU work (launcher/process-group check)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"])
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    wl = args.workload
    backend = args.backend if args.backend != "auto" else ("gloo" if args.dry_run else "nccl")
    D = Dist(world, local, backend) if world > 1 else None
    ranks_seen = D.world if D is not None else 1

    if args.dry_run:
        out = bench_dry(args, wl, rank, world, D, args.steps, args.warmup)
    elif wl == "batch":
        out = bench_batch(args, rank, world, local, D, args.steps, args.warmup, not args.no_cpu_baseline)
        if not args.no_extra and world > 1:
            rep = bench_single(args, "c3", rank, world, local, D, args.steps, args.warmup, False)
            if out is not None:
                out["c3_replicas"] = {k: rep[k] for k in ("value", "unit", "ms_per_step", "scaling", "config",
                                                          "iterations_per_step", "roofline", "iteration_roofline")}
    elif wl == "c5":
        out = bench_c5(args, rank, world, local, D, args.steps, args.warmup)
    else:
        out = bench_single(args, wl, rank, world, local, D, args.steps, args.warmup, not args.no_cpu_baseline)
        if not args.no_extra and wl == "c3":
            # the C4 strong-scaling batch at every N: the 1024 plots dealt over the ranks
            b = bench_batch(args, rank, world, local, D, max(3, args.steps // 2), 1, False)
            if out is not None:
                out["batch"] = {k: b[k] for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "scaling",
                                                  "config", "iterations_per_step", "nn_calls_per_step",
                                                  "correspondences_per_s", "roofline", "iteration_roofline",
                                                  "kernel_ms")}
                if world == 1:
                    out["batch_shares"] = batch_shares(args, local, b)
    if out is not None:
        out["ranks_seen"] = ranks_seen
        print(json.dumps(out), flush=True)
    if D is not None:
        D.close()


if __name__ == "__main__":
    main()
