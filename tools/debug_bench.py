"""Repeat the bench step with a sync + state check after every run (fault isolation)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import bench
from coregistrationgame_amd import _lib, synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
prof = int(sys.argv[3]) if len(sys.argv) > 3 else 0
p = synth.make_plot(n, n, 0.6, 1_000_000, md=3)
ctx = _lib.Context(0, 2)
src0 = [bench.DevArray(ctx, p.source[:, j]) for j in range(3)]
src = [bench.DevArray(ctx, p.source[:, j]) for j in range(3)]
tgt = [bench.DevArray(ctx, p.target[:, j]) for j in range(3)]
if prof:
    ctx.profile_enable(prof)
for s in range(steps):
    t0 = time.perf_counter()
    src[0].copy_from(src0[0]); src[1].copy_from(src0[1])
    ctx.set_target_device(tgt[0].ptr, tgt[1].ptr, tgt[2].ptr, n, 3)
    st = ctx.run_device(src[0].ptr, src[1].ptr, src[2].ptr, n, [3.0, 0.95], 1e-6, 1000)
    ctx.synchronize()
    print(f"step {s}: {st['n_nn_calls']} NN calls, {st['n_fits']} fits, k={st['k_last']}, "
          f"{1e3*(time.perf_counter()-t0):.2f} ms, gpu {st['gpu_ms']:.2f} ms", flush=True)
if prof:
    print(ctx.profile_report())
