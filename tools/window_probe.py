"""Window probe (tools only): how many rows lie between consecutive FRMSD thresholds of the
C3 loop, and how flat the FRMSD curve is around each minimum.  Steps the reference loop
(ficp.py:122-154) with the CPU oracle's NN / fit / apply and numpy prefix sums, and prints
per NN call: k, the threshold distance, the rows between the previous and this threshold,
and the rows on each side of k whose FRMSD lies within 1e-9 / 1e-6 (relative) of the min.

usage: python tools/window_probe.py [n] [lam0]
"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
import ficp_oracle as orc  # noqa: E402
from coregistrationgame_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    p = synth.make_plot(n, n, 0.6, 1_000_000, md=3)
    src = p.source.copy()
    tgt = p.target
    N = len(src)
    prev_t = None
    call = 0
    for stage, lam in enumerate((3.0, 0.95)):
        cur = None
        it = 0
        first = True
        while True:
            idx, d, _ = orc.nn(src, tgt, 3, nthreads=8)
            order = np.argsort(d, kind="stable")
            ds = d[order]
            S = np.cumsum(ds * ds)
            k = np.arange(1, N + 1, dtype=np.float64)
            f = (1.0 / (k / N) ** lam) * np.sqrt(S / k)
            kb = int(np.argmin(f)) + 1
            fb = f[kb - 1]
            dt = ds[kb - 1]
            near9 = np.nonzero(f <= fb * (1 + 1e-9))[0]
            near6 = np.nonzero(f <= fb * (1 + 1e-6))[0]
            between = None
            if prev_t is not None:
                lo, hi = min(prev_t, dt), max(prev_t, dt)
                between = int(np.count_nonzero((d >= lo) & (d <= hi)))
            # rows within +-x (relative) of the threshold distance
            w = [int(np.count_nonzero(np.abs(d - dt) <= x * dt)) for x in (1e-4, 1e-3, 1e-2)]
            print(f"call {call:2d} st {stage} k={kb} d_t={dt:.9f} moved_rows={between} "
                  f"near1e-9=[{near9.min() + 1 - kb},{near9.max() + 1 - kb}] "
                  f"near1e-6=[{near6.min() + 1 - kb},{near6.max() + 1 - kb}] "
                  f"rows(+-1e-4,1e-3,1e-2 rel)={w}", flush=True)
            prev_t = dt
            call += 1
            if first:
                first = False
                if kb == 0:
                    break
                cur = fb
            else:
                if cur - fb <= 1e-6:
                    break
                cur = fb
                it += 1
            sel = order[:kb]
            T = orc.fit_rigid2d(src[sel], tgt[idx[sel]])
            src = orc.apply_xy(src, T)


if __name__ == "__main__":
    main()
