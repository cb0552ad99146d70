"""Golden fixtures for Plot.get_transform (trees.py:248-280) from the REFERENCE.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_transforms.py

The reference's Plot/Tree classes are imported from /root/reference purely to produce
input/expected-output vectors. Trees are loaded at (x, y) and moved by a known rigid
motion, with or without a flip (coordinate_flip). The reference's own get_transform
gives R, t. Writes transforms.npz: per case the loaded xy, the current xy, the flipped
flag, and R, t.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("FICP_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REF))

import trees as ref_trees  # noqa: E402  (reference, build container only)


def main():
    rng = np.random.default_rng(31)
    out = {}
    cases = 0
    for n in (1, 2, 3, 17, 120):
        for flip in (False, True):
            for geo in (False, True):
                p = ref_trees.Plot(cases, center=(0.0, 0.0))
                xy = rng.uniform(-15, 15, (n, 2)) + ((420000.0, 6483000.0) if geo else (0.0, 0.0))
                for i, (x, y) in enumerate(xy):
                    t = ref_trees.Tree(f"t{i}", float(x), float(y))
                    t.height = 10.0
                    p.append_tree(t)
                p.center = tuple(p.current_center)
                if flip:
                    p.coordinate_flip()
                th = rng.uniform(-0.3, 0.3)
                c, s = np.cos(th), np.sin(th)
                R = np.array([[c, -s], [s, c]])
                cur = np.array([[t.currentx, t.currenty] for t in p.trees]) @ R.T + rng.uniform(-3, 3, 2)
                cur += rng.normal(0, 0.05, cur.shape)
                p.update_tree_positions(cur)
                Rr, tr, fl = p.get_transform()
                key = f"c{cases}"
                out[f"{key}/xy"] = xy
                out[f"{key}/cur"] = np.array([[t.currentx, t.currenty] for t in p.trees])
                out[f"{key}/flipped"] = np.array(bool(fl))
                out[f"{key}/R"] = np.asarray(Rr, dtype=float)
                out[f"{key}/t"] = np.asarray(tr, dtype=float)
                cases += 1
    np.savez_compressed(HERE / "transforms.npz", **out)
    print(cases, "cases")


if __name__ == "__main__":
    main()
