#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration for the NN kernel's access width (8 B per lane):
ficp_apply_device over two columns of n doubles reads exactly 16 n bytes and writes 16 n
bytes with 8-B-per-lane coalesced loads and stores (k_apply_inplace).  Run under
rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE); the ratio counter / known bytes is the
correction MI355X_MICROARCH.md asks to measure before trusting an absolute."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from coregistrationgame_amd import _lib  # noqa: E402

n = 1 << 24  # 2 x 128 MiB: past the 256 MiB Infinity Cache together with the writes
ctx = _lib.Context(0, 0)
ptrs = []
for _ in range(2):
    p = _lib.C.c_void_p()
    _lib._check(_lib.lib().ficp_dev_alloc(ctx.h, 8 * n, _lib.C.byref(p)))
    h = np.random.default_rng(1).random(n)
    _lib._check(_lib.lib().ficp_memcpy_h2d(ctx.h, p, h.ctypes.data_as(_lib.C.c_void_p), 8 * n))
    ptrs.append(p.value)
T = np.array([1, 0, 1e-3, 0, 1, -1e-3, 0, 0, 1], dtype=np.float64)
for _ in range(4):
    ctx.apply_device(ptrs[0], ptrs[1], n, T)
ctx.synchronize()
print({"kernel": "k_apply_inplace", "read_bytes": 16 * n, "write_bytes": 16 * n})
