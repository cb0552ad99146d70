"""CPU-side checks of the drop-in boundary (no GPU needed).

* libficp.so loads and exports every entry point include/ficp.h declares;
* the facade keeps the reference's constructor contract, attributes and empty-input
  behaviour (ficp.py:34-44, 56-57, 66-68, 75-77, 125-126; tests/test_ficp.py:104-126);
* without a GPU the compute methods raise instead of silently running on the CPU.
"""
import ctypes
import subprocess

import numpy as np
import pytest

from coregistrationgame_amd import FractionalICP, _lib, synth


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert L.ficp_version() == 100


def test_exported_symbols_match_header_exactly():
    """nm: the .so exports no extern "C" ficp_* symbol the header does not declare."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if ln.split()[-1].startswith("ficp_")})
    assert exported == _lib.header_symbols()


def test_constructor_contract():
    src = synth.make_cloud(20, 1)
    icp = FractionalICP(src, src[:10, :2])
    assert icp.match_dims == 2
    assert (icp.lambda_val, icp.threshold, icp.max_iterations, icp.allow_reflection) == (3.0, 1e-6, 1000, False)
    assert icp.source is not src and icp.source.dtype == np.float64
    assert FractionalICP(src, src).match_dims == 3
    with pytest.raises(ValueError, match=r"source and target must be 2D arrays \(N, D\)\."):
        FractionalICP(np.zeros(3), src)
    with pytest.raises(ValueError, match=r"source and target must be 2D arrays \(N, D\)\."):
        FractionalICP(src, np.zeros((2, 2, 2)))


def test_empty_source_returns_empty_alignment():
    """tests/test_ficp.py:104-112 (no device work needed)."""
    source = np.empty((0, 3))
    target = synth.make_cloud(n=5, seed=42)
    icp = FractionalICP(source.copy(), target)
    aligned = icp.run()
    assert aligned.shape == source.shape
    assert aligned.size == 0
    assert icp.lambda_val == 0.95


def test_empty_target_produces_no_correspondences():
    """tests/test_ficp.py:115-126"""
    source = synth.make_cloud(n=4, seed=24)
    target = np.empty((0, 3))
    icp = FractionalICP(source.copy(), target)
    corr, dist = icp.find_correspondences(source, target)
    frac, num = icp.find_optimal_fraction(corr, dist)
    assert corr.shape == (0, target.shape[1])
    assert dist.size == 0
    assert frac == 0.0 and num == 0
    out = icp.run()
    np.testing.assert_array_equal(out, source)
    assert icp.frmsd(0.5, 0, source[:0], source[:0]) == float("inf")


def test_no_cpu_fallback_without_gpu():
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    icp = FractionalICP(synth.make_cloud(50, 2), synth.make_cloud(50, 3))
    with pytest.raises(_lib.FicpError):
        icp.run()
    with pytest.raises(_lib.FicpError):
        icp.find_correspondences(icp.source, icp.target)


def test_stats_struct_layout():
    """ctypes mirror of struct ficp_stats has the C layout (offsets of the trace pointers)."""
    assert ctypes.sizeof(_lib.Stats) == 4 * 4 + 8 + 16 + 72 + 8 + 8 + 5 * 8 + 4 * 8 + 8
    assert _lib.Stats.host_ms.offset == 4 * 4 + 8 + 16 + 72 + 8 + 8 + 5 * 8


def test_copy_array_is_np_array_semantics():
    """_lib.copy_array stands in for ficp.py:34-35's np.array(x, dtype=float): a float64
    copy for every input kind (pooled pinned memory only where a GPU runtime gives it)."""
    from coregistrationgame_amd import _lib
    big = np.random.default_rng(0).random((50_000, 3))  # 1.2 MB: the pooled size class
    for x in (big, big[:, :2], big.astype(np.float32), [[1, 2], [3, 4]], np.arange(6).reshape(3, 2)):
        y = _lib.copy_array(x)
        ref = np.array(x, dtype=float)
        assert y.dtype == np.float64 and y.shape == ref.shape and np.array_equal(y, ref)
        if isinstance(x, np.ndarray):
            assert not np.shares_memory(y, x)
