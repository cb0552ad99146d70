"""Drop-in module: `from ficp import FractionalICP` (app.py:20, tests/test_ficp.py:9).

Re-exports the MI355X engine's FractionalICP, which keeps the reference class
surface of ficp.py:5-154 (see coregistrationgame_amd/ficp.py).
"""
from coregistrationgame_amd.ficp import FractionalICP  # noqa: F401

__all__ = ["FractionalICP"]
