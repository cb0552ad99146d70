"""coregistrationgame_amd -- MI355X-native Fractional ICP engine.

Drop-in for the reference's `ficp.FractionalICP` (ficp.py:5-154): see
`coregistrationgame_amd.ficp`.  Compute runs in libficp.so (HIP, gfx950) behind
the C ABI of include/ficp.h.
"""
from .batch import FractionalICPBatch  # noqa: F401
from .ficp import FractionalICP  # noqa: F401

__all__ = ["FractionalICP", "FractionalICPBatch"]
