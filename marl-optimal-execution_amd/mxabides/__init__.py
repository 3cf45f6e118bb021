"""mxabides — MI355X-native vectorised ABIDES market step (host package).

The simulation runs in libmxa (HIP, gfx950); this package is the thin host layer that
mirrors the reference's entry points.  See DESIGN.md.
"""
from ._lib import CONFIG_IDS, MxaError, build_id, load  # noqa: F401
from .market import VecMarket  # noqa: F401

__all__ = ["VecMarket", "MxaError", "CONFIG_IDS", "build_id", "load"]
