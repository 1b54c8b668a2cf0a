"""dpathsim -- MI355X-native APVPA PathSim engine (drop-in for DPathSim_APVPA.py's hot path).

Host side in Python (this package) over the C ABI of libdpathsim.so
(include/dpathsim.h, HIP kernels for gfx950).  See DESIGN.md.
"""
from .graph import APTPA, APVPA, METAPATHS, Graph, MetaPath, TypedTables  # noqa: F401

__all__ = ["Graph", "MetaPath", "TypedTables", "APVPA", "APTPA", "METAPATHS"]
