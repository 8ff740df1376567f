"""lbm_amd -- host side of the MI355X-native D2Q9-BGK engine.

The compute path is liblbm_hip.so (hand-written gfx950 HIP behind the C ABI
in include/lbm_hip.h); this package only binds it (native), mirrors the
reference host's problem I/O (io) and restates the reference gate (check).
Importing it needs no GPU; native.load_library() is called on first use.
"""
from . import check, io, native  # noqa: F401
from .io import Params, init_cells, read_obstacles, reynolds_number, write_average_velocities, write_results  # noqa: F401

__all__ = ["io", "check", "native", "Params", "read_obstacles", "init_cells", "reynolds_number",
           "write_average_velocities", "write_results"]
