"""round_amd — MI355X-native batched Heard-Of executor and Spec checker for PSync.

The product is the C-ABI library round_amd/libpsg.so (HIP kernels for gfx950,
include/psg.h). This package holds its ctypes binding (round_amd.lib) and a
host-side mirror of the reference's Algorithm/Round plugin interface
(round_amd.psync).
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
