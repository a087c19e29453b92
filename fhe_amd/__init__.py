"""fhe_amd -- MI355X (gfx950) TFHE gate-bootstrapping engine.

Python host-side mirror over the C-ABI in include/fhe_hip.h (libfhe_amd.so,
built in-tree by ``fhe_amd.build.build()``).  The compute path is the HIP
library only: there is no CPU fallback, and every entry point raises if the
native library is missing or returns an error.
"""
from ._lib import FheHipError, lib, lib_path  # noqa: F401
from .ntt import NttPlan  # noqa: F401

__all__ = ["FheHipError", "lib", "lib_path", "NttPlan"]
