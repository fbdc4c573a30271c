"""siril_amd -- MI355X-native engine for Siril's per-pixel rejection stack.

The compute path is libsirilgpu.so (hand-written HIP for gfx950, C-ABI in
include/sirilgpu.h).  This package is the Python host layer over that ABI:
`stacking` mirrors Siril's stacking interface.  There is no CPU fallback.
"""
from . import stacking  # noqa: F401
from ._lib import LIB_PATH, SgpuError, lib  # noqa: F401
from .stacking import (Context, Normalization, Rejection, StackingArgs, StackResult,  # noqa: F401
                       stack_mean_with_rejection, stack_median)

__all__ = ["stacking", "Context", "Rejection", "Normalization", "StackingArgs", "StackResult",
           "stack_mean_with_rejection", "stack_median", "SgpuError", "lib", "LIB_PATH"]
