"""The C-ABI library: loads, exports every symbol include/sirilgpu.h declares,
and reports the absence of a device loudly (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "sirilgpu.h")).read()
    # function declarations: a return type at line start, then the name and "("
    return sorted(set(re.findall(r"^(?:int|void|long|double|float|const char)\s*\*?\s*(sgpu_[a-z_0-9]+)\(", txt, re.M)))


def test_header_symbols_exported():
    from siril_amd import _lib
    L = _lib.lib()
    declared = _declared()
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.EXPORTS)


def test_no_device_is_an_error_not_a_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from siril_amd import SgpuError, stacking
    from siril_amd._lib import lib
    assert lib().sgpu_device_count() == 0
    with pytest.raises(SgpuError) as e:
        stacking.Context(0)
    assert e.value.code == -20
