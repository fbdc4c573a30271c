"""The C-ABI library: loads, exports every symbol include/sirilgpu.h declares,
and reports the absence of a device loudly (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "sirilgpu.h")).read()
    # function declarations: a return type at line start, then the name and "("
    return sorted(set(re.findall(r"^(?:int|void|long|double|float|uint16_t|const char|sgpu_context)\s*\*?\s*(sgpu_[a-z_0-9]+)\(", txt, re.M)))


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


def test_row_band_partition_matches_python():
    """sgpu_row_bands (the C-ABI multi-device split) == distributed.row_bands,
    and the bands cover the block exactly (stacking_blocks_test.c:50-63 style)."""
    from siril_amd.distributed import row_bands
    from siril_amd.stacking import row_bands_c
    for rows in (1, 2, 7, 100, 4000, 4001):
        for parts in (1, 2, 3, 4, 8):
            b = row_bands_c(rows, parts)
            assert b == row_bands(rows, parts)
            assert b[0][0] == 0 and b[-1][1] == rows
            assert all(b[i][1] == b[i + 1][0] for i in range(parts - 1))
            assert max(y1 - y0 for y0, y1 in b) - min(y1 - y0 for y0, y1 in b) <= 1


def test_multi_init_without_device_is_an_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from siril_amd import SgpuError
    from siril_amd.stacking import MultiContext
    with pytest.raises(SgpuError):
        MultiContext([0, 1])
