"""Sort networks pruned to the real slots (stack_sorted_impl.h oem_sort<E, RS>,
rs_pick), checked on the host build of the kernels'
header: every compiled bound sorts a column whose slots >= RS are +Inf
padding exactly like the full network (= numpy's sort), including columns
with ties, zeros-as-missing (+Inf inside the real slots) and signed values,
and rs_pick never returns a bound below ceil(N / G)."""
import ctypes as C

import numpy as np
import pytest


def _bounds(E):
    return list(range(36, 65, 4)) if E == 64 else list(range(72, 129, 8))


@pytest.mark.parametrize("E", [64, 128])
def test_pruned_network_sorts_like_the_full_one(hostsim, E):
    S = hostsim
    S.sim_sort_rs.restype = C.c_int
    S.sim_sort_rs.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int]
    rng = np.random.default_rng(E)
    for rs in _bounds(E):
        for trial in range(40):
            v = np.full(E, np.inf, np.float32)
            kind = trial % 4
            if kind == 0:
                v[:rs] = rng.random(rs, dtype=np.float32)
            elif kind == 1:
                v[:rs] = rng.integers(0, 5, rs).astype(np.float32)          # heavy ties
            elif kind == 2:
                v[:rs] = rng.normal(size=rs).astype(np.float32)            # signed
            else:
                v[:rs] = rng.random(rs, dtype=np.float32)
                v[rng.integers(0, rs, rs // 3)] = np.inf                   # missing samples inside
            w = v.copy()
            assert S.sim_sort_rs(w.ctypes.data_as(C.POINTER(C.c_float)), E, rs) == 0
            np.testing.assert_array_equal(w, np.sort(v), err_msg=f"E={E} rs={rs} kind={kind}")


def test_rs_pick_bounds(hostsim):
    S = hostsim
    S.sim_rs_pick.restype = C.c_int
    S.sim_rs_pick.argtypes = [C.c_int, C.c_int, C.c_int]
    # (NP, G) shapes that have E = 64 or 128 slots per lane
    for NP, G in [(64, 1), (128, 1), (128, 2), (256, 2), (256, 4), (512, 4), (512, 8), (1024, 8)]:
        E = NP // G
        for N in range(NP // 2 + 1, NP + 1):
            rs = S.sim_rs_pick(E, G, N)
            need = -(-N // G)
            assert need <= rs <= E
            if rs < E:
                assert rs in _bounds(E)
    assert S.sim_rs_pick(32, 1, 20) == 32                                   # no variants below E = 64
