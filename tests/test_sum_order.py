"""Summation order of the reference's `omp simd` reductions (CPU).

Siril sums with `#pragma omp simd reduction(+:...)` from 24 samples on in
siril_stats_float_sd (algos/statistics.h:93-101) and from 16 kept samples on
in mean_and_reject's mean (stacking/median_and_mean.c:1085-1090).  Its order
is the build's vectorised reduction, not the sequential one.  The oracle
restates the sequential order by default; or_set_simd_lanes selects a model
of the default x86-64 (SSE2) build's reduction order (oracle/stack_ref.c).

Two facts are checked on the sum-order stress columns of
tests/test_stack_gpu.py::test_sum_order_stress (inexact f64 sums: negative
values, near-mean ties, tiny and huge values):
  * every pixel the sorted path keeps (the per-pixel kernel logic compiled
    for the host, tests/hostsim) equals the oracle in BOTH orders: SumGuard's
    order-independence proof holds for the reference's SIMD order too;
  * the residue -- pixels whose result differs between the two orders -- is
    counted and printed; such pixels are always among the deferred ones, and
    for them the engine reproduces the sequential order.
"""
import ctypes as C

import numpy as np
import pytest

FP = C.POINTER(C.c_float)
IP = C.POINTER(C.c_int)


def _stress_frames(rng, n, cols):
    kind = rng.integers(0, 4, cols)
    lvl = np.where(kind == 0, 1e-3, np.where(kind == 1, 0.05, np.where(kind == 2, 1e-20, 3.0)))
    spread = np.where(kind == 3, 1e-6, 0.1) * lvl
    x = lvl[None, :] + spread[None, :] * rng.standard_normal((n, cols))
    x -= np.where(kind == 0, 1.1e-3, 0.0)[None, :]
    m = rng.random(x.shape) < 0.04
    x[m] += (rng.uniform(2, 8, int(m.sum())) * np.broadcast_to(np.abs(lvl)[None, :], x.shape)[m])
    big = rng.random(x.shape) < 0.002
    x[big] *= 1e6
    x = x.astype(np.float32)
    x[rng.random(x.shape) < 0.01] = 0
    return x


def residue(oracle, fr, rt, lanes=4, sig=(3.0, 3.0)):
    """(pixels, pixels whose output or rejection counts differ between the
    sequential and the lanes-wide SIMD order, outputs of both)."""
    try:
        seq = oracle.stack_rows(fr, rt, sig, output_norm=True, nthreads=8)
        oracle.set_simd_lanes(lanes)
        vec = oracle.stack_rows(fr, rt, sig, output_norm=True, nthreads=8)
    finally:
        oracle.set_simd_lanes(0)
    diff = (seq[0].view(np.uint32) != vec[0].view(np.uint32)) | (seq[1] != vec[1]) | (seq[2] != vec[2])
    return diff.size, int(diff.sum()), seq, vec


def test_simd_order_model_changes_only_order_dependent_sums(oracle):
    """The model is a pure re-association: on columns whose sums are exact
    (positive, narrow binade span) both orders agree bit for bit."""
    rng = np.random.default_rng(1)
    fr = (0.05 + 0.005 * rng.standard_normal((100, 8, 512))).astype(np.float32)
    fr = np.clip(fr, 1e-3, 1)
    for rt in (2, 5):
        _, bad, _, _ = residue(oracle, fr, rt)
        assert bad == 0
    # ... and it is not the identity on inexact sums: [2^60, 1, -2^60, 1] x 6
    # sums to 1 sequentially, to 12 in 4 lanes ((l0 + l2) + (l1 + l3))
    x = np.ascontiguousarray(np.array([2.0 ** 60, 1.0, -2.0 ** 60, 1.0] * 6, np.float32))
    assert oracle.lib().or_sum_f(x.ctypes.data_as(FP), len(x)) == 1.0
    oracle.set_simd_lanes(4)
    try:
        assert oracle.lib().or_sum_f(x.ctypes.data_as(FP), len(x)) == 12.0
    finally:
        oracle.set_simd_lanes(0)


@pytest.mark.parametrize("n,rt", [(12, 5), (24, 2), (100, 5), (100, 2)])
def test_kept_pixels_are_order_independent(oracle, hostsim, n, rt):
    rng = np.random.default_rng(4242 + n + rt)
    cols = 1 << 15
    fr = _stress_frames(rng, n, cols).reshape(n, 1, cols)
    total, bad, seq, vec = residue(oracle, fr, rt)
    flat = np.ascontiguousarray(fr.reshape(n, cols))
    res = np.zeros(cols)
    a, b, st = (np.zeros(cols, np.int32) for _ in range(3))
    crit = np.zeros(1, np.float32)
    hostsim.sim_pixels(rt, flat.ctypes.data_as(FP), n, cols, 3.0, 3.0, crit.ctypes.data_as(FP), 0., 0.,
                       res.ctypes.data_as(C.POINTER(C.c_double)), a.ctypes.data_as(IP), b.ctypes.data_as(IP),
                       st.ctypes.data_as(IP))
    kept = st == 0
    got = res.astype(np.float32).view(np.uint32)
    for out, rl, rh, _ in (seq, vec):
        assert not (kept & (got != out.reshape(-1).view(np.uint32))).any()
        assert not (kept & ((a != rl.reshape(-1)) | (b != rh.reshape(-1)))).any()
    differ = (seq[0].view(np.uint32) != vec[0].view(np.uint32)).reshape(-1)
    assert not (differ & kept).any()                 # the residue lies in the deferred set
    print(f"simd-order residue N={n} rt={rt}: {bad} of {total} columns differ between the sequential and "
          f"the 4-lane order; {int((~kept).sum())} deferred")
