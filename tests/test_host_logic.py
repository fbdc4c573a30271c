"""Host-side logic of the Python mirror (no device needed)."""
import numpy as np

from siril_amd import stacking as S


def test_round_to_int_half_away_from_zero():
    assert [S.round_to_int(v) for v in (0.5, 1.5, -0.5, -1.5, 2.4999, -2.5)] == [1, 2, -1, -2, 2, -3]


def test_shifts_from_registration():
    sh = S.shifts_from_registration([0.0, 1.49, -3.5, 10.0], offset0=2, upscale_at_stacking=False)
    assert sh.tolist() == [-2, -1, -6, 8]
    assert S.shifts_from_registration([1.25], upscale_at_stacking=True).tolist() == [3]


def test_gesd_critical_values_match_oracle(oracle):
    for n, s0, a in [(22, 0.32, 0.05), (25, 0.32, 0.05), (100, 0.32, 0.05), (100, 0.3, 0.05), (400, 0.1, 0.01)]:
        assert np.array_equal(S.gesd_critical_values(n, s0, a), oracle.gesd_critical_values(n, s0, a))


def test_params_marshalling():
    args = S.StackingArgs(S.Rejection.SIGMA, (2.0, 3.5), S.Normalization.ADDITIVE_SCALING,
                          scale=np.ones(4), offset=np.zeros(4), shiftx=np.arange(4))
    keep = S._Keep()
    p = S._params(args, S.METHOD_MEAN, 4, keep)
    assert p.type_of_rejection == 2 and p.normalize == 3
    assert abs(p.sig[0] - 2.0) < 1e-7 and abs(p.sig[1] - 3.5) < 1e-7
    assert p.shiftx[3] == 3 and p.scale[0] == 1.0 and not p.weights


def test_registration_matrices():
    from siril_amd import registration as R
    H = R.set_shifts(3.0, 5.0, top_down=False)
    assert R.translation_from_H(H) == (3.0, 5.0)
    assert R.translation_from_H(R.set_shifts(3.0, 5.0, top_down=True)) == (3.0, -5.0)


def test_row_bands_cover_the_image():
    """The properties src/tests/stacking_blocks_test.c checks for Siril's
    block planner (stack_compute_parallel_blocks), on the multi-GPU row bands:
    adjacent bands cover every row once, one band per rank, balanced."""
    from siril_amd.distributed import row_bands
    for h, world in [(1000, 1), (1000, 8), (4000, 8), (7, 3), (3, 8), (4001, 7)]:
        bands = row_bands(h, world)
        assert len(bands) == world
        y = 0
        for y0, y1 in bands:
            assert y0 == y and y1 >= y0
            y = y1
        assert y == h
        sizes = [b1 - b0 for b0, b1 in bands]
        assert max(sizes) - min(sizes) <= 1


def test_dft_oracle_recovers_shifts():
    from oracle import dft_ref
    from siril_amd import synth
    base = synth.star_field(64, 64, nstars=30)
    fr = synth.shifted_frames(base, [(0, 0), (5, -9), (-32, 32)])
    assert dft_ref.dft_shift(fr[0], fr[1])[:2] == (-5, 9)
    assert dft_ref.dft_shift(fr[0], fr[2])[:2] == (32, 32)      # -32 == 32 (mod 64), not > S/2
