"""The CPU restatement (oracle/) pinned against the reference's own tests.

* rejection_test.c known answers (GESDT, PERCENTILE, LINEARFIT) through the
  restated apply_rejection_float / mean_and_reject;
* sorting.c:58-110 property: quickmedian agrees with the median of a full
  sort for every size 1..400 -- the float quickmedian, and the WORD
  quickmedian and histogram_median the reference's test itself runs.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "rejection_kats.json")))


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_rejection_kats(oracle, case):
    data = np.array(KATS[case["set"]], np.float32)
    mean, lo, hi = oracle.stack_column(data, case["rejection"], tuple(case["sig"]))
    assert (lo, hi) == tuple(case["rej"])
    assert abs(np.float32(mean) - np.float32(case["mean"])) <= case["tol"] * max(1.0, abs(case["mean"]))


def _median_sorted(a):
    s = np.sort(a)
    n = len(s)
    if n % 2:
        return float(s[(n - 1) // 2])
    return (float(s[n // 2 - 1]) + float(s[n // 2])) / 2.0


def test_quickmedian_matches_sort(oracle):
    # sorting.c:58-110 (that test uses WORD data; integers are exact in float too)
    rng = np.random.default_rng(0)
    for n in range(1, 401):
        a = rng.integers(0, 65535, n).astype(np.float32)
        qm = oracle.quickmedian(a)
        if n < 9 and n % 2 == 0:
            s = np.sort(a)
            expect = float(np.float32(s[n // 2 - 1] + s[n // 2])) / 2.0   # float add, sorting.c:512
        else:
            expect = _median_sorted(a)
        assert qm == expect, n


def _median_sorted_word(a):
    # median_from_sorted_array, sorting.c:37-43 (int sum of the two WORDs / 2.0)
    s = np.sort(a)
    n = len(s)
    if n % 2:
        return float(s[(n - 1) // 2])
    return (int(s[(n - 1) // 2]) + int(s[n // 2])) / 2.0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_word_medians_match_sort(oracle, seed):
    """sorting.c:45-98 (Sorting/Median): quickmedian(WORD) and
    histogram_median(WORD) both equal the median of a quicksort, sizes 1..400,
    data rand() % USHRT_MAX.  Covers the sortnet path (n < 9 for quickmedian,
    n < 10 for histogram_median, so case 9 of sortnet_median) and the
    Lomuto / histogram paths above."""
    rng = np.random.default_rng(100 + seed)
    for n in range(1, 401):
        a = rng.integers(0, 65535, n).astype(np.uint16)
        expect = _median_sorted_word(a)
        assert oracle.quickmedian_u16(a) == expect, ("quickmedian", n)
        assert oracle.histogram_median_u16(a) == expect, ("histogram_median", n)
    # ties and the extremes of the WORD range (values the rand() draw rarely
    # hits): the histogram's cumulative walk over repeated bins
    for n in range(1, 401):
        a = rng.choice(np.array([0, 1, 2, 65534, 65535], np.uint16), n)
        expect = _median_sorted_word(a)
        assert oracle.quickmedian_u16(a) == expect, ("quickmedian ties", n)
        assert oracle.histogram_median_u16(a) == expect, ("histogram_median ties", n)


def test_block_driver_matches_column(oracle):
    rng = np.random.default_rng(3)
    fr = (0.1 + 0.01 * rng.standard_normal((12, 3, 5))).astype(np.float32)
    fr[rng.random(fr.shape) < 0.05] = 0
    out, rl, rh, counts = oracle.stack_rows(fr, oracle.WINSORIZED, (3, 3), nthreads=2)
    tl = th = 0
    for y in range(3):
        for x in range(5):
            r, lo, hi = oracle.stack_column(fr[:, y, x], oracle.WINSORIZED, (3, 3))
            assert out[y, x] == np.float32(min(max(np.float32(r), 0), 1))
            assert (rl[y, x], rh[y, x]) == (lo, hi)
            tl += lo
            th += hi
    assert tuple(counts) == (tl, th)


def test_golden_vectors_regression(oracle):
    """Self-generated vectors (tests/golden/make_golden.py): the oracle must keep
    producing them (regression pin of the restatement itself)."""
    path = os.path.join(HERE, "golden", "columns.npz")
    g = np.load(path)
    cols, rtype, sig, expect, rej = g["cols"], g["rtype"], g["sig"], g["expect"], g["rej"]
    for i in range(len(cols)):
        n = int(g["n"][i])
        r, lo, hi = oracle.stack_column(cols[i, :n], int(rtype[i]), tuple(sig[i]),
                                        method=1 if rtype[i] == 16 else 0)
        assert np.float32(r) == expect[i] and (lo, hi) == tuple(rej[i]), i
