"""Residue of the reference's omp-simd summation order: on the
sum-order stress columns (tests/test_sum_order.py), the number of pixels whose
oracle result (mean bits or rejection counts) differs between the sequential
order and the L-lane vectorised-reduction model, L in {2, 4, 8}.  CPU only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import oracle as O  # noqa: E402
from test_sum_order import _stress_frames, residue  # noqa: E402

O.build()
total_cols = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
for n, rt in [(24, 2), (100, 5), (100, 2), (400, 5), (400, 2)]:
    rng = np.random.default_rng(4242 + n + rt)
    cols = total_cols if n < 400 else total_cols // 4
    chunk = 1 << 16
    res = {L: 0 for L in (2, 4, 8)}
    for c0 in range(0, cols, chunk):
        fr = _stress_frames(rng, n, chunk).reshape(n, 1, chunk)
        for L in res:
            res[L] += residue(O, fr, rt, lanes=L)[1]
    print(f"N={n} rt={rt}: {cols} columns; differ seq vs simd: " +
          ", ".join(f"L={L}: {v}" for L, v in res.items()), flush=True)
