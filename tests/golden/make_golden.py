"""Generate tests/golden/columns.npz: per-pixel columns and the oracle's
mean_and_reject / quickmedian results for every rejection type.  These are
SELF-GENERATED from the restatement (oracle/stack_ref.c), not reference
outputs; they pin the restatement against regressions and feed the GPU
parity tests.  Run: python tests/golden/make_golden.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

NMAX = 400


def column(rng, n, kind):
    x = (0.05 + 0.005 * rng.standard_normal(n)).astype(np.float32)
    if kind in (1, 2, 3):
        m = rng.random(n) < 0.05
        x[m] += rng.uniform(0.2, 0.6, int(m.sum())).astype(np.float32)
    if kind in (2, 3):
        x[rng.random(n) < 0.1] = 0
    if kind == 3:
        m = rng.random(n) < 0.3
        x[m] = rng.uniform(0, 1, int(m.sum())).astype(np.float32)
    if kind == 4:
        x[:] = np.float32(0.25)          # constant column
    if kind == 5:
        x = np.round(x * 40) / 40        # many ties
    return np.clip(x, 0, 1).astype(np.float32)


def main():
    rng = np.random.default_rng(20260821)
    rows = []
    sizes = list(range(2, 26)) + [31, 32, 33, 64, 100, 128, 129, 256, 400]
    for rt in [0, 1, 2, 3, 4, 5, 6, 7, 16]:
        sigs = [(0.32, 0.05)] if rt == 7 else ([(0.2, 0.1), (1.0, 1.0)] if rt == 1 else [(3.0, 3.0), (2.5, 2.5), (1.0, 1.0)])
        for sig in sigs:
            for n in sizes:
                if rt == 7 and n < 3:
                    continue
                for kind in range(6):
                    c = column(rng, n, kind)
                    if rt == 16:
                        r, lo, hi = O.stack_column(c, 0, sig, method=1)
                    else:
                        r, lo, hi = O.stack_column(c, rt, sig)
                    rows.append((c, n, rt, sig, np.float32(r), (lo, hi)))
    cols = np.zeros((len(rows), NMAX), np.float32)
    for i, r in enumerate(rows):
        cols[i, :r[1]] = r[0]
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "columns.npz"),
                        cols=cols, n=np.array([r[1] for r in rows], np.int32),
                        rtype=np.array([r[2] for r in rows], np.int32),
                        sig=np.array([r[3] for r in rows], np.float32),
                        expect=np.array([r[4] for r in rows], np.float32),
                        rej=np.array([r[5] for r in rows], np.int32))
    print(len(rows), "vectors")


if __name__ == "__main__":
    main()
