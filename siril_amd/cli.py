"""Headless entry point: `python -m siril_amd.cli stack <seq> rej w 3 3 [-nonorm | -norm=addscale [-fastnorm]] -32b [-out=file]`
(the scripting command of Siril's siril-cli for the stacking step; see
siril_amd/sequence.py).  Prints the output path and the rejection totals."""
import sys
import time


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] != "stack":
        print(__doc__, file=sys.stderr)
        return 2
    from siril_amd.sequence import run_command
    t0 = time.perf_counter()
    out, (lo, hi) = run_command(" ".join(argv))
    print(f"Stacked to {out} in {time.perf_counter() - t0:.3f} s; rejected low {lo}, high {hi}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
