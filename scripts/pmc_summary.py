"""Summarise rocprofv3 --pmc CSVs for one kernel (per-dispatch averages).

usage: python scripts/pmc_summary.py KERNEL_SUBSTRING DIR [DIR ...]
HBM traffic per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads half the
bytes of a wide coalesced stream on gfx950 -> doubled; WRITE_SIZE exact.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirs, ksub):
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if ksub in row.get("Kernel_Name", ""):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ksub, dirs = sys.argv[1], sys.argv[2:]
    avg = load(dirs, ksub)
    out = {"kernel": ksub, "per_dispatch": avg}
    if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
        out["bytes_per_launch"] = int(2 * avg.get("FETCH_SIZE", 0) * 1024 + avg.get("WRITE_SIZE", 0) * 1024)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
