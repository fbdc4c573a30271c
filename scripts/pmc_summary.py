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
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # VALU issue utilisation: a wave64 VALU instruction occupies its SIMD
        # 4 cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
        cycles = avg["GRBM_GUI_ACTIVE"] / 8.0
        out["valu_busy"] = round(avg["SQ_INSTS_VALU"] * 4.0 / (cycles * 1024.0), 4)
        out["valu_insts_per_wave"] = round(avg["SQ_INSTS_VALU"] / max(1.0, avg.get("SQ_WAVES", 1.0)), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
