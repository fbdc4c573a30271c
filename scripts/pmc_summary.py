"""Summarise rocprofv3 --pmc CSVs for one kernel (per-dispatch averages).

usage: python scripts/pmc_summary.py KERNEL_SUBSTRING CONFIG DIR [DIR ...]

HBM traffic per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads half the
bytes of a wide coalesced stream on gfx950 -> doubled; WRITE_SIZE exact.
VALU issue: SQ_INSTS_VALU wave-instructions per dispatch against the chip's
issue peak (1024 SIMDs x 2.4 GHz / 2 cycles per wave64 f32 instruction =
1.2288e12 wave-instructions/s, MI355X_MICROARCH.md: v_fma_f32 wave64 2 cyc
throughput); lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x
SQ_ACTIVE_INST_VALU) (active lanes per issued VALU instruction: the divergence
waste of data-dependent loops).  The record carries the hash of the kernel
sources (bench.kernel_source_hash) so bench.py ignores a stale profile.
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VALU_PEAK = 1024 * 2.4e9 / 2


def load(dirs, ksub):
    vals = defaultdict(list)
    names = set()
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if ksub in row.get("Kernel_Name", ""):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                    names.add(row["Kernel_Name"])
    load.totals = {k: sum(v) for k, v in vals.items()}      # every matching dispatch of the run
    return {k: sum(v) / len(v) for k, v in vals.items()}, sorted(names)


def main():
    ksub, cfg, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    avg, names = load(dirs, ksub)
    from bench import kernel_source_hash
    try:
        head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                              cwd=ROOT).stdout.strip() or None
    except OSError:
        head = None
    out = {"config": cfg, "kernel": names[0] if names else ksub, "kernel_source_hash": kernel_source_hash(),
           "commit": head, "per_dispatch": avg}
    if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
        out["bytes_per_launch"] = int(2 * avg.get("FETCH_SIZE", 0) * 1024 + avg.get("WRITE_SIZE", 0) * 1024)
    tot = getattr(load, "totals", {})
    if len(names) > 1 and "SQ_INSTS_VALU" in tot:
        # several kernels of one step (the moment path: prep, rounds, tails):
        # the run is one step (bench --steps 1 --warmup 0), so the totals are
        # per step; lane utilisation weighted by instructions
        out["kernels"] = names
        out["valu_wave_insts_step"] = tot["SQ_INSTS_VALU"]
        if tot.get("SQ_THREAD_CYCLES_VALU") and tot.get("SQ_ACTIVE_INST_VALU"):
            out["valu_lane_utilisation_step"] = round(tot["SQ_THREAD_CYCLES_VALU"] / (64.0 * tot["SQ_ACTIVE_INST_VALU"]), 4)
        if tot.get("SQ_WAIT_ANY") and tot.get("SQ_WAVE_CYCLES"):
            out["wait_any_frac_step"] = round(tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"], 4)
    if "SQ_INSTS_VALU" in avg:
        out["valu_wave_insts"] = avg["SQ_INSTS_VALU"]
        out["valu_peak_wave_insts_per_s"] = VALU_PEAK
        out["valu_insts_per_wave"] = round(avg["SQ_INSTS_VALU"] / max(1.0, avg.get("SQ_WAVES", 1.0)), 1)
    if avg.get("SQ_THREAD_CYCLES_VALU") and avg.get("SQ_ACTIVE_INST_VALU"):
        # active lanes per issued VALU instruction / 64 (gfx950 has no
        # SQ_INST_CYCLES_VALU; SQ_ACTIVE_INST_VALU ~= SQ_INSTS_VALU there)
        out["valu_lane_utilisation"] = round(avg["SQ_THREAD_CYCLES_VALU"] / (64.0 * avg["SQ_ACTIVE_INST_VALU"]), 4)
    if "GRBM_GUI_ACTIVE" in avg:
        out["gui_active_cycles_per_xcd"] = avg["GRBM_GUI_ACTIVE"] / 8.0
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            # matrix-core busy cycles (summed over the SIMDs) over the
            # dispatch's cycles on all 1024 SIMDs
            out["mfma_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8.0 * 1024), 4)
    cfg_src = os.environ.get("PMC_SOURCE_CONFIG")
    if cfg_src:
        from bench import aux_source_hash
        out["kernel_source_hash"] = aux_source_hash(cfg_src)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
