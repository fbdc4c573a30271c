"""Per-kernel HBM traffic of one bench step from rocprofv3 --pmc CSVs.

usage: python scripts/pmc_traffic_summary.py CONFIG DIR [DIR ...]

Only the library's kernels (demangled names in namespace sgpu::) count; the
torch kernels that build the synthetic input are left out.  Bytes per
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) doubled (gfx950 tallies the 128-B
requests of wide streaming reads at 64 B), WRITE_SIZE as is; other access
widths are uncalibrated there, so `fetch_kb_raw` is kept beside the doubled
figure.  `scope` sums the kernels bench.py's roofline for CONFIG covers
(bench.AUX_TRAFFIC_SCOPE); the record carries the hash of the sources those
kernels are built from so that a stale profile is ignored.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)\(", name)
    return m.group(1) if m else name.split("(")[0]


def main():
    cfg, dirs = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: {"dispatches": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "n_fetch": 0, "n_write": 0})
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if "sgpu::" not in k:
                    continue
                c = row["Counter_Name"]
                if c not in ("FETCH_SIZE", "WRITE_SIZE"):
                    continue
                e = per[short(k)]
                e[c] += float(row["Counter_Value"])
                e["n_fetch" if c == "FETCH_SIZE" else "n_write"] += 1
    import bench
    scope = bench.AUX_TRAFFIC_SCOPE.get(cfg, "")
    kernels, total, in_scope = {}, 0, 0
    for k, e in sorted(per.items(), key=lambda kv: -(2 * kv[1]["FETCH_SIZE"] + kv[1]["WRITE_SIZE"])):
        nb = int(2 * e["FETCH_SIZE"] * 1024 + e["WRITE_SIZE"] * 1024)     # totals over the step
        n = max(e["n_fetch"], e["n_write"])
        kernels[k] = {"dispatches": n, "bytes_per_step": nb, "bytes_per_dispatch": nb // max(1, n),
                      "fetch_kb_raw": round(e["FETCH_SIZE"], 1), "write_kb": round(e["WRITE_SIZE"], 1)}
        total += nb
        if scope and re.search(scope, k):
            in_scope += nb
    out = {"config": cfg, "source_hash": bench.aux_source_hash(cfg), "steps": 1, "scope_regex": scope,
           "bytes_per_step_scope": in_scope, "bytes_per_step_all": total, "kernels": kernels}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
