"""Merge gpurun_out/<TAG>/tr_<config>/traffic.json records into
profiles/pmc_traffic_aux.json (the per-step HBM traffic bench.py reports).
usage: python scripts/merge_traffic.py TAG"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
dst = os.path.join(ROOT, "profiles", "pmc_traffic_aux.json")
out = json.load(open(dst)) if os.path.exists(dst) else {}
for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "tr_*", "traffic.json"))):
    t = json.load(open(f))
    keep = os.path.join("profiles", f"{tag}_traffic_{t['config']}.json")      # committed copy
    json.dump(t, open(os.path.join(ROOT, keep), "w"), indent=1)
    t["source"] = f"{keep} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one step)"
    out[t["config"]] = t
    print(t["config"], t["bytes_per_step_scope"])
json.dump(out, open(dst, "w"), indent=1)
