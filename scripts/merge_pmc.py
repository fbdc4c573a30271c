"""Merge gpurun_out/<TAG>/<DIR>/summary.json (scripts/pmc_summary.py) into
profiles/pmc_traffic.json under its config, keeping a committed copy
profiles/<TAG>_pmc_<config>.json.  usage: python scripts/merge_pmc.py TAG DIR"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, sub = sys.argv[1], sys.argv[2]
t = json.load(open(os.path.join(ROOT, "gpurun_out", tag, sub, "summary.json")))
keep = os.path.join("profiles", f"{tag}_pmc_{t['config']}.json")
json.dump(t, open(os.path.join(ROOT, keep), "w"), indent=1)
dst = os.path.join(ROOT, "profiles", "pmc_traffic.json")
out = json.load(open(dst)) if os.path.exists(dst) else {}
t["source"] = f"{keep} (rocprofv3 --pmc, one step)"
prev = out.get(t["config"], {})
for k in ("bytes_per_launch",):            # traffic of an earlier pass of the same sources
    if k in prev and k not in t and prev.get("kernel_source_hash") == t.get("kernel_source_hash"):
        t[k] = prev[k]
out[t["config"]] = t
json.dump(out, open(dst, "w"), indent=1)
print(t["config"], t.get("valu_wave_insts_step"), t.get("valu_lane_utilisation_step"), t.get("mfma_busy_frac"))
