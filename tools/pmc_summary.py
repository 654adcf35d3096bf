#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_lds_valu.sh) per workload and kernel.

Derived figures (gfx950; SQ_*_CYCLES and SQ_ACTIVE_INST_* count quad-cycles, MI355X_MICROARCH.md):
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE   (extra LDS cycles per LDS cycle)
  valu_lane_utilisation  = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   (divergence: 1 = no masked lanes)
  valu_insts_per_wave, lds_insts_per_wave, wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES, ...
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for d in sorted(glob.glob(os.path.join(root, "*_*"))):
    if not os.path.isdir(d):
        continue
    wl = os.path.basename(d).split("_")[0]
    agg = out.setdefault(wl, collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("shp::", "")
            if k.startswith("k_"):
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
res = {"method": "rocprofv3 --pmc, two passes of 8 SQ counters per workload (tools/pmc_lds_valu.sh); "
                 "sums over every dispatch of the run", "workloads": {}}
for wl, ks in out.items():
    wr = res["workloads"][wl] = {}
    for k, c in ks.items():
        e = {n: v for n, v in sorted(c.items())}
        w = c.get("SQ_WAVES", 0)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("SQ_ACTIVE_INST_VALU"):
            e["valu_lane_utilisation"] = c.get("SQ_THREAD_CYCLES_VALU", 0) / (64.0 * c["SQ_ACTIVE_INST_VALU"])
        if c.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
            e["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            e["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        if w:
            e["lds_insts_per_wave"] = c.get("SQ_INSTS_LDS", 0) / w
        wr[k] = e
print(json.dumps(res, indent=1))
