"""Summarize rocprofv3 PMC passes (gpurun_out/prof_<tag>/pmc*/pmc_counter_collection.csv)
into per-dispatch means for the classify kernel; writes <dir>/pmc_summary.json."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
vals = {}
meta = {}
for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
    per = {}
    for row in csv.DictReader(open(f)):
        if "k_classify" not in row["Kernel_Name"]:
            continue
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        meta["kernel"] = row["Kernel_Name"]
        meta["vgpr"] = row["VGPR_Count"]
        meta["sgpr"] = row["SGPR_Count"]
        meta["grid"] = row["Grid_Size"]
        meta["wg"] = row["Workgroup_Size"]
    for (disp, name), v in per.items():
        vals.setdefault(name, []).append(v)
out = {"meta": meta, "counters": {k: statistics.mean(v) for k, v in sorted(vals.items())},
       "dispatches": {k: len(v) for k, v in vals.items()}}
json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
