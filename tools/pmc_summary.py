"""Summarize rocprofv3 PMC passes (gpurun_out/prof_<tag>/pmc*/pmc_counter_collection.csv)
into per-dispatch means for the kernel named by argv[2] (default k_classify); writes <dir>/pmc_summary.json and
<dir>/traffic.json (HBM-side bytes per launch, corrected as MI355X_MICROARCH.md's
HBM section prescribes: FETCH_SIZE is KiB of 64-B-tallied 128-B requests on gfx950,
so it is doubled; WRITE_SIZE is taken as reported).  Infinity-Cache hits are
included in these counters (they count L2 -> fabric requests)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
KSUB = sys.argv[2] if len(sys.argv) > 2 else "k_classify"
CONF = sys.argv[3] if len(sys.argv) > 3 else "gpu"
vals = {}
meta = {}
for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
    per = {}
    for row in csv.DictReader(open(f)):
        if KSUB not in row["Kernel_Name"]:
            continue
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        meta["kernel"] = row["Kernel_Name"]
        meta["vgpr"] = row.get("VGPR_Count") or row.get("Arch_VGPR_Count")
        meta["sgpr"] = row.get("SGPR_Count")
        meta["grid"] = row["Grid_Size"]
        meta["wg"] = row["Workgroup_Size"]
        meta["lds"] = row.get("LDS_Block_Size") or row.get("Lds_Size")
    for (disp, name), v in per.items():
        vals.setdefault(name, []).append(v)
c = {k: statistics.mean(v) for k, v in sorted(vals.items())}
out = {"meta": meta, "counters": c, "dispatches": {k: len(v) for k, v in vals.items()}}
json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    fetch = 2.0 * c["FETCH_SIZE"] * 1024.0
    write = c["WRITE_SIZE"] * 1024.0
    t = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes_corrected": round(fetch),
         "write_bytes": round(write), "kernel": meta.get("kernel"),
         "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, tools/pmc_driver.py "
                   f"(CGPU_PMC_CONFIG={CONF}, 64M-tuple launches); FETCH_SIZE doubled per "
                   "MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B)"}
    if "TCC_HIT_sum" in c:
        t["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    json.dump(t, open(os.path.join(d, "traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
