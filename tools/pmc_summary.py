"""Summarize rocprofv3 PMC passes of one bench.py workload.

    python3 tools/pmc_summary.py <dir> <config> <skip_steps> <steps>

<dir>/pmc*/pmc_counter_collection.csv hold separate --pmc passes of
`bench.py --config <config> --warmup W --steps K` (tools/profile.sh).  Every
pass dispatches the same kernels in every step, so per kernel name the
dispatches split evenly into skip_steps + steps steps; the first skip_steps
steps (warmup, and the popularity-rebalance step of configs 2 / 5) are
dropped and the rest averaged.

Writes <dir>/pmc_summary.json (per kernel: dispatches per step, counter means
per dispatch) and <dir>/traffic.json:
  hbm_bytes_per_step   HBM-side bytes of ALL kernels of one step (the
                       bench's kernel_ms spans the same launches)
  hbm_bytes_per_launch the same for the dominant kernel alone, per dispatch
corrected as MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE is KiB
of 128-B requests tallied at 64 B on gfx950, so it is doubled; WRITE_SIZE is
taken as reported.  Infinity-Cache hits are included (the counters count
L2 -> fabric requests).  Both files carry the identity of the library the
passes loaded (cilium_amd.build.lib_identity): bench.py prints a traffic
figure only when it loaded that same library.
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cilium_amd.build import lib_identity  # noqa: E402

d, conf = sys.argv[1], sys.argv[2]
skip, steps = int(sys.argv[3]), int(sys.argv[4])
total_steps = skip + steps

# per pass: kernel -> dispatch id -> counter -> value (summed over instances)
per_kernel = {}
non_step = {}
meta = {}
for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
    rows = {}
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        disp = int(row["Dispatch_Id"])
        rows.setdefault(k, {}).setdefault(disp, {})
        c = row["Counter_Name"]
        rows[k][disp][c] = rows[k][disp].get(c, 0.0) + float(row["Counter_Value"])
        meta.setdefault(k, {"vgpr": row.get("VGPR_Count") or row.get("Arch_VGPR_Count"),
                            "sgpr": row.get("SGPR_Count"), "grid": row.get("Grid_Size"),
                            "wg": row.get("Workgroup_Size"),
                            "lds": row.get("LDS_Block_Size") or row.get("Lds_Size")})
    for k, disps in rows.items():
        ids = sorted(disps)
        if len(ids) % total_steps:
            # a one-off launch (the rebalance's slot init, a table upload):
            # not part of a step
            non_step[k] = len(ids)
            continue
        per_step = len(ids) // total_steps
        kept = ids[skip * per_step:]
        ent = per_kernel.setdefault(k, {"dispatches_per_step": per_step, "counters": {}})
        names = {c for i in kept for c in disps[i]}
        for c in names:
            ent["counters"][c] = statistics.mean(disps[i].get(c, 0.0) for i in kept)


def bytes_of(c):
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return None
    return 2.0 * c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0


ident = lib_identity()
summary = {"config": conf, "skip_steps": skip, "steps": steps, "library": ident,
           "kernels": {k: dict(v, meta=meta.get(k)) for k, v in sorted(per_kernel.items())},
           "non_step_dispatches": non_step}
json.dump(summary, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)

step_fetch = step_write = 0.0
dom, dom_b = None, -1.0
complete = True
for k, v in per_kernel.items():
    b = bytes_of(v["counters"])
    if b is None:
        complete = False
        continue
    step_fetch += v["dispatches_per_step"] * b[0]
    step_write += v["dispatches_per_step"] * b[1]
    if v["dispatches_per_step"] * (b[0] + b[1]) > dom_b:
        dom, dom_b = k, v["dispatches_per_step"] * (b[0] + b[1])
if complete and per_kernel:
    c = per_kernel[dom]["counters"]
    fb, wb = bytes_of(c)
    t = {"config": conf, "hbm_bytes_per_step": round(step_fetch + step_write),
         "fetch_bytes_per_step": round(step_fetch), "write_bytes_per_step": round(step_write),
         "dominant_kernel": dom, "hbm_bytes_per_launch": round(fb + wb),
         "fetch_bytes_corrected": round(fb), "write_bytes": round(wb),
         "library": ident,
         "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py --config "
                   f"{conf} ({skip} warmup steps dropped, {steps} averaged); FETCH_SIZE doubled per "
                   "MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B)"}
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        t["l2_hit_rate_dominant"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    if "TCC_EA0_ATOMIC_sum" in c:
        t["memory_side_atomics_dominant"] = round(c["TCC_EA0_ATOMIC_sum"])
    # whole-step sums over every kernel of a step (bench.py's atomic floor)
    def step_sum(name):
        vals = [v["dispatches_per_step"] * v["counters"][name] for v in per_kernel.values()
                if name in v["counters"]]
        return round(sum(vals)) if vals else None
    t["memory_side_atomics_per_step"] = step_sum("TCC_EA0_ATOMIC_sum")
    hits, miss = step_sum("TCC_HIT_sum"), step_sum("TCC_MISS_sum")
    t["l2_requests_per_step"] = hits + miss if hits is not None and miss is not None else None
    t["l2_misses_per_step"] = miss
    json.dump(t, open(os.path.join(d, "traffic.json"), "w"), indent=1)
print(json.dumps({k: v["dispatches_per_step"] for k, v in per_kernel.items()}, indent=1))
