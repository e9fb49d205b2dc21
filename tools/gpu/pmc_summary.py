"""Average rocprofv3 --pmc counter values per kernel and dispatch (tools/gpu/pmc.sh output).

    python tools/gpu/pmc_summary.py gpurun_out/pmc > profiles/<round>/pmc_counters.json
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for path in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
    per_dispatch = collections.defaultdict(float)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?").split("(")[0]
            key = (k, row.get("Dispatch_Id"), row.get("Counter_Name"))
            per_dispatch[key] += float(row.get("Counter_Value", 0) or 0)  # summed over XCD/SE instances
            meta.setdefault(k, {"grid": row.get("Grid_Size"), "vgpr": row.get("VGPR_Count"),
                                "agpr": row.get("Accum_VGPR_Count"), "scratch": row.get("Scratch_Size")})
    for (k, _, c), v in per_dispatch.items():
        acc[k][c].append(v)
out = {"note": "rocprofv3 --pmc, one counter group per run (tools/gpu/pmc.sh), one unloaded 64512-set verify "
               "call (tools/gpu/roof_call.py); values averaged per dispatch",
       "per_dispatch": {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in sorted(acc.items())},
       "kernel_meta": meta}
d = out["per_dispatch"]
for k, cs in d.items():
    if cs.get("SQ_WAVE_CYCLES"):
        cs["frac_valu_active"] = cs.get("SQ_ACTIVE_INST_VALU", 0) / cs["SQ_WAVE_CYCLES"]
        cs["frac_wait_any"] = cs.get("SQ_WAIT_ANY", 0) / cs["SQ_WAVE_CYCLES"]
print(json.dumps(out, indent=1))
