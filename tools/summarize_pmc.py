"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) for one kernel into JSON.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half of
the bytes of a wide (16 B/lane) coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KB)
is exact for 16 B/lane stores.  Usage: summarize_pmc.py PMCDIR KERNEL_SUBSTR OUT.json [FLOPS]"""
import csv
import glob
import json
import sys

d, sub, out = sys.argv[1], sys.argv[2], sys.argv[3]
flops = float(sys.argv[4]) if len(sys.argv) > 4 else None
vals = {}
for f in glob.glob(d + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
res = {"kernel_substr": sub, "dispatches": {k: len(v) for k, v in vals.items()}, "counters_avg": avg}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    res["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
    res["fetch_bytes_corrected_x2"] = avg["FETCH_SIZE"] * 1024 * 2
    res["write_bytes"] = avg["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = res["fetch_bytes_corrected_x2"] + res["write_bytes"]
    res["note"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts half the bytes of 16-B/lane "
                   "coalesced reads); gathered table rows are served partly from the 256 MB Infinity Cache, "
                   "which the memory-side counters include")
if flops:
    res["flops_per_launch"] = flops
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
